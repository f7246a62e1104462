"""bf16-storage mode (BASELINE configs[4]: bf16 storage, f32 accumulate) — not run by the
reference (fp32 only), so reference-unpinned; pinned here against the fp32 path:

* pg_gemm_bf16 vs a float64 product of the same bf16 operands: f32 outputs within the
  f32-accumulation bound 2e-6 sqrt(K) (|A| |B|); bf16 outputs within one bf16 rounding
  of that. Every transposition (row images and ds_read_b64_tr_b16 k images), ragged
  M / N / K tails, every epilogue, split-K.
* pg_spmm_max_fwd_bf16 / pg_spmm_max_bwd_bf16 vs the fp32 kernels (bit-exact vs the
  oracle) on the bf16 values widened to f32: bit-identical after rounding the fp32
  result to bf16 (the max is a selection; the backward sums in the same f32 order).
"""
import numpy as np
import pytest
import torch

from conftest import hub_graph

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


def _ref(A, B, ta, tb):
    a = A.double().t() if ta else A.double()
    b = B.double().t() if tb else B.double()
    return a @ b, a.abs() @ b.abs()


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(1000, 256, 512), (4104, 520, 264), (200, 72, 1000), (64, 8, 8),
                                   (65544, 520, 136), (36000, 512, 576), (36000, 520, 584)])
# (36000, 512, 576) and (36000, 520, 584) run on 256 x 256 tiles (pick_tile needs K >= 384;
# A B^T there: the ping-pong kernel), the latter with a ragged N and K % 64 != 0 (its
# partial store and K-tail zero fill)
def test_gemm_bf16_f32_out(ta, tb, M, N, K):
    from plagnn import ops

    A = _bf((K, M) if ta else (M, K), M + K)
    B = _bf((N, K) if tb else (K, N), N + 3 * K)
    got = ops.gemm_bf16(A, B, ta, tb, split_k=1).double()
    ref, mag = _ref(A, B, ta, tb)
    bound = 2e-6 * np.sqrt(K) * mag + 1e-30
    assert bool(((got - ref).abs() <= bound).all()), float(((got - ref).abs() / bound).max())


@pytest.mark.parametrize("ta,tb", [(False, True), (True, False), (False, False)])
@pytest.mark.parametrize("M", [3000, 70000])  # 128 x 128 and 256 x 256 tiles
def test_gemm_bf16_bf16_out_epilogues(ta, tb, M):
    from plagnn import _lib, ops

    N, K = 264, 520
    A = _bf((K, M) if ta else (M, K), 5)
    B = _bf((N, K) if tb else (K, N), 6)
    bias = torch.randn(N, device=DEV)
    ref, mag = _ref(A, B, ta, tb)
    tol = 2e-6 * np.sqrt(K) * mag
    # bias + leaky_relu, bf16 out
    got = ops.gemm_bf16(A, B, ta, tb, out_dtype=torch.bfloat16, bias=bias, act=_lib.PG_ACT_LEAKY).double()
    r = ref + bias.double()
    r = torch.where(r > 0, r, r * 0.01)
    assert bool(((got - r).abs() <= r.abs() * 2.0 ** -8 + tol).all())
    # relu
    got = ops.gemm_bf16(A, B, ta, tb, out_dtype=torch.bfloat16, bias=bias, act=_lib.PG_ACT_RELU).double()
    r = (ref + bias.double()).clamp_min(0)
    assert bool(((got - r).abs() <= r.abs() * 2.0 ** -8 + tol).all())
    # fused leaky' with a bf16 activation output, f32 out
    y = _bf((M, N), 7)
    got = ops.gemm_bf16(A, B, ta, tb, act=_lib.PG_ACT_LEAKY, dact=y).double()
    r = torch.where(y.double() > 0, ref, ref * 0.01)
    assert bool(((got - r).abs() <= tol + 1e-30).all())
    # beta = 1 into a bf16 C
    c0 = _bf((M, N), 8)
    c = c0.clone()
    ops.gemm_bf16(A, B, ta, tb, out=c, beta=1.0)
    r = ref + c0.double()
    assert bool(((c.double() - r).abs() <= r.abs() * 2.0 ** -8 + tol).all())


def test_gemm_bf16_rowsum_and_split_k():
    """Weight-gradient shape: dW = dY^T X with K = nodes, both operands k images,
    bias gradient as the row sums of dY^T, split-K with an ordered combine."""
    from plagnn import ops

    Nn, Fo, Fi = 24000, 264, 512
    dY = _bf((Nn, Fo), 11)
    X = _bf((Nn, Fi), 12)
    ref, mag = _ref(dY, X, True, False)
    for sk in (1, 7, None):
        rs = torch.empty(Fo, device=DEV)
        got = ops.gemm_bf16(dY, X, True, False, rowsum=rs, split_k=sk).double()
        assert bool(((got - ref).abs() <= 2e-6 * np.sqrt(Nn) * mag).all()), sk
        rref = dY.double().sum(0)
        assert bool(((rs.double() - rref).abs() <= 2e-6 * np.sqrt(Nn) * dY.double().abs().sum(0)).all()), sk
    a = ops.gemm_bf16(dY, X, True, False, split_k=9)
    b = ops.gemm_bf16(dY, X, True, False, split_k=9)
    assert torch.equal(a, b)  # deterministic


@pytest.mark.parametrize("case", ["grouped", "mixed"])
def test_gemm_bf16_group(case):
    """pg_gemm_bf16_group on the cfg5 step's weight-gradient shapes (K = nodes, both
    operands k images, row sums; liner2's 16 x 104 product runs alone, a 256 x 256 tile
    would waste 39x its area; one part with beta = 1): within the f32-accumulation bound
    of a float64 product of the same bf16 values, deterministic. `mixed` (one part with B
    stored [n][k]) runs every part one by one as pg_gemm_bf16."""
    from plagnn import _lib
    from plagnn._lib import call, ptr

    Nn = 40000
    shapes = [(512, 1024), (504, 504), (512, 1024), (512, 512), (104, 512), (16, 104)]
    parts = (_lib.PgGemmPart * len(shapes))()
    keep = []
    for i, (M, N) in enumerate(shapes):
        tb = case == "mixed" and i == 2
        A = _bf((Nn, M), 40 + i)
        B = _bf((N, Nn) if tb else (Nn, N), 60 + i)
        C = torch.randn(M, N, device=DEV)
        beta = 1.0 if i == 1 else 0.0
        rs = torch.empty(M, device=DEV)
        q = parts[i]
        q.transa, q.transb, q.M, q.N, q.K = 1, int(tb), M, N, Nn
        q.A, q.lda, q.B, q.ldb = ptr(A), A.stride(0), ptr(B), B.stride(0)
        q.beta, q.C, q.ldc, q.rowsum = beta, ptr(C), C.stride(0), ptr(rs)
        keep.append((A, B, tb, C, C.clone(), rs, beta))
    n = len(shapes)
    ws = torch.empty(int(_lib.lib().pg_gemm_bf16_group_workspace(parts, n)), dtype=torch.uint8, device=DEV)
    st = _lib.stream_handle(torch.device(DEV))
    call("pg_gemm_bf16_group", parts, n, ptr(ws), ws.numel(), st)
    first = [(C.clone(), rs.clone()) for (_, _, _, C, _, rs, _) in keep]
    for (_, _, _, C, C0, _, _) in keep:
        C.copy_(C0)
    call("pg_gemm_bf16_group", parts, n, ptr(ws), ws.numel(), st)
    torch.cuda.synchronize()
    for (A, B, tb, C, C0, rs, beta), (c1, r1) in zip(keep, first):
        assert torch.equal(C, c1) and torch.equal(rs, r1)
        ref, mag = _ref(A, B, True, tb)
        assert bool(((C.double() - ref - beta * C0.double()).abs()
                     <= 2e-6 * np.sqrt(Nn) * mag + 1e-6 * beta * C0.double().abs()).all())
        a64 = A.double()
        assert bool(((rs.double() - a64.sum(0)).abs() <= 2e-6 * np.sqrt(Nn) * a64.abs().sum(0)).all())


@pytest.mark.parametrize("ta,tb", [(True, False), (False, False), (True, True)])
def test_gemm_bf16_256_tiles_rowsum_unsplit(ta, tb):
    """256 x 256 tiles without split-K (>= 256 tiles) in the k-image transpositions (the
    two-phase kernel), with the row sums of op(A) and a ragged K tail."""
    from plagnn import ops

    M, N, K = 2056, 8192, 520
    A = _bf((K, M) if ta else (M, K), 21)
    B = _bf((N, K) if tb else (K, N), 22)
    rs = torch.empty(M, device=DEV)
    got = ops.gemm_bf16(A, B, ta, tb, rowsum=rs, split_k=1).double()
    ref, mag = _ref(A, B, ta, tb)
    assert bool(((got - ref).abs() <= 2e-6 * np.sqrt(K) * mag + 1e-30).all())
    a64 = A.double().t() if ta else A.double()
    assert bool(((rs.double() - a64.sum(1)).abs() <= 2e-6 * np.sqrt(K) * a64.abs().sum(1)).all())


def test_gemm_bf16_rejects_unaligned_extents():
    from plagnn import _lib, ops

    A = _bf((64, 20), 1)  # K = 20 not a multiple of 8
    B = _bf((20, 64), 2)
    with pytest.raises(_lib.PlagnnError):
        ops.gemm_bf16(A, B)


@pytest.mark.parametrize("F,weighted", [(64, False), (256, False), (512, True), (1000, False)])
def test_spmm_max_bf16_matches_fp32_kernels(F, weighted):
    import plagnn
    from plagnn import ops

    n = 700
    src, dst = hub_graph(n, 2000, seed=F)
    g = plagnn.CSRGraph(src, dst, n)
    dg = g.on(DEV)
    gen = torch.Generator().manual_seed(F)
    X = torch.randn(n, F, generator=gen)
    X[torch.rand(n, F, generator=gen) < 0.4] = 0.0
    Xb = X.to(torch.bfloat16).to(DEV)
    ew = None
    if weighted:
        ew = dg.edge_weight_slots(torch.rand(g.num_edges, generator=gen) + 0.5)
    out_b, arg_b = ops.spmm_max(dg, Xb, ew)
    out_f, arg_f = ops.spmm_max(dg, Xb.float(), ew)
    assert torch.equal(arg_b, arg_f)
    assert torch.equal(out_b, out_f.to(torch.bfloat16))
    # backward: relu' mask from a bf16 "P", bf16 upstream gradient
    dout = torch.randn(n, F, generator=gen).to(torch.bfloat16).to(DEV)
    mask = Xb
    dx_b = ops.spmm_max_backward(dg, arg_b, dout, ew, mask=mask)
    dx_f = ops.spmm_max_backward(dg, arg_f, dout.float(), ew, mask=mask.float())
    assert dx_b.dtype == torch.bfloat16
    assert torch.equal(dx_b, dx_f.to(torch.bfloat16))


def test_cast_bf16_gather():
    from plagnn import ops

    src = torch.randn(1000, device=DEV)
    idx = torch.tensor([5, -1, 999, 0, 5], dtype=torch.int32, device=DEV)
    got = ops.cast_bf16(src, idx)
    ref = torch.stack([src[5], src.new_zeros(()), src[999], src[0], src[5]]).to(torch.bfloat16)
    assert torch.equal(got, ref)
    assert torch.equal(ops.cast_bf16(src), src.to(torch.bfloat16))
