"""The fused MLP head (pg_mlp_l1_head, ABI 12; pg_mlp_l1_head_ex with W1's pieces kept by
pg_adam_apply_l1, ABI 13): liner1's forward, the head (liner2 +
sigmoid + train/val multi_loss + dZ + dA4) and liner1's input gradient through the top SAGE
layer's leaky_relu, in one launch. It computes both products exactly as the three-piece
GEMM does (same split, same 16-k steps and MFMA sequence, zero past K), so a TrainEngine
step with it must equal the same step with the separate launches (two pg_gemm_f32 calls +
pg_mlp_head) BIT FOR BIT: A4, dA4, prob, dZ, both losses, the top layer's dY and every
gradient. Shapes: the cfg2 dims at full size (N = 24,041: 752 blocks, a ragged last block),
the reference dims (F3 = 200: a K tail inside a 16-k step, one partial 256-column chunk),
cfg3's hidden 512 (two K chunks and two column chunks), a narrow MLP (K1 = 28) and 3
classes, on small random graphs (N not a multiple of 32). The oracle parity of the step
itself is tests/test_gpu_engine.py / test_gpu_fullsize.py (which run the fused path)."""
import numpy as np
import pytest
import torch

from conftest import random_graph

pytestmark = pytest.mark.gpu


def _engine_pair(dims, n, e, seed):
    import oracle
    import plagnn

    src, dst = random_graph(n, e, seed, self_loop=False)
    rng = np.random.default_rng(seed)
    x = torch.from_numpy(rng.standard_normal((n, dims[0])).astype(np.float32))
    labels = torch.from_numpy((rng.random((n, dims[-1])) < 0.3).astype(np.float32))
    w = oracle.weight_cal(labels.numpy().astype(np.float64))
    idx = rng.permutation(n)
    tr, va = idx[: n // 2], idx[n // 2: n // 2 + n // 5]
    loops = np.arange(n)
    g = plagnn.CSRGraph(np.concatenate([src, loops]), np.concatenate([dst, loops]), n)
    from plagnn.model import GNN

    torch.manual_seed(seed)
    params = GNN(list(dims)).state_dict()
    out = []
    for fused in (True, False):
        cls = type("E", (plagnn.TrainEngine,), {"FUSED_L1_HEAD": fused})
        out.append(cls(g, x, labels, dims, w, tr, va, device="cuda", params=params))
    return out


def _run(eng):
    eng.forward()
    eng.backward()
    torch.cuda.synchronize()
    top = eng.L - 1
    r = {"A4": eng.A4, "dA4": eng.dA4, "prob": eng.prob, "dZ": eng.dZ, "loss": eng.loss,
         "dY_top": eng.DYP[top][:, :eng.pd[top + 1]]}
    r.update({"grad." + k: v for k, v in eng.grads().items()})
    return {k: v.detach().cpu().clone() for k, v in r.items()}


@pytest.mark.parametrize("dims,n,e", [
    ((31, 24, 20, 16, 10, 12), 600, 6000),
    ((64, 48, 200, 100, 12), 1000, 12000),          # F3 = 200: K tail, a partial column chunk
    ((40, 512, 100, 12), 777, 7000),                 # F3 = 512: two K chunks, two column chunks
    ((33, 60, 28, 3), 97, 900),                      # K1 = 28, C = 3, 4 blocks (last ragged)
])
def test_fused_head_equals_separate_launches_bitwise(dims, n, e):
    fused, sep = _engine_pair(dims, n, e, seed=len(dims) + n)
    assert fused._l1_fused() and not sep._l1_fused()
    a, b = _run(fused), _run(sep)
    for k in b:
        assert torch.equal(a[k], b[k]), f"{k}: fused != separate (max diff {(a[k] - b[k]).abs().max().item():.3e})"
    assert fused.flops_per_step() + fused.head_flops_per_step() == sep.flops_per_step()


@pytest.mark.parametrize("dims,n,e", [((31, 24, 20, 16, 10, 12), 600, 6000), ((64, 48, 200, 100, 12), 1000, 12000)])
def test_fused_head_steps_equal_separate_bitwise(dims, n, e):
    """Three whole training steps: the fused engine's head reads W1's pieces that its Adam
    (pg_adam_apply_l1) rewrote, the separate engine's GEMMs split W1 themselves; parameters,
    moments and losses stay bitwise equal."""
    fused, sep = _engine_pair(dims, n, e, seed=n)
    assert fused.l1_pieces is not None and sep.l1_pieces is None
    for _ in range(3):
        fused.step_eager()
        sep.step_eager()
    torch.cuda.synchronize()
    for a, b in ((fused.flat, sep.flat), (fused.m, sep.m), (fused.v, sep.v)):
        assert torch.equal(a, b)
    assert fused.losses() == sep.losses()


@pytest.mark.parametrize("F3,K1,ldw1,off", [(256, 100, 256, 1000), (200, 28, 204, 37), (512, 128, 512, 0)])
def test_adam_apply_l1_equals_adam_and_split(F3, K1, ldw1, off):
    """pg_adam_apply_l1 == pg_adam_apply on every parameter and moment (bitwise), and the
    pieces it leaves == pg_mlp_l1_split of the updated W1 (bitwise, pads included)."""
    from plagnn import _lib

    L = _lib.lib()
    g = torch.Generator(device="cpu").manual_seed(F3 + K1)
    n = off + K1 * ldw1 + 333
    p0 = torch.randn(n, generator=g).cuda()
    gr = torch.randn(n, generator=g).cuda()
    m0 = torch.randn(n, generator=g).cuda() * 0.1
    v0 = torch.rand(n, generator=g).cuda() * 0.01
    st = torch.zeros(4, device="cuda")
    assert L.pg_adam_prepare(st.data_ptr(), 1e-3, 0.9, 0.999, None) == 0
    nb = int(L.pg_mlp_l1_pieces_bytes(F3, K1))
    pieces = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    ref = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    W1 = lambda p: p[off:off + K1 * ldw1].view(K1, ldw1)  # noqa: E731
    # the pieces start as the split of the old W1 (the pads are the split's zeros)
    assert L.pg_mlp_l1_split(W1(p0).data_ptr(), ldw1, F3, K1, pieces.data_ptr(), None) == 0
    a = [t.clone() for t in (p0, m0, v0)]
    b = [t.clone() for t in (p0, m0, v0)]
    assert L.pg_adam_apply_l1(a[0].data_ptr(), gr.data_ptr(), a[1].data_ptr(), a[2].data_ptr(), n, st.data_ptr(),
                              0.9, 0.999, 1e-8, 0.0, off, ldw1, F3, K1, pieces.data_ptr(), None) == 0
    assert L.pg_adam_apply(b[0].data_ptr(), gr.data_ptr(), b[1].data_ptr(), b[2].data_ptr(), n, st.data_ptr(),
                           0.9, 0.999, 1e-8, 0.0, None) == 0
    assert L.pg_mlp_l1_split(W1(b[0]).data_ptr(), ldw1, F3, K1, ref.data_ptr(), None) == 0
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert not torch.equal(a[0], p0)
    assert torch.equal(pieces, ref)
    # W1 outside the n parameters, misaligned pieces: refused
    assert L.pg_adam_apply_l1(a[0].data_ptr(), gr.data_ptr(), a[1].data_ptr(), a[2].data_ptr(), n, st.data_ptr(),
                              0.9, 0.999, 1e-8, 0.0, n - 10, ldw1, F3, K1, pieces.data_ptr(), None) != 0
    assert L.pg_adam_apply_l1(a[0].data_ptr(), gr.data_ptr(), a[1].data_ptr(), a[2].data_ptr(), n, st.data_ptr(),
                              0.9, 0.999, 1e-8, 0.0, off, ldw1, F3, K1, pieces.data_ptr() + 16, None) != 0


def test_fused_head_full_size_cfg2_bitwise_and_replay():
    """cfg2 at full size (N = 24,041, 3 x 256, MLP 256 -> 100 -> 12): fused == separate bit
    for bit after a forward + backward, and the fused engine's captured step replays equal
    its eager steps."""
    import plagnn
    from plagnn import workload as W

    wl = W.build("cfg2", device="cuda")
    engs = []
    for fused in (True, False):
        cls = type("E", (plagnn.TrainEngine,), {"FUSED_L1_HEAD": fused})
        engs.append(cls(wl.graph(), torch.from_numpy(wl.ds.feat), torch.from_numpy(wl.ds.loc.astype(np.float32)),
                        wl.dims, wl.class_weight, wl.train_index, wl.val_index, device="cuda", seed=0))
    a, b = _run(engs[0]), _run(engs[1])
    for k in b:
        assert torch.equal(a[k], b[k]), f"{k}: fused != separate"
    # graph replay == eager on the fused engine (two more steps each, from equal states)
    e0 = engs[0]
    e0.adam()
    cls = type("E", (plagnn.TrainEngine,), {"FUSED_L1_HEAD": True})
    e1 = cls(wl.graph(), torch.from_numpy(wl.ds.feat), torch.from_numpy(wl.ds.loc.astype(np.float32)), wl.dims,
             wl.class_weight, wl.train_index, wl.val_index, device="cuda", params=e0.state_dict())
    e1.m.copy_(e0.m)
    e1.v.copy_(e0.v)
    e1.adam_state.copy_(e0.adam_state)
    e0.capture(warmup=0)
    for _ in range(2):
        e0.step()
        e1.step_eager()
    torch.cuda.synchronize()
    assert torch.equal(e0.flat, e1.flat)
    assert e0.losses() == e1.losses()


def test_mlp_l1_head_rejects_bad_shapes():
    from plagnn import _lib

    L = _lib.lib()
    ws = torch.zeros(int(L.pg_mlp_l1_head_workspace(64, 12, 256, 104)), dtype=torch.uint8, device="cuda")
    inp = torch.zeros(256, 256, device="cuda")   # every input operand (zeros), in bounds for 64 rows
    outs = [torch.zeros(64, 256, device="cuda") for _ in range(3)]  # A4, dA4, dH3
    loss = torch.zeros(2, device="cuda")
    rs = torch.zeros(64, dtype=torch.int8, device="cuda")
    p = inp.data_ptr()

    def args(F3, K1, C):
        return (p, 256, 64, F3, p, 256, p, K1, outs[0].data_ptr(), 256, p, 256, p, C, p, 256, p, rs.data_ptr(), 0, 0,
                None, 0, None, 0, outs[1].data_ptr(), 256, outs[2].data_ptr(), 256, 0.01, loss.data_ptr(),
                ws.data_ptr(), ws.numel(), None, 0.0, 0.0, 0.0, None)

    assert L.pg_mlp_l1_head(*args(256, 104, 12)) == 0
    torch.cuda.synchronize()
    assert not outs[0].any() and not outs[2].any()
    for bad in ((254, 104, 12), (256, 129, 12), (256, 104, 17)):
        assert L.pg_mlp_l1_head(*args(*bad)) != 0
    short = list(args(256, 104, 12))
    short[-6] = ws.numel() - 1  # workspace one byte short
    assert L.pg_mlp_l1_head(*short) != 0


def test_adam_scalars_folded_into_head_equal_separate_prepare():
    """FOLD_ADAM_PREP: inside a training step the fused head's final kernel forms the Adam
    scalars (pg_adam_prepare's work). Three steps (eager, then captured replays) must leave
    the parameters, moments and step count bitwise where the separate prepare launch leaves
    them; a bare forward() must not advance the step count."""
    import plagnn

    dims = (31, 24, 20, 16, 10, 12)
    engs = []
    for fold in (True, False):
        e, _ = _engine_pair(dims, 600, 6000, seed=5)
        e.FOLD_ADAM_PREP = fold
        engs.append(e)
    for e in engs:
        e.step_eager()
        e.capture(warmup=1)
        e.step()
        e.step()
    torch.cuda.synchronize()
    a, b = engs
    for name in ("flat", "m", "v", "adam_state"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert a.adam_state[0].item() == 4.0  # 1 eager + 1 capture warm-up + 2 replays
    before = a.adam_state.clone()
    a.forward()
    torch.cuda.synchronize()
    assert torch.equal(a.adam_state, before)
    assert isinstance(a, plagnn.TrainEngine)
