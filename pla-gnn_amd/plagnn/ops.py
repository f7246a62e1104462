"""Tensor-level operations over the C-ABI, and their autograd wrappers.

Every GPU operation here is a call into libplagnn.so on torch's current stream; there is
no fallback to another implementation. Tensors on the CPU device (the reference's
``-d cpu``, code/main_normal.py:30) go to the library's ``*_cpu`` entry points for the
message passing and to torch-CPU for the dense algebra, as DGL's CPU backend does.
"""
from __future__ import annotations

import weakref
from typing import Optional, Tuple

import torch

from . import _lib
from ._lib import call, ptr
from .graph import DeviceGraph

LEAKY_SLOPE = 0.01  # F.leaky_relu default (code/model.py:21-27)


def round4(n: int) -> int:
    return (n + 3) // 4 * 4


def _ld(t: torch.Tensor) -> int:
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("expected a row-major 2-D tensor with unit column stride")
    return t.stride(0)


def _stream(t: torch.Tensor):
    return _lib.stream_handle(t.device)


_scratch = {}


def _workspace(nbytes: int, device) -> Optional[torch.Tensor]:
    """Library scratch for one call: one buffer per (device, stream), grown on demand and
    reused by every later call on that stream (stream order makes the reuse safe), so the
    drop-in path's autograd functions allocate nothing per call. During HIP-graph capture a
    call gets a fresh buffer from the graph's private pool instead: a cached buffer would
    be shared between the graph's replays and eager calls that can run beside them."""
    if nbytes <= 0:
        return None
    device = torch.device(device)
    if device.type == "cuda" and torch.cuda.is_current_stream_capturing():
        return torch.empty(int(nbytes), dtype=torch.uint8, device=device)
    key = (str(device), torch.cuda.current_stream(device).cuda_stream if device.type == "cuda" else 0)
    buf = _scratch.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(int(nbytes), 1 << 20), dtype=torch.uint8, device=device)
        _scratch[key] = buf
    return buf


def _check_device(dg: DeviceGraph, *ts):
    for t in ts:
        if t is not None and t.device != dg.device:
            raise ValueError(f"tensor on {t.device}, graph on {dg.device}")
        if t is not None and t.dtype not in (torch.float32, torch.bfloat16, torch.int16, torch.int32,
                                             torch.int64):
            raise TypeError(f"unsupported dtype {t.dtype}")


# ------------------------------------------------------------------ message passing
def spmm_max(dg: DeviceGraph, X: torch.Tensor, ew_slots: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None, argpos: Optional[torch.Tensor] = None,
             dead_none: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """out[v] = max over in-edges of X[u] (* w), argpos = winning in-row position.
    DGL update_all(copy_u|u_mul_e, max) (code/model.py:20,22,24). `dead_none`
    (PG_ARG_DEAD_NONE, GPU): a zero maximum records no winner."""
    if X.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError("spmm_max: float32 or bfloat16 features expected")
    bf = X.dtype == torch.bfloat16
    _check_device(dg, X, ew_slots)
    n, F = dg.num_nodes, X.shape[1]
    if X.shape[0] != n:
        raise ValueError(f"spmm_max: X has {X.shape[0]} rows, graph has {n} nodes")
    if out is None:
        out = torch.empty(n, F, dtype=X.dtype, device=X.device)
    if argpos is None:
        argpos = torch.empty(n, F, dtype=dg.arg_dtype, device=X.device)
    g = dg.fwd.struct(ew_slots)
    if bf and not dg.is_cuda:
        raise TypeError("spmm_max: bfloat16 storage runs on the GPU only")
    if dg.is_cuda:
        ws_n = _lib.lib().pg_spmm_max_fwd_workspace(g, F, dg.arg_kind)
        ws = _workspace(ws_n, X.device)
        kind = dg.arg_kind | (_lib.PG_ARG_DEAD_NONE if dead_none else 0)
        call("pg_spmm_max_fwd_bf16" if bf else "pg_spmm_max_fwd", g, ptr(X), _ld(X), F, ptr(out), _ld(out), ptr(argpos), _ld(argpos),
             kind, ptr(ws), ws_n, _stream(X))
    else:
        call("pg_spmm_max_fwd_cpu", g, ptr(X), _ld(X), F, ptr(out), _ld(out), ptr(argpos),
             _ld(argpos), dg.arg_kind)
    return out, argpos


def spmm_max_backward(dg: DeviceGraph, argpos: torch.Tensor, dout: torch.Tensor,
                      ew_slots: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None,
                      dx: Optional[torch.Tensor] = None, fwd_out: Optional[torch.Tensor] = None,
                      dead_none: bool = False) -> torch.Tensor:
    """dX of the max aggregation (DGL GSpMM.backward: scatter_add_ through argX),
    gathered per source in ascending destination order; optional fused relu' mask
    (mask[u,f] > 0). With `fwd_out` (the forward's output; needs mask = the forward's
    input) entries whose maximum is 0 are skipped: they contribute nothing (the mask is
    still applied). `dead_none`: the records come from spmm_max(..., dead_none=True) (the
    same skip made by the forward; needs mask = a relu output >= 0, which is then implied
    and not read)."""
    _check_device(dg, argpos, dout, ew_slots, mask)
    bf = dout.dtype == torch.bfloat16
    if bf and ((mask is not None and mask.dtype != torch.bfloat16) or not dg.is_cuda):
        raise TypeError("spmm_max_backward: bfloat16 storage (GPU) needs a bfloat16 mask")
    n, F = dg.num_nodes, dout.shape[1]
    if dx is None:
        dx = torch.empty(n, F, dtype=dout.dtype, device=dout.device)
    g = dg.fwd.struct(ew_slots)
    gt = dg.bwd.struct(None)
    ldm = _ld(mask) if mask is not None else 0
    if dg.is_cuda:
        ws_n = _lib.lib().pg_spmm_max_bwd_workspace(gt, F)
        ws = _workspace(ws_n, dout.device)
        ldf = _ld(fwd_out) if fwd_out is not None else 0
        kind = dg.arg_kind | (_lib.PG_ARG_DEAD_NONE if dead_none else 0)
        call("pg_spmm_max_bwd_bf16" if bf else "pg_spmm_max_bwd", g, gt, ptr(argpos), _ld(argpos), kind, ptr(dout), _ld(dout),
             F, ptr(mask), ldm, ptr(fwd_out), ldf, ptr(dx), _ld(dx), ptr(ws), ws_n, _stream(dout))
    else:
        call("pg_spmm_max_bwd_cpu", g, gt, ptr(argpos), _ld(argpos), dg.arg_kind, ptr(dout),
             _ld(dout), F, ptr(mask), ldm, ptr(dx), _ld(dx))
    return dx


def spmm_max_backward_scatter(dg: DeviceGraph, argpos: torch.Tensor, dout: torch.Tensor,
                              ew_slots: Optional[torch.Tensor] = None) -> torch.Tensor:
    """DGL-form backward with float atomics (non-deterministic summation order)."""
    if not dg.is_cuda:
        raise ValueError("scatter backward is a GPU-only entry point")
    F = dout.shape[1]
    dx = torch.empty(dg.num_nodes, F, dtype=torch.float32, device=dout.device)
    call("pg_spmm_max_bwd_scatter", dg.fwd.struct(ew_slots), ptr(argpos), _ld(argpos), dg.arg_kind,
         ptr(dout), _ld(dout), F, ptr(dx), _ld(dx), dg.num_nodes, _stream(dout))
    return dx


def spmm_sum(dg: DeviceGraph, X: torch.Tensor, mean: bool = False,
             ew_slots: Optional[torch.Tensor] = None, transpose: bool = False,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sum/mean aggregation (copy_u|u_mul_e, sum|mean). With transpose=True it runs on the
    out-CSR: the backward of the forward aggregation (mean -> per-term 1/deg(dst))."""
    _check_device(dg, X, ew_slots)
    F = X.shape[1]
    if out is None:
        out = torch.empty(dg.num_nodes, F, dtype=torch.float32, device=X.device)
    csr = dg.bwd if transpose else dg.fwd
    g = csr.struct(ew_slots)
    norm_mode = (2 if transpose else 1) if mean else 0
    norm_ptr = dg.fwd.ptr if (mean and transpose) else None
    if dg.is_cuda:
        ws_n = _lib.lib().pg_spmm_sum_workspace(g, F)
        ws = _workspace(ws_n, X.device)
        call("pg_spmm_sum", g, ptr(X), _ld(X), F, norm_mode, ptr(norm_ptr), ptr(out), _ld(out),
             ptr(ws), ws_n, _stream(X))
    else:
        call("pg_spmm_sum_cpu", g, ptr(X), _ld(X), F, norm_mode, ptr(norm_ptr), ptr(out), _ld(out))
    return out


def argpos_to_src(dg: DeviceGraph, argpos: torch.Tensor) -> torch.Tensor:
    """DGL's argX (int64 source ids; -1 where a row has no in-edge)."""
    n, F = argpos.shape
    argx = torch.empty(n, F, dtype=torch.int64, device=argpos.device)
    g = dg.fwd.struct(None)
    if dg.is_cuda:
        call("pg_argpos_to_src", g, ptr(argpos), _ld(argpos), dg.arg_kind, F, ptr(argx), F,
             _stream(argpos))
    else:
        call("pg_argpos_to_src_cpu", g, ptr(argpos), _ld(argpos), dg.arg_kind, F, ptr(argx), F)
    return argx


# ------------------------------------------------------------------ dense
def _split_k(M: int, N: int, K: int) -> int:
    """K-split for long-K products (weight gradients): the library's recommendation
    (pg_gemm_f32_split_k: ~3 workgroups per CU, slices of >= 96 K entries)."""
    return int(_lib.lib().pg_gemm_f32_split_k(M, N, K))


def gemm(A: torch.Tensor, B: torch.Tensor, transa: bool = False, transb: bool = False,
         out: Optional[torch.Tensor] = None, alpha: float = 1.0, beta: float = 0.0,
         bias: Optional[torch.Tensor] = None, act: int = _lib.PG_ACT_NONE,
         slope: float = LEAKY_SLOPE, split_k: Optional[int] = None,
         dact: Optional[torch.Tensor] = None, rowsum: Optional[torch.Tensor] = None) -> torch.Tensor:
    """C = alpha*op(A)@op(B) + beta*C (+bias, act): f32 GEMM on the GPU (three-piece bf16 MFMA
    products where the operands are aligned, the f32 MFMA kernel otherwise; f32 accuracy) or
    torch-CPU (CPU device). With `dact` (an activation output) the result is instead
    multiplied by act'(dact): the fused activation backward. With `rowsum`, also
    rowsum[m] = sum_k op(A)[m][k] (bias gradients of a weight-gradient product)."""
    M = A.shape[1] if transa else A.shape[0]
    K = A.shape[0] if transa else A.shape[1]
    Kb = B.shape[1] if transb else B.shape[0]
    N = B.shape[0] if transb else B.shape[1]
    if K != Kb:
        raise ValueError(f"gemm: inner dims {K} vs {Kb}")
    if out is None:
        if beta != 0.0:
            raise ValueError("gemm: beta != 0 needs out")
        out = torch.empty(M, N, dtype=torch.float32, device=A.device)
    if A.device.type != "cuda":
        a = A.t() if transa else A
        b = B.t() if transb else B
        r = alpha * (a @ b)
        if beta != 0.0:
            r = r + beta * out
        if bias is not None:
            r = r + bias
        if dact is not None:
            r = torch.where(dact > 0, r, r * slope if act == _lib.PG_ACT_LEAKY else r * 0)
        elif act == _lib.PG_ACT_RELU:
            r = torch.relu(r)
        elif act == _lib.PG_ACT_LEAKY:
            r = torch.nn.functional.leaky_relu(r, slope)
        out.copy_(r)
        if rowsum is not None:
            rowsum.copy_((A.t() if transa else A).sum(1))
        return out
    if split_k is None:
        split_k = 1 if (bias is not None or act != _lib.PG_ACT_NONE or dact is not None
                        or beta not in (0.0, 1.0)) else _split_k(M, N, K)
    ws_n = _lib.lib().pg_gemm_f32_workspace(M, N, K, split_k)
    ws = _workspace(ws_n, A.device)
    ep = _lib.epilogue(bias, act, slope, dact, rowsum)
    call("pg_gemm_f32", int(transa), int(transb), M, N, K, alpha, ptr(A), _ld(A), ptr(B), _ld(B),
         beta, ptr(out), _ld(out), ep, split_k, ptr(ws), ws_n, _stream(A))
    return out


PG_ERR_UNSUPPORTED = -2


def gemm_cat(A1: torch.Tensor, A2: torch.Tensor, B1: torch.Tensor, B2: torch.Tensor, transb: bool = False,
             out: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None,
             act: int = _lib.PG_ACT_NONE) -> Optional[torch.Tensor]:
    """C = [A1 | A2] @ op([B1 ; B2]) (+ bias, leaky_relu) without building either
    concatenation (pg_gemm_f32_cat, GPU). Returns None when the library does not take these
    operands (PG_ERR_UNSUPPORTED: the caller concatenates instead)."""
    M, K1 = A1.shape
    K2 = A2.shape[1]
    N = B1.shape[0] if transb else B1.shape[1]
    if A2.shape[0] != M or (B1.shape[1] if transb else B1.shape[0]) != K1 or \
            (B2.shape[1] if transb else B2.shape[0]) != K2 or (B2.shape[0] if transb else B2.shape[1]) != N:
        raise ValueError("gemm_cat: shapes do not concatenate")
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=A1.device)
    ep = _lib.epilogue(bias, act, LEAKY_SLOPE)
    rc = _lib.lib().pg_gemm_f32_cat(int(transb), M, N, K1, K2, 1.0, ptr(A1), _ld(A1), ptr(A2), _ld(A2), ptr(B1),
                                    _ld(B1), ptr(B2), _ld(B2), 0.0, ptr(out), _ld(out), ep, _stream(A1))
    if rc == PG_ERR_UNSUPPORTED:
        return None
    _lib.check(rc, "pg_gemm_f32_cat")
    return out


def gemm_group(parts) -> None:
    """Several split-K products in one launch + one combine (pg_gemm_f32_group): each part
    (A, B, C, transa, transb, beta, rowsum) computes C = op(A) op(B) (+ C when beta = 1) and
    rowsum = the row sums of op(A) when given. The weight gradients of a layer's backward."""
    if not parts:
        return
    dev = parts[0][0].device
    if dev.type != "cuda":
        for A, B, C, ta, tb, beta, rs in parts:
            gemm(A, B, transa=ta, transb=tb, out=C, beta=beta, rowsum=rs)
        return
    arr = (_lib.PgGemmPart * len(parts))()
    for q, (A, B, C, ta, tb, beta, rs) in zip(arr, parts):
        q.transa, q.transb = int(ta), int(tb)
        q.M = A.shape[1] if ta else A.shape[0]
        q.K = A.shape[0] if ta else A.shape[1]
        q.N = B.shape[0] if tb else B.shape[1]
        q.A, q.lda, q.B, q.ldb = ptr(A), _ld(A), ptr(B), _ld(B)
        q.beta, q.C, q.ldc, q.rowsum = beta, ptr(C), _ld(C), ptr(rs)
    ws_n = _lib.lib().pg_gemm_f32_group_workspace(arr, len(parts))
    ws = _workspace(ws_n, dev)
    call("pg_gemm_f32_group", arr, len(parts), ptr(ws), ws_n, _stream(parts[0][0]))


def gemm_bf16(A: torch.Tensor, B: torch.Tensor, transa: bool = False, transb: bool = False,
              out: Optional[torch.Tensor] = None, out_dtype=torch.float32, alpha: float = 1.0,
              beta: float = 0.0, bias: Optional[torch.Tensor] = None, act: int = _lib.PG_ACT_NONE,
              slope: float = LEAKY_SLOPE, split_k: Optional[int] = None,
              dact: Optional[torch.Tensor] = None, rowsum: Optional[torch.Tensor] = None
              ) -> torch.Tensor:
    """pg_gemm_bf16: bfloat16 operands, f32 accumulate on v_mfma_f32_32x32x16_bf16, output
    float32 or bfloat16 (`out` / `out_dtype`), the same epilogues as gemm() (bias f32, dact
    bfloat16, rowsum f32)."""
    if A.dtype != torch.bfloat16 or B.dtype != torch.bfloat16 or A.device.type != "cuda":
        raise TypeError("gemm_bf16: bfloat16 operands on a HIP device expected")
    M = A.shape[1] if transa else A.shape[0]
    K = A.shape[0] if transa else A.shape[1]
    Kb = B.shape[1] if transb else B.shape[0]
    N = B.shape[0] if transb else B.shape[1]
    if K != Kb:
        raise ValueError(f"gemm_bf16: inner dims {K} vs {Kb}")
    if out is None:
        if beta != 0.0:
            raise ValueError("gemm_bf16: beta != 0 needs out")
        out = torch.empty(M, N, dtype=out_dtype, device=A.device)
    if out.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError("gemm_bf16: float32 or bfloat16 output")
    if dact is not None and dact.dtype != torch.bfloat16:
        raise TypeError("gemm_bf16: dact must be bfloat16")
    obf = out.dtype == torch.bfloat16
    if split_k is None:
        split_k = 1 if (obf or bias is not None or act != _lib.PG_ACT_NONE or dact is not None
                        or beta not in (0.0, 1.0)) else int(_lib.lib().pg_gemm_bf16_split_k(M, N, K))
    ws_n = _lib.lib().pg_gemm_bf16_workspace(M, N, K, split_k)
    ws = _workspace(ws_n, A.device)
    ep = _lib.epilogue(bias, act, slope, dact, rowsum)
    call("pg_gemm_bf16", int(transa), int(transb), M, N, K, alpha, ptr(A), _ld(A), ptr(B), _ld(B),
         beta, ptr(out), _ld(out), _lib.PG_DTYPE_BF16 if obf else _lib.PG_DTYPE_F32, ep, split_k,
         ptr(ws), ws_n, _stream(A))
    return out


def cast_bf16(src: torch.Tensor, index: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16(src[index]) (round to nearest even; index < 0 gives 0) with pg_cast_f32_bf16."""
    if src.dtype != torch.float32 or not src.is_contiguous():
        raise TypeError("cast_bf16: contiguous float32 source expected")
    n = index.numel() if index is not None else src.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.bfloat16, device=src.device)
    if index is not None and index.dtype != torch.int32:
        raise TypeError("cast_bf16: int32 index expected")
    call("pg_cast_f32_bf16", ptr(src), ptr(index), n, ptr(out), _stream(src))
    return out


def pad2d_group(parts) -> None:
    """dst[:rows, :cols] = src, the rest of dst zero, for each (src, dst) pair of 2-D f32
    tensors (unit column stride): one pg_pad2d_group launch per PG_PAD2D_MAX parts on the
    GPU, torch on the CPU."""
    parts = [(s.contiguous(), d) for s, d in parts]
    if not parts:
        return
    if parts[0][1].device.type != "cuda":
        for src, dst in parts:
            dst.zero_()
            dst[:src.shape[0], :src.shape[1]].copy_(src)
        return
    for i in range(0, len(parts), _lib.PG_PAD2D_MAX):
        chunk = parts[i:i + _lib.PG_PAD2D_MAX]
        arr = (_lib.PgPad2d * len(chunk))()
        for k, (src, dst) in enumerate(chunk):
            if dst.stride(1) != 1 or src.dtype != torch.float32 or dst.dtype != torch.float32:
                raise ValueError("pad2d_group: f32 operands with unit column stride expected")
            arr[k] = _lib.PgPad2d(ptr(src), _ld(src), src.shape[0], src.shape[1], ptr(dst), dst.stride(0),
                                  dst.shape[0], dst.shape[1])
        call("pg_pad2d_group", arr, len(chunk), _stream(chunk[0][1]))


def col_sum(x: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False
            ) -> torch.Tensor:
    rows, cols = x.shape
    if out is None:
        out = torch.empty(cols, dtype=torch.float32, device=x.device)
    if x.device.type != "cuda":
        s = x.sum(0)
        out.copy_(out + s if accumulate else s)
        return out
    ws_n = _lib.lib().pg_col_sum_workspace(rows, cols)
    ws = _workspace(ws_n, x.device)
    call("pg_col_sum", ptr(x), _ld(x), rows, cols, ptr(out), int(accumulate), ptr(ws), ws_n,
         _stream(x))
    return out


# ------------------------------------------------------------------ autograd
class MaxAggregate(torch.autograd.Function):
    """update_all(copy_u('h','m') | u_mul_e, max('m','neigh')) with the DGL backward."""

    @staticmethod
    def forward(ctx, X, dg, ew_slots):
        if ew_slots is not None and ew_slots.requires_grad:
            raise NotImplementedError("gradient w.r.t. edge weights of a max aggregation")
        out, argpos = spmm_max(dg, X.contiguous(), ew_slots)
        ctx.dg = dg
        ctx.save_for_backward(argpos, ew_slots)
        return out

    @staticmethod
    def backward(ctx, dout):
        argpos, ew_slots = ctx.saved_tensors
        dx = spmm_max_backward(ctx.dg, argpos, dout.contiguous(), ew_slots)
        return dx, None, None


class SumAggregate(torch.autograd.Function):
    """update_all(copy_u | u_mul_e, sum | mean); backward on the transposed CSR."""

    @staticmethod
    def forward(ctx, X, dg, ew_slots, mean):
        if ew_slots is not None and ew_slots.requires_grad:
            raise NotImplementedError("gradient w.r.t. edge weights of a sum aggregation")
        ctx.dg, ctx.mean = dg, mean
        ctx.save_for_backward(ew_slots)
        return spmm_sum(dg, X.contiguous(), mean, ew_slots)

    @staticmethod
    def backward(ctx, dout):
        (ew_slots,) = ctx.saved_tensors
        dx = spmm_sum(ctx.dg, dout.contiguous(), ctx.mean, ew_slots, transpose=True)
        return dx, None, None, None


def _padded(n: int, F: int, device) -> torch.Tensor:
    """(n, F) view of an (n, round4(F)) buffer whose pad columns are zero."""
    Fp = round4(F)
    buf = torch.empty(n, Fp, dtype=torch.float32, device=device)
    if Fp > F:
        buf[:, F:].zero_()
    return buf


def sage_width(F: int) -> int:
    """TrainEngine's SAGE input width: a multiple of 64 when that costs <= 2 % more columns
    (503 -> 512: whole SpMM feature tiles, the three-piece GEMM's aligned operands), else a
    multiple of 4. Pads are zero."""
    r64 = -(-F // 64) * 64
    return r64 if r64 <= 1.02 * F else round4(F)


# layer inputs that take no gradient (the features: the same tensor every epoch) keep their
# padded [H | M] buffer: {key: [HM, weakref(h), version, busy]}. A hit needs the SAME tensor
# object (identity through the weak reference, not only its address: a freed input's memory
# is handed to the next same-size allocation, which starts at the same version) with an
# unchanged version. A buffer whose forward saved it for a backward that has not run yet is
# busy (its M half must not be overwritten): another forward then gets a fresh buffer.
_HM_CACHE: dict = {}


def _hm_buffer(h: torch.Tensor, Fp: int, keep: bool):
    """([H | M] (N x 2Fp, H and its zero pad in the left half) for a SAGE layer's input h,
    the cache key it was marked busy under or None)."""
    N, Fin = h.shape
    key = (h.data_ptr(), tuple(h.shape), str(h.device), Fp) if not h.requires_grad else None
    if key is not None:
        hit = _HM_CACHE.get(key)
        if hit is not None and hit[1]() is h and hit[2] == h._version and not hit[3]:
            hit[3] = keep
            return hit[0], (key if keep else None)
    HM = torch.empty(N, 2 * Fp, dtype=torch.float32, device=h.device)
    HM[:, :Fin].copy_(h)
    if Fp > Fin:
        HM[:, Fin:Fp].zero_()
    if key is not None and (key not in _HM_CACHE or not _HM_CACHE[key][3]):
        if len(_HM_CACHE) > 8:
            _HM_CACHE.clear()
        _HM_CACHE[key] = [HM, weakref.ref(h), h._version, keep]
        return HM, (key if keep else None)
    return HM, None


def _hm_release(key) -> None:
    hit = _HM_CACHE.get(key) if key is not None else None
    if hit is not None:
        hit[3] = False


class SagePool(torch.autograd.Function):
    """One DGL 0.8.2 SAGEConv(in, out, 'pool') layer, forward and backward, on the
    engine's kernels (code/model.py:13-15):
        P = relu(h @ Wpool^T + bpool); M = max-aggregate(P); Y = h @ Wself^T + M @ Wneigh^T + b

    On a HIP device it runs TrainEngine's layouts: the input padded to sage_width (503 ->
    512, so the layer-1 products run the three-piece GEMM), fc_self + fc_neigh as ONE
    K = 2F product [H | M] [Wself | Wneigh]^T, dead-none max records (the backward reads no
    relu' mask), the weight gradients of fc_self and fc_neigh as one product dY^T [H | M],
    and the input gradient as one stacked product [dY | dP] [Wself ; Wpool]. On the CPU
    device: the plain composition (DGL's CPU backend role)."""

    @staticmethod
    def forward(ctx, h, w_pool, b_pool, w_self, w_neigh, bias, dg, ew_slots):
        h = h.contiguous()
        ctx.dg = dg
        ctx.has_bias = bias is not None
        if h.device.type == "cuda":
            return SagePool._forward_gpu(ctx, h, w_pool, b_pool, w_self, w_neigh, bias, dg, ew_slots)
        N, Fin = h.shape
        Fp = round4(Fin)
        Pb = _padded(N, Fin, h.device)
        gemm(h, w_pool, transb=True, out=Pb[:, :Fin], bias=b_pool, act=_lib.PG_ACT_RELU)
        Mb = torch.empty(N, Fp, dtype=torch.float32, device=h.device)
        argpos = torch.empty(N, Fp, dtype=dg.arg_dtype, device=h.device)
        spmm_max(dg, Pb, ew_slots, out=Mb, argpos=argpos)
        Y = gemm(h, w_self, transb=True)
        gemm(Mb[:, :Fin], w_neigh, transb=True, out=Y, beta=1.0, bias=bias)
        ctx.gpu = False
        ctx.save_for_backward(h, w_pool, w_self, w_neigh, Pb, Mb, argpos, ew_slots)
        return Y

    @staticmethod
    def _forward_gpu(ctx, h, w_pool, b_pool, w_self, w_neigh, bias, dg, ew_slots):
        N, Fin = h.shape
        Fp = sage_width(Fin)
        if Fp == Fin:
            out = SagePool._forward_gpu_cat(ctx, h, w_pool, b_pool, w_self, w_neigh, bias, dg, ew_slots)
            if out is not None:
                return out
        ctx.cat = False
        fpad = Fp - Fin
        keep = torch.is_grad_enabled() and any(ctx.needs_input_grad[:6])
        HM, ctx.hm_key = _hm_buffer(h, Fp, keep)
        # the padded weight images in one launch (pg_pad2d_group)
        Fo = w_self.shape[0]
        Wpool = torch.empty(Fp, Fp, dtype=torch.float32, device=h.device)
        bpool = torch.empty(Fp, dtype=torch.float32, device=h.device)
        Wcat = torch.empty(Fo, 2 * Fp, dtype=torch.float32, device=h.device)
        pad2d_group([(w_pool, Wpool), (b_pool.view(1, -1), bpool.view(1, -1)), (w_self, Wcat[:, :Fp]),
                     (w_neigh, Wcat[:, Fp:])])
        P = torch.empty(N, Fp, dtype=torch.float32, device=h.device)
        gemm(HM[:, :Fp], Wpool, transb=True, out=P, bias=bpool, act=_lib.PG_ACT_RELU)
        argpos = torch.empty(N, Fp, dtype=dg.arg_dtype, device=h.device)
        spmm_max(dg, P, ew_slots, out=HM[:, Fp:], argpos=argpos, dead_none=True)
        Y = gemm(HM, Wcat, transb=True, bias=bias)
        ctx.gpu = True
        ctx.save_for_backward(HM, P, argpos, Wpool, Wcat, ew_slots)
        ctx.fin = Fin
        return Y

    @staticmethod
    def _forward_gpu_cat(ctx, h, w_pool, b_pool, w_self, w_neigh, bias, dg, ew_slots):
        """A layer whose input needs no padding (4-aligned width): H is the caller's tensor
        and M its own buffer, fc_self + fc_neigh one product over the two K pieces
        ([H | M] [Wself | Wneigh]^T, pg_gemm_f32_cat), no [H | M] copy and no weight
        concatenation; where the library does not take the operands (a misaligned h or
        bias, an odd output width), the same product on the two concatenations, reusing P, M
        and argpos (the aggregation is not redone)."""
        N, Fin = h.shape
        w_pool, w_self, w_neigh = w_pool.contiguous(), w_self.contiguous(), w_neigh.contiguous()
        P = torch.empty(N, Fin, dtype=torch.float32, device=h.device)
        gemm(h, w_pool, transb=True, out=P, bias=b_pool.contiguous(), act=_lib.PG_ACT_RELU)
        M = torch.empty(N, Fin, dtype=torch.float32, device=h.device)
        argpos = torch.empty(N, Fin, dtype=dg.arg_dtype, device=h.device)
        spmm_max(dg, P, ew_slots, out=M, argpos=argpos, dead_none=True)
        Y = gemm_cat(h, M, w_self, w_neigh, transb=True, bias=bias)
        if Y is None:
            Y = gemm(torch.cat([h, M], 1), torch.cat([w_self, w_neigh], 1), transb=True, bias=bias)
        ctx.gpu = ctx.cat = True
        ctx.save_for_backward(h, M, P, argpos, w_pool, w_self, w_neigh, ew_slots)
        ctx.fin = Fin
        ctx.hm_key = None
        return Y

    @staticmethod
    def _backward_gpu_cat(ctx, dY):
        h, M, P, argpos, w_pool, w_self, w_neigh, ew_slots = ctx.saved_tensors
        dg, Fin = ctx.dg, ctx.fin
        dY = dY.contiguous()
        N, Fo = dY.shape
        need_h, need_wp, need_bp, need_ws, need_wn, need_b = ctx.needs_input_grad[:6]
        d_b = torch.empty(Fo, dtype=torch.float32, device=dY.device) if (need_b and ctx.has_bias) else None
        wgrads = []  # the layer's weight gradients, one grouped launch after the max backward
        d_ws = torch.empty(Fo, Fin, dtype=torch.float32, device=dY.device) if need_ws else None
        d_wn = torch.empty(Fo, Fin, dtype=torch.float32, device=dY.device) if need_wn else None
        if d_ws is not None:
            wgrads.append((dY, h, d_ws, True, False, 0.0, d_b))
        if d_wn is not None:
            wgrads.append((dY, M, d_wn, True, False, 0.0, d_b if d_ws is None else None))
        if d_b is not None and not wgrads:
            d_b = col_sum(dY)
        dM = gemm(dY, w_neigh)
        dP = torch.empty(N, Fin, dtype=torch.float32, device=dY.device)
        spmm_max_backward(dg, argpos, dM, ew_slots, mask=P, dx=dP, dead_none=True)
        d_bp = torch.empty(Fin, dtype=torch.float32, device=dY.device) if need_bp else None
        d_wp = None
        if need_wp:
            d_wp = torch.empty(Fin, Fin, dtype=torch.float32, device=dY.device)
            wgrads.append((dP, h, d_wp, True, False, 0.0, d_bp))
        elif d_bp is not None:
            d_bp = col_sum(dP)
        gemm_group(wgrads)
        d_h = None
        if need_h:  # [dY | dP] [Wself ; Wpool] over the two K pieces
            d_h = gemm_cat(dY, dP, w_self, w_pool)
            if d_h is None:
                d_h = gemm(torch.cat([dY, dP], 1), torch.cat([w_self, w_pool], 0))
        return d_h, d_wp, d_bp, d_ws, d_wn, d_b, None, None

    @staticmethod
    def backward(ctx, dY):
        if ctx.gpu and ctx.cat:
            return SagePool._backward_gpu_cat(ctx, dY)
        if ctx.gpu:
            return SagePool._backward_gpu(ctx, dY)
        h, w_pool, w_self, w_neigh, Pb, Mb, argpos, ew_slots = ctx.saved_tensors
        dg = ctx.dg
        dY = dY.contiguous()
        N, Fin = h.shape
        need_h, need_wp, need_bp, need_ws, need_wn, need_b = ctx.needs_input_grad[:6]
        d_b = torch.empty(dY.shape[1], dtype=torch.float32, device=dY.device) \
            if (need_b and ctx.has_bias) else None
        d_ws = gemm(dY, h, transa=True, rowsum=d_b) if need_ws else None
        d_wn = gemm(dY, Mb[:, :Fin], transa=True) if need_wn else None
        if d_b is not None and not need_ws:
            d_b = col_sum(dY)
        dMb = _padded(N, Fin, h.device)
        gemm(dY, w_neigh, out=dMb[:, :Fin])
        dPb = torch.empty_like(Pb)
        spmm_max_backward(dg, argpos, dMb, ew_slots, mask=Pb, dx=dPb)
        dP = dPb[:, :Fin]
        d_bp = torch.empty(Fin, dtype=torch.float32, device=dY.device) if need_bp else None
        d_wp = gemm(dP, h, transa=True, rowsum=d_bp) if need_wp else None
        if d_bp is not None and not need_wp:
            d_bp = col_sum(dP)
        d_h = None
        if need_h:
            d_h = gemm(dY, w_self)
            gemm(dP, w_pool, out=d_h, beta=1.0)
        return d_h, d_wp, d_bp, d_ws, d_wn, d_b, None, None

    @staticmethod
    def _backward_gpu(ctx, dY):
        HM, P, argpos, Wpool, Wcat, ew_slots = ctx.saved_tensors
        dg, Fin = ctx.dg, ctx.fin
        try:
            return SagePool._backward_gpu_body(ctx, dY, HM, P, argpos, Wpool, Wcat, ew_slots, dg, Fin)
        finally:
            _hm_release(ctx.hm_key)

    @staticmethod
    def _backward_gpu_body(ctx, dY, HM, P, argpos, Wpool, Wcat, ew_slots, dg, Fin):
        N, Fp = P.shape
        Fo = dY.shape[1]
        need_h, need_wp, need_bp, need_ws, need_wn, need_b = ctx.needs_input_grad[:6]
        # [dY | dP]: dY copied in, dP written by the max backward (only for the stacked
        # input-gradient product: the first layer's input, the features, takes none)
        if need_h:
            DYP = torch.empty(N, Fo + Fp, dtype=torch.float32, device=dY.device)
            DYP[:, :Fo].copy_(dY)
            dY = DYP[:, :Fo]
        else:
            dY = dY.contiguous()
            DYP = None
        d_b = torch.empty(Fo, dtype=torch.float32, device=dY.device) if (need_b and ctx.has_bias) else None
        d_ws = d_wn = None
        wgrads = []  # the layer's weight gradients, one grouped launch after the max backward
        if need_ws or need_wn:
            d_wcat = torch.empty(Fo, 2 * Fp, dtype=torch.float32, device=dY.device)
            wgrads.append((dY, HM, d_wcat, True, False, 0.0, d_b))  # [d Wself | d Wneigh]
            d_ws, d_wn = d_wcat[:, :Fin], d_wcat[:, Fp:Fp + Fin]
        elif d_b is not None:
            d_b = col_sum(dY)
        dM = gemm(dY, Wcat[:, Fp:])
        # dead-none records: the relu' mask of P is implied (P is not read)
        dP = DYP[:, Fo:] if DYP is not None else torch.empty(N, Fp, dtype=torch.float32, device=dY.device)
        spmm_max_backward(dg, argpos, dM, ew_slots, mask=P, dx=dP, dead_none=True)
        d_bp_p = torch.empty(Fp, dtype=torch.float32, device=dY.device) if need_bp else None
        d_wp = d_bp = None
        if need_wp:
            d_wp_p = torch.empty(Fp, Fp, dtype=torch.float32, device=dY.device)
            wgrads.append((dP, HM[:, :Fp], d_wp_p, True, False, 0.0, d_bp_p))
            d_wp = d_wp_p[:Fin, :Fin]
        elif d_bp_p is not None:
            d_bp_p = col_sum(dP)
        gemm_group(wgrads)
        if d_bp_p is not None:
            d_bp = d_bp_p[:Fin]
        d_h = None
        if need_h:  # one stacked product [dY | dP] [Wself ; Wpool]
            Wstack = torch.cat([Wcat[:, :Fp], Wpool], 0)
            d_h = gemm(DYP, Wstack)[:, :Fin]
        return d_h, d_wp, d_bp, d_ws, d_wn, d_b, None, None
