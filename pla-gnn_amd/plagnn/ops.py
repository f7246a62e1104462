"""Tensor-level operations over the C-ABI, and their autograd wrappers.

Every GPU operation here is a call into libplagnn.so on torch's current stream; there is
no fallback to another implementation. Tensors on the CPU device (the reference's
``-d cpu``, code/main_normal.py:30) go to the library's ``*_cpu`` entry points for the
message passing and to torch-CPU for the dense algebra, as DGL's CPU backend does.
"""
from __future__ import annotations

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
    input, a relu output >= 0) entries whose maximum is 0 are skipped: they contribute
    nothing, and the mask is implied by the skip (not read). `dead_none`: the records come
    from spmm_max(..., dead_none=True) (the same skip without fwd_out; needs mask)."""
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


class SagePool(torch.autograd.Function):
    """One DGL 0.8.2 SAGEConv(in, out, 'pool') layer, forward and backward, on the
    engine's kernels (code/model.py:13-15):
        P = relu(h @ Wpool^T + bpool); M = max-aggregate(P); Y = h @ Wself^T + M @ Wneigh^T + b
    """

    @staticmethod
    def forward(ctx, h, w_pool, b_pool, w_self, w_neigh, bias, dg, ew_slots):
        h = h.contiguous()
        N, Fin = h.shape
        Fout = w_self.shape[0]
        Fp = round4(Fin)
        Pb = _padded(N, Fin, h.device)
        gemm(h, w_pool, transb=True, out=Pb[:, :Fin], bias=b_pool, act=_lib.PG_ACT_RELU)
        Mb = torch.empty(N, Fp, dtype=torch.float32, device=h.device)
        argpos = torch.empty(N, Fp, dtype=dg.arg_dtype, device=h.device)
        spmm_max(dg, Pb, ew_slots, out=Mb, argpos=argpos)
        Y = gemm(h, w_self, transb=True)
        gemm(Mb[:, :Fin], w_neigh, transb=True, out=Y, beta=1.0, bias=bias)
        ctx.dg = dg
        ctx.save_for_backward(h, w_pool, w_self, w_neigh, Pb, Mb, argpos, ew_slots)
        ctx.has_bias = bias is not None
        return Y

    @staticmethod
    def backward(ctx, dY):
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
