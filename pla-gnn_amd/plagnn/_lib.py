"""ctypes binding of libplagnn.so (the C-ABI declared in include/plagnn.h).

torch is imported first on purpose: libplagnn.so links the HIP runtime by SONAME
(libamdhip64.so.7) and must bind to the copy PyTorch already loaded, so both share one
runtime, one device context and the same streams.
"""
from __future__ import annotations

import ctypes
import os
import warnings

import torch  # noqa: F401  (load order: see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
ABI_VERSION = 13  # pg_version() of the library this package binds (include/plagnn.h)
# PLAGNN_LIB overrides the library path (A/B builds of tuning variants)
LIB_PATH = os.environ.get("PLAGNN_LIB") or os.path.join(_HERE, "libplagnn.so")

PG_ARG_U16 = 16
PG_ARG_I32 = 32
PG_ARG_DEAD_NONE = 0x100  # flag: a zero maximum records no winner (include/plagnn.h)
PG_DTYPE_F32 = 0
PG_DTYPE_BF16 = 1
PG_ACT_NONE = 0
PG_ACT_RELU = 1
PG_ACT_LEAKY = 2


class PgCsr(ctypes.Structure):
    """pg_csr_t (include/plagnn.h)."""

    _fields_ = [
        ("n_rows", ctypes.c_int64),
        ("n_cols", ctypes.c_int64),
        ("nnz", ctypes.c_int64),
        ("ptr", ctypes.c_void_p),
        ("col", ctypes.c_void_p),
        ("eslot", ctypes.c_void_p),
        ("epos", ctypes.c_void_p),
        ("ew", ctypes.c_void_p),
        ("items", ctypes.c_void_p),
        ("n_items", ctypes.c_int64),
        ("merges", ctypes.c_void_p),
        ("n_merges", ctypes.c_int64),
        ("n_slots", ctypes.c_int64),
        ("max_deg", ctypes.c_int32),
        ("chunk", ctypes.c_int32),
    ]


class PgGemmEpilogue(ctypes.Structure):
    """pg_gemm_epilogue_t (include/plagnn.h)."""

    _fields_ = [
        ("bias", ctypes.c_void_p),
        ("act", ctypes.c_int),
        ("slope", ctypes.c_float),
        ("dact", ctypes.c_void_p),
        ("lddact", ctypes.c_int64),
        ("rowsum", ctypes.c_void_p),
    ]


class PgPad2d(ctypes.Structure):
    """pg_pad2d_t (include/plagnn.h)."""

    _fields_ = [
        ("src", ctypes.c_void_p),
        ("lds", ctypes.c_int64),
        ("rows", ctypes.c_int64),
        ("cols", ctypes.c_int64),
        ("dst", ctypes.c_void_p),
        ("ldd", ctypes.c_int64),
        ("drows", ctypes.c_int64),
        ("dcols", ctypes.c_int64),
    ]


PG_PAD2D_MAX = 8

_i = ctypes.c_int
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f = ctypes.c_float
_d = ctypes.c_double
_sz = ctypes.c_size_t
_vp = ctypes.c_void_p
_csr = ctypes.POINTER(PgCsr)
class PgGemmPart(ctypes.Structure):
    """pg_gemm_part_t (include/plagnn.h): A, B f32 or bf16 bits, C f32."""

    _fields_ = [
        ("transa", ctypes.c_int32),
        ("transb", ctypes.c_int32),
        ("M", ctypes.c_int64),
        ("N", ctypes.c_int64),
        ("K", ctypes.c_int64),
        ("A", ctypes.c_void_p),
        ("lda", ctypes.c_int64),
        ("B", ctypes.c_void_p),
        ("ldb", ctypes.c_int64),
        ("beta", ctypes.c_float),
        ("C", ctypes.c_void_p),
        ("ldc", ctypes.c_int64),
        ("rowsum", ctypes.c_void_p),
    ]


class PgSplitkJob(ctypes.Structure):
    """pg_splitk_job_t (include/plagnn.h)."""

    _fields_ = [
        ("ws", ctypes.c_void_p),
        ("split_k", ctypes.c_int),
        ("M", ctypes.c_int64),
        ("N", ctypes.c_int64),
        ("alpha", ctypes.c_float),
        ("beta", ctypes.c_float),
        ("C", ctypes.c_void_p),
        ("ldc", ctypes.c_int64),
        ("rowsum", ctypes.c_void_p),
    ]


_ep = ctypes.POINTER(PgGemmEpilogue)

# name -> (restype, argtypes); every symbol of include/plagnn.h
SIGNATURES = {
    "pg_csr_from_coo": (_i, [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp]),
    "pg_csr_transpose": (_i, [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp]),
    "pg_schedule_count": (_i, [_vp, _i64, _i32, _vp, _vp, _vp, _vp]),
    "pg_schedule_build": (_i, [_vp, _i64, _i32, _vp, _vp]),
    "pg_spmm_max_fwd_workspace": (_sz, [_csr, _i64, _i]),
    "pg_spmm_max_fwd": (_i, [_csr, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _i, _vp, _sz, _vp]),
    "pg_spmm_max_bwd_workspace": (_sz, [_csr, _i64]),
    "pg_spmm_max_bwd": (_i, [_csr, _csr, _vp, _i64, _i, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _i64,
                             _vp, _sz, _vp]),
    "pg_gemm_f32_partials": (_i, [_i, _i, _i64, _i64, _i64, _vp, _i64, _vp, _i64, ctypes.POINTER(PgGemmEpilogue),
                                  _i, _vp, _sz, ctypes.POINTER(ctypes.c_int), _vp]),
    "pg_gemm_splitk_reduce_batch": (_i, [ctypes.POINTER(PgSplitkJob), _i, _vp]),
    "pg_gemm_f32_group_workspace": (_sz, [ctypes.POINTER(PgGemmPart), _i]),
    "pg_gemm_f32_group": (_i, [ctypes.POINTER(PgGemmPart), _i, _vp, _sz, _vp]),
    "pg_gemm_bf16_group_workspace": (_sz, [ctypes.POINTER(PgGemmPart), _i]),
    "pg_gemm_bf16_group": (_i, [ctypes.POINTER(PgGemmPart), _i, _vp, _sz, _vp]),
    "pg_csr_spmm_f64": (_i, [_i64, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _i64, _vp]),
    "pg_spmm_max_bwd_scatter": (_i, [_csr, _vp, _i64, _i, _vp, _i64, _i64, _vp, _i64, _i64, _vp]),
    "pg_spmm_sum_workspace": (_sz, [_csr, _i64]),
    "pg_spmm_sum": (_i, [_csr, _vp, _i64, _i64, _i, _vp, _vp, _i64, _vp, _sz, _vp]),
    "pg_argpos_to_src": (_i, [_csr, _vp, _i64, _i, _i64, _vp, _i64, _vp]),
    "pg_bias_act": (_i, [_vp, _i64, _i64, _i64, _vp, _i, _f, _vp]),
    "pg_act_bwd": (_i, [_vp, _i64, _vp, _i64, _i64, _i64, _i, _f, _vp]),
    "pg_col_sum_workspace": (_sz, [_i64, _i64]),
    "pg_col_sum": (_i, [_vp, _i64, _i64, _i64, _vp, _i, _vp, _sz, _vp]),
    "pg_sigmoid_multi_loss_workspace": (_sz, [_i64, _i32]),
    "pg_sigmoid_multi_loss": (_i, [_vp, _i64, _i64, _i32, _vp, _i64, _vp, _vp, _i64, _vp, _i64,
                                   _vp, _vp, _i64, _vp, _sz, _vp]),
    "pg_mlp_head_workspace": (_sz, [_i64, _i32]),
    "pg_mlp_head": (_i, [_vp, _i64, _i64, _i32, _i, _vp, _i64, _vp, _i32, _vp, _i64, _vp, _vp, _i64, _i64,
                         _vp, _i64, _vp, _i64, _vp, _vp, _i64, _f, _vp, _vp, _sz, _vp]),
    "pg_mlp_l1_head_workspace": (_sz, [_i64, _i32, _i32, _i32]),
    "pg_mlp_l1_head": (_i, [_vp, _i64, _i64, _i32, _vp, _i64, _vp, _i32, _vp, _i64, _vp, _i64, _vp, _i32, _vp,
                            _i64, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _f, _vp,
                            _vp, _sz, _vp, _d, _d, _d, _vp]),
    "pg_mlp_l1_pieces_bytes": (_sz, [_i32, _i32]),
    "pg_mlp_l1_split": (_i, [_vp, _i64, _i32, _i32, _vp, _vp]),
    "pg_mlp_l1_head_ex": (_i, [_vp, _i64, _i64, _i32, _vp, _i64, _vp, _i32, _vp, _i64, _vp, _i64, _vp, _i32, _vp,
                               _i64, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _f, _vp,
                               _vp, _sz, _vp, _d, _d, _d, _vp, _vp]),
    "pg_adam_apply_l1": (_i, [_vp, _vp, _vp, _vp, _i64, _vp, _d, _d, _d, _d, _i64, _i64, _i32, _i32, _vp, _vp]),
    "pg_adam_prepare": (_i, [_vp, _d, _d, _d, _vp]),
    "pg_adam_apply": (_i, [_vp, _vp, _vp, _vp, _i64, _vp, _d, _d, _d, _d, _vp]),
    "pg_gemm_f32_split_k": (_i, [_i64, _i64, _i64]),
    "pg_ecc": (_i, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _d, _vp, _vp]),
    "pg_loc_eval_workspace": (_sz, [_i64, _i32]),
    "pg_loc_correction": (_i, [_vp, _i64, _i64, _i32, _d, _vp, _i64, _vp, _sz, _vp]),
    "pg_loc_performance": (_i, [_vp, _i64, _vp, _i64, _i64, _i32, _vp, _vp, _sz, _vp]),
    "pg_perturb_workspace": (_sz, [_i64]),
    "pg_perturb_prepare": (_i, [_vp, _vp, _i64, _i32, _d, _vp, _vp, _vp]),
    "pg_perturb_sum": (_i, [_vp, _vp, _vp, _vp, _i64, _i32, _d, _i, _d, _vp, _vp, _sz, _vp]),
    "pg_perturb_count": (_i, [_vp, _vp, _vp, _vp, _i64, _i32, _d, _vp, _vp, _vp, _d, _d, _vp, _vp]),
    "pg_perturb_fill": (_i, [_vp, _vp, _vp, _vp, _i64, _i32, _d, _vp, _vp, _vp, _d, _d, _vp, _vp, _vp,
                             _vp]),
    "pg_gemm_f32_workspace": (_sz, [_i64, _i64, _i64, _i]),
    "pg_gemm_f32": (_i, [_i, _i, _i64, _i64, _i64, _f, _vp, _i64, _vp, _i64, _f, _vp, _i64, _ep,
                         _i, _vp, _sz, _vp]),
    "pg_gemm_f32_cat": (_i, [_i, _i64, _i64, _i64, _i64, _f, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _f, _vp,
                             _i64, _ep, _vp]),
    "pg_gemm_bf16_split_k": (_i, [_i64, _i64, _i64]),
    "pg_gemm_bf16_workspace": (_sz, [_i64, _i64, _i64, _i]),
    "pg_gemm_bf16": (_i, [_i, _i, _i64, _i64, _i64, _f, _vp, _i64, _vp, _i64, _f, _vp, _i64, _i, _ep,
                          _i, _vp, _sz, _vp]),
    "pg_spmm_max_fwd_bf16": (_i, [_csr, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _i, _vp, _sz, _vp]),
    "pg_spmm_max_bwd_bf16": (_i, [_csr, _csr, _vp, _i64, _i, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _vp,
                                  _i64, _vp, _sz, _vp]),
    "pg_cast_f32_bf16": (_i, [_vp, _vp, _i64, _vp, _vp]),
    "pg_cast_bf16_f32": (_i, [_vp, _i64, _vp, _vp]),
    "pg_pad2d_group": (_i, [ctypes.POINTER(PgPad2d), _i, _vp]),
    "pg_spmm_max_fwd_cpu": (_i, [_csr, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _i]),
    "pg_spmm_max_bwd_cpu": (_i, [_csr, _csr, _vp, _i64, _i, _vp, _i64, _i64, _vp, _i64, _vp, _i64]),
    "pg_spmm_sum_cpu": (_i, [_csr, _vp, _i64, _i64, _i, _vp, _vp, _i64]),
    "pg_argpos_to_src_cpu": (_i, [_csr, _vp, _i64, _i, _i64, _vp, _i64]),
    "pg_last_error_string": (ctypes.c_char_p, []),
    "pg_version": (_i, []),
}

_LIB = None


class PlagnnError(RuntimeError):
    pass


def lib():
    """Load libplagnn.so. Raises (never falls back) when it has not been built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise PlagnnError(
                f"{LIB_PATH} is missing: build the HIP extension first "
                "(make -C pla-gnn_amd, or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        missing = []
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("PLAGNN_LIB") and not hasattr(L, name):
                missing.append(name)  # an older A/B build (scripts/*_ab.sh) without this entry point
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        abi = int(L.pg_version()) if hasattr(L, "pg_version") else -1
        if abi != ABI_VERSION or missing:
            # only reachable through PLAGNN_LIB (the product library exports every symbol or
            # getattr above raised): say what this build lacks instead of failing later
            warnings.warn(f"{LIB_PATH}: ABI {abi} (this package expects {ABI_VERSION}); "
                          f"{len(missing)} declared entry points missing: {', '.join(missing[:12])}"
                          f"{' ...' if len(missing) > 12 else ''}", RuntimeWarning, stacklevel=2)
        _LIB = L
    return _LIB


def check(rc: int, name: str) -> None:
    if rc != 0:
        msg = lib().pg_last_error_string().decode(errors="replace")
        raise PlagnnError(f"{name} failed (code {rc}): {msg}")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)


def stream_handle(device: torch.device):
    """hipStream_t of torch's current stream on `device` (as an int for ctypes)."""
    return torch.cuda.current_stream(device).cuda_stream


def epilogue(bias=None, act: int = PG_ACT_NONE, slope: float = 0.01, dact=None, rowsum=None):
    """pg_gemm_epilogue_t from tensors (or None)."""
    e = PgGemmEpilogue()
    e.bias = ptr(bias)
    e.act = act
    e.slope = slope
    e.dact = ptr(dact)
    e.lddact = dact.stride(0) if dact is not None else 0
    e.rowsum = ptr(rowsum)
    return e


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()
