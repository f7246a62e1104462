"""Probe (variant build: make variant V=planes VSRC=gemm_x3 VFLAGS="-fno-slp-vectorize
-DPG_X3_PLANES_PROBE=1"): the three-piece GEMM fed with pre-split bf16 pieces by LDS-DMA
against the shipped kernel (split in registers) on the cfg2 forward / input-gradient shapes.
Usage: PLAGNN_LIB=.../libplagnn_planes.so python scripts/probes/x3_planes_probe.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import torch  # noqa: E402

from plagnn import _lib, ops  # noqa: E402


def pieces(x):
    h = x.to(torch.bfloat16)
    r = x - h.float()
    m = r.to(torch.bfloat16)
    lo = (r - m.float()).to(torch.bfloat16)
    return torch.stack([h, m, lo]).contiguous()


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


L = _lib.lib()
L.pg_x3_planes_probe.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
st = torch.cuda.current_stream().cuda_stream
for name, tb, M, N, K in [("fwd.pool", 1, 24041, 504, 504), ("fwd.cat", 1, 24041, 256, 1008),
                          ("dgrad.cat", 0, 24041, 1008, 256), ("dgrad.pool", 0, 24041, 504, 504),
                          ("fwd.pool2", 1, 24041, 256, 256), ("fwd.cat2", 1, 24041, 256, 512),
                          ("square", 0, 4096, 4096, 4096)]:
    A = torch.randn(M, K, device="cuda")
    B = torch.randn((N, K) if tb else (K, N), device="cuda")
    C = torch.empty(M, N, device="cuda")
    C2 = torch.empty(M, N, device="cuda")
    Ap, Bp = pieces(A), pieces(B)
    t_reg = timeit(lambda: ops.gemm(A, B, transb=bool(tb), out=C))
    res = {}
    for bm, bn in [(128, 128), (128, 64), (64, 64)]:
        f = lambda: L.pg_x3_planes_probe(tb, M, N, K, Ap.data_ptr(), Ap[0].numel(), K, Bp.data_ptr(),  # noqa: E731
                                         Bp[0].numel(), B.shape[1], C2.data_ptr(), N, bm, bn, st)
        assert f() == 0
        res[(bm, bn)] = timeit(f)
    torch.cuda.synchronize()
    err = float((C2 - C).abs().max() / C.abs().max())
    fl = 2.0 * M * N * K
    best = min(res.values())
    print(f"{name:10s} {M}x{N}x{K} tb{tb}: registers {t_reg:7.1f} us ({fl / t_reg / 1e6:6.1f} TF); pieces by DMA "
          + " ".join(f"{bm}x{bn} {t:7.1f}" for (bm, bn), t in res.items())
          + f" -> {fl / best / 1e6:6.1f} TF; max|diff|/max {err:.1e}", flush=True)
