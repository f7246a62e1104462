"""Per-step clock stamps of the register-staged three-piece GEMM (probe build:
make variant V=stamp VSRC=gemm_x3 VFLAGS="-fno-slp-vectorize -DPG_X3_DMA=0 -DPG_X3_STAMP=1").
Prints, for blocks 0..63 (wave 0), the median cycles of each step phase: load+frag+MFMA
issue, the wait for the next tile's global loads, split+store; and the prologue / epilogue.
Usage: PLAGNN_LIB=.../libplagnn_stamp.so python scripts/probes/x3_stamps.py M N K ta tb"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from plagnn import _lib, ops  # noqa: E402

M, N, K, ta, tb = (int(x) for x in sys.argv[1:6])
A = torch.randn((K, M) if ta else (M, K), device="cuda")
B = torch.randn((N, K) if tb else (K, N), device="cuda")
C = torch.empty(M, N, device="cuda")
for _ in range(5):
    ops.gemm(A, B, transa=bool(ta), transb=bool(tb), out=C)
torch.cuda.synchronize()
buf = np.zeros((64, 66, 4), np.uint64)
lib = _lib.lib()
lib.pg_x3_stamps.argtypes = [ctypes.c_void_p]
assert lib.pg_x3_stamps(buf.ctypes.data) == 0
nk = (K + 15) // 16
st = buf.astype(np.int64)
steps = st[:, 1:nk + 1, :]
a = np.median(steps[:, :, 1] - steps[:, :, 0], axis=0)
c = np.median(steps[:, :, 3] - steps[:, :, 1], axis=0)  # wait for the loads
b = np.median(steps[:, :, 2] - steps[:, :, 3], axis=0)  # split + store
tot = np.median(steps[:, -1, 2] - st[:, 0, 0])
print(f"shape {M}x{N}x{K} ta{ta} tb{tb}: steps {nk}, blocks 0..63 median total loop {tot} cycles")
print(f"prologue (first tile) median {np.median(steps[:, 0, 0] - st[:, 0, 0]):.0f}")
print("step: mfma-phase  split+store  load-wait   (median over blocks; every 4th step)")
for t in range(0, min(nk, 64), 4):
    print(f"  {t:3d}: {a[t]:8.0f} {b[t]:8.0f} {c[t]:8.0f}")
print(f"mean per step: mfma-phase {a.mean():.0f}, split+store {b.mean():.0f}, load-wait {c.mean():.0f}")
print(f"epilogue median {np.median(st[:, 65, 1] - st[:, 65, 0]):.0f}")
starts = st[:, 0, 0] - st[:, 0, 0].min()
print(f"block start spread (cycles): {np.percentile(starts, [0, 50, 100])}")
