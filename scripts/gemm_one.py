"""Run one GEMM shape repeatedly through ops.gemm (for rocprofv3 counter passes).
Usage: python scripts/gemm_one.py M N K ta tb [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import torch  # noqa: E402

from plagnn import ops  # noqa: E402

M, N, K, ta, tb = (int(x) for x in sys.argv[1:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
A = torch.randn((K, M) if ta else (M, K), device="cuda")
B = torch.randn((N, K) if tb else (K, N), device="cuda")
C = torch.empty(M, N, device="cuda")
for _ in range(reps):
    ops.gemm(A, B, transa=bool(ta), transb=bool(tb), out=C)
torch.cuda.synchronize()
print("ok", M, N, K, ta, tb)
