"""bf16 GEMM micro-benchmark (pg_gemm_bf16) on the cfg5 step shapes (N = 384,656 rows,
hidden 512) and a square product, HIP-event timed, against torch.mm (hipBLASLt) on the
same bf16 operands (A/B library variants with PLAGNN_LIB).
Usage (GPU box): python scripts/gemm_bf16_bench.py [--rows 384656]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import torch  # noqa: E402

from plagnn import ops  # noqa: E402


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=384656)
    ap.add_argument("--no-torch", action="store_true")
    a = ap.parse_args()
    n = a.rows
    cases = [("fwd.cat", False, True, n, 512, 1024), ("fwd.pool", False, True, n, 512, 512),
             ("dgrad.stack", False, False, n, 512, 1024), ("dgrad.neigh", False, False, n, 512, 512),
             ("wgrad.cat", True, False, 512, 1024, n), ("square", False, True, 8192, 8192, 8192)]
    print(f"{'op':12} {'ta':>2} {'tb':>2} {'M':>7} {'N':>5} {'K':>7} {'mine_us':>8} {'TF':>6} {'torch_us':>8} {'TF':>6}")
    for name, ta, tb, M, N, K in cases:
        A = torch.randn((K, M) if ta else (M, K), device="cuda").to(torch.bfloat16)
        B = torch.randn((N, K) if tb else (K, N), device="cuda").to(torch.bfloat16)
        C = torch.empty(M, N, device="cuda", dtype=torch.float32 if name.startswith("wgrad") else torch.bfloat16)
        tm = timeit(lambda: ops.gemm_bf16(A, B, ta, tb, out=C))
        a_ = A.t() if ta else A
        b_ = B.t() if tb else B
        Ct = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        tt = float("nan") if a.no_torch else timeit(lambda: torch.mm(a_, b_, out=Ct))
        fl = 2.0 * M * N * K
        print(f"{name:12} {int(ta):>2} {int(tb):>2} {M:>7} {N:>5} {K:>7} {tm*1e3:8.1f} {fl/tm/1e9:6.1f} "
              f"{tt*1e3:8.1f} {fl/tt/1e9:6.1f}", flush=True)
        del A, B, C, Ct


if __name__ == "__main__":
    main()
