"""GEMM micro-benchmark on the shapes of one PLA-GNN training step (cfg2 dims):
plagnn's fp32 MFMA kernel vs torch.mm (hipBLASLt) on the same operands, HIP-event timed.
Usage (GPU box): python scripts/gemm_bench.py [--dims 503,256,256,256,100,12]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import torch  # noqa: E402

from plagnn import ops  # noqa: E402


def shapes(dims, N=24041):
    r4 = lambda d: (d + 3) // 4 * 4  # noqa: E731
    pd = [r4(d) for d in dims]
    out = []
    L = len(dims) - 3
    for l in range(L):
        Fi, Fo = pd[l], pd[l + 1]
        out += [("fwd.pool", False, True, N, Fi, Fi), ("fwd.cat", False, True, N, Fo, 2 * Fi),
                ("wgrad.cat", True, False, Fo, 2 * Fi, N), ("dgrad.cat", False, False, N, 2 * Fi, Fo),
                ("wgrad.pool", True, False, Fi, Fi, N), ("dgrad.pool", False, False, N, Fi, Fi)]
    out += [("fwd.liner1", False, True, N, pd[-2], pd[-3]), ("fwd.liner2", False, True, N, pd[-1], pd[-2]),
            ("wgrad.liner1", True, False, pd[-2], pd[-3], N), ("dgrad.liner1", False, False, N, pd[-3], pd[-2])]
    return out


def timeit(fn, reps=20):
    for _ in range(3):
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
    ap.add_argument("--dims", default="503,256,256,256,100,12")
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--square", type=int, default=4096, help="also time an NxNxN NN GEMM (0: skip)")
    ap.add_argument("--err", action="store_true", help="also report the error against a float64 product")
    args = ap.parse_args()
    dims = [int(x) for x in args.dims.split(",")]
    extra = [("square", False, False, args.square, args.square, args.square)] if args.square else []
    tot_m = tot_t = 0.0
    print(f"{'op':14} {'ta':>2} {'tb':>2} {'M':>6} {'N':>5} {'K':>6} {'mine_us':>8} {'TF':>6} {'torch_us':>8} {'TF':>6}"
          + ("  rel_fro   max/scale" if args.err else ""))
    seen = set()
    for name, ta, tb, M, N, K in shapes(dims) + extra:
        key = (ta, tb, M, N, K)
        if key in seen:
            continue
        seen.add(key)
        A = torch.randn((K, M) if ta else (M, K), device="cuda")
        B = torch.randn((N, K) if tb else (K, N), device="cuda")
        C = torch.empty(M, N, device="cuda")
        tm = timeit(lambda: ops.gemm(A, B, transa=ta, transb=tb, out=C))
        a_ = A.t() if ta else A
        b_ = B.t() if tb else B
        tt = float("nan") if args.no_torch else timeit(lambda: torch.mm(a_, b_, out=C))
        fl = 2.0 * M * N * K
        if name != "square":
            tot_m += tm
            tot_t += tt
        err = ""
        if args.err:
            ops.gemm(A, B, transa=ta, transb=tb, out=C)
            ref = torch.mm(a_.double(), b_.double())
            scale = torch.mm(a_.double().abs(), b_.double().abs())  # sum |a b| per output
            d = (C.double() - ref)
            err = f"  {float(d.norm() / ref.norm()):.2e}  {float((d.abs() / scale).max()):.2e}"
        print(f"{name:14} {int(ta):>2} {int(tb):>2} {M:>6} {N:>5} {K:>6} {tm*1e3:8.1f} {fl/tm/1e9:6.1f} {tt*1e3:8.1f} {fl/tt/1e9:6.1f}" + err)
    print(f"total (unique shapes): mine {tot_m*1e3:.1f} us, torch {tot_t*1e3:.1f} us")


if __name__ == "__main__":
    main()
