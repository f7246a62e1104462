"""Max-aggregation forward (bf16 storage) on a BASELINE workload's graph (default cfg5, RMAT
x16), HIP-event timed, per feature width, with algorithmic GB/s (SURVEY.md §8d bytes).
A/B library variants with PLAGNN_LIB. Usage (GPU box): python scripts/fwd_bf16_bench.py [config]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import torch  # noqa: E402

from plagnn import ops  # noqa: E402
from plagnn import workload as W  # noqa: E402


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    wl = W.build(sys.argv[1] if len(sys.argv) > 1 else "cfg5", device="cuda")
    dg = wl.graph().on("cuda")
    N, E = dg.num_nodes, dg.num_edges
    gen = torch.Generator(device="cuda").manual_seed(0)
    for F in (512,):
        P = torch.relu(torch.randn(N, F, device="cuda", generator=gen)).to(torch.bfloat16)
        out = torch.empty_like(P)
        arg = torch.empty(N, F, dtype=dg.arg_dtype, device="cuda")
        t = timeit(lambda: ops.spmm_max(dg, P, out=out, argpos=arg, dead_none=True))
        fb = 4 * (N + 1) + 4 * E + 2 * F * E + 2 * F * N + 2 * F * N
        print(f"N={N} E'={E} F={F}: fwd {t:8.1f} us, {fb / t / 1e3:8.1f} GB/s algorithmic", flush=True)


if __name__ == "__main__":
    main()
