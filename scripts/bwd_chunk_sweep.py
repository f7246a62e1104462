"""Max-backward time on S0 per backward chunk (CSRGraph(chunk_bwd=...)): the engine's call
(dead-none records, implied relu' mask), HIP-event timed, per feature width.
Usage (GPU box): python scripts/bwd_chunk_sweep.py [chunk ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import torch  # noqa: E402

import plagnn  # noqa: E402
from plagnn import data, ops  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    chunks = [int(c) for c in sys.argv[1:]] or [32, 48, 64, 96, 128, 192]
    ds = data.make_dataset("s0")
    src, dst = ds.edges_with_self_loops()
    N = ds.n
    gen = torch.Generator(device="cuda").manual_seed(0)
    for F in (256, 512):
        P = torch.relu(torch.randn(N, F, device="cuda", generator=gen))
        P[:, ::4] = 0.0
        dZ = torch.randn(N, F, device="cuda", generator=gen)
        line = [f"F={F:4d}"]
        for c in chunks:
            dg = plagnn.CSRGraph(src, dst, N, chunk_bwd=c).on("cuda")
            _, arg = ops.spmm_max(dg, P, dead_none=True)
            dx = torch.empty_like(P)
            t = timeit(lambda: ops.spmm_max_backward(dg, arg, dZ, None, mask=P, dx=dx, dead_none=True))
            line.append(f"chunk {c}: {t:6.1f} us ({dg.bwd.n_merges} split rows)")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
