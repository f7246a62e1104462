"""Max-backward micro-benchmark (the engine's call: dead-none records, implied relu' mask):
S0 at F = 256 / 512 (f32) and RMAT x16 at F = 512 (bf16), HIP-event timed per call, with
the algorithmic bytes of SURVEY.md §8d (4(N+1) + 8E' + (2+4+4+4) F N for f32). Run under
`rocprofv3 --kernel-trace --stats` for the per-pass split (pack, pull, merge).  python scripts/bwd_bench.py [s0|rmat|all] [reps] [backward chunks, comma list]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import torch  # noqa: E402

import plagnn  # noqa: E402
from plagnn import data, ops  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def run(kind, widths, bf16, reps, chunk_bwd):
    ds = data.make_dataset(kind)
    src, dst = ds.edges_with_self_loops()
    g = plagnn.CSRGraph(src, dst, ds.n, chunk_bwd=chunk_bwd)
    dg = g.on("cuda")
    N, E = ds.n, g.num_edges
    print(f"graph {kind}: N={N} E'={E} max_in={g.fwd.max_deg} max_out={g.bwd.max_deg} "
          f"bwd items={g.bwd.n_items} split={g.bwd.n_merges} (chunk {chunk_bwd})", flush=True)
    gen = torch.Generator(device="cuda").manual_seed(1)
    for F in widths:
        dt = torch.bfloat16 if bf16 else torch.float32
        P = torch.relu(torch.randn(N, F, device="cuda", generator=gen)).to(dt)
        P[:, ::4] = 0  # dead features: their maxima are 0 (no records)
        _, arg = ops.spmm_max(dg, P, dead_none=True)
        dZ = torch.randn(N, F, device="cuda", generator=gen).to(dt)
        dX = torch.empty_like(P)
        gs, gts = dg.fwd.struct(None), dg.bwd.struct(None)
        ws = torch.empty(plagnn.lib().pg_spmm_max_bwd_workspace(gts, F), dtype=torch.uint8, device="cuda")
        fn = "pg_spmm_max_bwd_bf16" if bf16 else "pg_spmm_max_bwd"
        kind_flag = dg.arg_kind | plagnn._lib.PG_ARG_DEAD_NONE
        st = plagnn._lib.stream_handle(P.device)

        def bwd():
            plagnn._lib.call(fn, gs, gts, arg.data_ptr(), F, kind_flag, dZ.data_ptr(), F, F, P.data_ptr(), F,
                             None, F, dX.data_ptr(), F, ws.data_ptr(), ws.numel(), st)

        t = timeit(bwd, reps)
        es = P.element_size()
        algo = 4 * (N + 1) + 8 * E + (2 + es + es + es) * F * N
        live = int((arg != -1).sum()) if arg.dtype == torch.int16 else -1
        print(f"{kind} F={F} {'bf16' if bf16 else 'f32'}: {t * 1e3:8.1f} us/call  "
              f"{algo / t / 1e6:7.1f} GB/s algorithmic  live entries {live} ({live / (N * F):.2f} of N*F)",
              flush=True)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    chunks = [int(c) for c in (sys.argv[3] if len(sys.argv) > 3 else "128").split(",")]
    for c in chunks:
        if which in ("s0", "all"):
            run("s0", (256, 512), False, reps, c)
        if which in ("rmat", "all"):
            run("rmat", (512,), True, reps, c)


if __name__ == "__main__":
    main()
