"""SpMM-max micro-benchmark on the S0 graph: forward and backward per feature width,
HIP-event timed, with algorithmic GB/s (SURVEY.md §8d byte model). Run it with
PLAGNN_SPMM_FTILE / PLAGNN_BWD_PATH set to A/B the tuning knobs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import torch  # noqa: E402

import plagnn  # noqa: E402
from plagnn import data, ops  # noqa: E402


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
    kind = sys.argv[1] if len(sys.argv) > 1 else "s0"
    ds = data.make_dataset(kind)
    src, dst = ds.edges_with_self_loops()
    g = plagnn.CSRGraph(src, dst, ds.n)
    dg = g.on("cuda")
    N, E = ds.n, g.num_edges
    print(f"graph {kind}: N={N} E'={E} max_deg={g.fwd.max_deg} split_rows={g.fwd.n_merges} "
          f"env FTILE={os.environ.get('PLAGNN_SPMM_FTILE', '-')} BWD={os.environ.get('PLAGNN_BWD_PATH', '-')}")
    for F in (256, 504, 512):
        P = torch.relu(torch.randn(N, F, device="cuda"))
        P[:, ::4] = 0.0  # dead features (relu never fires): their maxima are all 0
        out = torch.empty_like(P)
        arg = torch.empty(N, F, dtype=dg.arg_dtype, device="cuda")
        tf = timeit(lambda: ops.spmm_max(dg, P, out=out, argpos=arg))
        dZ = torch.randn(N, F, device="cuda")
        dX = torch.empty_like(P)
        ws = torch.empty(plagnn.lib().pg_spmm_max_bwd_workspace(dg.bwd.struct(None), F),
                         dtype=torch.uint8, device="cuda")

        def bwd():
            plagnn._lib.call("pg_spmm_max_bwd", dg.fwd.struct(None), dg.bwd.struct(None), arg.data_ptr(), F,
                             dg.arg_kind, dZ.data_ptr(), F, F, P.data_ptr(), F,
                             out.data_ptr() if skip_zero else None, F, dX.data_ptr(), F,
                             ws.data_ptr(), ws.numel(), plagnn._lib.stream_handle(P.device))
        skip_zero = False
        tb = timeit(bwd)
        skip_zero = True
        tbz = timeit(bwd)
        ts = timeit(lambda: ops.spmm_max_backward_scatter(dg, arg, dZ, None))
        fb = 4 * (N + 1) + 4 * E + 4 * F * E + 4 * F * N + 2 * F * N
        print(f"F={F:4d} fwd {tf*1e3:8.1f} us {fb/tf/1e6:8.1f} GB/s | bwd {tb*1e3:8.1f} us "
              f"(skipping zero maxima {tbz*1e3:8.1f} us) | "
              f"scatter(atomics, incl. zero-fill) {ts*1e3:8.1f} us")


if __name__ == "__main__":
    main()
