"""Does a HIP graph run two independent branches at once, and what does the max aggregation
(MALL-bound gather) leave for a GEMM beside it? On S0 at F = 256: the SpMM alone, the GEMM
(N x 256 x 256, K-half of fwd.cat) alone, both on one stream, and both as forked branches
of one captured graph. Usage: python scripts/probes/overlap_probe.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import torch  # noqa: E402

import plagnn  # noqa: E402
from plagnn import data, ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
F = 256
ds = data.make_dataset("s0")
src, dst = ds.edges_with_self_loops()
g = plagnn.CSRGraph(src, dst, ds.n)
dg = g.on("cuda")
torch.manual_seed(0)
P = torch.relu(torch.randn(ds.n, F, device="cuda"))
out = torch.empty_like(P)
arg = torch.empty(ds.n, F, dtype=dg.arg_dtype, device="cuda")
H = torch.randn(ds.n, 256, device="cuda")
W = torch.randn(256, 256, device="cuda") * 0.05
Y = torch.empty(ds.n, 256, device="cuda")
H2 = torch.randn(ds.n, 512, device="cuda")
W2 = torch.randn(256, 512, device="cuda") * 0.05
Y2 = torch.empty(ds.n, 256, device="cuda")
out2 = torch.empty_like(P)
arg2 = torch.empty_like(arg)
side = torch.cuda.Stream()


def spmm():
    ops.spmm_max(dg, P, out=out, argpos=arg, dead_none=True)


def gemm():
    ops.gemm(H, W, transb=True, out=Y)


def gemm2():
    ops.gemm(H, W, transb=True, out=Y2)


def spmm2():
    ops.spmm_max(dg, H, out=out2, argpos=arg2, dead_none=True)


def gemm_big():
    ops.gemm(H2, W2, transb=True, out=Y)


def forked(a, b):
    def f():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            b()
        a()
        cur.wait_stream(side)
    return f


def seq(*fs):
    def f():
        for x in fs:
            x()
    return f


def timed_eager(fn, inner=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        for _ in range(inner):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / inner)
    ts.sort()
    return ts[len(ts) // 2]


def timed(fn, inner=10):
    if os.environ.get("OVL_EAGER"):
        return timed_eager(fn, inner)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(inner):
            fn()
    for _ in range(3):
        gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        gr.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / inner)
    ts.sort()
    return ts[len(ts) // 2]


res = {}
res["spmm"] = timed(spmm)
res["gemm_k256"] = timed(gemm)
res["gemm_k512"] = timed(gemm_big)
res["seq_spmm_gemm_k256"] = timed(seq(spmm, gemm))
res["fork_spmm_gemm_k256"] = timed(forked(spmm, gemm))
res["fork_gemm_k256_spmm"] = timed(forked(gemm, spmm))
res["seq_spmm_gemm_k512"] = timed(seq(spmm, gemm_big))
res["fork_spmm_gemm_k512"] = timed(forked(spmm, gemm_big))
res["seq_gemm_gemm"] = timed(seq(gemm, gemm2))
res["fork_gemm_gemm"] = timed(forked(gemm, gemm2))
res["seq_spmm_spmm"] = timed(seq(spmm, spmm2))
res["fork_spmm_spmm"] = timed(forked(spmm, spmm2))
for k, v in res.items():
    print(f"{k:24s} {v:8.1f} us")
