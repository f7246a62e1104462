"""The max aggregation forward (and optionally backward) on S0 at one feature width,
repeated, for rocprofv3 counter passes. Usage: python scripts/probes/spmm_one.py [F] [reps] [bwd]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import torch  # noqa: E402

import plagnn  # noqa: E402
from plagnn import data, ops  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ds = data.make_dataset("s0")
src, dst = ds.edges_with_self_loops()
g = plagnn.CSRGraph(src, dst, ds.n)
dg = g.on("cuda")
torch.manual_seed(0)
P = torch.relu(torch.randn(ds.n, F, device="cuda"))
out = torch.empty_like(P)
arg = torch.empty(ds.n, F, dtype=dg.arg_dtype, device="cuda")
for _ in range(reps):
    ops.spmm_max(dg, P, out=out, argpos=arg, dead_none=True)
if len(sys.argv) > 3:
    dZ = torch.randn(ds.n, F, device="cuda")
    dX = torch.empty_like(P)
    for _ in range(reps):
        ops.spmm_max_backward(dg, arg, dZ, mask=P, dx=dX, dead_none=True)
torch.cuda.synchronize()
print("ok", F)
