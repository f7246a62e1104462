"""Does a node relabeling speed up the max aggregation? Times the forward (and backward)
SpMM on the cfg2 S0 graph and the cfg5 RMAT x16 graph as generated (random ids), after a
reverse Cuthill-McKee relabeling, and after a degree-descending relabeling. Each row keeps
its in-edges in edge-id order (the relabeled graph is built from the same COO in the same
order), so the results are the same up to the row permutation. Usage: python reorder_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
from scipy.sparse.csgraph import reverse_cuthill_mckee  # noqa: E402
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
    return a.elapsed_time(b) / reps * 1e3


def run(name, ds, F, dtype):
    n = ds.n
    src = np.concatenate([ds.row.astype(np.int64), np.arange(n)])
    dst = np.concatenate([ds.col.astype(np.int64), np.arange(n)])
    A = sp.csr_matrix((np.ones(len(ds.row)), (ds.row, ds.col)), shape=(n, n))
    t0 = time.time()
    rcm = reverse_cuthill_mckee(A, symmetric_mode=True)
    t_rcm = time.time() - t0
    deg = np.bincount(ds.row, minlength=n)
    orders = {"ids": np.arange(n), "rcm": np.ascontiguousarray(rcm).astype(np.int64),
              "degree": np.argsort(-deg, kind="stable")}
    X0 = torch.randn(n, F, device="cuda").to(dtype)
    for oname, order in orders.items():
        new = np.empty(n, np.int64)
        new[order] = np.arange(n)  # old id -> new id
        g = plagnn.CSRGraph(new[src], new[dst], n)
        dg = g.on("cuda")
        X = X0[torch.as_tensor(order, device="cuda")]  # row new holds old row order[new]
        out, arg = ops.spmm_max(dg, X)
        tf = timeit(lambda: ops.spmm_max(dg, X, out=out, argpos=arg))
        dout = torch.randn_like(out)
        tb = timeit(lambda: ops.spmm_max_backward(dg, arg, dout)) if dtype == torch.float32 else float("nan")
        print(f"{name:5s} F={F} {str(dtype)[6:]:8s} {oname:7s} fwd {tf:8.1f} us  bwd {tb:8.1f} us"
              + (f"  (rcm {t_rcm:.1f} s on the host)" if oname == "rcm" else ""), flush=True)


torch.manual_seed(0)
run("S0", data.make_dataset("s0"), 256, torch.float32)
run("S0", data.make_dataset("s0"), 512, torch.float32)
run("RMAT", data.make_dataset("rmat"), 256, torch.bfloat16)
run("RMAT", data.make_dataset("rmat"), 256, torch.float32)
