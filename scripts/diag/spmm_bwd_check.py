"""Diagnostic: each layer's max-aggregation backward of one TrainEngine step (dP, with the
relu' mask and the zero-maximum skip) against the oracle's scatter_add_ on the engine's own
operands (its argmax records, upstream gradient and edge weights). Usage:
  python scripts/diag/spmm_bwd_check.py [config]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
import plagnn  # noqa: E402
from plagnn import ops, workload  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
wl = workload.build(cfg, device="cuda")
x = torch.from_numpy(wl.ds.feat)
labels = torch.from_numpy(wl.ds.loc.astype(np.float32))
g = wl.graph()
eng = plagnn.TrainEngine(g, x, labels, wl.dims, wl.class_weight, wl.train_index, wl.val_index, device="cuda",
                         edge_weight=wl.edge_weight, seed=1)
eng.forward()
eng.backward()
torch.cuda.synchronize()
src, dst, w = wl.edges_without_loops()
og = oracle.OracleGraph(src, dst, wl.n, edge_weight=w)
ptr = g.fwd.ptr.astype(np.int64)
eid = g.eid.astype(np.int64)
outdeg = np.diff(g.bwd.ptr)
for l in range(eng.L):
    F = eng.dims[l]
    Fi = eng.pd[l]
    pos = eng.arg[l][:, :F].to(torch.int32).cpu().numpy() & 0xFFFF
    argx = ops.argpos_to_src(eng.dg, eng.arg[l][:, :F].contiguous()).cpu().numpy()
    slot = ptr[:-1, None] + pos
    arge = eid[np.minimum(slot, len(eid) - 1)]
    dM = eng.dHM[l][:, Fi:Fi + F].contiguous().cpu().numpy()
    P = eng.Pl[l][:, :F].cpu().numpy()
    M = eng.HM[l][:, Fi:Fi + F].cpu().numpy()
    ref = oracle.spmm_max_bwd(og, argx, arge, dM, use_weight=w is not None)
    ref = np.where(P > 0, ref, 0.0).astype(np.float32)
    got = eng.dP[l][:, :F].cpu().numpy()
    d = np.abs(got.astype(np.float64) - ref)
    bad = np.argwhere(d > 0)
    print(f"layer {l + 1}: F {F}, max |diff| {d.max():.3e}, differing entries {len(bad)}, "
          f"zero maxima {(M == 0).sum()}, bias-sum diff {abs(got.astype(np.float64).sum(0) - ref.astype(np.float64).sum(0)).max():.3e}")
    if len(bad):
        rows = np.unique(bad[:, 0])
        print(f"   rows {len(rows)}: out-degree of the worst {outdeg[bad[np.argmax(d[bad[:, 0], bad[:, 1]]), 0]]}, "
              f"out-degrees (first 10) {outdeg[rows[:10]].tolist()}, split threshold {g.bwd.chunk}")
        i, f = np.unravel_index(np.argmax(d), d.shape)
        print(f"   worst ({i},{f}): got {got[i, f]:.9e} ref {ref[i, f]:.9e} P {P[i, f]:.3e}")
