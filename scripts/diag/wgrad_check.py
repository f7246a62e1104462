"""Diagnostic: every weight gradient of one TrainEngine step recomputed in float64 from the
engine's own operands (dY / dP and [H | M]), to localise a GEMM error. Usage:
  python scripts/diag/wgrad_check.py [config]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import plagnn  # noqa: E402
from plagnn import workload  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "ref"
wl = workload.build(cfg, device="cuda")
x = torch.from_numpy(wl.ds.feat)
labels = torch.from_numpy(wl.ds.loc.astype(np.float32))
eng = plagnn.TrainEngine(wl.graph(), x, labels, wl.dims, wl.class_weight, wl.train_index, wl.val_index,
                         device="cuda", edge_weight=wl.edge_weight, seed=1)
eng.forward()
eng.backward()
torch.cuda.synchronize()


def report(name, G, A, B, rowsum=None):
    ref = A.double().t() @ B.double()
    g = G.double()
    err = (g - ref).abs()
    scale = ref.abs().max().item()
    i, j = np.unravel_index(int(err.argmax()), err.shape)
    bad = (err > 1e-5 * scale).nonzero()
    rows = sorted(set(bad[:, 0].tolist()))
    cols = sorted(set(bad[:, 1].tolist()))
    print(f"{name}: shape {tuple(g.shape)} max err {err.max().item():.3e} (rel {err.max().item() / scale:.2e}) at "
          f"({i},{j}); entries > 1e-5 rel: {len(bad)}; rows {rows[:8]}..{len(rows)} cols {cols[:8]}..{len(cols)}")
    if rowsum is not None:
        rs = A.double().sum(0)
        e2 = (rowsum.double() - rs).abs().max().item()
        print(f"   rowsum err {e2:.3e} (scale {rs.abs().max().item():.3e})")


pd = eng.pd
dY = eng.dA3
for l in reversed(range(eng.L)):
    p = f"conv{l + 1}."
    Fi = pd[l]
    HM = eng.HM[l]
    report(p + "Wcat", eng.G[p + "Wcat"], dY, HM, eng.G[p + "b"])
    report(p + "Wpool", eng.G[p + "Wpool"], eng.dP[l], HM[:, :Fi], eng.G[p + "bpool"])
    if l > 0:
        dY = eng.dHM[l][:, :Fi]
report("liner1.W", eng.G["liner1.W"], eng.dA4, eng.A3, eng.G["liner1.b"])
report("liner2.W", eng.G["liner2.W"], eng.dZ, eng.A4, eng.G["liner2.b"])
