"""Winner-list statistics of the SpMM max backward on the bench graph after a few steps:
per (destination row, in-row position) how many features that edge wins."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import plagnn  # noqa: E402
from plagnn import data  # noqa: E402
from plagnn.train import fold_splits, weight_cal  # noqa: E402

ds = data.make_dataset("s0", seed=70)
src, dst = ds.edges_with_self_loops()
g = plagnn.CSRGraph(src, dst, ds.n)
label = [int(i) for i in ds.labelled]
tr, va = next(fold_splits(label, 10, 12))
eng = plagnn.TrainEngine(g, torch.from_numpy(ds.feat), torch.from_numpy(ds.loc.astype(np.float32)),
                         [503, 256, 256, 256, 100, 12], weight_cal(ds.loc), tr, va, lr=5e-5, device="cuda")
for _ in range(3):
    eng.step_eager()
torch.cuda.synchronize()
ptr = g.fwd.ptr
deg = np.diff(ptr)
for l in range(eng.L):
    a = eng.arg[l].cpu().numpy().astype(np.int64) & 0xFFFF
    N, F = a.shape
    F = eng.dims[l]
    a = a[:, :F]
    key = np.repeat(np.arange(N), F) * 70000 + a.reshape(-1)
    _, cnt = np.unique(key, return_counts=True)
    print(f"layer {l + 1} F={F}: (row,pos) lists {len(cnt)} of E'={g.num_edges}; mean {cnt.mean():.2f}"
          f" median {np.median(cnt):.0f} p99 {np.percentile(cnt, 99):.0f} max {cnt.max()}; "
          f"lists > 64: {(cnt > 64).sum()} holding {cnt[cnt > 64].sum() / cnt.sum():.1%} of entries; "
          f"winner = self-loop {(a == (deg[:, None] - 1)).mean():.1%}, pos 0 {(a == 0).mean():.1%}")
