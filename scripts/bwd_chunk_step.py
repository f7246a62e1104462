"""The cfg2 step's max-backward group time per backward chunk, in ONE process (engines built
on graphs with different CSRGraph(chunk_bwd=...), each captured; group_times alternated).
Usage (GPU box): python scripts/bwd_chunk_step.py [chunk ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import plagnn  # noqa: E402
from plagnn import workload as W  # noqa: E402


def main():
    chunks = [int(c) for c in sys.argv[1:]] or [48, 64, 96, 128]
    wl = W.build(os.environ.get("CONFIG", "cfg2"), device="cuda")
    engines = {}
    for c in chunks:
        g = plagnn.CSRGraph(wl.src, wl.dst, wl.ds.n, chunk_bwd=c)
        e = plagnn.TrainEngine(g, torch.from_numpy(wl.ds.feat), torch.from_numpy(wl.ds.loc.astype(np.float32)),
                               wl.dims, wl.class_weight, wl.train_index, wl.val_index, lr=5e-5, device="cuda",
                               edge_weight=wl.edge_weight)
        e.capture(warmup=2)
        for _ in range(3):
            e.step()
        engines[c] = e
    res = {c: [] for c in chunks}
    for _ in range(3):
        for c, e in engines.items():
            gt = e.group_times(groups=("spmm_max_bwd",), reps=10)
            res[c].append(gt["spmm_max_bwd"]["ms"])
    for c in chunks:
        print(f"chunk {c:4d}: spmm_max_bwd {np.median(res[c]) * 1e3:7.1f} us/step  {[round(x * 1e3, 1) for x in res[c]]}",
              flush=True)


if __name__ == "__main__":
    main()
