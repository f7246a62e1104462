"""Run the fused MLP head (pg_mlp_l1_head) of the cfg2 engine repeatedly (rocprofv3 passes).
Usage: python scripts/probes/mlp_head_one.py [reps] [config]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import plagnn  # noqa: E402
from plagnn import workload as W  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = sys.argv[2] if len(sys.argv) > 2 else "cfg2"
wl = W.build(cfg, device="cuda")
eng = plagnn.TrainEngine(wl.graph(), torch.from_numpy(wl.ds.feat), torch.from_numpy(wl.ds.loc.astype(np.float32)),
                         wl.dims, wl.class_weight, wl.train_index, wl.val_index, device="cuda", seed=0)
eng.forward()
torch.cuda.synchronize()
for _ in range(reps):
    eng._mlp_l1_head()
torch.cuda.synchronize()
print("ok", cfg, reps)
