"""Per-group step times (TrainEngine.group_times: graph-replayed launch groups) of one config
for the library named by PLAGNN_LIB (the product build when unset). One JSON line per run,
so scripts/group_ab.sh can alternate library variants across processes.
Usage (GPU box): CONFIG=cfg2 python scripts/group_ab.py [label]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import plagnn  # noqa: E402
from plagnn import workload as W  # noqa: E402


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(os.environ.get("PLAGNN_LIB", "base"))
    cfg = os.environ.get("CONFIG", "cfg2")
    wl = W.build(cfg, device="cuda")
    Engine = plagnn.TrainEngineBF16 if wl.bf16 else plagnn.TrainEngine
    if os.environ.get("PG_REDUCE_INLINE") is not None:  # A/B of the split-K combine placement
        plagnn.TrainEngine.REDUCE_INLINE = os.environ["PG_REDUCE_INLINE"] == "1"
        label += f"+inline{os.environ['PG_REDUCE_INLINE']}"
    if os.environ.get("PG_GROUP_WGRAD") is not None:  # A/B of the grouped weight gradients
        plagnn.TrainEngine.GROUP_WGRAD = os.environ["PG_GROUP_WGRAD"] == "1"
        label += f"+group{os.environ['PG_GROUP_WGRAD']}"
    if wl.bf16 and os.environ.get("PG_STACK_T") is not None:  # A/B of the stacked-weight layout
        plagnn.TrainEngineBF16.STACK_T = os.environ["PG_STACK_T"] == "1"
        label += f"+stackT{os.environ['PG_STACK_T']}"
    e = Engine(wl.graph(), torch.from_numpy(wl.ds.feat), torch.from_numpy(wl.ds.loc.astype(np.float32)),
               wl.dims, wl.class_weight, wl.train_index, wl.val_index, lr=5e-5, device="cuda",
               edge_weight=wl.edge_weight)
    e.capture(warmup=2)
    for _ in range(5):
        e.step()
    torch.cuda.synchronize()
    groups = tuple(os.environ.get("PG_GROUPS", "gemm,spmm_max_fwd,spmm_max_bwd").split(","))
    res = {g: [] for g in groups}
    for _ in range(int(os.environ.get("ROUNDS", "3"))):
        gt = e.group_times(groups=groups, reps=10)
        for g in groups:
            if g in gt:
                res[g].append(round(gt[g]["ms"] * 1e3, 2))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        e.step()
    b.record()
    torch.cuda.synchronize()
    out = {"label": label, "config": cfg, "step_ms": round(a.elapsed_time(b) / 50, 4),
           "us_per_step": {g: sorted(v)[len(v) // 2] for g, v in res.items() if v}, "all": res}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
