"""Prototype: the pull's work items cut by EXPECTED list entries instead of edge count.
An out-edge u -> v of the transposed CSR carries about F_live / deg_in(v) winning entries
(v's features are won by its deg_in(v) in-neighbours), so its cost is modelled as
1 + beta * (F / deg_in(v)) / 64 (a descriptor, plus 64-entry segments); rows are cut
greedily at `budget` cost units and items ordered by cost, heaviest first. Compared with
the edge-count schedule (chunk 64) on the cfg2 step's max-backward group, in ONE process.
Usage (GPU box): python scripts/probes/bwd_sched_step.py. Result (round 3): no gain
(best 257.6 vs 259.5 us per step)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import plagnn  # noqa: E402
from plagnn import workload as W  # noqa: E402


def weighted_schedule(tptr, tcol, deg_in, F, beta, budget):
    items, merges = [], []
    slot = 0
    cost_of = []
    for u in range(len(tptr) - 1):
        b, e = int(tptr[u]), int(tptr[u + 1])
        if e == b:
            items.append((u, b, e, -1)); cost_of.append(0.0)
            continue
        c = 1.0 + beta * (F / np.maximum(deg_in[tcol[b:e]], 1)) / 64.0
        total = float(c.sum())
        if total <= budget:
            items.append((u, b, e, -1)); cost_of.append(total)
            continue
        cum = np.cumsum(c)
        cuts = [b]
        base = 0.0
        for i in range(e - b):
            if cum[i] - base > budget and b + i > cuts[-1]:
                cuts.append(b + i)
                base = cum[i - 1]
        cuts.append(e)
        n = len(cuts) - 1
        merges.append((u, slot, n, 0))
        for i in range(n):
            k0, k1 = cuts[i], cuts[i + 1]
            items.append((u, k0, k1, slot + i))
            cost_of.append(float(c[k0 - b:k1 - b].sum()))
        slot += n
    order = np.argsort(-np.asarray(cost_of), kind="stable")
    it = np.asarray(items, np.int32)[order].reshape(-1)
    mg = np.asarray(merges if merges else [(0, 0, 0, 0)], np.int32).reshape(-1)
    return it, len(items), mg, len(merges), slot


def make_engine(wl, g):
    e = plagnn.TrainEngine(g, torch.from_numpy(wl.ds.feat), torch.from_numpy(wl.ds.loc.astype(np.float32)),
                           wl.dims, wl.class_weight, wl.train_index, wl.val_index, lr=5e-5, device="cuda",
                           edge_weight=wl.edge_weight)
    e.capture(warmup=2)
    for _ in range(3):
        e.step()
    return e


def main():
    wl = W.build(os.environ.get("CONFIG", "cfg2"), device="cuda")
    variants = {"chunk64": None}
    for beta in (1.0, 2.0, 4.0):
        for budget in (48, 64, 96):
            variants[f"b{beta:g}_B{budget}"] = (beta, budget)
    engines = {}
    for name, v in variants.items():
        g = plagnn.CSRGraph(wl.src, wl.dst, wl.ds.n)
        if v is not None:
            deg_in = np.diff(g.fwd.ptr)
            it, ni, mg, nm, ns = weighted_schedule(g.bwd.ptr, g.bwd.col, deg_in, 256, *v)
            h = g.bwd
            h.items, h.n_items, h.merges, h.n_merges, h.n_slots = it, ni, mg, nm, ns
        engines[name] = (make_engine(wl, g), g.bwd.n_items, g.bwd.n_merges)
        print(f"{name}: {engines[name][1]} items, {engines[name][2]} split rows", flush=True)
    res = {k: [] for k in engines}
    for _ in range(3):
        for k, (e, _, _) in engines.items():
            res[k].append(e.group_times(groups=("spmm_max_bwd",), reps=10)["spmm_max_bwd"]["ms"])
    for k in engines:
        print(f"{k:12s}: spmm_max_bwd {np.median(res[k]) * 1e3:7.1f} us/step", flush=True)


if __name__ == "__main__":
    main()
