#!/usr/bin/env python3
"""PLA-GNN training-step benchmark on MI355X (BASELINE.json metric).

metric: edges aggregated / s per training epoch, full graph. One step = one full-graph
training epoch of the reference (code/train.py:197-207: zero_grad, forward, multi_loss on
the train rows, backward, Adam.step, val loss on the same logits); edges per step =
L_sage * E' (E' = PPI edges + N self-loops). Workload (BASELINE configs[1]): synthetic
PPI stand-in S0 (N = 24,041, power-law, mean degree 50, E' ~ 1.23 M), 3 SAGE-pool layers
of hidden 256 (503 -> 256 -> 256 -> 256, MLP 256 -> 100 -> 12), fp32.

Multi-GPU (torch.distributed.run, one rank per GPU, RCCL): every rank trains a full-graph
replica on its own graph (rank r: synthetic seed 70 + r, the perturbation-graph replicas
of BASELINE configs[3]) with ONE all-reduce (average) of the flat gradient bucket per step
before Adam; weak scaling. value = sum over ranks of edges / max-over-ranks time.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pla-gnn_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

CONFIGS = {
    # name: (graph kind, dims, description)
    "cfg2": ("s0", [503, 256, 256, 256, 100, 12],
             "S0 PPI stand-in (N=24041, mean deg 50), 3x SAGE-pool hidden 256, fp32"),
    "ref": ("s0", [503, 400, 300, 200, 100, 12],
            "S0 PPI stand-in, reference dims GNN32(503,400,300,200,100,12), fp32"),
    "cfg3": ("s0", [503, 512, 512, 512, 100, 12],
             "S0 perturbed (+-3% edges), ECC edge weights (pg_ecc, u_mul_e max), hidden 512, fp32"),
    "cfg5": ("rmat", [503, 512, 512, 512, 100, 12],
             "RMAT x16 PPI (N=384656, a,b,c,d=.57,.19,.19,.05, mean deg 50), hidden 512, bf16 storage, f32 accumulate"),
    "cfg5-f32": ("rmat", [503, 512, 512, 512, 100, 12],
                 "RMAT x16 PPI (N=384656, a,b,c,d=.57,.19,.19,.05, mean deg 50), hidden 512, fp32"),
}
BF16_CONFIGS = {"cfg5"}  # BASELINE configs[4]: "hidden=512 bf16"
PEAK_HBM_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_F32_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32 MFMA (= vector) dense peak
# MI355X_MICROARCH.md: bf16 MFMA ~2.5 PF dense = 256 CUs x 4 SIMDs x (2*32*32*16 flops per
# 32-cycle v_mfma_f32_32x32x16_bf16) x 2.4 GHz
PEAK_BF16_TFLOPS = 2516.6


def _group(name: str, gemm_group: str = "gemm_f32") -> str:
    if name.startswith("gemm"):
        return gemm_group
    return name.split(".")[0]


def _cfg3_graph(ds, seed):
    """the S0 graph perturbed (about 3 % of the undirected edges removed
    and as many random ones added, the ΔPCC-style topology change of
    data_preprocess.py:217-257), its edge clustering coefficients computed on the GPU
    (pg_ecc, data_preprocess.py:175-214) as edge weights; self-loops weigh 1.0."""
    from scipy.sparse import coo_matrix

    from plagnn import ecc

    rng = np.random.default_rng(seed)
    n = ds.n
    r, c = ds.row.astype(np.int64), ds.col.astype(np.int64)
    up = r < c
    ur, uc = r[up], c[up]
    keep = rng.random(len(ur)) >= 0.03
    na = int((~keep).sum())
    ar, ac = rng.integers(0, n, na), rng.integers(0, n, na)
    ok = ar != ac
    ur = np.concatenate([ur[keep], np.minimum(ar[ok], ac[ok])])
    uc = np.concatenate([uc[keep], np.maximum(ar[ok], ac[ok])])
    a = coo_matrix((np.ones(2 * len(ur), np.int64), (np.concatenate([ur, uc]), np.concatenate([uc, ur]))),
                   shape=(n, n)).tocsr()
    a.data[:] = 1
    a = a.tocoo()
    e = ecc.edge_clustering_coefficients(a).tocsr()
    src, dst = a.row.astype(np.int64), a.col.astype(np.int64)
    w = np.asarray(e[src, dst]).ravel().astype(np.float32)
    loops = np.arange(n, dtype=np.int64)
    src = np.concatenate([src, loops])
    dst = np.concatenate([dst, loops])
    w = np.concatenate([w, np.ones(n, np.float32)])
    return src, dst, torch.from_numpy(w)


def cpu_baseline(ds, dims, train_idx, w, seconds: float = 15.0):
    """The oracle (C restatement of DGL's CPU loops + torch-CPU fp32 dense algebra) timed
    on this host on the same graph and dims; bounded to ~`seconds` of work."""
    import oracle

    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    og = oracle.OracleGraph(ds.row, ds.col, ds.n)
    x = torch.from_numpy(ds.feat)
    labels = torch.from_numpy(ds.loc.astype(np.float32))
    p = oracle.init_params(dims, seed=0)
    keys = list(p)
    m = [torch.zeros_like(p[k]) for k in keys]
    v = [torch.zeros_like(p[k]) for k in keys]
    times = []
    t_start = time.perf_counter()
    step = 0
    while True:
        t0 = time.perf_counter()
        _, _, grads = oracle.train_step(og, x, labels, train_idx, w, p)
        step += 1
        oracle.adam_step_torch110([p[k] for k in keys], [grads[k] for k in keys], m, v, step, 5e-5)
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > seconds or step >= 5:
            break
    t = float(np.median(times))
    L = len(dims) - 3
    return {"value": L * og.num_edges / t, "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": f"{step} full training step(s) of the oracle on the same S0 graph and dims "
                      f"(median {t:.2f} s/step; SpMM in single-thread C, dense in torch-CPU with "
                      f"{threads} threads)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--breakdown-reps", type=int, default=5)
    ap.add_argument("--dump-breakdown", default="", help="write the per-launch-site breakdown (JSON)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)

    import plagnn
    from plagnn import data
    from plagnn.train import fold_splits, weight_cal

    kind, dims, desc = CONFIGS[args.config]
    ds = data.make_dataset(kind, seed=70 + rank)
    src, dst = ds.edges_with_self_loops()
    graph = plagnn.CSRGraph(src, dst, ds.n)
    label = [int(i) for i in ds.labelled]
    train_idx, val_idx = next(fold_splits(label, 10, 12))  # round 1, fold 1 (train.py:162-178)
    w = weight_cal(ds.loc)
    ew = None
    if args.config == "cfg3":
        src, dst, ew = _cfg3_graph(ds, 70 + rank)
        graph = plagnn.CSRGraph(src, dst, ds.n)
    bf16 = args.config in BF16_CONFIGS
    Engine = plagnn.TrainEngineBF16 if bf16 else plagnn.TrainEngine
    gemm_group = "gemm_bf16" if bf16 else "gemm_f32"
    engine = Engine(graph, torch.from_numpy(ds.feat), torch.from_numpy(ds.loc.astype(np.float32)),
                                dims, w, train_idx, val_idx, lr=5e-5, device=dev, edge_weight=ew,
                                seed=rank)
    allreduce = None
    if dist is not None:
        from plagnn.dist import allreduce_mean as allreduce

    n_cap_warm = min(2, args.warmup)
    engine.capture(warmup=n_cap_warm, allreduce=allreduce)
    for _ in range(args.warmup - n_cap_warm):
        engine.step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        engine.step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    edges = torch.tensor([float(engine.edges_per_step)], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(edges, op=dist.ReduceOp.SUM)
    t_max = t.item()
    value = edges.item() * args.steps / t_max
    loss_tr, loss_va = engine.losses()
    if not (np.isfinite(loss_tr) and np.isfinite(loss_va)):
        raise SystemExit(f"non-finite loss after training: {loss_tr}, {loss_va}")

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    # per-kernel HIP-event breakdown (eager diagnostic steps, after the timed region)
    bd = engine.kernel_breakdown(args.breakdown_reps)
    if args.dump_breakdown:
        with open(args.dump_breakdown, "w") as f:
            json.dump(bd, f, indent=1)
    groups = {}
    for name, r in bd.items():
        gname = _group(name, gemm_group)
        g = groups.setdefault(gname, {"ms": 0.0, "work": 0.0, "launches": 0.0})
        g["ms"] += r["ms"]
        g["work"] += r["work"]
        g["launches"] += r["calls"]
    dom = max(groups, key=lambda k: groups[k]["ms"])

    def roof(gname):
        g = groups[gname]
        sec = g["ms"] / 1e3
        if gname == gemm_group:
            # algorithmic flops at the true (unpadded) dims, not the padded launch shapes
            ach = engine.flops_per_step() / sec / 1e12
            peak = PEAK_BF16_TFLOPS if bf16 else PEAK_F32_TFLOPS
            return {"kernel": gname, "bound": "mfma", "achieved": round(ach, 2), "peak": peak,
                    "unit": "TFLOP/s", "frac": round(ach / peak, 4),
                    "launches_per_step": g["launches"], "ms_per_step": round(g["ms"], 4)}
        ach = g["work"] / sec / 1e9
        return {"kernel": gname, "bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS,
                "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4),
                "launches_per_step": g["launches"], "ms_per_step": round(g["ms"], 4)}

    traffic = None
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    rf = roof(dom)
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f)
        traffic = tj.get(args.config, {}).get(dom)
    rf["traffic"] = traffic

    cpu = None
    if world == 1 and not args.no_cpu_baseline and args.config in ("cfg2", "ref"):
        cpu = cpu_baseline(ds, dims, train_idx, w)

    out = {
        "metric": "edges aggregated/sec per training epoch, full PPI graph",
        "value": round(value, 1),
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if bf16 else "f32",
        "data": "synthetic (seeded power-law PPI stand-in; real PPI/GEO/UniProt inputs are not shipped)",
        "config": {"workload": f"{args.config}: {desc}", "nodes": ds.n, "edges_with_self_loops": graph.num_edges,
                   "sage_layers": len(dims) - 3, "dims": dims, "edges_per_step": engine.edges_per_step,
                   "parallelism": f"replicas{world}+grad-allreduce" if world > 1 else "single"},
        "roofline": rf,
        "spmm_roofline": {k: roof(k) for k in ("spmm_max_fwd", "spmm_max_bwd") if k in groups},
        "kernels_ms_per_step": {k: round(v["ms"], 4) for k, v in sorted(groups.items(), key=lambda kv: -kv[1]["ms"])},
        "cpu_baseline": cpu,
        "loss": {"train": loss_tr, "val": loss_va},
    }
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
