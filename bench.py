#!/usr/bin/env python3
"""PLA-GNN training-step benchmark on MI355X (BASELINE.json metric).

metric: edges aggregated / s per training epoch, full graph. One step = one full-graph
training epoch of the reference (code/train.py:197-207: zero_grad, forward, multi_loss on
the train rows, backward, Adam.step, val loss on the same logits); edges per step =
L_sage * E' (E' = PPI edges + N self-loops). Default workload (BASELINE configs[1]):
synthetic PPI stand-in S0 (N = 24,041, power-law, mean degree 50, E' ~ 1.23 M), 3 SAGE-pool
layers of hidden 256 (503 -> 256 -> 256 -> 256, MLP 256 -> 100 -> 12), fp32. The other
configs are plagnn.workload.CONFIGS (--config).

Multi-GPU (torch.distributed.run, one rank per GPU), --mode:
  replicas (default, Mode A): the reference's own parallelism — its 10 rounds x 10 folds
    are independent trainings (code/train.py:162-178), so rank r trains job r (round
    r // 10, fold r % 10) on its own full-graph replica with its own initial parameters,
    with NO collective. Weak scaling: value = sum over ranks of edges / max-over-ranks time.
  dp (Mode B; the default for cfg4, BASELINE configs[3]): one shared model; every rank
    starts from rank 0's parameters and each step ends with ONE RCCL all-reduce (average)
    of the flat gradient bucket before Adam. cfg4: rank r trains perturbation graph
    r % 4 (different graphs: value = sum over ranks, weak scaling); other configs: rank r
    trains the rows train_index[r::world] of the same graph, every rank repeating the same
    full-graph forward/backward, so value = ONE model's edges / time (strong scaling).

At N = 1 the line also carries `sub_configs`: ref (the reference dims), cfg3 (hidden
512, edge-weighted) and cfg5 (RMAT x16, bf16), each timed the same way in a child process
started before this process touches the GPU (as is the drop-in leg), so that every GEMM
dispatch of this process belongs to the headline engine's steps.

Beside the engine's number (`value`), rank 0 at N = 1 also reports
  * `dropin`: the unmodified reference loop on the dgl shim (plagnn.model + torch Adam,
    exactly what main_normal.py -d cuda runs, code/train.py:197-207);
  * `epoch_with_eval`: the reference-faithful epoch with its per-epoch evaluation
    (code/train.py:210-218) on the device kernels;
  * `cpu_baseline`: the oracle run as DGL's CPU backend runs it (OpenMP rows + torch-CPU).

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

PEAK_HBM_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_F32_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32 MFMA (= vector) dense peak
# MI355X_MICROARCH.md: bf16 MFMA ~2.5 PF dense = 256 CUs x 4 SIMDs x (2*32*32*16 flops per
# 32-cycle v_mfma_f32_32x32x16_bf16) x 2.4 GHz
PEAK_BF16_TFLOPS = 2516.6
# The aligned f32 GEMMs run as three-piece bf16 splits (gemm_x3.hip): 6 bf16 MFMA products per
# f32 block, so their own ceiling is the bf16 peak / 6 in f32-equivalent flops
X3_CEILING_TFLOPS = PEAK_BF16_TFLOPS / 6
ALPHA = 0.1               # main_normal.py -a default (code/main_normal.py:29)
# MI355X_MICROARCH.md "Indexed rows": rows gathered from an XCD's L2 16.8-18.8 TB/s chip-wide
# (a uniformly random 38 MB table from the Infinity Cache: 8.6 TB/s)
L2_GATHER_GBS = 17800.0
# the same section: uniformly random rows of a 151 MB table (Infinity-Cache resident) 7.4-7.9
# TB/s; rows of a buffer far larger than the Infinity Cache 5.5-5.8 TB/s (register gather)
MALL_GATHER_GBS = 7900.0
HBM_GATHER_GBS = 5800.0
MALL_BYTES = 256 << 20


def gather_regime(n_rows: int, elem_bytes: int):
    """The random-row gather ceiling that applies to the max forward, chosen by the bytes of
    one 256-column feature tile of X (the table one gather pass draws rows from): up to
    32 MiB the library cuts the tile's columns into 256-B slices dealt to the XCDs (S0: 6.2 MB
    per slice, L2 hit 0.77 with the power-law reuse), so the L2-served rate applies; up to the
    256 MiB Infinity Cache the 151-MB random-row rate; beyond it the HBM random-row rate.
    Returns (bound, peak GB/s, peak_is)."""
    tile = n_rows * 256 * elem_bytes
    if tile <= 32 << 20:
        return "l2_gather", L2_GATHER_GBS, (f"L2-served random-row gather ceiling (MI355X_MICROARCH.md, indexed rows): "
                                            f"a {tile / 2**20:.1f} MiB feature tile, sliced over the XCDs")
    if tile <= MALL_BYTES:
        return "mall_gather", MALL_GATHER_GBS, (f"Infinity-Cache random-row gather ceiling, 151 MB table "
                                                f"(MI355X_MICROARCH.md, indexed rows: 7.4-7.9 TB/s): a {tile / 2**20:.0f} MiB "
                                                f"feature tile fits the 256 MiB Infinity Cache, not the 4 MiB L2s")
    return "hbm_gather", HBM_GATHER_GBS, (f"HBM random-row gather rate (MI355X_MICROARCH.md: 5.5-5.8 TB/s): a "
                                          f"{tile / 2**20:.0f} MiB feature tile exceeds the Infinity Cache")


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_threads() -> int:
    """The threads this job may use: OMP_NUM_THREADS when the launcher sets it (the GPU box
    sets it to the job's CPU share), else the CPUs in this process's affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_baseline(wl, dims, seconds: float = 20.0, min_steps: int = 5):
    """The oracle run the way DGL's CPU backend runs the reference step: SpMM-max rows under
    OpenMP, backward via torch-CPU scatter_add_, dense algebra in torch-CPU fp32, with every
    CPU thread of the job; median of >= min_steps full steps (bounded by `seconds`). Also
    the reference-faithful epoch: the step plus code/train.py:210-214's evaluation
    (protein_loc_correction with its per-row loop, performances_record on the train and
    val rows)."""
    import oracle

    threads = _cpu_threads()
    torch.set_num_threads(threads)
    os.environ["OMP_NUM_THREADS"] = str(threads)
    src, dst, w = wl.edges_without_loops()
    og = oracle.OracleGraph(src, dst, wl.n, edge_weight=w)
    use_w = w is not None
    x = torch.from_numpy(wl.ds.feat)
    labels = torch.from_numpy(wl.ds.loc.astype(np.float32))
    p = oracle.init_params(dims, seed=0)
    keys = list(p)
    m = [torch.zeros_like(p[k]) for k in keys]
    v = [torch.zeros_like(p[k]) for k in keys]
    times, eval_times = [], []
    t_start = time.perf_counter()
    step = 0
    while True:
        t0 = time.perf_counter()
        logits, _, grads = oracle.train_step(og, x, labels, wl.train_index, wl.class_weight, p, use_weight=use_w,
                                             parallel=True)
        step += 1
        oracle.adam_step_torch110([p[k] for k in keys], [grads[k] for k in keys], m, v, step, 5e-5)
        oracle.multi_loss(logits[wl.val_index], labels[wl.val_index], wl.class_weight)
        t1 = time.perf_counter()
        times.append(t1 - t0)
        if step <= 2:  # the reference-faithful epoch's evaluation, timed on two epochs
            pred = oracle.protein_loc_correction(logits, ALPHA, rowwise=True)
            oracle.performances_record(labels[wl.train_index], pred[wl.train_index])
            oracle.performances_record(labels[wl.val_index], pred[wl.val_index])
            eval_times.append(time.perf_counter() - t1)
        if step >= min_steps and time.perf_counter() - t_start > seconds:
            break
        if step >= 50:
            break
    t = float(np.median(times))
    t_eval = float(np.median(eval_times))
    L = len(dims) - 3
    return {"value": round(L * og.num_edges / t, 1), "unit": "edges/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "nproc": os.cpu_count(), "ms_per_step": round(t * 1e3, 2),
            "steps_timed": step, "epoch_with_eval_ms": round((t + t_eval) * 1e3, 2),
            "sample": f"median of {step} full training steps of the oracle on the same graph and dims "
                      f"(SpMM-max rows OpenMP-parallel C, backward torch scatter_add_, dense torch-CPU fp32, "
                      f"{threads} threads); epoch_with_eval adds code/train.py:210-214's evaluation "
                      f"(per-row loops, median of {len(eval_times)})"}


def dropin_leg(wl, dims, dev, steps: int, warmup: int):
    """What `main_normal.py -d cuda` runs per epoch (code/train.py:197-207) on the dgl shim:
    GNN32/GNN module, multi_loss, autograd, torch.optim.Adam, val loss on the same logits."""
    import dgl
    from plagnn.model import GNN
    from plagnn.train import multi_loss

    if wl.edge_weight is not None:
        return None  # the reference's SAGEConv('pool') call takes no edge weights
    src, dst, _ = wl.edges_without_loops()
    g = dgl.add_self_loop(dgl.graph((torch.from_numpy(src), torch.from_numpy(dst)), num_nodes=wl.n)).to(dev)
    features = torch.from_numpy(wl.ds.feat).to(dev)
    labels = torch.from_numpy(wl.ds.loc.astype(np.float32)).to(dev)
    tr = torch.as_tensor(wl.train_index, device=dev)
    va = torch.as_tensor(wl.val_index, device=dev)
    torch.manual_seed(0)
    model = GNN(dims).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=5e-5)

    def epoch():
        opt.zero_grad()
        model.train()
        logits = model(g, features)
        train_loss = multi_loss(logits[tr], labels[tr], wl.class_weight)
        train_loss.backward()
        opt.step()
        model.eval()
        val_loss = multi_loss(logits[va], labels[va], wl.class_weight)
        return train_loss, val_loss

    for _ in range(warmup):
        epoch()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        tl, vl = epoch()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    L = len(dims) - 3
    return {"ms_per_step": round(ms, 4), "value": round(L * (len(wl.src)) / ms * 1e3, 1), "unit": "edges/s",
            "loss": {"train": float(tl.detach()), "val": float(vl.detach())},
            "what": "unmodified reference epoch body on the dgl shim: plagnn.model + multi_loss + autograd + "
                    "torch.optim.Adam (code/train.py:197-207)"}


def dropin_epoch_with_eval(wl, dims, dev, epochs: int = 2) -> dict:
    """The epoch a `main_normal.py -d cuda` user pays (code/train.py:197-218): the shim step
    (plagnn.model + multi_loss + autograd + Adam) plus the reference's own per-epoch
    evaluation as its code runs it: protein_loc_correction's per-row loop over all N rows
    (train.py:36-38) and performances_record's host copies and per-row loops on the train
    and val rows (52-53, 60-78), then the two loss values read on the host (217-218).
    Median of `epochs` epochs after one warm-up epoch (each takes seconds)."""
    import dgl
    from plagnn.model import GNN
    from plagnn.train import loc_correction_per_row, multi_loss, performances_per_row

    src, dst, _ = wl.edges_without_loops()
    g = dgl.add_self_loop(dgl.graph((torch.from_numpy(src), torch.from_numpy(dst)), num_nodes=wl.n)).to(dev)
    features = torch.from_numpy(wl.ds.feat).to(dev)
    labels = torch.from_numpy(wl.ds.loc.astype(np.float32)).to(dev)
    tr = torch.as_tensor(wl.train_index, device=dev)
    va = torch.as_tensor(wl.val_index, device=dev)
    torch.manual_seed(0)
    model = GNN(dims).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=5e-5)
    times, evals = [], []
    for e in range(epochs + 1):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        opt.zero_grad()
        model.train()
        logits = model(g, features)
        train_loss = multi_loss(logits[tr], labels[tr], wl.class_weight)
        train_loss.backward()
        opt.step()
        model.eval()
        val_loss = multi_loss(logits[va], labels[va], wl.class_weight)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        pred = loc_correction_per_row(logits.detach(), ALPHA)
        performances_per_row(labels[tr], pred[tr.cpu()])
        performances_per_row(labels[va], pred[va.cpu()])
        train_loss.item(), val_loss.item()
        t2 = time.perf_counter()
        if e > 0:
            times.append(t2 - t0)
            evals.append(t2 - t1)
    return {"ms": round(float(np.median(times)) * 1e3, 2), "eval_ms": round(float(np.median(evals)) * 1e3, 2),
            "epochs": epochs,
            "what": "shim step + the reference's per-epoch evaluation as its code runs it (per-row Python loops over "
                    "the N rows and the labelled rows, host copies; code/train.py:19-86, 197-218)"}


def dropin_device_time(wl, dims, dev, reps: int = 20) -> float:
    """The device time of the shim model's forward + backward alone (without the reference's
    multi_loss host loop and Adam): zero_grad + model(g, features).backward(G) with a fixed
    upstream gradient G, issued `reps` times back to back between two HIP events after a
    warm-up. zero_grad as the reference's epoch does it (code/train.py:197, optimizer.
    zero_grad() on the installed torch: gradients set to None, so backward writes them
    instead of adding into the previous ones). The host issues one iteration in well under
    the device time, so the queue stays full and the events see device time."""
    import dgl
    from plagnn.model import GNN

    src, dst, _ = wl.edges_without_loops()
    g = dgl.add_self_loop(dgl.graph((torch.from_numpy(src), torch.from_numpy(dst)), num_nodes=wl.n)).to(dev)
    features = torch.from_numpy(wl.ds.feat).to(dev)
    torch.manual_seed(0)
    model = GNN(dims).to(dev)
    dlog = torch.randn(wl.n, dims[-1], device=dev) * 1e-3
    for _ in range(5):
        model.zero_grad()
        model(g, features).backward(dlog)
    torch.cuda.synchronize(dev)
    ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ea.record()
    for _ in range(reps):
        model.zero_grad()
        model(g, features).backward(dlog)
    eb.record()
    torch.cuda.synchronize(dev)
    return ea.elapsed_time(eb) / reps


def epoch_with_eval_leg(engine, wl, dev, epochs: int = 20):
    """The reference-faithful epoch (code/train.py:197-218): the engine's step, then
    protein_loc_correction on all logits and performances_record on the train and val rows
    (device kernels, plagnn.loc_eval), and the two loss values read on the host."""
    from plagnn import loc_eval

    labels = torch.from_numpy(wl.ds.loc.astype(np.float32)).to(dev)
    tr = torch.as_tensor(wl.train_index, device=dev)
    va = torch.as_tensor(wl.val_index, device=dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(epochs):
        engine.step()
        pred = loc_eval.protein_loc_correction(engine.logits(), ALPHA)
        loc_eval.performances_record(labels[tr], pred[tr])
        loc_eval.performances_record(labels[va], pred[va])
        engine.losses()
    torch.cuda.synchronize(dev)
    return round((time.perf_counter() - t0) / epochs * 1e3, 4)


def _roofline(engine, gt, bf16):
    """Roofline of each launch group from TrainEngine.group_times (the group's launches of
    one step, replayed as a graph: the benchmark's own execution), with the algorithmic
    work of SURVEY.md §8(d) at the true dims."""
    L = engine.L
    work = {"gemm": float(engine.flops_per_step()),
            "spmm_max_fwd": float(sum(engine.spmm_bytes(l) for l in range(L))),
            "spmm_max_bwd": float(sum(engine.spmm_bwd_bytes(l) for l in range(L))),
            "adam": 16.0 * engine.flat.numel(),
            "head": float(engine.head_flops_per_step())}
    gemm_group = "gemm_bf16" if bf16 else "gemm_f32"
    groups = {}
    for gname, r in gt.items():
        name = gemm_group if gname == "gemm" else gname
        groups[name] = {"ms": r["ms"], "launches": r["launches"], "work": work.get(gname, 0.0)}

    def roof(gname):
        g = groups[gname]
        sec = g["ms"] / 1e3
        base = {"kernel": gname, "launches_per_step": g["launches"], "ms_per_step": round(g["ms"], 4),
                "us_per_launch": round(g["ms"] * 1e3 / g["launches"], 2)}
        if gname == gemm_group:
            # algorithmic flops at the true (unpadded) dims, not the padded launch shapes
            ach = g["work"] / sec / 1e12
            r = {"bound": "mfma", "achieved": round(ach, 2), "unit": "TFLOP/s", **base,
                 "flops_per_step": int(g["work"]),
                 "compulsory_bytes_per_launch": round(engine.gemm_bytes_per_step() / g["launches"])}
            if bf16:
                r.update(peak=PEAK_BF16_TFLOPS, frac=round(ach / PEAK_BF16_TFLOPS, 4))
            else:
                # the pipe the kernel runs on: three-piece bf16 products (6 per f32 block)
                r.update(peak=round(X3_CEILING_TFLOPS, 1), frac=round(ach / X3_CEILING_TFLOPS, 4),
                         peak_is="bf16 MFMA peak / 6 (three-piece f32 split, gemm_x3.hip)",
                         peak_f32_mfma=PEAK_F32_TFLOPS, frac_vs_f32_mfma=round(ach / PEAK_F32_TFLOPS, 4))
            return r
        if gname == "head":
            # the fused MLP head (pg_mlp_l1_head): liner1's forward and input-gradient products
            # (three-piece MFMA) with the loss in between; its flops against the same ceiling
            ach = g["work"] / sec / 1e12
            return {"bound": "mfma", "achieved": round(ach, 2), "unit": "TFLOP/s", **base,
                    "flops_per_step": int(g["work"]), "peak": round(X3_CEILING_TFLOPS, 1),
                    "frac": round(ach / X3_CEILING_TFLOPS, 4),
                    "what": "liner1 forward + liner2/sigmoid/multi_loss/dZ/dA4 + liner1 input gradient, one launch "
                            "(+ the loss reduction); flops of the two liner1 products"}
        ach = g["work"] / sec / 1e9
        if gname == "spmm_max_fwd":
            # per-edge row gathers (SURVEY.md §8d bytes) are served mostly by the L2s and the
            # 256 MiB Infinity Cache, not HBM (PMC: the fabric sees a quarter of them on S0):
            # the bound is the random-row gather rate of the regime the feature tile's size
            # puts it in; the HBM figure stays beside it
            bound, peak, peak_is = gather_regime(engine.N, 2 if bf16 else 4)
            return {"bound": bound, "achieved": round(ach, 1), "peak": peak, "unit": "GB/s",
                    "frac": round(ach / peak, 4), **base, "bytes_per_step": int(g["work"]),
                    "peak_is": peak_is, "peak_hbm": PEAK_HBM_GBS, "frac_vs_hbm": round(ach / PEAK_HBM_GBS, 4)}
        return {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(ach / PEAK_HBM_GBS, 4), **base, "bytes_per_step": int(g["work"])}

    return groups, roof


def _traffic(config, group, calls_per_step):
    """HBM bytes per library call (as `achieved`: a call can be several kernel dispatches) of
    `group` from the committed PMC passes (profiles/pmc_traffic.json, scripts/pmc_traffic.sh:
    2 FETCH_SIZE + WRITE_SIZE of every dispatch of the group, per step), or None."""
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(tfile):
        return None
    with open(tfile) as f:
        b = json.load(f).get(config, {}).get("bytes_per_step", {}).get(group)
    if b is None or not calls_per_step:
        return None
    return round(b / calls_per_step)


def _job_of(rank, mode):
    return rank if mode == "replicas" else 0


def _median_ms(evs):
    return float(np.median([a.elapsed_time(b) for a, b in evs])) if evs else None


def run(args, rank, world, dev, dist, mode, breakdown=True):
    """Build, capture and time one config; returns the result dict (rank 0) or None.
    breakdown=False (the N > 1 dp leg beside the replicas headline): no per-group timing,
    the line's timing fields plus the all-reduce's own time."""
    import plagnn
    from plagnn import workload as W

    job = _job_of(rank, mode)
    wl = W.build(args.config, rank=rank, device=dev, job=job)
    if mode == "dp" and world > 1 and args.config != "cfg4":
        wl.train_index = wl.train_index[rank::world]  # the fold's train rows sharded over ranks
    graph = wl.graph()
    dims, bf16 = wl.dims, wl.bf16
    if wl.conv != "pool":
        raise SystemExit(f"--config {args.config}: TrainEngine runs SAGEConv 'pool' layers; {wl.conv} runs on the "
                         f"dgl shim (tests/test_gpu_graphconv.py)")
    Engine = plagnn.TrainEngineBF16 if bf16 else plagnn.TrainEngine
    engine = Engine(graph, torch.from_numpy(wl.ds.feat), torch.from_numpy(wl.ds.loc.astype(np.float32)),
                    dims, wl.class_weight, wl.train_index, wl.val_index, lr=5e-5, device=dev,
                    edge_weight=wl.edge_weight, seed=job)
    allreduce = None
    if dist is not None and mode == "dp":
        from plagnn import dist as pdist

        engine.broadcast_params()  # identical starting replicas
        # two gradient buckets (top SAGE layer + MLP, then the layers below); over RCCL both
        # all-reduces are captured into the step graph, the first under the rest of the backward
        allreduce = pdist.BucketAllReduce(engine.gflat, engine.grad_buckets())

    if args.eager:  # PMC passes: every launch a plain dispatch (counters see graph replays poorly)
        for _ in range(args.warmup):
            engine.step_eager(allreduce)
    else:
        n_cap_warm = min(2, args.warmup)
        engine.capture(warmup=n_cap_warm, allreduce=allreduce)
        for _ in range(args.warmup - n_cap_warm):
            engine.step()
    step = (lambda: engine.step_eager(allreduce)) if args.eager else engine.step
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    edges = torch.tensor([float(engine.edges_per_step)], dtype=torch.float64, device=dev)
    summed = world > 1 and (mode == "replicas" or args.config == "cfg4")
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if summed:
            dist.all_reduce(edges, op=dist.ReduceOp.SUM)
    t_max = t.item()
    value = edges.item() * args.steps / t_max
    # per-step distribution (median of >= 50 steps), after the timed region:
    # each step bracketed by HIP events on the stream the graphs replay on
    n_med = max(50, args.steps)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_med)]
    for ea, eb in evs:
        ea.record()
        step()
        eb.record()
    torch.cuda.synchronize(dev)
    per_step = np.array(sorted(ea.elapsed_time(eb) for ea, eb in evs))
    med = float(np.median(per_step))
    step_dist = {"steps": n_med, "median_ms": round(med, 4),
                 "p10_ms": round(float(np.percentile(per_step, 10)), 4),
                 "p90_ms": round(float(np.percentile(per_step, 90)), 4),
                 "value_at_median": round(edges.item() / (med / 1e3), 1)}
    allreduce_ms = None
    if allreduce is not None and not args.eager:
        if engine.allreduce_in_graph:
            # the collective is inside the step graph: time the same bucket all-reduces alone,
            # eagerly on the replay stream, as many times (the gradients are rewritten by the
            # next step's backward, so averaging them again changes nothing that is kept)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_med)]
            for ea, eb in evs:
                ea.record()
                allreduce()
                eb.record()
            torch.cuda.synchronize(dev)
            ar = torch.tensor([_median_ms(evs)], dtype=torch.float64, device=dev)
        else:
            # between the two replayed graphs: HIP events around it on the replay stream, over
            # as many more steps (each rank's median, then the max over ranks)
            engine.ar_events = []
            for _ in range(n_med):
                step()
            torch.cuda.synchronize(dev)
            ar = torch.tensor([_median_ms(engine.ar_events)], dtype=torch.float64, device=dev)
            engine.ar_events = None
        dist.all_reduce(ar, op=dist.ReduceOp.MAX)
        allreduce_ms = ar.item()
    loss_tr, loss_va = engine.losses()
    if not (np.isfinite(loss_tr) and np.isfinite(loss_va)):
        raise SystemExit(f"non-finite loss after training: {loss_tr}, {loss_va}")
    if dist is not None and mode == "dp":
        # every rank must hold bitwise the same parameters after the timed steps: the
        # element-wise MIN and MAX over ranks of the whole flat buffer (as int32 bits) agree
        bits = engine.flat.view(torch.int32)
        lo, hi = bits.clone(), bits.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        if not torch.equal(lo, hi):
            raise SystemExit(f"replicas diverged at {int((lo != hi).sum())} of {bits.numel()} parameters")
    if dist is not None:
        dist.barrier()
    if rank != 0:
        return None
    ar_info = None
    if allreduce_ms is not None:
        nbytes = engine.gflat.numel() * engine.gflat.element_size()
        inside = engine.allreduce_in_graph
        ar_info = {"ms_per_step": round(allreduce_ms, 4), "bytes": nbytes,
                   "op": f"AVG, {len(allreduce.buckets)} f32 buckets of one flat buffer "
                         f"({', '.join(str((b - a) * 4) for a, b in allreduce.buckets)} B)",
                   "in_step_graph": inside,
                   "timing": ("the collective alone: HIP events around the buckets' eager all-reduces on the replay "
                              "stream, median over steps, max over ranks; in the step it runs inside the graph on a "
                              "communication stream, the first bucket beside the rest of the backward"
                              if inside else
                              "HIP events around the eager all-reduce between the two replayed graphs, "
                              "median over steps, max over ranks"),
                   "share_of_step": round(allreduce_ms / med, 4)}
    if not breakdown:
        return {"value": round(value, 1), "unit": "edges/s", "ms_per_step": round(t_max / args.steps * 1e3, 4),
                "step_distribution": step_dist,
                "scaling": "strong" if not summed else "weak",
                "overhead_only": not summed,
                "what": ("one shared model; every rank runs the full-graph step on its shard of the train rows, "
                         f"one {'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()} all-reduce of the "
                         "gradients per step; value = ONE model's edges/s, so it cannot exceed the N = 1 value: "
                         "this leg measures what the collective costs (overhead only), not a speed-up"
                         if not summed else "a different graph per rank; value sums the ranks"),
                "allreduce": ar_info, "loss": {"train": loss_tr, "val": loss_va}}

    # per-group times after the timed region, on rank 0 only (without the collective): each
    # group's launches of one step captured as a graph and replayed back to back
    gt = engine.group_times(reps=args.breakdown_reps)
    if args.dump_breakdown:  # per launch site, eager steps (diagnostic)
        with open(args.dump_breakdown, "w") as f:
            json.dump(engine.kernel_breakdown(5), f, indent=1)
    groups, roof = _roofline(engine, gt, bf16)
    dom = max(groups, key=lambda k: groups[k]["ms"])
    gemm_name = "gemm_bf16" if bf16 else "gemm_f32"
    rf = roof(dom)
    rf["timing"] = ("HIP events around back-to-back replays of a graph holding this group's launches of one step "
                    "(the step's own buffers), per step")
    rf["traffic"] = _traffic(args.config, dom, rf.get("launches_per_step"))
    if world > 1:
        par = (f"replicas{world}: independent (round, fold) trainings, no collective" if mode == "replicas" else
               f"dp{world}: shared model, one gradient all-reduce per step, "
               + ("a different perturbation graph per rank" if args.config == "cfg4" else "train rows sharded"))
    else:
        par = "single"
    return {
        "metric": "edges aggregated/sec per training epoch, full PPI graph",
        "value": round(value, 1),
        "pid": os.getpid(),
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_max / args.steps * 1e3, 4),
        "step_distribution": step_dist,
        "higher_is_better": True,
        "scaling": "strong" if (world > 1 and not summed) else "weak",
        "vs_baseline": None,
        "dtype": "bf16" if bf16 else "f32",
        "data": "synthetic (seeded power-law PPI stand-in; real PPI/GEO/UniProt inputs are not shipped)",
        "config": {"workload": f"{args.config}: {wl.desc}", "nodes": wl.n, "edges_with_self_loops": graph.num_edges,
                   "graph_variant_rank0": wl.variant, "sage_layers": len(dims) - 3, "dims": dims,
                   "edges_per_step": engine.edges_per_step, "mode": mode if world > 1 else "single",
                   "parallelism": par},
        "roofline": rf,
        "spmm_roofline": {k: roof(k) for k in ("spmm_max_fwd", "spmm_max_bwd") if k in groups},
        # the GEMM group's own roofline when another group dominates (cfg5)
        "gemm_roofline": roof(gemm_name) if gemm_name in groups and gemm_name != dom else None,
        "head_roofline": roof("head") if groups.get("head", {}).get("work") else None,
        "kernels_ms_per_step": {k: round(v["ms"], 4) for k, v in sorted(groups.items(), key=lambda kv: -kv[1]["ms"])},
        "allreduce": ar_info,
        "loss": {"train": loss_tr, "val": loss_va},
        "_engine": engine,
        "_wl": wl,
    }


def _child(args, extra):
    """Run this script in a child process (started before this process initialises the GPU,
    so the GEMM dispatches of this process are the headline engine's alone); its JSON line."""
    import subprocess

    cmd = [sys.executable, os.path.abspath(__file__), "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--no-cpu-baseline", "--no-legs", "--sub-configs", "", "--breakdown-reps", str(args.breakdown_reps)] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise SystemExit(f"child {extra} failed (rc {r.returncode}):\n{r.stderr[-3000:]}")
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


def sub_configs(args):
    """The other single-GPU configs, each in a child process of its own, timed with the same
    steps / warm-up."""
    out = {}
    for name in [c for c in args.sub_configs.split(",") if c]:
        t0 = time.perf_counter()
        res = _child(args, ["--config", name])
        keep = ("value", "unit", "ms_per_step", "step_distribution", "dtype", "config", "roofline", "spmm_roofline",
                "gemm_roofline", "head_roofline", "kernels_ms_per_step", "loss")
        out[name] = {k: res[k] for k in keep}
        out[name]["child_wall_s"] = round(time.perf_counter() - t0, 1)
        print(f"sub-config {name}: {res['ms_per_step']} ms/step", file=sys.stderr, flush=True)
    return out


def _device(local_rank: int) -> torch.device:
    """One rank per GPU; more ranks than GPUs (a rehearsal of the N-rank flow on a smaller
    box, with PLAGNN_BENCH_BACKEND=gloo) share them round-robin."""
    local_dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_dev)
    return torch.device("cuda", local_dev)


def _device_info(dev) -> dict:
    props = torch.cuda.get_device_properties(dev)
    return {"device": dev.index, "name": props.name, "pci_bus_id": getattr(props, "pci_bus_id", None),
            "uuid": str(getattr(props, "uuid", ""))}


def guarded_dp_leg(args, rank, world, dev, dist, ctrl):
    """The N > 1 RCCL data-parallel leg beside the replicas headline, as a leg: a failure
    (on any rank) is recorded as {"error": ...} and the headline still prints. Every rank
    takes the same path: each reports ok / failed over `ctrl` (a gloo group, usable even
    when the RCCL communicator is what failed) and all of them agree on the outcome."""
    err = None
    res = None
    try:
        res = run(args, rank, world, dev, dist, "dp", breakdown=False)
    except (Exception, SystemExit) as e:  # run() raises SystemExit on diverged replicas
        err = f"rank {rank}: {type(e).__name__}: {e}"[-500:]
        print(f"dp leg failed on {err}", file=sys.stderr, flush=True)
    # (without a gloo group the default one carries it: a device tensor for RCCL)
    on_dev = ctrl is None and dist.get_backend() == "nccl"
    flag = torch.tensor([1 if err else 0], dtype=torch.int32, device=dev if on_dev else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=ctrl)
    if flag.item():
        return {"error": err or "failed on another rank (see its stderr)"} if rank == 0 else None
    return res


def main(argv=None):
    from plagnn import workload as W

    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg2", choices=sorted(W.CONFIGS))
    ap.add_argument("--mode", default="auto", choices=["auto", "replicas", "dp"],
                    help="N > 1: replicas = independent (round, fold) trainings, dp = shared model + all-reduce "
                         "(auto: dp for cfg4, replicas otherwise)")
    ap.add_argument("--sub-configs", default="ref,cfg3,cfg5",
                    help="N = 1: other configs timed in child processes (comma list, '' for none)")
    ap.add_argument("--eager", action="store_true", help="no HIP graph (PMC counter passes)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-legs", action="store_true", help="skip the drop-in and epoch-with-eval legs")
    ap.add_argument("--breakdown-reps", type=int, default=5, help="replays of each launch-group timing graph")
    ap.add_argument("--dump-breakdown", default="", help="write the per-launch-site breakdown (JSON)")
    ap.add_argument("--dropin-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--chunk-bwd", type=int, default=0, help=argparse.SUPPRESS)  # tuning experiments
    ap.add_argument("--bwd-trans-min", type=int, default=-1, help=argparse.SUPPRESS)  # A/B: transposed descriptors from E
    ap.add_argument("--separate-l1-head", action="store_true", help=argparse.SUPPRESS)  # A/B: unfused MLP head
    ap.add_argument("--separate-adam-prep", action="store_true", help=argparse.SUPPRESS)  # A/B: own prepare launch
    ap.add_argument("--split-l1-per-call", action="store_true", help=argparse.SUPPRESS)  # A/B: head splits W1
    args = ap.parse_args(argv)
    if args.separate_l1_head:
        import plagnn.engine

        plagnn.engine.TrainEngine.FUSED_L1_HEAD = False
    if args.separate_adam_prep:
        import plagnn.engine

        plagnn.engine.TrainEngine.FOLD_ADAM_PREP = False
    if args.split_l1_per_call:
        import plagnn.engine

        plagnn.engine.TrainEngine.KEEP_L1_PIECES = False
    if args.bwd_trans_min >= 0:
        import plagnn.graph

        plagnn.graph.TRANS_MIN_EDGES = args.bwd_trans_min
    if args.chunk_bwd:
        import plagnn.graph

        plagnn.graph.CHUNK_BWD_OVERRIDE = args.chunk_bwd

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    mode = args.mode if args.mode != "auto" else ("dp" if args.config == "cfg4" else "replicas")
    if args.dropin_only:
        wl = W.build(args.config, device="cuda")
        out = dropin_leg(wl, wl.dims, torch.device("cuda"), steps=min(args.steps, 20), warmup=3)
        if out is not None:
            out["model_fwd_bwd_device_ms"] = round(dropin_device_time(wl, wl.dims, torch.device("cuda")), 4)
            out["epoch_with_reference_eval"] = dropin_epoch_with_eval(wl, wl.dims, torch.device("cuda"))
        print(json.dumps(out))
        return
    subs = sub_configs(args) if (world == 1 and args.sub_configs) else None
    dropin = None
    if world == 1 and not args.no_legs and not W.CONFIGS[args.config][2]:
        try:
            dropin = _child(args, ["--config", args.config, "--dropin-only"])
        except SystemExit as e:  # a leg, not the headline: report it and go on
            dropin = {"error": str(e)[-500:]}
    dev = _device(local_rank)
    dist = None
    ctrl = None  # control-flag group (gloo) for the guarded dp leg
    if world > 1:
        import torch.distributed as dist

        backend = os.environ.get("PLAGNN_BENCH_BACKEND", "nccl")  # nccl = RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
            try:
                ctrl = dist.new_group(backend="gloo")
            except Exception as e:  # noqa: BLE001 — the dp leg's flag then goes over RCCL itself
                print(f"gloo control group unavailable ({e}); dp-leg status over {backend}", file=sys.stderr)
        else:
            dist.init_process_group(backend)

    dist_info = None
    if dist is not None:
        me = {"rank": rank, "local_rank": local_rank, **_device_info(dev)}
        every = [None] * world
        dist.all_gather_object(every, me)
        dist_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "ranks": every}
    out = run(args, rank, world, dev, dist, mode)
    # N > 1: the RCCL data-parallel leg in the same job, after the replicas headline; a leg,
    # so its failure is reported in the line and does not cost the headline
    dp_leg = None
    if world > 1 and mode == "replicas" and args.mode == "auto":
        dp_leg = guarded_dp_leg(args, rank, world, dev, dist, ctrl)
    if out is None:
        _finish(dist)
        return
    engine, wl = out.pop("_engine"), out.pop("_wl")
    if dist_info is not None:
        out["dist"] = dist_info
    if dp_leg is not None:
        out["dp"] = dp_leg
    legs = {}
    if world == 1 and not args.no_legs:
        legs["epoch_with_eval_ms"] = epoch_with_eval_leg(engine, wl, dev)
        if dropin is not None:
            # the engine's forward + backward (every group but Adam; the head includes its
            # fused loss) against the shim model's forward + backward device time
            eng = sum(v for k, v in out["kernels_ms_per_step"].items() if k != "adam")
            dropin["engine_fwd_bwd_device_ms"] = round(eng, 4)
            if dropin.get("model_fwd_bwd_device_ms"):
                dropin["model_vs_engine"] = round(dropin["model_fwd_bwd_device_ms"] / eng, 3)
            legs["dropin"] = dropin
            # beside the engine's epoch with eval: the epoch a main_normal.py -d cuda user pays
            ref_ep = dropin.get("epoch_with_reference_eval")
            if ref_ep:
                legs["dropin_epoch_with_reference_eval_ms"] = ref_ep["ms"]
    out.update(legs)
    cpu = None
    if world == 1 and not args.no_cpu_baseline and not args.config.startswith("cfg5"):
        cpu = cpu_baseline(wl, wl.dims)
    out["cpu_baseline"] = cpu
    if subs is not None:
        out["sub_configs"] = subs
    loss = out.pop("loss")
    out["loss"] = loss
    print(json.dumps(out), flush=True)
    _finish(dist)


def _finish(dist) -> None:
    """Tear the process group down after the line is out; a communicator left broken by a
    failed leg must not turn a printed result into a failed run."""
    if dist is None:
        return
    try:
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        print(f"destroy_process_group: {e}", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
