"""The engine's multi-GPU path (bench.py --gpus N): world_size 2 over gloo with both ranks
on cuda:0. Every rank builds a TrainEngine on its own graph from the same parameters,
captures the step with a two-bucket plagnn.dist.BucketAllReduce (gloo: forward+backward
graph with the weight gradients in two grouped launches, the buckets' all-reduces, the Adam
graph) and replays it. Checked against the serial computation on the
oracle: p_{t+1} = Adam(p_t, (g_rank0(p_t) + g_rank1(p_t)) / 2) for both steps, and the two
ranks must hold bitwise identical parameters afterwards."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, ROOT, random_graph

pytestmark = pytest.mark.gpu
DIMS = (31, 24, 20, 16, 10, 12)
LR = 1e-3
DEV = "cuda"


def _problem(rank):
    n = 400
    src, dst = random_graph(n, 4000, seed=200 + rank, self_loop=False)
    rng = np.random.default_rng(rank)
    x = torch.from_numpy(rng.standard_normal((n, DIMS[0])).astype(np.float32))
    labels = torch.from_numpy((rng.random((n, DIMS[-1])) < 0.3).astype(np.float32))
    tr = list(range(0, n, 2))
    va = list(range(1, n, 4))
    return src, dst, n, x, labels, tr, va


def _weights():
    return np.linspace(0.5, 3.0, DIMS[-1])


def _params():
    from plagnn.model import GNN

    torch.manual_seed(0)
    return {k: v.detach().clone() for k, v in GNN(list(DIMS)).state_dict().items()}


def _worker(rank, world, port, outdir):
    import sys

    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import plagnn
    from plagnn import dist as pdist

    torch.cuda.set_device(0)
    assert pdist.init("gloo")
    src, dst, n, x, labels, tr, va = _problem(rank)
    loops = np.arange(n)
    g = plagnn.CSRGraph(np.concatenate([src, loops]), np.concatenate([dst, loops]), n)
    eng = plagnn.TrainEngine(g, x, labels, DIMS, _weights(), tr, va, lr=LR, device="cuda:0", params=_params())
    pdist.broadcast_([eng.flat])
    ar = pdist.BucketAllReduce(eng.gflat, eng.grad_buckets())
    assert len(ar.buckets) == 2 and not ar.capturable  # gloo: between the two graphs
    eng.capture(warmup=1, allreduce=ar)
    assert not eng.allreduce_in_graph
    eng.step()
    torch.cuda.synchronize()
    torch.save({k: v.cpu() for k, v in eng.state_dict().items()}, os.path.join(outdir, f"rank{rank}.pt"))
    torch.distributed.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_engine_two_rank_allreduce_matches_serial_adam(tmp_path, oracle_mod):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    for k in got[0]:
        assert torch.equal(got[0][k], got[1][k]), f"ranks diverged on {k}"
    p = _params()
    keys = list(p)
    m = [torch.zeros_like(p[k]) for k in keys]
    v = [torch.zeros_like(p[k]) for k in keys]
    probs = [_problem(r) for r in range(world)]
    last_avg = None
    for step in (1, 2):
        gs = []
        for src, dst, n, x, labels, tr, va in probs:
            og = oracle_mod.OracleGraph(src, dst, n)
            gs.append(oracle_mod.train_step(og, x, labels, tr, _weights(), p)[2])
        avg = {k: (gs[0][k] + gs[1][k]) / 2 for k in keys}
        params = [p[k] for k in keys]
        oracle_mod.adam_step_torch110(params, [avg[k] for k in keys], m, v, step, LR)
        p = dict(zip(keys, params))
        last_avg = avg
    for k in keys:
        scale = max(p[k].abs().max().item(), 1e-12)
        g = last_avg[k]
        settled = g.abs() > 1e-4 * max(g.abs().max().item(), 1e-30)
        err = ((got[0][k].double() - p[k].double()).abs() * settled).max().item()
        assert err <= 1e-4 * scale, f"{k}: {err:.3e} vs scale {scale:.3e}"


def _worker_cfg4(rank, world, port, outdir):
    """Rank r trains cfg4 replica r + 1 (GSE30931 / GSE27182 PPI_inter, reference dims)."""
    import sys

    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import plagnn
    from plagnn import dist as pdist
    from plagnn import workload
    from test_gpu_fullsize import _engine_signs

    torch.cuda.set_device(0)
    assert pdist.init("gloo")
    wl = workload.build("cfg4", rank=rank + 1, device="cuda:0")
    sd = torch.load(os.path.join(outdir, "sd.pt"), weights_only=True)
    if rank == 1:  # a different start everywhere but rank 0: the broadcast must fix it
        sd = {k: v + 0.01 for k, v in sd.items()}
    eng = plagnn.TrainEngine(wl.graph(), torch.from_numpy(wl.ds.feat), torch.from_numpy(wl.ds.loc.astype(np.float32)),
                             wl.dims, wl.class_weight, wl.train_index, wl.val_index, lr=5e-5, device="cuda:0",
                             params=sd)
    eng.broadcast_params()
    eng.forward()
    eng.backward()
    torch.cuda.synchronize()
    signs = {k: torch.from_numpy(v) if isinstance(v, np.ndarray) else v for k, v in _engine_signs(eng).items()}
    local = {k: v.cpu() for k, v in eng.grads().items()}
    pdist.allreduce_mean(eng.gflat)
    eng.adam()
    torch.cuda.synchronize()
    step1 = {k: v.cpu() for k, v in eng.state_dict().items()}
    eng.capture(warmup=0, allreduce=pdist.allreduce_mean)
    eng.step()
    torch.cuda.synchronize()
    step2 = {k: v.cpu() for k, v in eng.state_dict().items()}
    torch.save({"signs": signs, "local": local, "step1": step1, "step2": step2},
               os.path.join(outdir, f"cfg4_rank{rank}.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(600)
def test_cfg4_two_replicas_allreduce_matches_serial_adam(tmp_path, oracle_mod):
    """BASELINE configs[3] on two ranks: each holds a DIFFERENT cfg4 perturbation graph
    (GSE30931 and GSE27182 PPI_inter, N = 24,041, reference dims). Checked: each rank's
    local gradient against the oracle's on its own graph (the bars of
    test_gpu_fullsize._check_step), the step-1 parameters against serial Adam on the
    oracle's averaged gradients, and bitwise agreement of the ranks after a second,
    graph-captured step."""
    from plagnn import workload
    from test_gpu_fullsize import LR, _check_signs, _close_judged, _oracle_graph, _Yardstick

    world = 2
    dims = workload.CONFIGS["cfg4"][1]
    sd = oracle_mod.init_params(dims, seed=20)
    torch.save(sd, tmp_path / "sd.pt")
    mp.start_processes(_worker_cfg4, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = [torch.load(tmp_path / f"cfg4_rank{r}.pt", weights_only=True) for r in range(world)]
    for k in got[0]["step2"]:
        assert torch.equal(got[0]["step2"][k], got[1]["step2"][k]), f"ranks diverged on {k}"
    ref = []
    for r in range(world):
        wl = workload.build("cfg4", rank=r + 1, device=DEV)
        og = _oracle_graph(oracle_mod, wl)
        x = torch.from_numpy(wl.ds.feat)
        labels = torch.from_numpy(wl.ds.loc.astype(np.float32))
        signs = {k: v.numpy() if k.endswith("argpos") else v for k, v in got[r]["signs"].items()}
        _, _, g = oracle_mod.train_step(og, x, labels, wl.train_index, wl.class_weight, sd, signs=signs)
        _check_signs(signs)
        s64 = {k: v for k, v in signs.items() if not k.startswith("_")}
        exact = _Yardstick(lambda og=og, x=x, labels=labels, wl=wl, s64=s64: oracle_mod.train_step(
            og, x, labels, wl.train_index, wl.class_weight, sd, dtype=torch.float64, signs=s64))
        for k, v in g.items():
            _close_judged(got[r]["local"][k], v, lambda k=k, exact=exact: exact.get()[2][k], name=f"rank{r} grad {k}")
        ref.append(g)
    keys = list(sd)
    zeros = lambda: [torch.zeros_like(sd[k]) for k in keys]  # noqa: E731
    avg = {k: (ref[0][k] + ref[1][k]) / 2 for k in keys}
    p_ref = [sd[k].clone() for k in keys]
    oracle_mod.adam_step_torch110(p_ref, [avg[k] for k in keys], zeros(), zeros(), 1, LR)
    own = {k: (got[0]["local"][k] + got[1]["local"][k]) / 2 for k in keys}
    p_own = [sd[k].clone() for k in keys]
    oracle_mod.adam_step_torch110(p_own, [own[k] for k in keys], zeros(), zeros(), 1, LR)
    for k, pr, po in zip(keys, p_ref, p_own):
        for r in range(world):
            p1 = got[r]["step1"][k].double()
            scale = max(pr.abs().max().item(), 1e-12)
            g = avg[k].double()
            settled = g.abs() > 1e-4 * max(g.abs().max().item(), 1e-30)
            err = ((p1 - pr.double()).abs() * settled).max().item()
            assert err <= 1e-4 * scale, f"rank{r} adam {k}: {err:.3e} vs scale {scale:.3e}"
            assert (p1 - po.double()).abs().max().item() <= 1e-6 * scale, f"rank{r} adam(own grads) {k}"


def _worker_rccl_one_rank(rank, world, port, outdir):
    """RCCL with ONE rank (a one-GPU box cannot hold two RCCL ranks): the all-reduce of
    both buckets captured INTO the step graph on the communication stream (the N > 1
    path of bench.py), against the same engine run eagerly with the buckets reduced on the
    step's stream. An average over one rank is the identity, so the two must agree bitwise."""
    import sys

    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import plagnn
    from plagnn import dist as pdist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    src, dst, n, x, labels, tr, va = _problem(0)
    loops = np.arange(n)
    g = plagnn.CSRGraph(np.concatenate([src, loops]), np.concatenate([dst, loops]), n)
    out = {}
    for mode in ("graph", "eager"):
        eng = plagnn.TrainEngine(g, x, labels, DIMS, _weights(), tr, va, lr=LR, device="cuda:0", params=_params())
        ar = pdist.BucketAllReduce(eng.gflat, eng.grad_buckets())
        assert ar.capturable and len(ar.buckets) == 2
        if mode == "graph":
            eng.capture(warmup=1, allreduce=ar)
            assert eng.allreduce_in_graph
            for _ in range(3):
                eng.step()
        else:
            for _ in range(4):
                eng._uses_buckets(ar)
                eng.forward()
                eng.backward()
                ar()
                eng.adam()
        torch.cuda.synchronize()
        out[mode] = {k: v.cpu() for k, v in eng.state_dict().items()}
    torch.save(out, os.path.join(outdir, "rccl1.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_allreduce_in_step_graph_one_rank(tmp_path):
    mp.start_processes(_worker_rccl_one_rank, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True,
                       start_method="spawn")
    got = torch.load(tmp_path / "rccl1.pt", weights_only=True)
    for k, v in got["eager"].items():
        assert torch.equal(got["graph"][k], v), f"in-graph RCCL step differs from the eager one on {k}"


def test_engine_rejects_buckets_it_does_not_launch():
    """the backward launches the all-reduce of bucket i by position, so a bucket
    list other than grad_buckets() (one bucket for a two-bucket engine, or the two in the
    natural order, whose lower range the backward has not written at the first launch) must
    be rejected before anything runs; and bucket 0's launch point must find every gradient
    of its range pending in the flush it follows."""
    import plagnn
    from plagnn import dist as pdist

    src, dst, n, x, labels, tr, va = _problem(0)
    loops = np.arange(n)
    g = plagnn.CSRGraph(np.concatenate([src, loops]), np.concatenate([dst, loops]), n)
    eng = plagnn.TrainEngine(g, x, labels, DIMS, _weights(), tr, va, lr=LR, device="cuda:0", params=_params())
    (a, nn_), (z, a2) = eng.grad_buckets()
    assert nn_ == eng.gflat.numel() and z == 0 and a2 == a
    for bad in ([(0, nn_)], [(0, a), (a, nn_)]):
        ar = pdist.BucketAllReduce(eng.gflat, bad)
        with pytest.raises(ValueError, match="grad_buckets"):
            eng.capture(warmup=1, allreduce=ar)
        with pytest.raises(ValueError, match="grad_buckets"):
            eng.step_eager(ar)
    assert eng.steps_done == 0
    # the boundary check itself: with the top layer's parts dropped from the flush, bucket 0
    # is not fully written, and the check says which gradients are missing
    eng._uses_buckets(pdist.BucketAllReduce(eng.gflat, eng.grad_buckets()))
    eng.forward()
    eng._parts = []
    with pytest.raises(RuntimeError, match="liner1.W"):
        eng._check_bucket_pending(0)
    eng._parts = []


def _worker_guard_nccl(rank, world, port, outdir):
    """bench.py's N > 1 dp-leg guard over a real RCCL default group (one rank: a one-GPU box
    holds one RCCL rank) with its gloo control group, as the driver's 8-GPU runs set it up."""
    import json
    import sys

    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch.distributed as dist

    import bench

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    ctrl = dist.new_group(backend="gloo")

    def boom(*a, **k):
        raise RuntimeError("injected dp-leg failure")

    bench.run = boom
    out = {"with_gloo": bench.guarded_dp_leg(None, 0, 1, dev, dist, ctrl),
           "rccl_only": bench.guarded_dp_leg(None, 0, 1, dev, dist, None)}
    bench.run = lambda *a, **k: {"value": 1.0}
    out["ok"] = bench.guarded_dp_leg(None, 0, 1, dev, dist, ctrl)
    with open(os.path.join(outdir, "guard.json"), "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_bench_dp_guard_over_rccl_one_rank(tmp_path):
    import json

    mp.start_processes(_worker_guard_nccl, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True,
                       start_method="spawn")
    got = json.load(open(tmp_path / "guard.json"))
    assert "injected dp-leg failure" in got["with_gloo"]["error"]
    assert "injected dp-leg failure" in got["rccl_only"]["error"]
    assert got["ok"] == {"value": 1.0}
