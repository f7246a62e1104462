"""The engine's multi-GPU path (bench.py --gpus N): world_size 2 over gloo with both ranks
on cuda:0. Every rank builds a TrainEngine on its own graph from the same parameters,
captures the step with `allreduce=allreduce_mean` (forward+backward graph, the bucket
all-reduce, the Adam graph) and replays it. Checked against the serial computation on the
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
    eng.capture(warmup=1, allreduce=pdist.allreduce_mean)
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
