"""Multi-process (world_size 2, gloo on CPU) check of the data-parallel path: every rank
trains a full-graph replica of its own graph, gradients are averaged in one bucket
all-reduce before Adam (plagnn.dist), and the result equals the serial computation on
the oracle: params_after = Adam(params, (g_rank0 + g_rank1) / 2)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, ROOT, random_graph

DIMS = (11, 8, 8, 8, 6, 12)


def _problem(rank):
    n = 70
    src, dst = random_graph(n, 400, seed=100 + rank, self_loop=False)
    rng = np.random.default_rng(rank)
    x = torch.from_numpy(rng.standard_normal((n, DIMS[0])).astype(np.float32))
    labels = torch.from_numpy((rng.random((n, DIMS[-1])) < 0.4).astype(np.float32))
    idx = list(range(0, n, 2))
    return src, dst, n, x, labels, idx


def _weights():
    return np.linspace(0.5, 3.0, DIMS[-1])


def _worker(rank, world, port, outdir):
    import sys

    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import dgl
    from plagnn import dist as pdist
    from plagnn.model import GNN
    from plagnn.train import multi_loss

    assert pdist.init("gloo")
    torch.manual_seed(0)
    model = GNN(list(DIMS))
    pdist.broadcast_(list(model.parameters()))
    src, dst, n, x, labels, idx = _problem(rank)
    g = dgl.add_self_loop(dgl.graph((src, dst), num_nodes=n))
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    bucket = pdist.GradBucket(model.parameters())
    opt.zero_grad()
    loss = multi_loss(model(g, x)[idx], labels[idx], _weights())
    loss.backward()
    bucket.allreduce()
    opt.step()
    torch.save({k: v.detach().clone() for k, v in model.state_dict().items()},
               os.path.join(outdir, f"rank{rank}.pt"))
    torch.distributed.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_two_rank_gradient_allreduce_matches_serial(tmp_path, oracle_mod):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    got = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    for k in got[0]:
        assert torch.equal(got[0][k], got[1][k]), f"ranks diverged on {k}"
    # serial reference on the oracle
    from plagnn.model import GNN

    torch.manual_seed(0)
    p0 = {k: v.detach().clone() for k, v in GNN(list(DIMS)).state_dict().items()}
    grads = []
    for r in range(world):
        src, dst, n, x, labels, idx = _problem(r)
        og = oracle_mod.OracleGraph(src, dst, n)
        _, _, gr = oracle_mod.train_step(og, x, labels, idx, _weights(), p0)
        grads.append(gr)
    avg = {k: (grads[0][k] + grads[1][k]) / 2 for k in p0}
    opt_params = {k: v.clone().requires_grad_(True) for k, v in p0.items()}
    opt = torch.optim.Adam(list(opt_params.values()), lr=1e-2)
    for k, v in opt_params.items():
        v.grad = avg[k]
    opt.step()
    for k in p0:
        torch.testing.assert_close(got[0][k], opt_params[k].detach(), rtol=1e-5, atol=1e-6, msg=k)


def _worker_buckets(rank, world, port, outdir):
    import sys

    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from plagnn import dist as pdist

    assert pdist.init("gloo")
    rng = np.random.default_rng(10 + rank)
    base = torch.from_numpy(rng.standard_normal(50_000).astype(np.float32) * np.float32(1e3) ** rng.integers(-2, 3, 50_000))
    flat = base.clone()
    pdist.allreduce_mean(flat)
    two = base.clone()
    # TrainEngine.grad_buckets' shape: a tail (top layer + MLP) first, then the head
    ar = pdist.BucketAllReduce(two, [(31_232, 50_000), (0, 31_232)])
    assert not ar.capturable
    ar(two)
    torch.save({"flat": flat, "two": two}, os.path.join(outdir, f"b{rank}.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_bucket_allreduce_equals_flat_bitwise(tmp_path):
    """The dp step's gradient all-reduce in two buckets (plagnn.dist.BucketAllReduce, as
    TrainEngine reduces its top layer + MLP bucket before the rest of the backward has run)
    equals one all-reduce of the whole flat buffer bit for bit, on every rank (gloo, two
    ranks: each element is the same two-term sum either way)."""
    world = 2
    mp.start_processes(_worker_buckets, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    got = [torch.load(tmp_path / f"b{r}.pt", weights_only=True) for r in range(world)]
    for r in range(world):
        assert torch.equal(got[r]["two"], got[r]["flat"]), f"rank {r}: bucketed != flat"
        assert torch.equal(got[r]["two"], got[0]["two"])
