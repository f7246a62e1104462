"""bench.py at N > 1 (what the driver's 8-GPU SCALE runs): the RCCL dp leg runs after the
replicas headline in the same processes, and its failure must not cost the headline line.
Two ranks over gloo on the CPU run bench.main() with the engine replaced by a stand-in
whose dp leg raises (on every rank, or on rank 1 only); rank 0 must still print the
replicas headline (value, dist) with the leg recorded as {"error": ...}, and both ranks
must exit with rc 0. Also the engine's bucket guard: an all-reduce whose
buckets are not TrainEngine.grad_buckets() is rejected before anything is launched."""
import contextlib
import json
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _fake_run(fail_on):
    def run(args, rank, world, dev, dist, mode, breakdown=True):
        t = torch.ones(1)
        dist.all_reduce(t)  # the headline's max-over-ranks collective, as run() has
        if mode == "dp" and rank in fail_on:
            raise RuntimeError("injected dp-leg failure")
        if mode == "dp":
            return {"value": 1.0, "ms_per_step": 1.0} if rank == 0 else None
        if rank != 0:
            return None
        return {"metric": "edges aggregated/sec per training epoch, full PPI graph", "value": 2.0e9 * world,
                "unit": "edges/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": 1.0, "config": {"mode": mode}, "_engine": None, "_wl": None,
                "loss": {"train": 0.5, "val": 0.6}}
    return run


def _worker(rank, world, port, outdir, fail_on):
    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PLAGNN_BENCH_BACKEND="gloo")
    import bench

    bench.run = _fake_run(set(fail_on))
    bench._device = lambda local_rank: torch.device("cpu")
    bench._device_info = lambda dev: {"device": None, "name": "cpu"}
    with open(os.path.join(outdir, f"out{rank}.txt"), "w") as f, contextlib.redirect_stdout(f):
        bench.main(["--gpus", str(world), "--steps", "2", "--warmup", "1"])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fail_on", [(0, 1), (1,), ()], ids=["every-rank", "rank1-only", "no-failure"])
def test_dp_leg_failure_keeps_headline(tmp_path, fail_on):
    world = 2
    # join=True raises if any rank exits non-zero
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), fail_on), nprocs=world, join=True,
                       start_method="spawn")
    lines = [ln for ln in (tmp_path / "out0.txt").read_text().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, lines
    out = json.loads(lines[0])
    assert out["value"] == 4.0e9 and out["n_gpus"] == world
    assert out["dist"]["world_size"] == world and len(out["dist"]["ranks"]) == world
    if fail_on:
        assert "error" in out["dp"], out["dp"]
        if 0 in fail_on:
            assert "injected dp-leg failure" in out["dp"]["error"]
    else:
        assert out["dp"] == {"value": 1.0, "ms_per_step": 1.0}
    assert not [ln for ln in (tmp_path / "out1.txt").read_text().splitlines() if ln.startswith("{")]


class _Bucketed:
    def __init__(self, buckets):
        self.buckets = buckets


def test_engine_rejects_foreign_buckets():
    """TrainEngine._uses_buckets on the engine's own logic (the class needs a HIP device to
    build, so a stand-in carries grad_buckets()): the backward launches bucket i by position,
    so one bucket over the whole buffer, or the two buckets in another order, must raise;
    the engine's own list and a plain function (eager, no buckets) are taken."""
    from plagnn.engine import TrainEngine

    class Eng:
        def grad_buckets(self):
            return [(700, 1000), (0, 700)]

    e = Eng()
    for bad in ([(0, 1000)], [(0, 700), (700, 1000)], [(700, 1000)]):
        with pytest.raises(ValueError, match="grad_buckets"):
            TrainEngine._uses_buckets(e, _Bucketed(bad))
    TrainEngine._uses_buckets(e, _Bucketed([(700, 1000), (0, 700)]))
    assert e._split_buckets
    TrainEngine._uses_buckets(e, lambda flat: None)
    assert not e._split_buckets
    TrainEngine._uses_buckets(e, None)
    assert not e._split_buckets
