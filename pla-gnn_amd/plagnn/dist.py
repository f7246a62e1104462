"""Multi-GPU data parallelism for the PLA-GNN step: one process per GPU, full-graph
replicas, ONE gradient all-reduce per step.

The reference is single-process. Its graph fits one MI355X many
times over, so nothing is partitioned: every rank holds a whole graph (its own
perturbation replica, or the same graph with its own training rows) and computes its
local loss; the only exchange is the average of the flat gradient bucket before Adam
(BASELINE configs[3]). Backend "nccl" is RCCL on ROCm (xGMI); "gloo" runs the same code
on CPU for tests.
"""
from __future__ import annotations

import os
from typing import Iterable, Optional

import torch
import torch.distributed as dist


def env_rank():
    """(rank, world_size, local_rank) from torch.distributed.run's environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: Optional[str] = None, device: Optional[torch.device] = None) -> bool:
    """Initialise the default process group when WORLD_SIZE > 1. Returns True if
    distributed. MASTER_ADDR/MASTER_PORT come from the launcher (use 127.0.0.1)."""
    rank, world, _ = env_rank()
    if world <= 1:
        return False
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if (device is not None and device.type == "cuda") else "gloo"
        kw = {"device_id": device} if backend == "nccl" and device is not None else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return True


def _average(t: torch.Tensor) -> None:
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.AVG)
    else:  # gloo has no AVG
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.div_(dist.get_world_size())


def allreduce_mean(t: torch.Tensor) -> torch.Tensor:
    """In-place average over ranks (one collective on the whole bucket)."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        _average(t)
    return t


class BucketAllReduce:
    """The step's gradient all-reduce as several buckets of one flat buffer, each averaged
    as soon as the backward has finished it (TrainEngine.grad_buckets: the top SAGE layer +
    the MLP first, then the layers below), so the first bucket's collective overlaps the
    rest of the backward.

    * RCCL (backend "nccl"): `launch(i)` issues bucket i's all-reduce on a communication
      stream that forks from the current one, `join()` makes the current stream wait for
      it. Both are capturable, so TrainEngine.capture() puts the whole dp step, collective
      included, into ONE HIP graph.
    * gloo (CPU collectives: tests, rehearsals): not capturable; `__call__` averages the
      buckets one after the other on the current stream, between the two graphs.
    Averaging is element-wise, so splitting the buffer changes no value when each element's
    sum runs in the same rank order (two ranks: always; tests/test_dist.py)."""

    def __init__(self, flat: torch.Tensor, buckets):
        self.flat = flat
        self.buckets = [(int(a), int(b)) for a, b in buckets if b > a]
        # (a one-rank RCCL group still runs the collective: captured and replayed in
        # tests/test_gpu_dist_engine.py::test_rccl_allreduce_in_step_graph_one_rank)
        self.active = dist.is_initialized()
        self.capturable = flat.is_cuda and self.active and dist.get_backend() == "nccl"
        self.stream = torch.cuda.Stream(flat.device) if self.capturable else None

    def view(self, i: int) -> torch.Tensor:
        a, b = self.buckets[i]
        return self.flat[a:b]

    def launch(self, i: int) -> None:
        """Bucket i's all-reduce on the communication stream (RCCL), ordered after the work
        issued so far on the current stream."""
        cur = torch.cuda.current_stream(self.flat.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            _average(self.view(i))

    def join(self) -> None:
        torch.cuda.current_stream(self.flat.device).wait_stream(self.stream)

    def __call__(self, flat: Optional[torch.Tensor] = None) -> None:
        """Every bucket, in order, on the current stream (eager; any backend)."""
        if flat is not None and flat.data_ptr() != self.flat.data_ptr():
            raise ValueError("BucketAllReduce: another buffer than the one it was built for")
        if self.active:
            for i in range(len(self.buckets)):
                _average(self.view(i))


def broadcast_(tensors: Iterable[torch.Tensor], src: int = 0) -> None:
    if dist.is_initialized() and dist.get_world_size() > 1:
        for t in tensors:
            dist.broadcast(t, src)


class GradBucket:
    """Flat all-reduce of an nn.Module's gradients (drop-in training loop, autograd path):
    grads are copied into one contiguous bucket, averaged in one collective, copied back."""

    def __init__(self, params: Iterable[torch.nn.Parameter]):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)

    def allreduce(self) -> None:
        off = 0
        for p in self.params:
            k = p.numel()
            g = p.grad if p.grad is not None else torch.zeros_like(p)
            self.flat[off:off + k].copy_(g.reshape(-1))
            off += k
        allreduce_mean(self.flat)
        off = 0
        for p in self.params:
            k = p.numel()
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            p.grad.copy_(self.flat[off:off + k].view_as(p))
            off += k
