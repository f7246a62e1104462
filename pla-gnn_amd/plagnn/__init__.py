"""plagnn — MI355X-native message-passing engine for the PLA-GNN training hot path.

  CSRGraph     host CSR/transposed CSR + schedules, uploaded per device (graph.py)
  ops          C-ABI calls (SpMM max/sum, GEMM, ...) and autograd wrappers (ops.py)
  GNN32, GNN   the reference's model on the engine's SAGEConv (model.py)
  TrainEngine  the whole training step, explicit and HIP-graph captured (engine.py)
  TrainEngineBF16  the same step in bf16 storage, f32 accumulate (engine_bf16.py)
  data         synthetic PPI stand-ins in the reference's on-disk formats (data.py)
"""
from ._lib import PlagnnError, lib  # noqa: F401
from . import ops  # noqa: F401
from .graph import CSRGraph, DeviceGraph  # noqa: F401


def __getattr__(name):
    # model/engine import the dgl shim; resolve lazily to avoid an import cycle
    if name in ("GNN32", "GNN"):
        from . import model

        return getattr(model, name)
    if name == "TrainEngine":
        from .engine import TrainEngine

        return TrainEngine
    if name == "TrainEngineBF16":
        from .engine_bf16 import TrainEngineBF16

        return TrainEngineBF16
    raise AttributeError(name)
