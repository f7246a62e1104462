"""Drop-in subset of the DGL 0.8.2 Python API that quinlanW/PLA-GNN uses, backed by the
MI355X message-passing engine (``plagnn``).

The reference touches exactly this surface:
  import dgl                                         code/utils.py:4, main_normal.py:9-15
  dgl.graph((start, end), num_nodes=N)               code/utils.py:44
  dgl.add_self_loop(g)                               code/utils.py:45
  g.nodes[list(range(N))].data[key] = tensor         code/utils.py:46, 49
  g.ndata['feat'], g.ndata['loc']                    code/train.py:145-146, 179
  g.to(device)                                       code/main_normal.py:66
  dgl.seed(seed)                                     code/main_normal.py:15
  from dgl.nn.pytorch import SAGEConv                code/model.py:7
  SAGEConv(in, out, 'pool')(g, h)                    code/model.py:13-15, 20-24
plus ``update_all`` with ``dgl.function`` builtins (copy_u / u_mul_e with sum / mean /
max), which SAGEConv itself is defined by.

Message passing on a CUDA (HIP) device always runs in libplagnn.so; a missing library is
an error, never a silent fallback.
"""
from __future__ import annotations

import contextlib
from typing import Dict, Optional

import numpy as np
import torch

from . import function  # noqa: F401  (dgl.function)
from . import nn  # noqa: F401  (dgl.nn)

__version__ = "0.8.2+plagnn"

_SEED: Optional[int] = None


def seed(val: int) -> None:
    """dgl.seed: DGL seeds its own C RNG (used by samplers). Nothing on the full-graph
    training path draws from it; the value is recorded for completeness."""
    global _SEED
    _SEED = int(val)


def _engine():
    import plagnn  # deferred: keeps `import dgl` cheap and the load order torch -> lib

    return plagnn


class _Frame(dict):
    """ndata / edata: name -> tensor whose first dimension is the node/edge count."""

    def __init__(self, n: int, kind: str):
        super().__init__()
        self._n = n
        self._kind = kind

    def __setitem__(self, key, value):
        if not isinstance(value, torch.Tensor):
            value = torch.as_tensor(value)
        if value.shape[0] != self._n:
            raise ValueError(f"{self._kind} data '{key}' has {value.shape[0]} rows, expected {self._n}")
        super().__setitem__(key, value)


class _NodeDataView:
    def __init__(self, g: "DGLGraph", ids):
        self._g = g
        self._ids = ids

    def __getitem__(self, key):
        t = self._g.ndata[key]
        return t if self._ids is None else t[self._index(t.device)]

    def __setitem__(self, key, value):
        if not isinstance(value, torch.Tensor):
            value = torch.as_tensor(value)
        n = self._g.num_nodes()
        idx = self._ids
        if idx is not None:
            ids = torch.as_tensor(idx, dtype=torch.int64).reshape(-1)
            if ids.numel() == n and bool((ids == torch.arange(n)).all()):
                idx = None  # full, in order (code/utils.py:46, 49 pass list(range(N)))
        if idx is None:
            self._g.ndata[key] = value
            return
        if key in self._g.ndata:
            self._g.ndata[key][self._index(self._g.ndata[key].device)] = value.to(self._g.ndata[key].device)
        else:
            buf = torch.zeros((n,) + tuple(value.shape[1:]), dtype=value.dtype, device=value.device)
            buf[self._index(value.device)] = value
            self._g.ndata[key] = buf

    def _index(self, device):
        return torch.as_tensor(self._ids, dtype=torch.int64, device=device)

    def keys(self):
        return self._g.ndata.keys()


class _NodeSpace:
    def __init__(self, g: "DGLGraph", ids):
        self.data = _NodeDataView(g, ids)


class _NodeView:
    def __init__(self, g: "DGLGraph"):
        self._g = g

    def __getitem__(self, ids):
        if isinstance(ids, slice) and ids == slice(None):
            ids = None
        return _NodeSpace(self._g, ids)

    def __call__(self):
        return torch.arange(self._g.num_nodes(), device=self._g.device)

    def __len__(self):
        return self._g.num_nodes()


class DGLGraph:
    """Homogeneous graph: COO edge list (edge id = position), node/edge frames, and the
    engine's CSR (built on first message passing, shared by every ``.to()`` copy)."""

    def __init__(self, src: torch.Tensor, dst: torch.Tensor, num_nodes: int, device=None,
                 _csr_cache=None):
        self._src = src.to(torch.int64)
        self._dst = dst.to(torch.int64)
        self._n = int(num_nodes)
        self._device = torch.device(device) if device is not None else self._src.device
        self.ndata = _Frame(self._n, "node")
        self.edata = _Frame(int(self._src.numel()), "edge")
        self._csr_cache = _csr_cache if _csr_cache is not None else {}

    # --- structure -------------------------------------------------------------------
    def num_nodes(self, ntype=None) -> int:
        return self._n

    number_of_nodes = num_nodes

    def num_edges(self, etype=None) -> int:
        return int(self._src.numel())

    number_of_edges = num_edges

    @property
    def device(self) -> torch.device:
        return self._device

    @property
    def idtype(self):
        return torch.int64

    @property
    def nodes(self) -> _NodeView:
        return _NodeView(self)

    @property
    def srcdata(self):
        return self.ndata

    @property
    def dstdata(self):
        return self.ndata

    def edges(self, form: str = "uv", order: str = "eid"):
        if form != "uv":
            raise NotImplementedError("edges(form != 'uv')")
        return self._src.to(self._device), self._dst.to(self._device)

    def in_degrees(self, v=None):
        d = torch.bincount(self._dst.cpu(), minlength=self._n).to(self._device)
        return d if v is None else d[torch.as_tensor(v, device=self._device)]

    def out_degrees(self, u=None):
        d = torch.bincount(self._src.cpu(), minlength=self._n).to(self._device)
        return d if u is None else d[torch.as_tensor(u, device=self._device)]

    def is_homogeneous(self) -> bool:
        return True

    # --- placement -------------------------------------------------------------------
    def to(self, device, **kwargs) -> "DGLGraph":
        device = torch.device(device)
        g = DGLGraph(self._src, self._dst, self._n, device=device, _csr_cache=self._csr_cache)
        for k, v in self.ndata.items():
            g.ndata[k] = v.to(device)
        for k, v in self.edata.items():
            g.edata[k] = v.to(device)
        if device.type == "cuda":
            self._engine_graph().on(device)  # upload the CSR once, eagerly (main_normal.py:66)
        return g

    def cpu(self) -> "DGLGraph":
        return self.to("cpu")

    def cuda(self, device=None) -> "DGLGraph":
        return self.to(torch.device("cuda") if device is None else device)

    # --- engine bridge ------------------------------------------------------------------
    def _engine_graph(self):
        if "host" not in self._csr_cache:
            self._csr_cache["host"] = _engine().CSRGraph(
                self._src.cpu().numpy(), self._dst.cpu().numpy(), self._n)
        return self._csr_cache["host"]

    def _device_graph(self, device=None):
        return self._engine_graph().on(device if device is not None else self._device)

    # --- message passing ----------------------------------------------------------------
    @contextlib.contextmanager
    def local_scope(self):
        nd, ed = dict(self.ndata), dict(self.edata)
        try:
            yield
        finally:
            dict.clear(self.ndata)
            dict.update(self.ndata, nd)
            dict.clear(self.edata)
            dict.update(self.edata, ed)

    def update_all(self, message_func, reduce_func, apply_node_func=None, etype=None):
        from .function import _Message, _Reduce

        if not isinstance(message_func, _Message) or not isinstance(reduce_func, _Reduce):
            raise NotImplementedError("update_all supports dgl.function builtins only")
        if reduce_func.msg != message_func.out:
            raise ValueError("reduce function reads a message the message function does not write")
        X = self.ndata[message_func.lhs]
        ew = None
        if message_func.op == "u_mul_e":
            ew = self.edata[message_func.rhs]
            if ew.dim() > 1:
                if ew.numel() != ew.shape[0]:
                    raise NotImplementedError("u_mul_e with multi-dimensional edge features")
                ew = ew.reshape(-1)
        shape = X.shape
        X2 = X.reshape(shape[0], -1)
        dg = self._device_graph(X.device)
        ews = dg.edge_weight_slots(ew)
        eng = _engine()
        if reduce_func.op == "max":
            out = eng.ops.MaxAggregate.apply(X2.float(), dg, ews)
        else:
            out = eng.ops.SumAggregate.apply(X2.float(), dg, ews, reduce_func.op == "mean")
        out = out.to(X.dtype).reshape(shape)
        self.ndata[reduce_func.out] = out
        if apply_node_func is not None:
            self.ndata.update(apply_node_func(_NodeBatch(self)))

    def __repr__(self):
        return (f"Graph(num_nodes={self._n}, num_edges={self.num_edges()},\n"
                f"      ndata_schemes={ {k: (tuple(v.shape[1:]), v.dtype) for k, v in self.ndata.items()} }\n"
                f"      edata_schemes={ {k: (tuple(v.shape[1:]), v.dtype) for k, v in self.edata.items()} })")


class _NodeBatch:
    def __init__(self, g: DGLGraph):
        self.data = g.ndata


def _as_ids(x) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(torch.int64).reshape(-1)
    return torch.as_tensor(np.asarray(x, dtype=np.int64)).reshape(-1)


def graph(data, num_nodes: Optional[int] = None, idtype=None, device=None, **kwargs) -> DGLGraph:
    """dgl.graph((U, V), num_nodes=N): edge i goes U[i] -> V[i] (code/utils.py:44)."""
    if isinstance(data, tuple) and len(data) == 2:
        src, dst = _as_ids(data[0]), _as_ids(data[1])
    else:
        raise NotImplementedError("dgl.graph: only the (src, dst) form is supported")
    if src.numel() != dst.numel():
        raise ValueError("dgl.graph: src and dst lengths differ")
    n = int(num_nodes) if num_nodes is not None else (
        int(max(src.max().item(), dst.max().item())) + 1 if src.numel() else 0)
    if src.numel() and (int(src.min()) < 0 or int(dst.min()) < 0 or
                        int(src.max()) >= n or int(dst.max()) >= n):
        raise ValueError("dgl.graph: node id out of range")
    g = DGLGraph(src.cpu(), dst.cpu(), n)
    return g.to(device) if device is not None else g


def add_self_loop(g: DGLGraph, etype=None) -> DGLGraph:
    """dgl.add_self_loop (code/utils.py:45): one loop per node appended, so the new
    edges get ids E..E+N-1 (existing loops are kept; duplicates allowed). Edge features
    of the new loops are zero-filled, as DGL does."""
    n = g.num_nodes()
    loops = torch.arange(n, dtype=torch.int64)
    ng = DGLGraph(torch.cat([g._src.cpu(), loops]), torch.cat([g._dst.cpu(), loops]), n,
                  device=g.device)
    for k, v in g.ndata.items():
        ng.ndata[k] = v
    for k, v in g.edata.items():
        pad = torch.zeros((n,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
        ng.edata[k] = torch.cat([v, pad])
    return ng


def remove_self_loop(g: DGLGraph, etype=None) -> DGLGraph:
    keep = g._src != g._dst
    ng = DGLGraph(g._src[keep], g._dst[keep], g.num_nodes(), device=g.device)
    for k, v in g.ndata.items():
        ng.ndata[k] = v
    for k, v in g.edata.items():
        ng.edata[k] = v[keep.to(v.device)]
    return ng


__all__ = ["DGLGraph", "graph", "add_self_loop", "remove_self_loop", "seed", "function", "nn"]
