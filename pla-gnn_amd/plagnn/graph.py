"""Graph storage for the message-passing engine.

Host side: the COO edge list (self-loops already appended, code/utils.py:44-45) becomes
an in-CSR (DGL's CSC: rows = destinations, each row in ascending edge id) and its
transpose (rows = sources, destinations ascending, with the in-CSR slot of every edge),
plus the longest-first work schedules the kernels consume. All of it is built by the
C-ABI host entry points (pg_csr_from_coo / pg_csr_transpose / pg_schedule_*).

Device side: one ``DeviceGraph`` per torch device, uploaded once and cached; int32 ids
throughout (DGL uses int64), the compact per-row argmax positions are u16 whenever the
largest in-degree allows (else int32).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from ._lib import PgCsr, call

# in-CSR entries per forward work item before a row is split (CSRGraph(chunk=...))
DEFAULT_CHUNK = 256
# out-CSR entries per backward work item, its work is data-dependent (CSRGraph(chunk_bwd=...);
# None = by graph size). Measured with the dense pull (scripts/bwd_bench.py, per call): S0
# (24 041 nodes) F = 256: 68.0 / 66.0 / 72.1 / 101.6 us at 64 / 128 / 256 / 512 (hub
# sources serialise on one wave past 128); RMAT x16 (384 656 nodes) F = 512 bf16: 1504 /
# 1375 / 1308 / 1275 us: finer items pay off only while the graph alone does not fill the
# chip.
DEFAULT_CHUNK_BWD = None


CHUNK_BWD_OVERRIDE: Optional[int] = None  # tuning experiments (bench.py --chunk-bwd)
# graphs from this many edges (self-loops included) get transposed max-backward descriptors
TRANS_MIN_EDGES = 1 << 22


def default_chunk_bwd(num_nodes: int) -> int:
    if CHUNK_BWD_OVERRIDE:
        return CHUNK_BWD_OVERRIDE
    return 64 if num_nodes <= 65536 else 512


def _np_ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _schedule(ptr: np.ndarray, chunk: int):
    n_rows = len(ptr) - 1
    n_items = ctypes.c_int64()
    n_merges = ctypes.c_int64()
    n_slots = ctypes.c_int64()
    max_deg = ctypes.c_int32()
    call("pg_schedule_count", _np_ptr(ptr), n_rows, chunk, ctypes.byref(n_items),
         ctypes.byref(n_merges), ctypes.byref(n_slots), ctypes.byref(max_deg))
    items = np.zeros(max(1, n_items.value) * 4, np.int32)
    merges = np.zeros(max(1, n_merges.value) * 4, np.int32)
    call("pg_schedule_build", _np_ptr(ptr), n_rows, chunk, _np_ptr(items), _np_ptr(merges))
    return items, n_items.value, merges, n_merges.value, n_slots.value, max_deg.value


class HostCsr:
    """One CSR direction with its schedule, in host memory (numpy int32)."""

    def __init__(self, ptr, col, eslot, n_cols: int, chunk: int, epos=None):
        self.ptr, self.col, self.eslot, self.epos = ptr, col, eslot, epos
        self.n_rows = len(ptr) - 1
        self.n_cols = int(n_cols)
        self.nnz = int(len(col))
        self.chunk = int(chunk)
        (self.items, self.n_items, self.merges, self.n_merges, self.n_slots,
         self.max_deg) = _schedule(ptr, chunk)


class DeviceCsr:
    """A HostCsr uploaded to one device; ``struct()`` gives the pg_csr_t view."""

    def __init__(self, h: HostCsr, device: torch.device):
        def up(a):
            return None if a is None else torch.from_numpy(a).to(device)

        self.device = device
        self.ptr, self.col, self.eslot, self.epos = up(h.ptr), up(h.col), up(h.eslot), up(h.epos)

        self.items, self.merges = up(h.items), up(h.merges)
        self.n_rows, self.n_cols, self.nnz = h.n_rows, h.n_cols, h.nnz
        self.n_items, self.n_merges, self.n_slots = h.n_items, h.n_merges, h.n_slots
        self.max_deg, self.chunk = h.max_deg, h.chunk

    def struct(self, ew: Optional[torch.Tensor] = None) -> PgCsr:
        """The pg_csr_t view (cached per edge-weight pointer: it holds raw pointers only)."""
        key = _lib.ptr(ew)
        cache = self.__dict__.setdefault("_structs", {})
        s = cache.get(key)
        if s is None:
            s = cache[key] = self._make_struct(ew)
        return s

    def _make_struct(self, ew: Optional[torch.Tensor]) -> PgCsr:
        s = PgCsr()
        s.n_rows, s.n_cols, s.nnz = self.n_rows, self.n_cols, self.nnz
        s.ptr = _lib.ptr(self.ptr)
        s.col = _lib.ptr(self.col)
        s.eslot = _lib.ptr(self.eslot)
        s.epos = _lib.ptr(self.epos)
        s.ew = _lib.ptr(ew)
        s.items = _lib.ptr(self.items)
        s.n_items = self.n_items
        s.merges = _lib.ptr(self.merges) if self.n_merges > 0 else 0
        s.n_merges = self.n_merges
        s.n_slots = self.n_slots
        s.max_deg = self.max_deg
        s.chunk = self.chunk
        return s


class CSRGraph:
    """In-CSR + out-CSR of a directed graph given as COO (src -> dst), host resident."""

    def __init__(self, src, dst, num_nodes: int, chunk: int = DEFAULT_CHUNK,
                 chunk_bwd: Optional[int] = DEFAULT_CHUNK_BWD, bwd_trans: Optional[bool] = None):
        src = np.ascontiguousarray(np.asarray(src, dtype=np.int64))
        dst = np.ascontiguousarray(np.asarray(dst, dtype=np.int64))
        if src.shape != dst.shape or src.ndim != 1:
            raise ValueError("src and dst must be 1-D arrays of equal length")
        n = int(num_nodes)
        E = len(src)
        ptr = np.zeros(n + 1, np.int32)
        col = np.zeros(max(E, 1), np.int32)
        eid = np.zeros(max(E, 1), np.int32)
        call("pg_csr_from_coo", _np_ptr(src), _np_ptr(dst), E, n, n, _np_ptr(ptr), _np_ptr(col),
             _np_ptr(eid))
        col, eid = col[:E], eid[:E]
        tptr = np.zeros(n + 1, np.int32)
        tcol = np.zeros(max(E, 1), np.int32)
        tslot = np.zeros(max(E, 1), np.int32)
        tpos = np.zeros(max(E, 1), np.int32)
        call("pg_csr_transpose", _np_ptr(ptr), _np_ptr(col), n, n, E, _np_ptr(tptr), _np_ptr(tcol),
             _np_ptr(tslot), _np_ptr(tpos))
        self.num_nodes = n
        self.num_edges = E
        self.eid = eid  # in-CSR slot -> edge id
        # the in-CSR slots' transposed indices (pg_csr_t.epos of the in-CSR): with them the
        # max backward stores each live edge's list descriptor where the pull reads it in
        # order (coalesced) instead of at the slot (one random read per edge), at the price
        # of clearing the descriptor array and scattered descriptor stores. Measured per step:
        # RMAT x16 (19.6 M edges) 3.28 -> 2.90 ms, S0 (1.23 M edges, its descriptors stay in
        # the caches) 0.232 -> 0.238 ms: on by default from TRANS_MIN_EDGES edges
        if bwd_trans is None:
            bwd_trans = E >= TRANS_MIN_EDGES
        einv = None
        if bwd_trans and E > 0:
            einv = np.empty(E, np.int32)
            einv[tslot[:E]] = np.arange(E, dtype=np.int32)
        self.bwd_trans = einv is not None
        self.fwd = HostCsr(ptr, col, None, n, chunk, epos=einv)
        if chunk_bwd is None:
            chunk_bwd = default_chunk_bwd(n)
        self.bwd = HostCsr(tptr, tcol[:E], tslot[:E], n, chunk_bwd, epos=tpos[:E])
        # argmax records hold positions inside in-CSR rows: u16 while every row is shorter
        # than 0xFFFF entries (0xFFFF = no winner)
        self.arg_kind = _lib.PG_ARG_U16 if self.fwd.max_deg < 0xFFFF else _lib.PG_ARG_I32
        self._dev: Dict[str, "DeviceGraph"] = {}

    def on(self, device) -> "DeviceGraph":
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        key = str(device)
        if key not in self._dev:
            self._dev[key] = DeviceGraph(self, device)
        return self._dev[key]

    def in_degrees(self) -> np.ndarray:
        return np.diff(self.fwd.ptr)

    def out_degrees(self) -> np.ndarray:
        return np.diff(self.bwd.ptr)


class DeviceGraph:
    def __init__(self, g: CSRGraph, device: torch.device):
        self.device = device
        self.num_nodes = g.num_nodes
        self.num_edges = g.num_edges
        self.arg_kind = g.arg_kind
        self.arg_dtype = torch.int16 if g.arg_kind == _lib.PG_ARG_U16 else torch.int32
        self.fwd = DeviceCsr(g.fwd, device)
        self.bwd = DeviceCsr(g.bwd, device)
        self.eid = torch.from_numpy(g.eid.astype(np.int64)).to(device)

    @property
    def is_cuda(self) -> bool:
        return self.device.type == "cuda"

    def edge_weight_slots(self, edge_weight: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """Edge weights given per edge id (DGL order) -> in-CSR slot order, f32 contiguous."""
        if edge_weight is None:
            return None
        w = edge_weight.reshape(-1)
        if w.numel() != self.num_edges:
            raise ValueError(f"edge_weight has {w.numel()} entries, graph has {self.num_edges} edges")
        return w.to(device=self.device, dtype=torch.float32).index_select(0, self.eid).contiguous()
