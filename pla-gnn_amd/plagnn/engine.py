"""TrainEngine — the full PLA-GNN training step as one explicit, graph-captured sequence of
engine kernels.

One step is exactly the reference's epoch body (code/train.py:197-207):
  optimizer.zero_grad(); logits = model(g, features)            (model.py:19-31)
  train_loss = multi_loss(logits[train_index], labels[train_index], w); backward(); Adam.step()
  val_loss = multi_loss(logits[val_index], ...)                 (same pre-step logits)
computed without autograd: forward and backward are written out layer by layer and the
whole step is captured once into a HIP graph (torch.cuda.CUDAGraph) and replayed.

Layout in HBM (fp32, row-major; every width padded to a multiple of 4 with zero pads that
stay exactly zero through forward, backward and Adam):
  * SAGE layer l (Fi -> Fo): HM_l[N][2Fi] = [H_l | M_l] — the layer input H_l (written
    there by the previous layer's GEMM epilogue) beside the max-aggregated neighbourhood
    M_l (written there by the SpMM); parameters Wpool[Fi][Fi], bpool[Fi],
    Wcat[Fo][2Fi] = [Wself | Wneigh], b[Fo]: fc_self + fc_neigh + bias is ONE K = 2Fi GEMM
    over HM. P_l[N][Fi] = relu(fc_pool), argpos_l[N][Fi] (u16 winning in-row positions).
  * All parameters live in ONE flat buffer (Adam is one launch; a multi-GPU all-reduce is
    one bucket), gradients in a second one with the same layout.
  * Fusions: bias + relu / leaky_relu in the forward GEMM epilogues; leaky_relu' in the
    epilogue of the GEMM producing each activation gradient; the bias gradients
    (sum of dY over nodes) as row sums of the weight-gradient GEMM's A operand; relu' of
    fc_pool inside the SpMM backward.
"""
from __future__ import annotations

import contextlib
import ctypes
from collections import defaultdict
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib, ops
from ._lib import PG_ARG_DEAD_NONE as DEAD_NONE, call, ptr
from .graph import CSRGraph, DeviceGraph
from .ops import LEAKY_SLOPE, round4

RELU, LEAKY, NONE = _lib.PG_ACT_RELU, _lib.PG_ACT_LEAKY, _lib.PG_ACT_NONE
MAX_GROUP_PARTS = 16  # pg_gemm_*_group: up to 16 parts per call (include/plagnn.h)


def launch_group(site: str) -> str:
    """Kernel group of a launch site name: every GEMM launch ('gemm.*') is 'gemm', the rest
    their prefix ('spmm_max_fwd.l1' -> 'spmm_max_fwd')."""
    return "gemm" if site.startswith("gemm") else site.split(".")[0]


class _Flat:
    """Named views into one flat fp32 buffer (256-B aligned), plus named sub-views
    (row ranges / column prefixes) of those blocks."""

    def __init__(self):
        self.layout: List = []  # (name, shape)
        self.offsets: Dict[str, int] = {}
        self.subs: List = []  # (name, parent, row0, row1, ncols)
        self.size = 0

    def add(self, name, shape):
        n = int(np.prod(shape))
        self.layout.append((name, tuple(shape)))
        self.offsets[name] = self.size
        self.size += (n + 63) // 64 * 64

    def sub(self, name, parent, row0, row1, ncols=None):
        self.subs.append((name, parent, row0, row1, ncols))

    def views(self, buf: torch.Tensor) -> Dict[str, torch.Tensor]:
        v = {name: buf[self.offsets[name]:self.offsets[name] + int(np.prod(sh))].view(*sh)
             for name, sh in self.layout}
        for name, parent, r0, r1, nc in self.subs:
            t = v[parent][r0:r1]
            v[name] = t if nc is None else t[:, :nc]
        return v


class TrainEngine:
    REDUCE_INLINE = False  # True: each split-K combine right after its partials (A/B knob)
    # True: every weight gradient of the step in one grouped split-K launch at the end of the
    # backward (pg_gemm_f32_group); False: one split-K launch per product (A/B knob)
    GROUP_WGRAD = True
    # liner1's forward, the head and liner1's input gradient as one launch (pg_mlp_l1_head:
    # bitwise the separate x3 GEMMs + pg_mlp_head); False: three launches (A/B knob)
    FUSED_L1_HEAD = True
    # with it, the fused head's final kernel also forms the step's Adam scalars (pg_adam_prepare's
    # work): one launch fewer per step (A/B knob)
    FOLD_ADAM_PREP = True
    # with it, W1's bf16 pieces live in their own buffer, rewritten by the step's Adam
    # (pg_adam_apply_l1), so the head splits nothing: one launch fewer per step (A/B knob)
    KEEP_L1_PIECES = True
    _fold_prep = False             # set by the step paths (step_eager, capture, group_times)
    _prepped = False               # the head of this step formed the Adam scalars
    WIDTH_ALIGN = 4  # every padded width is a multiple of this
    _cur = ""                      # launch site being issued (_t)
    _filter: Optional[str] = None  # group_times: issue only this launch group
    _issued = 0
    _rec: Optional[list] = None    # gemm_bytes_per_step's dry-run record
    _split_buckets = False         # dp: the weight gradients as two grouped launches (grad_buckets)
    _ar_inline = None              # dp over RCCL: the BucketAllReduce launched from inside the backward

    def __init__(self, graph: CSRGraph, features: torch.Tensor, labels: torch.Tensor,
                 dims: Sequence[int], class_weight, train_index, val_index=None,
                 lr: float = 5e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 device="cuda", edge_weight: Optional[torch.Tensor] = None,
                 params: Optional[Dict[str, torch.Tensor]] = None, seed: int = 0):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("TrainEngine runs on a HIP device; use the dgl shim for -d cpu")
        self.dims = list(dims)
        self.L = len(self.dims) - 3
        if self.L < 1:
            raise ValueError("dims = [in, h_1, ..., h_L, h_mlp, classes] with L >= 1")
        N = graph.num_nodes
        self.N = N
        self.dg: DeviceGraph = graph.on(self.device)
        self.ews = self.dg.edge_weight_slots(edge_weight)
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)
        C = self.dims[-1]
        self.C = C
        dev = self.device
        a = self.WIDTH_ALIGN
        pd = [(d + a - 1) // a * a for d in self.dims]
        # SAGE layer inputs: a multiple of 64 when that costs <= 2 % more columns (503 -> 512):
        # whole feature tiles for the SpMM kernels; pads are zero and stay zero
        for l in range(self.L):
            r64 = -(-self.dims[l] // 64) * 64
            if r64 <= 1.02 * self.dims[l]:
                pd[l] = r64
        self.pd = pd

        # ---- parameters (flat, padded) ----
        # per SAGE layer one block [Wcat ; Wpool | 0] of (Fo + Fi) x 2Fi: Wcat = [Wself | Wneigh]
        # in rows [0, Fo), Wpool in rows [Fo, Fo + Fi) x columns [0, Fi) (the rest is a zero
        # pad that stays zero), so that its left half [Wself ; Wpool] is the B operand of the
        # stacked input gradient dH = ([dY | dP] [Wself ; Wpool]) * leaky'(H)
        fl = _Flat()
        for l in range(self.L):
            Fi, Fo = pd[l], pd[l + 1]
            q = f"conv{l + 1}."
            fl.add(q + "Wcp", (Fo + Fi, 2 * Fi))
            fl.sub(q + "Wcat", q + "Wcp", 0, Fo)
            fl.sub(q + "Wpool", q + "Wcp", Fo, Fo + Fi, Fi)
            fl.sub(q + "Wstack", q + "Wcp", 0, Fo + Fi, Fi)
            fl.add(q + "bpool", (Fi,))
            fl.add(q + "b", (Fo,))
        fl.add("liner1.W", (pd[-2], pd[-3]))
        fl.add("liner1.b", (pd[-2],))
        fl.add("liner2.W", (pd[-1], pd[-2]))
        fl.add("liner2.b", (pd[-1],))
        self.flat_layout = fl
        self.flat = torch.zeros(fl.size, dtype=torch.float32, device=dev)
        self.gflat = torch.zeros_like(self.flat)
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        self.adam_state = torch.zeros(4, dtype=torch.float32, device=dev)
        self.P = fl.views(self.flat)
        self.G = fl.views(self.gflat)
        if params is None:
            from .model import GNN

            torch.manual_seed(seed)
            params = GNN(self.dims).state_dict()
        self.load_state_dict(params)

        # ---- inputs ----
        if tuple(features.shape) != (N, self.dims[0]):
            raise ValueError(f"features must be ({N}, {self.dims[0]})")
        self.labels = torch.zeros(N, pd[-1], dtype=torch.float32, device=dev)
        self.labels[:, :C] = labels.to(dev, torch.float32)
        cw = np.asarray(class_weight, dtype=np.float64)
        if cw.shape != (C,):
            raise ValueError(f"class_weight must have {C} entries")
        cwp = np.empty(2 * C, np.float32)
        cwp[0::2] = cw.astype(np.float32)          # (float)w_c
        cwp[1::2] = (cw + 1.0).astype(np.float32)  # (float)(w_c + 1)
        self.cw = torch.from_numpy(cwp).to(dev)
        self.train_index = torch.as_tensor(np.asarray(train_index, np.int32), device=dev)
        self.val_index = None if val_index is None else torch.as_tensor(
            np.asarray(val_index, np.int32), device=dev)
        # per-row set for the fused head: 1 = train, 2 = val, 0 = neither
        rs = np.zeros(N, np.int8)
        rs[np.asarray(train_index, np.int64)] = 1
        if val_index is not None:
            vi = np.asarray(val_index, np.int64)
            if np.any(rs[vi] == 1):
                raise ValueError("train and val rows overlap")
            rs[vi] = 2
        self.row_set = torch.from_numpy(rs).to(dev)
        self.n_train = len(np.asarray(train_index))
        self.n_val = 0 if val_index is None else len(np.asarray(val_index))
        self._alloc_buffers(features)
        self._alloc_workspace()
        # W1's bf16 pieces for the fused head, kept current by the step's Adam
        # (pg_adam_apply_l1) instead of split in every head call (pg_mlp_l1_split here and
        # whenever the parameters are written from outside the step)
        self.l1_pieces: Optional[torch.Tensor] = None
        if self._l1_fused() and self.KEEP_L1_PIECES:
            nb = int(_lib.lib().pg_mlp_l1_pieces_bytes(self.pd[-3], self.pd[-2]))
            self.l1_pieces = torch.zeros(nb, dtype=torch.uint8, device=dev)
            self._split_l1()
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.graph_adam: Optional[torch.cuda.CUDAGraph] = None
        self.allreduce = None
        # [(start, end)] HIP events around each replayed step's gradient all-reduce, when a
        # list is set (bench.py's dp leg)
        self.ar_events: Optional[list] = None
        self.steps_done = 0
        self._timing: Optional[list] = None  # [(name, work, start_event, end_event)]

    def _alloc_buffers(self, features: torch.Tensor) -> None:
        N, pd, dev = self.N, self.pd, self.device
        # ---- activations ----
        f32 = dict(dtype=torch.float32, device=dev)
        self.HM, self.Pl, self.arg = [], [], []
        for l in range(self.L):
            Fi = pd[l]
            self.HM.append(torch.zeros(N, 2 * Fi, **f32))
            self.Pl.append(torch.zeros(N, Fi, **f32))
            self.arg.append(torch.zeros(N, Fi, dtype=self.dg.arg_dtype, device=dev))
        self.HM[0][:, :self.dims[0]] = features.to(dev, torch.float32)
        self.A3 = torch.zeros(N, pd[-3], **f32)
        self.A4 = torch.zeros(N, pd[-2], **f32)
        self.prob = torch.zeros(N, pd[-1], **f32)
        self.loss = torch.zeros(2, **f32)  # [train, val]
        # backward buffers: DYP_l = [dY_l | dP_l] (the gradients at layer l's pre-activation
        # output and at P_l, side by side: the stacked input-gradient product's A operand),
        # dM_l the gradient at the aggregated neighbourhood
        self.dZ = torch.zeros(N, pd[-1], **f32)
        self.dA4 = torch.zeros(N, pd[-2], **f32)
        self.DYP = [torch.zeros(N, pd[l + 1] + pd[l], **f32) for l in range(self.L)]
        self.dM = [torch.zeros(N, pd[l], **f32) for l in range(self.L)]

    def _alloc_workspace(self) -> None:
        # ---- workspace (one buffer, sized for the largest call) ----
        N, pd, C, dev = self.N, self.pd, self.C, self.device
        L = _lib.lib()
        need = 0
        for l in range(self.L):
            Fi = pd[l]
            need = max(need, L.pg_spmm_max_fwd_workspace(self.dg.fwd.struct(self.ews), Fi, self.dg.arg_kind))
            need = max(need, L.pg_spmm_max_bwd_workspace(self.dg.bwd.struct(None), Fi))
        self._gemm_plans = {}
        # weight gradients' split-K combines deferred to one batched launch per step
        self._slabs: Dict[str, torch.Tensor] = {}
        self._jobs: list = []
        self._parts: list = []
        for (M_, N_, K_) in self._wgrad_shapes():
            sk = ops._split_k(M_, N_, K_)
            self._gemm_plans[(M_, N_, K_)] = sk
            need = max(need, L.pg_gemm_f32_workspace(M_, N_, K_, sk))
        if self.GROUP_WGRAD:
            # the grouped launches' slabs, sized from the shapes alone (transposed A, plain B)
            self.gws = torch.empty(self._group_ws_bytes(L.pg_gemm_f32_group_workspace), dtype=torch.uint8,
                                   device=dev)
        need = max(need, L.pg_sigmoid_multi_loss_workspace(N, C), L.pg_mlp_head_workspace(N, C),
                   L.pg_mlp_l1_head_workspace(N, C, pd[-3], pd[-2]))
        self.ws = torch.zeros(max(int(need), 256), dtype=torch.uint8, device=dev)
        self.ws_bytes = self.ws.numel()

    def _wgrad_groupings(self):
        """The weight-gradient parts (shapes, in the order the backward issues them) of every
        grouped launch the step can make: all of them at once (one bucket), or [top SAGE layer
        + MLP] and [the layers below] (two buckets, grad_buckets), each chunked to the
        library's part limit."""
        sh = self._wgrad_shapes()
        L = self.L
        order = [sh[-1], sh[-2]] + [x for l in reversed(range(L)) for x in (sh[2 * l], sh[2 * l + 1])]
        groups = [order]
        if L > 1:
            groups += [order[:4], order[4:]]
        out = []
        for g in groups:
            out += [g[i:i + MAX_GROUP_PARTS] for i in range(0, len(g), MAX_GROUP_PARTS)]
        return out

    def _group_ws_bytes(self, ws_fn) -> int:
        need = 0
        for g in self._wgrad_groupings():
            parts = (_lib.PgGemmPart * len(g))()
            for i, (M_, N_, K_) in enumerate(g):
                parts[i].transa, parts[i].transb, parts[i].M, parts[i].N, parts[i].K = 1, 0, M_, N_, K_
            n = int(ws_fn(parts, len(g)))
            if n == 0:
                raise ValueError(f"grouped weight gradients: no workspace size for {len(g)} parts")
            need = max(need, n)
        return need

    def grad_buckets(self):
        """Ranges of the flat gradient buffer in the order the backward completes them: the
        top SAGE layer + the MLP (their weight gradients are done once the top layer's max
        backward has run: one contiguous tail of the flat layout), then the layers below.
        One bucket for a one-layer model."""
        n = self.gflat.numel()
        if self.L < 2:
            return [(0, n)]
        off = self.flat_layout.offsets[f"conv{self.L}.Wcp"]
        return [(off, n), (0, off)]

    # ------------------------------------------------------------------ parameters
    def _wgrad_shapes(self):
        pd, N = self.pd, self.N
        out = []
        for l in range(self.L):
            Fi, Fo = pd[l], pd[l + 1]
            out += [(Fo, 2 * Fi, N), (Fi, Fi, N)]
        out += [(pd[-2], pd[-3], N), (pd[-1], pd[-2], N)]
        return out

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        """Load DGL/GNN32-named parameters (code/model.py names) into the padded buffer."""
        with torch.no_grad():
            self.flat.zero_()
            for l in range(self.L):
                p = f"conv{l + 1}."
                fi, fo, Fi = self.dims[l], self.dims[l + 1], self.pd[l]
                self.P[p + "Wpool"][:fi, :fi] = sd[p + "fc_pool.weight"]
                self.P[p + "bpool"][:fi] = sd[p + "fc_pool.bias"]
                self.P[p + "Wcat"][:fo, :fi] = sd[p + "fc_self.weight"]
                self.P[p + "Wcat"][:fo, Fi:Fi + fi] = sd[p + "fc_neigh.weight"]
                if sd.get(p + "bias") is not None:
                    self.P[p + "b"][:fo] = sd[p + "bias"]
            d = self.dims
            self.P["liner1.W"][:d[-2], :d[-3]] = sd["liner1.weight"]
            self.P["liner1.b"][:d[-2]] = sd["liner1.bias"]
            self.P["liner2.W"][:d[-1], :d[-2]] = sd["liner2.weight"]
            self.P["liner2.b"][:d[-1]] = sd["liner2.bias"]
        if getattr(self, "l1_pieces", None) is not None:
            self._split_l1()

    def _split_l1(self) -> None:
        W1 = self.P["liner1.W"]
        self._call("pg_mlp_l1_split", ptr(W1), W1.stride(0), self.pd[-3], self.pd[-2], ptr(self.l1_pieces),
                   self._s())

    def _unpad(self, views: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        out = {}
        for l in range(self.L):
            p = f"conv{l + 1}."
            fi, fo, Fi = self.dims[l], self.dims[l + 1], self.pd[l]
            out[p + "fc_pool.weight"] = views[p + "Wpool"][:fi, :fi].clone()
            out[p + "fc_pool.bias"] = views[p + "bpool"][:fi].clone()
            out[p + "fc_neigh.weight"] = views[p + "Wcat"][:fo, Fi:Fi + fi].clone()
            out[p + "fc_self.weight"] = views[p + "Wcat"][:fo, :fi].clone()
            out[p + "bias"] = views[p + "b"][:fo].clone()
        d = self.dims
        out["liner1.weight"] = views["liner1.W"][:d[-2], :d[-3]].clone()
        out["liner1.bias"] = views["liner1.b"][:d[-2]].clone()
        out["liner2.weight"] = views["liner2.W"][:d[-1], :d[-2]].clone()
        out["liner2.bias"] = views["liner2.b"][:d[-1]].clone()
        return out

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return self._unpad(self.P)

    def params_updated(self) -> None:
        """Call after writing `flat` from outside the engine (e.g. a broadcast from rank 0):
        refreshes whatever the engine derives from the parameters (in fp32: W1's pieces)."""
        if self.l1_pieces is not None:
            self._split_l1()

    def broadcast_params(self, src: int = 0) -> None:
        """Every rank takes rank `src`'s parameters (multi-GPU replicas start identical)."""
        from . import dist as pdist

        pdist.broadcast_([self.flat], src)
        self.params_updated()

    def grads(self) -> Dict[str, torch.Tensor]:
        return self._unpad(self.G)

    @property
    def num_params(self) -> int:
        d = self.dims
        n = sum(d[l] * d[l] + d[l] + 2 * d[l] * d[l + 1] + d[l + 1] for l in range(self.L))
        return n + d[-3] * d[-2] + d[-2] + d[-2] * d[-1] + d[-1]

    # ------------------------------------------------------------------ timing
    @contextlib.contextmanager
    def _t(self, name: str, work: float = 0.0):
        """Marks one launch site; in diagnostic passes, HIP events around it on the engine's
        stream."""
        self._cur = name
        if self._timing is None:
            yield
            return
        st = torch.cuda.current_stream(self.device)
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(st)
        yield
        b.record(st)
        self._timing.append((name, work, a, b))

    def _call(self, fn: str, *args) -> None:
        """One library launch of the step (skipped when group_times captures another group)."""
        if self._filter is not None and launch_group(self._cur) != self._filter:
            return
        self._issued += 1
        call(fn, *args)

    def group_times(self, groups=("gemm", "spmm_max_fwd", "spmm_max_bwd", "head", "adam"), reps: int = 20,
                    warm: int = 2, copies: int = 10) -> Dict[str, Dict[str, float]]:
        """Time each launch group of the step AS THE REPLAYED GRAPH RUNS IT: for group g,
        `copies` steps are captured into one graph with only g's launches (in step order, on
        the step's own buffers), and that graph is replayed `reps` times back to back
        between two HIP events on the replay stream (no events sit between the launches; the
        graph launch overhead is spread over copies x launches). Returns {g: {ms (per
        step), launches (per step)}}. The others recompute the step's buffers from their
        current inputs; the Adam group's replays would train the model, so the parameters,
        moments and step count are restored afterwards (later measurements see the model the
        timed steps left)."""
        out = {}
        cur = torch.cuda.current_stream(self.device)
        s = torch.cuda.Stream(self.device)
        saved = [t.clone() for t in (self.flat, self.m, self.v, self.adam_state)] if "adam" in groups else None
        try:
            self._group_times(groups, reps, warm, copies, cur, s, out)
        finally:
            if saved is not None:
                torch.cuda.synchronize(self.device)
                for t, c in zip((self.flat, self.m, self.v, self.adam_state), saved):
                    t.copy_(c)
                self.params_updated()
                torch.cuda.synchronize(self.device)
        return out

    def _group_times(self, groups, reps, warm, copies, cur, s, out) -> None:
        for gname in groups:
            s.wait_stream(cur)
            self._filter, self._issued = gname, 0
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g, stream=s):
                    for _ in range(copies):
                        self._fold_prep = True  # as the step runs it
                        try:
                            self.forward()
                            self.backward()
                        finally:
                            self._fold_prep = False
                        self.adam()
            finally:
                self._filter = None
                self._prepped = False
            launches = self._issued // copies
            if launches == 0:
                continue
            for _ in range(warm):
                g.replay()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                g.replay()
            b.record()
            torch.cuda.synchronize(self.device)
            out[gname] = {"ms": a.elapsed_time(b) / (reps * copies), "launches": launches}
            del g

    def kernel_breakdown(self, reps: int = 5) -> Dict[str, Dict[str, float]]:
        """Per-launch-site mean duration (ms) and work over `reps` eager steps, timed with
        HIP events on the launch stream; each step is issued behind a GPU spin
        (torch.cuda._sleep) so that the host has queued the whole step before the GPU starts
        it. Returns {name: {ms, work, calls}} per step. A diagnostic of this process alone
        (no gradient all-reduce); the event packets between launches add a few us to each
        (group_times measures the replayed graph). Each timed step is a real training step."""
        acc: Dict[str, List[float]] = defaultdict(lambda: [0.0, 0.0, 0])
        for _ in range(reps):
            self._timing = []
            torch.cuda._sleep(20_000_000)
            self.step_eager(None)
            torch.cuda.synchronize(self.device)
            for name, work, a, b in self._timing:
                r = acc[name]
                r[0] += a.elapsed_time(b)
                r[1] += work
                r[2] += 1
            self._timing = None
        return {k: {"ms": v[0] / reps, "work": v[1] / reps, "calls": v[2] / reps} for k, v in acc.items()}

    # ------------------------------------------------------------------ kernels
    def _s(self):
        return _lib.stream_handle(self.device)

    def _rec_gemm(self, A, B, C, M, N, K, beta, dact) -> None:
        """gemm_bytes_per_step's dry run: the product's compulsory bytes (A, B read once, C
        written once, + C read for beta != 0, + the activation operand of a fused act')."""
        if self._rec is not None:
            b = A.element_size() * M * K + B.element_size() * K * N + C.element_size() * M * N
            b += (C.element_size() * M * N if beta != 0.0 else 0) + (dact.element_size() * M * N if dact is not None else 0)
            self._rec.append(b)

    def gemm_bytes_per_step(self) -> int:
        """Compulsory HBM bytes of the step's GEMM launches (each operand read once, each
        output written once, padded shapes), from a dry run that launches nothing."""
        self._rec, self._filter = [], "__dry_run__"
        jobs = list(getattr(self, "_jobs", []))
        try:
            self.forward()
            self.backward()
        finally:
            out, self._rec, self._filter = sum(self._rec), None, None
            if hasattr(self, "_jobs"):
                self._jobs = jobs
        return int(out)

    def _gemm(self, A, B, C, transa=False, transb=False, beta=0.0, bias=None, act=NONE, dact=None,
              rowsum=None, tag="gemm"):
        M = A.shape[1] if transa else A.shape[0]
        K = A.shape[0] if transa else A.shape[1]
        N = B.shape[0] if transb else B.shape[1]
        self._rec_gemm(A, B, C, M, N, K, beta, dact)
        # weight gradients (they feed only Adam) are recognised by their launch site, never by
        # shape: an input gradient of the same shape is read right after it is written
        wgrad = tag.startswith("gemm.wgrad")
        if wgrad and (bias is not None or act != NONE or dact is not None):
            raise ValueError(f"{tag}: a weight gradient takes no epilogue")
        sk = self._gemm_plans.get((M, N, K), 1) if wgrad else 1
        if self.GROUP_WGRAD and wgrad:
            q = _lib.PgGemmPart()
            q.transa, q.transb, q.M, q.N, q.K = int(transa), int(transb), M, N, K
            q.A, q.lda, q.B, q.ldb = ptr(A), A.stride(0), ptr(B), B.stride(0)
            q.beta, q.C, q.ldc, q.rowsum = beta, ptr(C), C.stride(0), ptr(rowsum)
            self._parts.append((q, 2.0 * M * N * K))
            return
        if sk > 1:
            self._gemm_partials(A, B, C, transa, transb, beta, rowsum, tag, M, N, K, sk)
            return
        ep = _lib.epilogue(bias, act, LEAKY_SLOPE, dact, rowsum)
        ws = self.ws
        with self._t(tag, 2.0 * M * N * K):
            self._call("pg_gemm_f32", int(transa), int(transb), M, N, K, 1.0, ptr(A), A.stride(0), ptr(B),
                 B.stride(0), beta, ptr(C), C.stride(0), ep, sk, ptr(ws), ws.numel(), self._s())

    def _gemm_partials(self, A, B, C, transa, transb, beta, rowsum, tag, M, N, K, sk) -> None:
        """A split-K weight gradient whose combine is deferred: the partial slabs go to this
        launch site's own workspace and one pg_gemm_splitk_reduce_batch at the end of the
        backward combines every weight gradient of the step (_reduce_deferred)."""
        slab = self._slabs.get(tag)
        if slab is None:
            slab = torch.empty(int(_lib.lib().pg_gemm_f32_workspace(M, N, K, sk)), dtype=torch.uint8,
                               device=self.device)
            self._slabs[tag] = slab
        used = ctypes.c_int(0)
        ep = _lib.epilogue(rowsum=rowsum)
        with self._t(tag, 2.0 * M * N * K):
            self._call("pg_gemm_f32_partials", int(transa), int(transb), M, N, K, ptr(A), A.stride(0), ptr(B),
                 B.stride(0), ep, sk, ptr(slab), slab.numel(), ctypes.byref(used), self._s())
        j = _lib.PgSplitkJob()
        j.ws, j.split_k, j.M, j.N = ptr(slab), used.value, M, N
        j.alpha, j.beta, j.C, j.ldc, j.rowsum = 1.0, beta, ptr(C), C.stride(0), ptr(rowsum)
        self._jobs.append(j)
        if self.REDUCE_INLINE:  # combine now, while the slabs are still in the caches
            self._reduce_deferred()

    def _reduce_deferred(self) -> None:
        parts, self._parts = self._parts, []
        for i in range(0, len(parts), MAX_GROUP_PARTS):  # the library's part limit per launch
            chunk = parts[i:i + MAX_GROUP_PARTS]
            arr = (_lib.PgGemmPart * len(chunk))(*[q for q, _ in chunk])
            with self._t("gemm.wgrad.group", sum(w for _, w in chunk)):
                self._call("pg_gemm_f32_group", arr, len(chunk), ptr(self.gws), self.gws.numel(), self._s())
        jobs, self._jobs = self._jobs, []
        for i in range(0, len(jobs), 16):
            part = jobs[i:i + 16]
            arr = (_lib.PgSplitkJob * len(part))(*part)
            with self._t("gemm.splitk_reduce"):
                self._call("pg_gemm_splitk_reduce_batch", arr, len(part), self._s())

    def forward(self) -> None:
        """Logits (self.prob) and both losses; dZ = d train_loss / d z."""
        st = self._s()
        g = self.dg.fwd.struct(self.ews)
        P, pd = self.P, self.pd
        for l in range(self.L):
            p = f"conv{l + 1}."
            Fi = pd[l]
            HM = self.HM[l]
            # P = relu(H Wpool^T + bpool)
            self._gemm(HM[:, :Fi], P[p + "Wpool"], self.Pl[l], transb=True, bias=P[p + "bpool"], act=RELU,
                       tag=f"gemm.fwd.pool.l{l + 1}")
            # M = max-aggregate(P) -> right half of HM
            with self._t(f"spmm_max_fwd.l{l + 1}", self.spmm_bytes(l)):
                self._call("pg_spmm_max_fwd", g, ptr(self.Pl[l]), Fi, Fi, ptr(HM[:, Fi:]), HM.stride(0),
                     ptr(self.arg[l]), Fi, self.dg.arg_kind | DEAD_NONE, ptr(self.ws), self.ws_bytes, st)
            # Y = [H | M] Wcat^T + b (fc_self + fc_neigh + bias), leaky_relu -> next input
            Fo = pd[l + 1]
            out = self.HM[l + 1][:, :Fo] if l + 1 < self.L else self.A3
            self._gemm(HM, P[p + "Wcat"], out, transb=True, bias=P[p + "b"], act=LEAKY,
                       tag=f"gemm.fwd.cat.l{l + 1}")
        if self._l1_fused():
            self._mlp_l1_head()
            return
        self._gemm(self.A3, P["liner1.W"], self.A4, transb=True, bias=P["liner1.b"], act=LEAKY,
                   tag="gemm.fwd.liner1")
        self._head(_lib.PG_DTYPE_F32, self.A4, self.dZ, None, self.dA4)

    def _l1_fused(self) -> bool:
        return self.FUSED_L1_HEAD and self.pd[-2] <= 128

    def _mlp_l1_head(self) -> None:
        """liner1 + liner2 + sigmoid + train/val loss + dZ + dA4 + liner1's input gradient
        through the top SAGE layer's leaky_relu (that layer's dY) in one launch
        (pg_mlp_l1_head; code/model.py:26-29, code/train.py:89-108, 199-207)."""
        P, pd, C = self.P, self.pd, self.C
        top = self.L - 1
        dH3 = self.DYP[top][:, :pd[top + 1]]
        # inside a training step (not a bare forward()): the Adam scalars too
        fold = self._fold_prep and self.FOLD_ADAM_PREP
        self._prepped = fold
        with self._t("head.l1", 2.0 * 2 * self.N * pd[-3] * pd[-2]):
            fn = "pg_mlp_l1_head" if self.l1_pieces is None else "pg_mlp_l1_head_ex"
            pieces = () if self.l1_pieces is None else (ptr(self.l1_pieces),)
            self._call(fn, ptr(self.A3), self.A3.stride(0), self.N, pd[-3], ptr(P["liner1.W"]),
                       P["liner1.W"].stride(0), ptr(P["liner1.b"]), pd[-2], ptr(self.A4), self.A4.stride(0),
                       ptr(P["liner2.W"]), pd[-2], ptr(P["liner2.b"]), C, ptr(self.labels), pd[-1], ptr(self.cw),
                       ptr(self.row_set), self.n_train, self.n_val, ptr(self.prob), pd[-1], ptr(self.dZ), pd[-1],
                       ptr(self.dA4), self.dA4.stride(0), ptr(dH3), dH3.stride(0), LEAKY_SLOPE, ptr(self.loss),
                       ptr(self.ws), self.ws_bytes, ptr(self.adam_state) if fold else None, self.lr, self.betas[0],
                       self.betas[1], *pieces, self._s())

    def _head(self, a_dtype, A4, dZ, dZb, dA4) -> None:
        """liner2 + sigmoid + train/val multi_loss + dZ + dA4 = (dZ W2) * leaky'(A4): one
        fused pass (pg_mlp_head; code/model.py:28-29, code/train.py:89-108, 199-207)."""
        P, pd, C = self.P, self.pd, self.C
        cp = pd[-1]
        with self._t("head"):
            self._call("pg_mlp_head", ptr(A4), A4.stride(0), self.N, pd[-2], a_dtype, ptr(P["liner2.W"]), pd[-2],
                 ptr(P["liner2.b"]), C, ptr(self.labels), cp, ptr(self.cw), ptr(self.row_set), self.n_train,
                 self.n_val, ptr(self.prob), cp, ptr(dZ), cp, ptr(dZb), ptr(dA4), dA4.stride(0), LEAKY_SLOPE,
                 ptr(self.loss), ptr(self.ws), self.ws_bytes, self._s())

    def backward(self) -> None:
        st = self._s()
        G, P, pd = self.G, self.P, self.pd
        g = self.dg.fwd.struct(self.ews)
        gt = self.dg.bwd.struct(None)
        # liner2: dW2 = dZ^T A4 (+ db2 = row sums of dZ^T); dA4 came from the fused head
        self._gemm(self.dZ, self.A4, G["liner2.W"], transa=True, rowsum=G["liner2.b"], tag="gemm.wgrad.liner2")
        # liner1
        self._gemm(self.dA4, self.A3, G["liner1.W"], transa=True, rowsum=G["liner1.b"], tag="gemm.wgrad.liner1")
        top = self.L - 1
        if not self._l1_fused():  # (fused: the head wrote the top layer's dY already)
            self._gemm(self.dA4, P["liner1.W"], self.DYP[top][:, :pd[top + 1]], act=LEAKY, dact=self.A3,
                       tag="gemm.dgrad.liner1")
        for l in reversed(range(self.L)):
            p = f"conv{l + 1}."
            Fi, Fo = pd[l], pd[l + 1]
            HM, DYP = self.HM[l], self.DYP[l]
            dY, dP = DYP[:, :Fo], DYP[:, Fo:]
            # d Wcat = dY^T [H | M], d b = sum_nodes dY
            self._gemm(dY, HM, G[p + "Wcat"], transa=True, rowsum=G[p + "b"], tag=f"gemm.wgrad.cat.l{l + 1}")
            # dM = dY Wneigh
            self._gemm(dY, P[p + "Wcat"][:, Fi:], self.dM[l], tag=f"gemm.dgrad.neigh.l{l + 1}")
            # max backward; the records say "none" where M = 0 (DEAD_NONE), so those entries are
            # skipped and the relu' mask of fc_pool (P >= 0) is implied
            with self._t(f"spmm_max_bwd.l{l + 1}", self.spmm_bwd_bytes(l)):
                self._call("pg_spmm_max_bwd", g, gt, ptr(self.arg[l]), Fi, self.dg.arg_kind | DEAD_NONE, ptr(self.dM[l]), Fi, Fi,
                     ptr(self.Pl[l]), Fi, None, 0, ptr(dP), DYP.stride(0), ptr(self.ws),
                     self.ws_bytes, st)
            # d Wpool = dP^T H, d bpool = sum_nodes dP
            self._gemm(dP, HM[:, :Fi], G[p + "Wpool"], transa=True, rowsum=G[p + "bpool"],
                       tag=f"gemm.wgrad.pool.l{l + 1}")
            self._wgrad_bucket_boundary(l)
            if l > 0:
                # dH = ([dY | dP] [Wself ; Wpool]) * leaky'(H), one K = Fo + Fi product: the
                # lower layer's dY (H is the previous layer's output)
                self._gemm(DYP, P[p + "Wstack"], self.DYP[l - 1][:, :Fi], act=LEAKY, dact=HM[:, :Fi],
                           tag=f"gemm.dgrad.stack.l{l + 1}")
        self._reduce_deferred()
        self._bucket_done(len(self.grad_buckets()) - 1)

    def _wgrad_bucket_boundary(self, l: int) -> None:
        """After the top SAGE layer's weight gradients are issued (dp with two buckets): run
        that bucket's grouped launch now, and with RCCL start its all-reduce, which then
        overlaps the rest of the backward."""
        if self._split_buckets and l == self.L - 1 and self.L > 1:
            self._check_bucket_pending(0)
            self._reduce_deferred()
            self._bucket_done(0)

    def _check_bucket_pending(self, i: int) -> None:
        """Bucket i's all-reduce may start only once every gradient inside its range has been
        issued: each parameter block in the range must be the output (or row-sum output) of a
        weight-gradient launch still pending in this flush (a Wcp block is written as its Wcat
        rows and its Wpool rows; its zero pad is never written). Ungrouped weight gradients
        (the GROUP_WGRAD = False A/B knob) were launched in stream order already."""
        if not self.GROUP_WGRAD:
            return
        a, b = self.grad_buckets()[i]
        pending = set()
        for q, _ in self._parts:
            pending.update((q.C or 0, q.rowsum or 0))
        for j in getattr(self, "_jobs", []):
            pending.update((j.C or 0, j.rowsum or 0))
        need = []
        for name, off in self.flat_layout.offsets.items():
            if a <= off < b:
                need += [name[:-3] + "Wcat", name[:-3] + "Wpool"] if name.endswith("Wcp") else [name]
        missing = [n for n in need if ptr(self.G[n]) not in pending]
        if missing:
            raise RuntimeError(f"gradient bucket {i} {a}:{b} would be all-reduced before {missing} are written")

    def _bucket_done(self, i: int) -> None:
        if self._ar_inline is not None and self._filter is None:
            self._ar_inline.launch(i)

    def adam(self) -> None:
        st = self._s()
        prepped, self._prepped = self._prepped, False
        with self._t("adam", 16.0 * self.flat.numel()):
            if not prepped:  # (else this step's head formed the scalars)
                self._call("pg_adam_prepare", ptr(self.adam_state), self.lr, self.betas[0], self.betas[1], st)
            if self.l1_pieces is not None:  # (also W1's pieces for the next step's head)
                W1 = self.P["liner1.W"]
                self._call("pg_adam_apply_l1", ptr(self.flat), ptr(self.gflat), ptr(self.m), ptr(self.v),
                           self.flat.numel(), ptr(self.adam_state), self.betas[0], self.betas[1], self.eps, 0.0,
                           (W1.data_ptr() - self.flat.data_ptr()) // 4, W1.stride(0), self.pd[-3], self.pd[-2],
                           ptr(self.l1_pieces), st)
                return
            self._call("pg_adam_apply", ptr(self.flat), ptr(self.gflat), ptr(self.m), ptr(self.v),
                 self.flat.numel(), ptr(self.adam_state), self.betas[0], self.betas[1], self.eps, 0.0, st)

    def _uses_buckets(self, allreduce) -> None:
        """A bucketed all-reduce must hold exactly grad_buckets(): the backward launches bucket
        i by position (bucket 0 at the top layer's boundary, the last one at the end), so any
        other list would reduce a range before the backward has written it, or index past it."""
        bk = getattr(allreduce, "buckets", None) if allreduce is not None else None
        if bk is not None:
            want = [tuple(int(v) for v in b) for b in self.grad_buckets()]
            got = [tuple(int(v) for v in b) for b in bk]
            if got != want:
                raise ValueError(f"all-reduce buckets {got} are not this engine's grad_buckets() {want}")
        self._split_buckets = bk is not None and len(bk) > 1

    def step_eager(self, allreduce=None) -> None:
        self._uses_buckets(allreduce)
        inline = allreduce is not None and getattr(allreduce, "capturable", False)
        self._ar_inline = allreduce if inline else None
        self._fold_prep = True
        try:
            self.forward()
            self.backward()
        finally:
            self._ar_inline = None
            self._fold_prep = False
        if inline:
            allreduce.join()
        elif allreduce is not None:
            allreduce(self.gflat)
        self.adam()
        self.steps_done += 1

    # ------------------------------------------------------------------ graph capture
    def capture(self, warmup: int = 2, allreduce=None) -> None:
        """Capture the step into HIP graphs. Warm-up steps run eagerly first (they are real
        training steps and count as such). With `allreduce` (multi-GPU data parallel): a
        capturable one (plagnn.dist.BucketAllReduce over RCCL) goes INTO the step's one
        graph, each gradient bucket's collective on a communication stream as soon as the
        backward has finished that bucket; any other (gloo, or a plain function) runs
        eagerly between two graphs, forward+backward and Adam."""
        self.allreduce = allreduce
        self._uses_buckets(allreduce)
        inline = allreduce is not None and getattr(allreduce, "capturable", False)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step_eager(allreduce)
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        self.graph_adam = None
        if allreduce is None or inline:
            with torch.cuda.graph(self.graph):
                self._ar_inline = allreduce if inline else None
                self._fold_prep = True
                try:
                    self.forward()
                    self.backward()
                finally:
                    self._ar_inline = None
                    self._fold_prep = False
                if inline:
                    allreduce.join()
                self.adam()
        else:
            with torch.cuda.graph(self.graph):
                self._fold_prep = True
                try:
                    self.forward()
                    self.backward()
                finally:
                    self._fold_prep = False
            self.graph_adam = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_adam):
                self.adam()

    @property
    def allreduce_in_graph(self) -> bool:
        return self.graph is not None and self.allreduce is not None and self.graph_adam is None

    def step(self) -> None:
        if self.graph is None:
            self.step_eager(self.allreduce)
            return
        self.graph.replay()
        if self.graph_adam is not None:
            if self.ar_events is not None:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                self.allreduce(self.gflat)
                b.record()
                self.ar_events.append((a, b))
            else:
                self.allreduce(self.gflat)
            self.graph_adam.replay()
        self.steps_done += 1

    def losses(self):
        return self.loss.detach().cpu().tolist()

    def logits(self) -> torch.Tensor:
        return self.prob[:, :self.C]

    # ------------------------------------------------------------------ accounting
    @property
    def edges_per_step(self) -> int:
        """Edges aggregated per training step: one aggregation per SAGE layer over E'
        (self-loops included) — SURVEY.md §8(d)."""
        return self.L * self.dg.num_edges

    def spmm_bytes(self, layer: int) -> int:
        """Algorithmic HBM bytes of one max-aggregation forward:
        4(N+1) + 4E' + s*F*E' + s*F*N + a*F*N, s = 4 (f32), a = argpos bytes, at the true
        (unpadded) width F."""
        N, E, F = self.N, self.dg.num_edges, self.dims[layer]
        a = 2 if self.dg.arg_kind == _lib.PG_ARG_U16 else 4
        return 4 * (N + 1) + 4 * E + 4 * F * E + 4 * F * N + a * F * N

    def spmm_bwd_bytes(self, layer: int) -> int:
        """Algorithmic bytes of one max backward: the upstream gradient
        and the argmax record read once (s*F*N + a*F*N), dX written once (s*F*N), plus
        the fused relu mask (s*F*N) and the transposed CSR (4(N+1) + 8E'), true width F."""
        N, E, F = self.N, self.dg.num_edges, self.dims[layer]
        a = 2 if self.dg.arg_kind == _lib.PG_ARG_U16 else 4
        return 4 * (N + 1) + 8 * E + (12 + a) * F * N

    def flops_per_step(self) -> int:
        """Flops of the step's GEMM launches at the true (unpadded) dims, forward + backward
        (layer-1 input gradient skipped, as autograd does for the constant features). liner2's
        forward and input-gradient products run inside the fused head, not as GEMMs, and are
        not counted; its weight gradient is."""
        N, d = self.N, self.dims
        f = 0
        for l in range(self.L):
            fi, fo = d[l], d[l + 1]
            fwd = 2 * N * fi * fi + 2 * N * (2 * fi) * fo
            wgrad = fwd
            igrad = 2 * N * fo * fi + (2 * N * fo * fi + 2 * N * fi * fi if l > 0 else 0)
            f += fwd + wgrad + igrad
        # liner1: forward, weight and input gradients (the forward and the input gradient run
        # inside the fused head when FUSED_L1_HEAD: head_flops_per_step)
        f += (1 if self._l1_fused() else 3) * 2 * N * d[-3] * d[-2]
        f += 2 * N * d[-2] * d[-1]       # liner2: weight gradient
        return f

    def head_flops_per_step(self) -> int:
        """Flops of the liner1 products inside the fused head (forward + input gradient, true
        dims), 0 when they run as GEMMs."""
        d = self.dims
        return 2 * 2 * self.N * d[-3] * d[-2] if self._l1_fused() else 0
