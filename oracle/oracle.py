"""ORACLE — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker (or the timed CPU baseline). The product
(``pla-gnn_amd/``) never imports it; its GPU path fails loudly when the HIP library is
missing instead of routing here.

CPU restatement of the reference's training hot path:

* graph construction — ``dgl.graph((start, end), num_nodes)`` + ``dgl.add_self_loop``
  (code/utils.py:44-45) with DGL's CSC in ascending edge id (C: ``oracle_csc_build``);
* ``SAGEConv(in, out, 'pool')`` of DGL 0.8.2.post1 (code/model.py:7, 13-15, 20-25):
  ``P = relu(fc_pool(h))``; ``update_all(copy_u('h','m'), max('m','neigh'))`` with argmax
  (C: ``oracle_spmm_max``); ``rst = fc_self(h) + fc_neigh(neigh) + bias``; backward of the
  max through ``scatter_add_`` on argX (C: ``oracle_spmm_max_bwd``);
* ``GNN32.forward`` (code/model.py:19-31): leaky_relu(0.01) after each conv and liner1,
  sigmoid at the end;
* ``multi_loss`` / ``weight_cal`` (code/train.py:89-126);
* ``torch.optim.Adam`` step as torch 1.10.0 computes it (code/train.py:180, 205).

Dense algebra runs in torch-CPU float32 (the "plain PyTorch fp32 reference"); the
message passing runs in the C restatement, single-threaded, in DGL's loop order. With
``parallel=True`` (bench.py's CPU baseline) the forward loop runs row-parallel under
OpenMP and the backward is torch-CPU ``scatter_add_``, as DGL's CPU backend runs them.

Pinning: ``multi_loss``/``weight_cal`` are checked against golden vectors produced by the
reference's own functions (tests/golden/gen_golden.py). The DGL message-passing
semantics are PARITY UNPINNED by reference tests (the reference has none and DGL is not
installable here); they are pinned by the known-answer tests in tests/test_oracle.py.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional, Tuple

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_i64p = ctypes.POINTER(ctypes.c_int64)
_f32p = ctypes.POINTER(ctypes.c_float)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build() -> str:
    """Compile the C restatement (gcc) into oracle/build/liboracle.so."""
    import subprocess

    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_csc_build.argtypes = [_i64p, _i64p, ctypes.c_int64, ctypes.c_int64, _i64p, _i64p, _i64p]
        L.oracle_csc_build.restype = ctypes.c_int
        L.oracle_spmm_max.argtypes = [_i64p, _i64p, _i64p, _f32p, _f32p, ctypes.c_int64, ctypes.c_int64,
                                      _f32p, _i64p, _i64p]
        L.oracle_spmm_max.restype = None
        L.oracle_spmm_max_omp.argtypes = L.oracle_spmm_max.argtypes
        L.oracle_spmm_max_omp.restype = None
        _d = ctypes.POINTER(ctypes.c_double)
        L.oracle_spmm_max_f64.argtypes = [_i64p, _i64p, _i64p, _d, _d, ctypes.c_int64, ctypes.c_int64, _d, _i64p,
                                          _i64p]
        L.oracle_spmm_max_f64.restype = None
        _i32p = ctypes.POINTER(ctypes.c_int32)
        L.oracle_spmm_max_align.argtypes = [_i64p, _i64p, _i64p, _f32p, _f32p, ctypes.c_int64, ctypes.c_int64,
                                            _i32p, _d, ctypes.c_double, _f32p, _i64p, _i64p, _i64p, _d]
        L.oracle_spmm_max_align.restype = ctypes.c_int64
        L.oracle_spmm_max_align_f64.argtypes = [_i64p, _i64p, _i64p, _d, _d, ctypes.c_int64, ctypes.c_int64, _i32p,
                                                _d, ctypes.c_double, _d, _i64p, _i64p, _i64p, _d]
        L.oracle_spmm_max_align_f64.restype = ctypes.c_int64
        L.oracle_spmm_max_bwd.argtypes = [_i64p, _i64p, _f32p, _f32p, _u8p, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_int64, _f32p]
        L.oracle_spmm_max_bwd.restype = None
        L.oracle_spmm_sum.argtypes = [_i64p, _i64p, _i64p, _f32p, _f32p, ctypes.c_int64, ctypes.c_int64,
                                      ctypes.c_int, _f32p]
        L.oracle_spmm_sum.restype = None
        _f64p = ctypes.POINTER(ctypes.c_double)
        L.oracle_ecc.argtypes = [_i64p, _i64p, _f64p, ctypes.c_int64, ctypes.c_double, _i64p, _i64p, _f64p]
        L.oracle_ecc.restype = ctypes.c_int64
        L.oracle_perturb_sd.argtypes = [_f64p, ctypes.c_int64, ctypes.c_int, ctypes.c_double, _f64p]
        L.oracle_perturb_sd.restype = None
        L.oracle_perturb_sum.argtypes = [_f64p, _f64p, _f64p, _f64p, ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                                         ctypes.c_int, ctypes.c_double, ctypes.c_int64, ctypes.c_int64]
        L.oracle_perturb_sum.restype = ctypes.c_double
        L.oracle_perturb_rows.argtypes = [_f64p, _f64p, _f64p, _f64p, ctypes.c_int64, ctypes.c_int,
                                          ctypes.c_double, _i64p, _i64p, _i64p, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_int64, ctypes.c_int64, _i64p, _i64p, _i64p,
                                          ctypes.c_int64]
        L.oracle_perturb_rows.restype = ctypes.c_int64
        _lib = L
    return _lib


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t) if a is not None else None


# ---------------------------------------------------------------- graph construction
class OracleGraph:
    """COO edge list + DGL-ordered CSC (int64 ids), as DGL 0.8 holds it."""

    def __init__(self, src, dst, num_nodes: int, self_loop: bool = True,
                 edge_weight: Optional[np.ndarray] = None):
        src = np.asarray(src, dtype=np.int64)
        dst = np.asarray(dst, dtype=np.int64)
        n = int(num_nodes)
        if self_loop:  # dgl.add_self_loop: loops appended, edge ids E..E+N-1 (utils.py:45)
            loops = np.arange(n, dtype=np.int64)
            src = np.concatenate([src, loops])
            dst = np.concatenate([dst, loops])
            if edge_weight is not None:
                edge_weight = np.concatenate([np.asarray(edge_weight, np.float32),
                                              np.ones(n, np.float32)])
        self.src, self.dst, self.n = src, dst, n
        self.ew = None if edge_weight is None else np.ascontiguousarray(edge_weight, np.float32)
        self.indptr = np.zeros(n + 1, np.int64)
        self.indices = np.zeros(len(src), np.int64)
        self.eids = np.zeros(len(src), np.int64)
        rc = lib().oracle_csc_build(_p(src, _i64p), _p(dst, _i64p), len(src), n,
                                    _p(self.indptr, _i64p), _p(self.indices, _i64p), _p(self.eids, _i64p))
        if rc != 0:
            raise ValueError("oracle_csc_build: bad edge list")

    @property
    def num_edges(self) -> int:
        return int(len(self.src))

    def in_degrees(self) -> np.ndarray:
        return np.diff(self.indptr)


# ---------------------------------------------------------------- message passing
def spmm_max(g: OracleGraph, X: np.ndarray, use_weight: bool = False, parallel: bool = False):
    """parallel=True: the OpenMP row-parallel form of the same loop (DGL's CPU backend;
    the timed CPU baseline), identical results."""
    if X.dtype == np.float64:  # the exact-arithmetic yardstick (row-parallel)
        X = np.ascontiguousarray(X)
        F = X.shape[1]
        out = np.empty((g.n, F), np.float64)
        argx = np.empty((g.n, F), np.int64)
        arge = np.empty((g.n, F), np.int64)
        w = g.ew.astype(np.float64) if use_weight else None
        d = ctypes.POINTER(ctypes.c_double)
        lib().oracle_spmm_max_f64(_p(g.indptr, _i64p), _p(g.indices, _i64p), _p(g.eids, _i64p), _p(w, d),
                                  _p(X, d), g.n, F, _p(out, d), _p(argx, _i64p), _p(arge, _i64p))
        return out, argx, arge
    X = np.ascontiguousarray(X, np.float32)
    F = X.shape[1]
    out = np.empty((g.n, F), np.float32)
    argx = np.empty((g.n, F), np.int64)
    arge = np.empty((g.n, F), np.int64)
    w = g.ew if use_weight else None
    fn = lib().oracle_spmm_max_omp if parallel else lib().oracle_spmm_max
    fn(_p(g.indptr, _i64p), _p(g.indices, _i64p), _p(g.eids, _i64p),
                          _p(w, _f32p), _p(X, _f32p), g.n, F, _p(out, _f32p), _p(argx, _i64p),
                          _p(arge, _i64p))
    return out, argx, arge


def spmm_max_bwd(g: OracleGraph, argx, arge, dZ: np.ndarray, use_weight: bool = False):
    dZ = np.ascontiguousarray(dZ, np.float32)
    F = dZ.shape[1]
    dX = np.empty((g.n, F), np.float32)
    has_in = (g.in_degrees() > 0).astype(np.uint8)
    w = g.ew if use_weight else None
    lib().oracle_spmm_max_bwd(_p(np.ascontiguousarray(argx), _i64p), _p(np.ascontiguousarray(arge), _i64p),
                              _p(w, _f32p), _p(dZ, _f32p), _p(has_in, _u8p), g.n, g.n, F, _p(dX, _f32p))
    return dX


def spmm_sum(g: OracleGraph, X: np.ndarray, mean: bool = False, use_weight: bool = False):
    X = np.ascontiguousarray(X, np.float32)
    out = np.empty((g.n, X.shape[1]), np.float32)
    w = g.ew if use_weight else None
    lib().oracle_spmm_sum(_p(g.indptr, _i64p), _p(g.indices, _i64p), _p(g.eids, _i64p), _p(w, _f32p),
                          _p(X, _f32p), g.n, X.shape[1], int(mean), _p(out, _f32p))
    return out


def spmm_max_align(g: OracleGraph, X: np.ndarray, use_weight: bool, hint: np.ndarray, scale: np.ndarray,
                   band: float, out, argx, arge) -> Tuple[int, int]:
    """In place: entries where `hint` (another computation's winning in-row positions,
    -1 = none) names a different candidate within `band` x the candidates' rounding scale
    (`scale`: n x F float64 running-error magnitudes of X, times |w| for weighted edges)
    of the maximum take it (oracle_spmm_max_align). Returns (changed, hard, max_gap): hard =
    the entries whose hint lies outside the band (real disagreements), max_gap = the largest
    gap / scale among the changed entries."""
    hint = np.ascontiguousarray(hint, np.int32)
    S = np.ascontiguousarray(scale, np.float64)
    F = X.shape[1]
    hard = ctypes.c_int64(0)
    gap = ctypes.c_double(0.0)
    d = ctypes.POINTER(ctypes.c_double)
    i32 = ctypes.POINTER(ctypes.c_int32)
    if X.dtype == np.float64:
        w = g.ew.astype(np.float64) if use_weight else None
        n = lib().oracle_spmm_max_align_f64(
            _p(g.indptr, _i64p), _p(g.indices, _i64p), _p(g.eids, _i64p), _p(w, d), _p(X, d), g.n, F,
            _p(hint, i32), _p(S, d), float(band), _p(out, d), _p(argx, _i64p), _p(arge, _i64p), ctypes.byref(hard),
            ctypes.byref(gap))
    else:
        w = g.ew if use_weight else None
        n = lib().oracle_spmm_max_align(
            _p(g.indptr, _i64p), _p(g.indices, _i64p), _p(g.eids, _i64p), _p(w, _f32p), _p(X, _f32p), g.n, F,
            _p(hint, i32), _p(S, d), float(band), _p(out, _f32p), _p(argx, _i64p), _p(arge, _i64p), ctypes.byref(hard),
            ctypes.byref(gap))
    return int(n), int(hard.value), float(gap.value)


class _MaxAggregate(torch.autograd.Function):
    """update_all(copy_u|u_mul_e, max) with DGL's GSpMM backward (scatter_add_ on argX).
    `align` (optional dict: hint, scale, band, counts) aligns near-tie winners with another
    computation (spmm_max_align) and receives the final argx / arge."""

    @staticmethod
    def forward(ctx, P, g, use_weight, parallel=False, align=None):
        Xn = np.ascontiguousarray(P.detach().numpy())
        out, argx, arge = spmm_max(g, Xn, use_weight, parallel)
        if align is not None:
            n, hard, gap = spmm_max_align(g, Xn, use_weight, align["hint"], align["scale"], align["band"], out,
                                          argx, arge)
            c = align["counts"]
            c["_ties"] = c.get("_ties", 0) + n
            c["_hard_ties"] = c.get("_hard_ties", 0) + hard
            c["_max_tie_ulps"] = max(c.get("_max_tie_ulps", 0.0), gap / U32)
            align["argx"], align["arge"] = argx, arge
        ctx.g, ctx.argx, ctx.arge, ctx.use_weight, ctx.parallel = g, argx, arge, use_weight, parallel
        return torch.from_numpy(out)

    @staticmethod
    def backward(ctx, dZ):
        if ctx.parallel or dZ.dtype == torch.float64:
            # DGL's own form: dX = zeros; dX.scatter_add_(0, argX, dZ [* w[argE]]) in torch-CPU
            dZ = dZ.contiguous()
            if ctx.use_weight:
                dZ = dZ * torch.from_numpy(ctx.g.ew).to(dZ.dtype)[torch.from_numpy(ctx.arge)]
            dX = torch.zeros_like(dZ).scatter_add_(0, torch.from_numpy(ctx.argx), dZ)
            return dX, None, None, None, None
        dX = spmm_max_bwd(ctx.g, ctx.argx, ctx.arge, dZ.contiguous().numpy(), ctx.use_weight)
        return torch.from_numpy(dX), None, None, None, None


# ---------------------------------------------------------------- model (code/model.py)
def leaky_relu(x):
    return torch.nn.functional.leaky_relu(x)  # negative_slope 0.01 (model.py:21,23,25,27)


# Decision alignment (parity tests at full size). Two float32 computations of the same
# algorithm round differently, so a relu / leaky_relu decision at a pre-activation near 0,
# or the winner among two nearly equal maximum candidates, can differ between them. Such a
# decision is taken from the other computation (`signs`) when it lies within BAND_ULPS
# units of 2^-24 x its running-error scale: the float64 sum of |terms| the value was
# formed from, propagated through the layers (|x| -> |h| |W|^T + |b| -> the winner's scale
# -> ...), i.e. a few ulp of the magnitudes that formed THAT value, not of the layer's
# largest value. Entries outside the band where the decisions differ count as "hard".
BAND_ULPS = 16.0
U32 = 2.0 ** -24


def _act(pre, slope, site, signs, scale=None, band_ulps: float = BAND_ULPS):
    """relu (slope 0) / leaky_relu of `pre`. With `signs` (site -> the other computation's
    "output > 0" mask) and `scale` (running-error scale of pre, float64), entries with
    |pre| <= band_ulps * 2^-24 * scale take that decision instead of their own.
    signs["_flips"] counts the changed decisions, signs["_hard_flips"] the differing ones
    outside the band, signs["_max_flip_ulps"] the largest |pre| / (2^-24 scale) among the
    changed ones."""
    if signs is None or site not in signs:
        return torch.relu(pre) if slope == 0.0 else torch.nn.functional.leaky_relu(pre, slope)
    with torch.no_grad():
        own = pre > 0
        eng = signs[site].to(own.device)
        ulps = pre.detach().abs().double() / (U32 * scale.clamp(min=1e-300))
        tiny = ulps <= band_ulps
        pos = torch.where(tiny, eng, own)
        changed = pos != own
        signs["_flips"] = signs.get("_flips", 0) + int(changed.sum())
        signs["_hard_flips"] = signs.get("_hard_flips", 0) + int(((eng != own) & ~tiny).sum())
        if bool(changed.any()):
            signs["_max_flip_ulps"] = max(signs.get("_max_flip_ulps", 0.0), float(ulps[changed].max()))
    return torch.where(pos, pre, pre * slope)


def _absmm(s: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """Running-error scale of s-scaled inputs times w^T: s |w|^T (float64)."""
    return s @ w.detach().abs().double().t()


def sage_pool(g: OracleGraph, h: torch.Tensor, p: Dict[str, torch.Tensor], prefix: str,
              use_weight: bool = False, parallel: bool = False, signs=None, sh: Optional[torch.Tensor] = None
              ):
    """DGL 0.8.2 SAGEConv(aggregator_type='pool', feat_drop=0, bias=True, norm=None,
    activation=None).forward(graph, feat[, edge_weight]). With `signs` and `sh` (the
    running-error scale of h) the decisions are aligned and (rst, scale of rst) returned."""
    pre = h @ p[prefix + "fc_pool.weight"].t() + p[prefix + "fc_pool.bias"]
    if signs is None:
        P = torch.relu(pre)
        neigh = _MaxAggregate.apply(P, g, use_weight, parallel, None)
        return neigh @ p[prefix + "fc_neigh.weight"].t() + h @ p[prefix + "fc_self.weight"].t() + p[prefix + "bias"]
    s_pool = _absmm(sh, p[prefix + "fc_pool.weight"]) + p[prefix + "fc_pool.bias"].detach().abs().double()
    P = _act(pre, 0.0, prefix + "pool", signs, s_pool)
    align = None
    if prefix + "argpos" in signs:
        align = {"hint": signs[prefix + "argpos"], "scale": s_pool.numpy(), "band": BAND_ULPS * U32, "counts": signs}
    neigh = _MaxAggregate.apply(P, g, use_weight, parallel, align)
    if align is not None:
        s_m = torch.gather(s_pool, 0, torch.from_numpy(align["argx"]))
        if use_weight:
            s_m = s_m * torch.from_numpy(np.abs(g.ew)).double()[torch.from_numpy(align["arge"])]
    else:
        s_m = torch.zeros_like(s_pool)
    rst = neigh @ p[prefix + "fc_neigh.weight"].t() + h @ p[prefix + "fc_self.weight"].t() + p[prefix + "bias"]
    s_rst = (_absmm(s_m, p[prefix + "fc_neigh.weight"]) + _absmm(sh, p[prefix + "fc_self.weight"])
             + p[prefix + "bias"].detach().abs().double())
    return rst, s_rst


class _SumAggregate(torch.autograd.Function):
    """update_all(copy_u|u_mul_e, sum|mean) (C: oracle_spmm_sum) with DGL's GSpMM backward:
    the same aggregation over the reversed graph, dX[u] = sum_{e = (u -> v)} w_e dZ[v]
    (mean: dZ[v] / max(in_deg(v), 1)), summed in edge-id order. Float64 inputs run the
    whole aggregation in torch float64 (the yardstick)."""

    @staticmethod
    def forward(ctx, X, g, use_weight, mean):
        ctx.g, ctx.use_weight, ctx.mean = g, use_weight, mean
        if X.dtype == torch.float64:
            return _sum_t(g, X, use_weight, mean)
        return torch.from_numpy(spmm_sum(g, X.detach().numpy(), mean=mean, use_weight=use_weight))

    @staticmethod
    def backward(ctx, dZ):
        g = ctx.g
        src, dst = torch.from_numpy(g.src), torch.from_numpy(g.dst)
        d = dZ
        if ctx.mean:
            deg = torch.from_numpy(np.maximum(g.in_degrees(), 1)).to(dZ.dtype)
            d = dZ / deg[:, None]
        m = d[dst]
        if ctx.use_weight:
            m = m * torch.from_numpy(g.ew).to(dZ.dtype)[:, None]
        return torch.zeros_like(dZ).index_add_(0, src, m), None, None, None


def _sum_t(g: OracleGraph, X: torch.Tensor, use_weight: bool, mean: bool) -> torch.Tensor:
    src, dst = torch.from_numpy(g.src), torch.from_numpy(g.dst)
    m = X[src]
    if use_weight:
        m = m * torch.from_numpy(g.ew).to(X.dtype)[:, None]
    out = torch.zeros_like(X).index_add_(0, dst, m)
    if mean:
        out = out / torch.from_numpy(np.maximum(g.in_degrees(), 1)).to(X.dtype)[:, None]
    return out


def out_degrees(g: OracleGraph) -> np.ndarray:
    return np.bincount(g.src, minlength=g.n)


def graph_conv(g: OracleGraph, feat: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
               norm: str = "both", use_weight: bool = False) -> torch.Tensor:
    """DGL 0.8.2 GraphConv.forward(graph, feat[, edge_weight]) (dgl/nn/pytorch/conv/
    graphconv.py; BASELINE configs[0], not run by the reference: reference-unpinned):
    norm 'left'/'both' scales the source features by out_degree.clamp(min=1)^-1/2 (or ^-1),
    the product with weight [in, out] runs BEFORE the sum aggregation when in_feats >
    out_feats and after it otherwise, norm 'right'/'both' scales by
    in_degree.clamp(min=1)^-1/2 (or ^-1), then + bias."""
    if norm in ("left", "both"):
        degs = torch.from_numpy(out_degrees(g)).to(feat.dtype).clamp(min=1)
        nrm = torch.pow(degs, -0.5) if norm == "both" else 1.0 / degs
        feat = feat * nrm.reshape(-1, 1)
    if weight.shape[0] > weight.shape[1]:
        rst = _SumAggregate.apply(feat @ weight, g, use_weight, False)
    else:
        rst = _SumAggregate.apply(feat, g, use_weight, False) @ weight
    if norm in ("right", "both"):
        degs = torch.from_numpy(g.in_degrees()).to(feat.dtype).clamp(min=1)
        nrm = torch.pow(degs, -0.5) if norm == "both" else 1.0 / degs
        rst = rst * nrm.reshape(-1, 1)
    if bias is not None:
        rst = rst + bias
    return rst


def sage_mean(g: OracleGraph, h: torch.Tensor, p: Dict[str, torch.Tensor], prefix: str, aggr: str = "mean",
              use_weight: bool = False) -> torch.Tensor:
    """DGL 0.8.2 SAGEConv(aggregator_type='mean' | 'gcn').forward (reference-unpinned; the
    reference runs 'pool' only): fc_neigh before the aggregation when in_feats > out_feats
    (lin_before_mp), after it otherwise; 'mean' = fc_self(h) + fc_neigh(mean over in-edges)
    + bias; 'gcn' = fc_neigh((sum over in-edges + h) / (in_degree + 1)) + bias."""
    wn = p[prefix + "fc_neigh.weight"]
    lin_before = wn.shape[1] > wn.shape[0]
    src = h @ wn.t() if lin_before else h
    if aggr == "mean":
        neigh = _SumAggregate.apply(src, g, use_weight, True)
    else:
        s = _SumAggregate.apply(src, g, use_weight, False)
        neigh = (s + src) / (torch.from_numpy(g.in_degrees()).to(h.dtype)[:, None] + 1)
    if not lin_before:
        neigh = neigh @ wn.t()
    rst = neigh if aggr == "gcn" else h @ p[prefix + "fc_self.weight"].t() + neigh
    return rst + p[prefix + "bias"]


def _graph_conv_scale(g: OracleGraph, sh: torch.Tensor, weight: torch.Tensor, bias, norm: str = "both",
                      use_weight: bool = False) -> torch.Tensor:
    """Running-error scale of graph_conv's output (the same operations on |values|)."""
    if norm in ("left", "both"):
        degs = torch.from_numpy(out_degrees(g)).double().clamp(min=1)
        sh = sh * (torch.pow(degs, -0.5) if norm == "both" else 1.0 / degs).reshape(-1, 1)
    wa = weight.detach().abs().double()
    r = _sum_t(g, sh @ wa, use_weight, False) if weight.shape[0] > weight.shape[1] else _sum_t(g, sh, use_weight,
                                                                                                False) @ wa
    if norm in ("right", "both"):
        degs = torch.from_numpy(g.in_degrees()).double().clamp(min=1)
        r = r * (torch.pow(degs, -0.5) if norm == "both" else 1.0 / degs).reshape(-1, 1)
    return r + (0.0 if bias is None else bias.detach().abs().double())


def _sage_mean_scale(g: OracleGraph, sh: torch.Tensor, p, prefix: str, aggr: str, use_weight: bool) -> torch.Tensor:
    wn = p[prefix + "fc_neigh.weight"]
    lin_before = wn.shape[1] > wn.shape[0]
    src = _absmm(sh, wn) if lin_before else sh
    if aggr == "mean":
        neigh = _sum_t(g, src, use_weight, True)
    else:
        neigh = (_sum_t(g, src, use_weight, False) + src) / (torch.from_numpy(g.in_degrees()).double()[:, None] + 1)
    if not lin_before:
        neigh = _absmm(neigh, wn)
    r = neigh if aggr == "gcn" else _absmm(sh, p[prefix + "fc_self.weight"]) + neigh
    return r + p[prefix + "bias"].detach().abs().double()


def gnn32_forward(g: OracleGraph, x: torch.Tensor, p: Dict[str, torch.Tensor],
                  use_weight: bool = False, parallel: bool = False, signs=None) -> torch.Tensor:
    """GNN32.forward (code/model.py:19-31), generalised to any number of conv layers and,
    for BASELINE configs[0] (reference-unpinned), to GraphConv / SAGEConv('mean'|'gcn')
    layers (told apart by their parameter names: conv<i>.weight = GraphConv, no
    fc_pool = SAGE mean, no fc_self = SAGE gcn).
    Activation sites for `signs` (decision alignment, see _act): conv<i>.pool (relu of
    fc_pool), conv<i>.out (the layer's leaky_relu), liner1; conv<i>.argpos the max
    aggregation's winners. The running-error scale of every value is carried beside it."""
    h = x
    sh = x.detach().abs().double() if signs is not None else None
    i = 1
    while f"conv{i}.bias" in p:
        q = f"conv{i}."
        s_y = None
        if q + "weight" in p:
            y = graph_conv(g, h, p[q + "weight"], p[q + "bias"], use_weight=use_weight)
            if signs is not None:
                s_y = _graph_conv_scale(g, sh, p[q + "weight"], p[q + "bias"], use_weight=use_weight)
        elif q + "fc_pool.weight" in p:
            r = sage_pool(g, h, p, q, use_weight, parallel, signs, sh)
            y, s_y = r if signs is not None else (r, None)
        else:
            aggr = "mean" if q + "fc_self.weight" in p else "gcn"
            y = sage_mean(g, h, p, q, aggr, use_weight)
            if signs is not None:
                s_y = _sage_mean_scale(g, sh, p, q, aggr, use_weight)
        h = _act(y, 0.01, q + "out", signs, s_y)
        sh = s_y
        i += 1
    pre = h @ p["liner1.weight"].t() + p["liner1.bias"]
    s1 = None if signs is None else _absmm(sh, p["liner1.weight"]) + p["liner1.bias"].detach().abs().double()
    h = _act(pre, 0.01, "liner1", signs, s1)
    h = h @ p["liner2.weight"].t() + p["liner2.bias"]
    return torch.sigmoid(h)


def init_params(dims, seed: int = 0, conv: str = "pool") -> Dict[str, torch.Tensor]:
    """Fresh parameters shaped like GNN32(dims[0], ..., num_classes); DGL 0.8 init
    (xavier_uniform gain sqrt(2) on fc_pool/fc_self/fc_neigh, zero SAGE bias). conv:
    'pool' (the reference), 'mean' / 'gcn' (SAGEConv variants) or 'graphconv' (GraphConv:
    weight [in, out] xavier_uniform gain 1; the biases drawn small and non-zero here so
    that their gradients are exercised)."""
    gen = torch.Generator().manual_seed(seed)
    n_conv = len(dims) - 3
    p: Dict[str, torch.Tensor] = {}

    def xavier(o, i, gain=2.0 ** 0.5):
        a = gain * (6.0 / (i + o)) ** 0.5
        return (torch.rand(o, i, generator=gen) * 2 - 1) * a

    def lin(o, i):
        b = 1.0 / i ** 0.5
        return (torch.rand(o, i, generator=gen) * 2 - 1) * b, (torch.rand(o, generator=gen) * 2 - 1) * b

    for li in range(n_conv):
        fi, fo = dims[li], dims[li + 1]
        pre = f"conv{li + 1}."
        if conv == "graphconv":
            p[pre + "weight"] = xavier(fi, fo, 1.0)
            p[pre + "bias"] = lin(fo, fo)[1] * 0.1
            continue
        if conv == "pool":
            p[pre + "fc_pool.weight"] = xavier(fi, fi)
            p[pre + "fc_pool.bias"] = lin(fi, fi)[1]
        p[pre + "fc_neigh.weight"] = xavier(fo, fi)
        if conv != "gcn":
            p[pre + "fc_self.weight"] = xavier(fo, fi)
        p[pre + "bias"] = torch.zeros(fo) if conv == "pool" else lin(fo, fo)[1] * 0.1
    w1, b1 = lin(dims[-2], dims[-3])
    w2, b2 = lin(dims[-1], dims[-2])
    p["liner1.weight"], p["liner1.bias"] = w1, b1
    p["liner2.weight"], p["liner2.bias"] = w2, b2
    return p


# ---------------------------------------------------------------- loss (code/train.py)
def multi_loss(input: torch.Tensor, target: torch.Tensor, i_weight) -> torch.Tensor:
    """code/train.py:89-108."""
    loss = 0
    for i in range(len(i_weight)):
        scl_input = input[:, i]
        scl_target = target[:, i]
        a = scl_target * torch.log(torch.clamp(scl_input, 1e-9, 10.)) * i_weight[i]
        b = (1 - scl_target) * torch.log(torch.clamp(1 - scl_input, 1e-9, 10.))
        scl_loss = (a + b) / (i_weight[i] + 1) * 2
        loss += -scl_loss.sum() / len(input)
    return loss


def weight_cal(loc_mat: np.ndarray) -> np.ndarray:
    """code/train.py:111-126: w_c = (n_labelled - n_c) / n_c (float64)."""
    class_num = loc_mat.sum(axis=0)
    sample_num = int((loc_mat.sum(axis=1) != 0).sum())
    return (sample_num - class_num) / class_num


# ---------------------------------------------------------------- optimiser
def adam_step_torch110(params, grads, exp_avg, exp_avg_sq, step: int, lr: float,
                       beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8):
    """torch 1.10.0 F.adam (single tensor), in place; step is the new step count."""
    import math

    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    for p, g, m, v in zip(params, grads, exp_avg, exp_avg_sq):
        m.mul_(beta1).add_(g, alpha=1 - beta1)
        v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(m, denom, value=-(lr / bc1))


# ---------------------------------------------------------------- one training step
def train_step(g: OracleGraph, x: torch.Tensor, labels: torch.Tensor, train_index,
               i_weight, p: Dict[str, torch.Tensor], use_weight: bool = False,
               parallel: bool = False, dtype=torch.float32, signs=None
               ) -> Tuple[torch.Tensor, torch.Tensor, Dict[str, torch.Tensor]]:
    """zero_grad -> forward -> multi_loss(train rows) -> backward (code/train.py:197-204).
    Returns (logits, loss, grads). parallel=True runs the message passing as DGL's CPU
    backend does (OpenMP rows forward, torch scatter_add_ backward): the CPU baseline.
    dtype=torch.float64 computes the same step in double precision (the yardstick the
    full-size tests use to judge two float32 results that differ by more than 1e-4).
    signs: another computation's decisions, taken where they lie within the rounding band
    (see _act / BAND_ULPS): "<site>" masks ("output > 0") and "conv<i>.argpos" (N x F int32
    in-row winner positions, spmm_max_align); the counts come back in its "_" keys."""
    if dtype != torch.float32:  # the float64 yardstick: every tensor and product in double
        x = x.to(dtype)
        p = {k: v.to(dtype) for k, v in p.items()}
        labels = labels.to(dtype)
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    logits = gnn32_forward(g, x, leaves, use_weight, parallel, signs)
    loss = multi_loss(logits[train_index], labels[train_index], i_weight)
    loss.backward()
    return logits.detach(), loss.detach(), {k: v.grad.detach() for k, v in leaves.items()}


# ---------------------------------------------------------------- §8f: ECC and eval
def edge_clustering_coefficients(ppi_net, epsilon: float = 0.0):
    """code/data_preprocess.py:175-214 (C restatement, oracle/ecc_oracle.c): scipy COO."""
    from scipy.sparse import coo_matrix

    csr = ppi_net.tocsr()
    n = csr.shape[0]
    indptr = np.ascontiguousarray(csr.indptr, np.int64)
    indices = np.ascontiguousarray(csr.indices, np.int64)
    data = np.ascontiguousarray(csr.data, np.float64)
    cap = max(1, 2 * len(indices))
    rows, cols = np.empty(cap, np.int64), np.empty(cap, np.int64)
    vals = np.empty(cap, np.float64)
    m = lib().oracle_ecc(_p(indptr, _i64p), _p(indices, _i64p), _p(data, ctypes.POINTER(ctypes.c_double)), n,
                         float(epsilon), _p(rows, _i64p), _p(cols, _i64p),
                         _p(vals, ctypes.POINTER(ctypes.c_double)))
    if m < 0:
        raise MemoryError("oracle_ecc")
    return coo_matrix((vals[:m], (rows[:m], cols[:m])), shape=csr.shape)


def protein_loc_correction(loc_proba: torch.Tensor, alpha: float, rowwise: bool = False) -> torch.Tensor:
    """code/train.py:19-39, the same torch-CPU float32 operations. By default the per-row
    threshold loop of the reference is one row-wise comparison; rowwise=True keeps the
    reference's Python loop over the rows (train.py:36-38: same result, its cost), which
    bench.py times for the reference-faithful epoch."""
    loc_proba = loc_proba.detach().cpu().float()
    min_proba = loc_proba.min(dim=0).values
    max_proba = loc_proba.max(dim=0).values
    new_proba = (loc_proba - min_proba) / (max_proba - min_proba)
    sum_proba = new_proba.sum(dim=1).reshape(-1, 1)
    new_proba = new_proba / sum_proba
    rmax = new_proba.max(dim=1).values
    rmin = new_proba.min(dim=1).values
    thresholds = rmax - (rmax - rmin) * alpha
    if rowwise:
        loc_pred = torch.zeros(loc_proba.shape)
        for row in range(len(loc_proba)):
            loc_pred[row][new_proba[row] > thresholds[row]] = 1.
        return loc_pred.double()
    return (new_proba > thresholds.reshape(-1, 1)).double()


def performances_record(loc_true: torch.Tensor, loc_pred: torch.Tensor):
    """code/train.py:42-86: aim / coverage / accuracy, float32 running sums in row order."""
    t = (loc_true.detach().cpu().long() == 1)
    p = (loc_pred.detach().cpu().long() == 1)
    aim = torch.zeros((), dtype=torch.float32)
    cov = torch.zeros((), dtype=torch.float32)
    acc = torch.zeros((), dtype=torch.float32)
    for i in range(len(t)):
        and_set = (t[i] & p[i]).sum().float()
        pred = p[i].sum().float()
        real = t[i].sum().float()
        or_set = (t[i] | p[i]).sum().float()
        if pred != 0:
            aim = aim + and_set / pred
        cov = cov + and_set / real
        acc = acc + and_set / or_set
    n = len(t)
    return float(aim / n), float(cov / n), float(acc / n)


# ---------------------------------------------------------------- §8f: topology perturbation
def pcc_matrix(expr) -> np.ndarray:
    """code/data_preprocess.py:166-169, verbatim numpy: np.corrcoef of the rows, diagonal
    and NaN set to 0 (dense N x N float64)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        c = np.corrcoef(np.asarray(expr, np.float64))
    np.fill_diagonal(c, 0)
    c[np.isnan(c)] = 0
    return c


def modify_network_topology(ppi_net, pcc_nor: np.ndarray, pcc_inter: np.ndarray, thr: float):
    """code/data_preprocess.py:217-257 on dense correlation matrices (numpy, verbatim
    operations): returns (scipy COO of the perturbed adjacency, (mean, std) of diff)."""
    from scipy.sparse import coo_matrix

    a = np.asarray(ppi_net.tocsr().todense())
    diff = pcc_inter - pcc_nor
    mean, std = np.mean(diff), np.std(diff)
    lo, hi = mean - thr * std, mean + thr * std
    res1 = np.logical_and(diff < lo, a == 1)
    res2 = np.logical_and(diff > hi, a == 0)
    a[res1] = 0
    a[res2] = 1
    return coo_matrix(a), (float(mean), float(std))


class PerturbStream:
    """The streaming C restatement (oracle/perturb_oracle.c) on centred expression rows:
    never stores an N x N matrix, so it runs at the full PPI size (CPU baseline)."""

    def __init__(self, ppi_net, expr_normal, expr_inter):
        def centred(e):
            x = np.array(e, dtype=np.float64, ndmin=2)
            x -= x.mean(axis=1)[:, None]
            return np.ascontiguousarray(x)

        self.xn, self.xi = centred(expr_normal), centred(expr_inter)
        self.n, self.S = self.xn.shape
        self.inv_fact = float(np.true_divide(1, self.S - 1))
        f64p = ctypes.POINTER(ctypes.c_double)
        self.sdn = np.empty(self.n)
        self.sdi = np.empty(self.n)
        lib().oracle_perturb_sd(_p(self.xn, f64p), self.n, self.S, self.inv_fact, _p(self.sdn, f64p))
        lib().oracle_perturb_sd(_p(self.xi, f64p), self.n, self.S, self.inv_fact, _p(self.sdi, f64p))
        csr = ppi_net.tocsr()
        csr.sum_duplicates()
        csr.sort_indices()
        self.ptr = np.ascontiguousarray(csr.indptr, np.int64)
        self.col = np.ascontiguousarray(csr.indices, np.int64)
        v = np.ascontiguousarray(csr.data, np.int64)
        self.val = None if np.all(v == 1) else v
        self._f = f64p

    def _base(self):
        f = self._f
        return (_p(self.xn, f), _p(self.xi, f), _p(self.sdn, f), _p(self.sdi, f), self.n, self.S, self.inv_fact)

    def row_sum(self, squared: bool, mean: float, r0: int, r1: int) -> float:
        return lib().oracle_perturb_sum(*self._base(), int(squared), float(mean), r0, r1)

    def stats(self, thr: float):
        nn = float(self.n) * float(self.n)
        mean = self.row_sum(False, 0.0, 0, self.n) / nn
        std = float(np.sqrt(self.row_sum(True, mean, 0, self.n) / nn))
        return mean, std, mean - thr * std, mean + thr * std

    def rows(self, lo: float, hi: float, r0: int, r1: int):
        cap = int(self.ptr[r1] - self.ptr[r0]) + (r1 - r0) * self.n
        cap = min(cap, (r1 - r0) * self.n)
        rr, cc, vv = (np.empty(max(cap, 1), np.int64) for _ in range(3))
        m = lib().oracle_perturb_rows(*self._base(), _p(self.ptr, _i64p), _p(self.col, _i64p),
                                      _p(self.val, _i64p), lo, hi, r0, r1, _p(rr, _i64p), _p(cc, _i64p),
                                      _p(vv, _i64p), len(rr))
        if m < 0:
            raise MemoryError("oracle_perturb_rows")
        return rr[:m], cc[:m], vv[:m]


# ---------------------------------------------------------------- PCA front end
def pca_randomized(mat, n_components: int, random_state: int = 42, n_oversamples: int = 10) -> np.ndarray:
    """CPU restatement of ``pca(mat, components)`` (code/data_preprocess.py:475-487), i.e.
    scikit-learn 1.1.1 (README.md:30) ``PCA(n_components, random_state=42).fit_transform``
    on the path its svd_solver='auto' takes for the reference's matrices (N = 24 041 > 500,
    250 < 0.8 N): ``_fit_truncated`` -> ``randomized_svd(X - mean, n_components,
    n_oversamples=10, n_iter='auto' (7 when n_components < 0.1 min(shape), else 4),
    power_iteration_normalizer='auto' (LU for n_iter > 2), flip_sign=True,
    random_state=RandomState(42))``: Gaussian test matrix ``normal(size=(n_features,
    n_components + 10))``, LU-normalised power iterations (``scipy.linalg.lu(.., permute_l=True)``),
    economic QR, SVD of ``Q^T X``, ``U = Q Uhat``, ``svd_flip`` u-based (1.1.1's rule: each
    column of U made positive at its largest |entry|), returned as ``U[:, :k] * S[:k]``.
    Pinned by tests/golden/pca.npz (the reference's own pca() under scikit-learn 1.7.2, the
    same algorithm with v-based signs)."""
    import scipy.linalg as sla
    import scipy.sparse as sp

    X = mat.toarray() if sp.issparse(mat) else np.asarray(mat)
    X = np.array(X, dtype=np.float64)
    n_samples, n_features = X.shape
    if not (max(X.shape) > 500 and 1 <= n_components < 0.8 * min(X.shape)):
        raise ValueError("pca_randomized: sklearn 1.1.1 would take the full-SVD path here")
    if n_samples < n_features:
        raise ValueError("pca_randomized: transposed randomized SVD not restated")
    X -= X.mean(axis=0)
    rs = np.random.RandomState(random_state)
    size = n_components + n_oversamples
    n_iter = 7 if n_components < 0.1 * min(X.shape) else 4
    Q = rs.normal(size=(n_features, size))
    for _ in range(n_iter):
        Q, _ = sla.lu(X @ Q, permute_l=True)
        Q, _ = sla.lu(X.T @ Q, permute_l=True)
    Q, _ = sla.qr(X @ Q, mode="economic")
    Uhat, s, _ = sla.svd(Q.T @ X, full_matrices=False)
    U = Q @ Uhat
    idx = np.argmax(np.abs(U), axis=0)
    U *= np.sign(U[idx, np.arange(U.shape[1])])
    return U[:, :n_components] * s[:n_components]
