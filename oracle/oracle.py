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
                                            _i32p, ctypes.c_double, _f32p, _i64p, _i64p]
        L.oracle_spmm_max_align.restype = ctypes.c_int64
        L.oracle_spmm_max_align_f64.argtypes = [_i64p, _i64p, _i64p, _d, _d, ctypes.c_int64, ctypes.c_int64, _i32p,
                                                ctypes.c_double, _d, _i64p, _i64p]
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


def spmm_max_align(g: OracleGraph, X: np.ndarray, use_weight: bool, hint: np.ndarray, tol: float,
                   out, argx, arge) -> int:
    """In place: entries where `hint` (another computation's winning in-row positions,
    -1 = none) names a candidate within tol * max|out| of the maximum take it (see
    oracle_spmm_max_align). Returns the number of changed entries."""
    hint = np.ascontiguousarray(hint, np.int32)
    F = X.shape[1]
    tol = float(tol) * float(np.abs(out).max(initial=0.0))
    if X.dtype == np.float64:
        d = ctypes.POINTER(ctypes.c_double)
        w = g.ew.astype(np.float64) if use_weight else None
        return int(lib().oracle_spmm_max_align_f64(
            _p(g.indptr, _i64p), _p(g.indices, _i64p), _p(g.eids, _i64p), _p(w, d), _p(X, d), g.n, F,
            _p(hint, ctypes.POINTER(ctypes.c_int32)), tol, _p(out, d), _p(argx, _i64p), _p(arge, _i64p)))
    w = g.ew if use_weight else None
    return int(lib().oracle_spmm_max_align(
        _p(g.indptr, _i64p), _p(g.indices, _i64p), _p(g.eids, _i64p), _p(w, _f32p), _p(X, _f32p), g.n, F,
        _p(hint, ctypes.POINTER(ctypes.c_int32)), tol, _p(out, _f32p), _p(argx, _i64p), _p(arge, _i64p)))


class _MaxAggregate(torch.autograd.Function):
    """update_all(copy_u|u_mul_e, max) with DGL's GSpMM backward (scatter_add_ on argX)."""

    @staticmethod
    def forward(ctx, P, g, use_weight, parallel=False, align=None):
        Xn = np.ascontiguousarray(P.detach().numpy())
        out, argx, arge = spmm_max(g, Xn, use_weight, parallel)
        if align is not None:  # (hint positions, tol, signs dict for the count)
            hint, tol, counts = align
            counts["_ties"] = counts.get("_ties", 0) + spmm_max_align(g, Xn, use_weight, hint, tol, out, argx, arge)
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


# Winner alignment band (spmm_max_align): a fraction of the aggregation's largest |value|.
# Float32 GEMM rounding moves P by ~1e-7 of that scale; near-ties seen differing between the
# engine and this oracle sat within 4e-8 of it.
WINNER_TOL = 1e-6


def _act(pre, slope, site, signs, sign_tol):
    """relu (slope 0) / leaky_relu of `pre`. With `signs` (site -> the other computation's
    "output > 0" mask), entries whose pre-activation lies within sign_tol * max|pre| of zero
    take that decision instead of their own: there the derivative (1 or slope) is decided by
    float32 rounding, not by the algorithm. signs["_flips"] counts the entries whose decision
    changed."""
    if signs is None or site not in signs:
        return torch.relu(pre) if slope == 0.0 else torch.nn.functional.leaky_relu(pre, slope)
    with torch.no_grad():
        own = pre > 0
        tiny = pre.abs() <= sign_tol * pre.abs().max()
        pos = torch.where(tiny, signs[site].to(own.device), own)
        signs["_flips"] = signs.get("_flips", 0) + int((pos != own).sum())
    return torch.where(pos, pre, pre * slope)


def sage_pool(g: OracleGraph, h: torch.Tensor, p: Dict[str, torch.Tensor], prefix: str,
              use_weight: bool = False, parallel: bool = False, signs=None, sign_tol: float = 0.0
              ) -> torch.Tensor:
    """DGL 0.8.2 SAGEConv(aggregator_type='pool', feat_drop=0, bias=True, norm=None,
    activation=None).forward(graph, feat[, edge_weight])."""
    P = _act(h @ p[prefix + "fc_pool.weight"].t() + p[prefix + "fc_pool.bias"], 0.0, prefix + "pool", signs,
             sign_tol)
    align = None
    if signs is not None and prefix + "argpos" in signs:
        align = (signs[prefix + "argpos"], WINNER_TOL, signs)
    neigh = _MaxAggregate.apply(P, g, use_weight, parallel, align)
    h_neigh = neigh @ p[prefix + "fc_neigh.weight"].t()
    rst = h @ p[prefix + "fc_self.weight"].t() + h_neigh
    return rst + p[prefix + "bias"]


def gnn32_forward(g: OracleGraph, x: torch.Tensor, p: Dict[str, torch.Tensor],
                  use_weight: bool = False, parallel: bool = False, signs=None,
                  sign_tol: float = 0.0) -> torch.Tensor:
    """GNN32.forward (code/model.py:19-31), generalised to any number of conv layers.
    Activation sites for `signs`: conv<i>.pool (relu of fc_pool), conv<i>.out (the layer's
    leaky_relu), liner1."""
    h = x
    i = 1
    while f"conv{i}.fc_pool.weight" in p:
        h = _act(sage_pool(g, h, p, f"conv{i}.", use_weight, parallel, signs, sign_tol), 0.01, f"conv{i}.out",
                 signs, sign_tol)
        i += 1
    h = _act(h @ p["liner1.weight"].t() + p["liner1.bias"], 0.01, "liner1", signs, sign_tol)
    h = h @ p["liner2.weight"].t() + p["liner2.bias"]
    return torch.sigmoid(h)


def init_params(dims, seed: int = 0) -> Dict[str, torch.Tensor]:
    """Fresh parameters shaped like GNN32(dims[0], ..., num_classes); DGL 0.8 init
    (xavier_uniform gain sqrt(2) on fc_pool/fc_self/fc_neigh, zero SAGE bias)."""
    gen = torch.Generator().manual_seed(seed)
    n_conv = len(dims) - 3
    p: Dict[str, torch.Tensor] = {}

    def xavier(o, i):
        a = (2.0 ** 0.5) * (6.0 / (i + o)) ** 0.5
        return (torch.rand(o, i, generator=gen) * 2 - 1) * a

    def lin(o, i):
        b = 1.0 / i ** 0.5
        return (torch.rand(o, i, generator=gen) * 2 - 1) * b, (torch.rand(o, generator=gen) * 2 - 1) * b

    for li in range(n_conv):
        fi, fo = dims[li], dims[li + 1]
        pre = f"conv{li + 1}."
        p[pre + "fc_pool.weight"] = xavier(fi, fi)
        p[pre + "fc_pool.bias"] = lin(fi, fi)[1]
        p[pre + "fc_neigh.weight"] = xavier(fo, fi)
        p[pre + "fc_self.weight"] = xavier(fo, fi)
        p[pre + "bias"] = torch.zeros(fo)
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
               parallel: bool = False, dtype=torch.float32, signs=None, sign_tol: float = 1e-5
               ) -> Tuple[torch.Tensor, torch.Tensor, Dict[str, torch.Tensor]]:
    """zero_grad -> forward -> multi_loss(train rows) -> backward (code/train.py:197-204).
    Returns (logits, loss, grads). parallel=True runs the message passing as DGL's CPU
    backend does (OpenMP rows forward, torch scatter_add_ backward): the CPU baseline.
    dtype=torch.float64 computes the same step in double precision (the yardstick the
    full-size tests use to judge two float32 results that differ by more than 1e-4).
    signs: see _act — the activation decisions of another computation at pre-activations
    within sign_tol * max|pre| of zero; "conv<i>.argpos" entries (N x F int32 in-row
    positions) do the same for the max aggregation's winners (spmm_max_align)."""
    if dtype != torch.float32:  # the float64 yardstick: every tensor and product in double
        x = x.to(dtype)
        p = {k: v.to(dtype) for k, v in p.items()}
        labels = labels.to(dtype)
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    logits = gnn32_forward(g, x, leaves, use_weight, parallel, signs, sign_tol)
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
