"""Topology perturbation on the GPU.

The reference builds, per drug dataset, two dense N x N Pearson matrices of the protein
expression rows (``construct_gcn_matrix``, code/data_preprocess.py:128-172: np.corrcoef,
diagonal and NaN set to 0) and perturbs the PPI topology by their difference
(``modify_network_topology``, code/data_preprocess.py:217-257): with
diff = pcc_inter - pcc_normal over all N x N entries,
  an edge is dropped when ppi == 1 and diff < mean(diff) - thr * std(diff),
  an edge is added   when ppi == 0 and diff > mean(diff) + thr * std(diff).
At N = 24 041 that is 2 x 4.6 GB of float64 correlations plus a dense difference and a
dense copy of the adjacency on the host. Here the same result comes from four fused HIP
passes over (i, j) that recompute the correlation from the centred N x S expression
rows (``pg_perturb_*``) — nothing N x N is ever stored.

``modify_network_topology_expr(ppi_net, expr_normal, expr_inter, thr)`` is the drop-in
for the reference's call at code/data_preprocess.py:326, taking the expression matrices
that ``construct_gcn_matrix`` returns alongside the correlation matrices; it returns the
same scipy COO matrix (row-major entries, int64 values) as
``modify_network_topology(ppi_net, coo(pcc(expr_normal)), coo(pcc(expr_inter)), thr)``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr


@dataclass
class PerturbStats:
    mean: float
    std: float
    lo_thr: float
    hi_thr: float
    removed: int
    added: int


def _centred(expr) -> np.ndarray:
    """X - X.mean(axis=1) exactly as np.cov does it (code/data_preprocess.py:166)."""
    x = np.array(expr, dtype=np.float64, ndmin=2)
    avg = x.mean(axis=1)
    x -= avg[:, None]
    return np.ascontiguousarray(x)


def modify_network_topology_expr(ppi_net, expr_normal, expr_inter, thr: float, device="cuda",
                                 return_stats: bool = False):
    from scipy.sparse import coo_matrix

    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError("perturb: GPU entry point (the CPU form is the reference's own code)")
    csr = ppi_net.tocsr()
    csr.sum_duplicates()  # tocsr() sums duplicates like the reference's .todense()
    csr.sort_indices()
    n = csr.shape[0]
    if csr.shape != (n, n):
        raise ValueError("perturb: square adjacency expected")
    xn, xi = _centred(expr_normal), _centred(expr_inter)
    if xn.shape != xi.shape or xn.shape[0] != n:
        raise ValueError("perturb: expression matrices must both be N x S")
    S = xn.shape[1]
    if not 2 <= S <= 8:
        raise ValueError("perturb: 2 <= samples <= 8")
    inv_fact = float(np.true_divide(1, S - 1))  # np.cov: c *= np.true_divide(1, fact)
    vals = np.asarray(csr.data).astype(np.int64)
    all_ones = bool(np.all(vals == 1))
    st = _lib.stream_handle(dev)
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    t_xn, t_xi = up(xn), up(xi)
    t_ptr, t_col = up(csr.indptr.astype(np.int32)), up(csr.indices.astype(np.int32))
    t_val = None if all_ones else up(vals)
    sdn = torch.empty(n, dtype=torch.float64, device=dev)
    sdi = torch.empty(n, dtype=torch.float64, device=dev)
    ws = torch.empty(max(1, int(_lib.lib().pg_perturb_workspace(n))), dtype=torch.uint8, device=dev)
    tot = torch.zeros(2, dtype=torch.float64, device=dev)
    call("pg_perturb_prepare", ptr(t_xn), ptr(t_xi), n, S, inv_fact, ptr(sdn), ptr(sdi), st)
    base = (ptr(t_xn), ptr(t_xi), ptr(sdn), ptr(sdi), n, S, inv_fact)
    # np.mean / np.std of the dense difference (code/data_preprocess.py:242-243)
    call("pg_perturb_sum", *base, 0, 0.0, ptr(tot[0:1]), ptr(ws), ws.numel(), st)
    nn = float(n) * float(n)
    mean = float(tot[0].item()) / nn
    call("pg_perturb_sum", *base, 1, mean, ptr(tot[1:2]), ptr(ws), ws.numel(), st)
    std = math.sqrt(float(tot[1].item()) / nn)
    thr = float(thr)
    lo, hi = mean - thr * std, mean + thr * std  # code/data_preprocess.py:244-245
    counts = torch.zeros(n, dtype=torch.int32, device=dev)
    call("pg_perturb_count", *base, ptr(t_ptr), ptr(t_col), ptr(t_val), lo, hi, ptr(counts), st)
    c = counts.cpu().numpy().astype(np.int64)
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(c, out=offs[1:])
    nnz = int(offs[-1])
    t_offs = up(offs)
    out_col = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
    out_val = torch.empty(max(nnz, 1), dtype=torch.int64, device=dev)
    call("pg_perturb_fill", *base, ptr(t_ptr), ptr(t_col), ptr(t_val), lo, hi, ptr(t_offs), ptr(out_col),
         ptr(out_val), st)
    cols = out_col[:nnz].cpu().numpy().astype(np.int32)
    data = out_val[:nnz].cpu().numpy()
    rows = np.repeat(np.arange(n, dtype=np.int32), c)
    res = coo_matrix((data, (rows, cols)), shape=(n, n))
    if not return_stats:
        return res
    # removed / added edges (directed entries) for reporting
    old = csr.copy()
    old.data = vals
    new = res.tocsr()
    removed = int(((old != 0).astype(np.int8) - (new != 0).astype(np.int8) > 0).sum())
    added = int(((new != 0).astype(np.int8) - (old != 0).astype(np.int8) > 0).sum())
    return res, PerturbStats(mean, std, lo, hi, removed, added)


def pcc_sd(expr, device="cuda") -> np.ndarray:
    """The per-row standard deviations the kernels use (sqrt of np.cov's diagonal);
    test hook for the prepare pass."""
    dev = torch.device(device)
    x = _centred(expr)
    n, S = x.shape
    t = torch.from_numpy(x).to(dev)
    a = torch.empty(n, dtype=torch.float64, device=dev)
    b = torch.empty(n, dtype=torch.float64, device=dev)
    call("pg_perturb_prepare", ptr(t), ptr(t), n, S, float(np.true_divide(1, S - 1)), ptr(a), ptr(b),
         _lib.stream_handle(dev))
    return a.cpu().numpy()


__all__ = ["modify_network_topology_expr", "PerturbStats", "pcc_sd"]
