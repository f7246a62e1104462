"""Edge clustering coefficient on the GPU.

Drop-in for the reference's ``edge_clustering_coefficients(ppi_net, epsilon=0)``
(code/data_preprocess.py:175-214): same input (a scipy sparse symmetric adjacency), same
output (a scipy COO matrix holding ecc(i, j) at every stored off-diagonal entry, both
directions), bit-exact values. The O(E·N) dense-row Python loop of the reference becomes
one HIP kernel (``pg_ecc``). Explicit zeros are dropped before the count (PPI matrices
store ones only).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr


def prepare(ppi_net):
    """Host-side CSR view with sorted unique columns, the mirror map and degrees."""
    csr = ppi_net.tocsr().astype(np.float64)
    csr.eliminate_zeros()
    csr.sort_indices()
    n = csr.shape[0]
    if csr.shape[0] != csr.shape[1]:
        raise ValueError("ecc: square adjacency expected")
    indptr = csr.indptr.astype(np.int32)
    indices = csr.indices.astype(np.int32)
    lens = np.diff(indptr)
    rows = np.repeat(np.arange(n, dtype=np.int64), lens)
    key = rows * n + indices
    mkey = indices.astype(np.int64) * n + rows
    mirror = np.searchsorted(key, mkey)
    if len(key) and (mirror.max() >= len(key) or not np.array_equal(key[mirror], mkey)):
        raise ValueError("ecc: the adjacency must be symmetric")
    deg = np.bincount(rows, weights=csr.data, minlength=n).astype(np.float64)
    order = np.argsort(-lens, kind="stable").astype(np.int32)
    return csr, indptr, indices, mirror.astype(np.int32), deg, order, rows


def edge_clustering_coefficients(ppi_net, epsilon: float = 0.0, device="cuda"):
    from scipy.sparse import coo_matrix

    csr, indptr, indices, mirror, deg, order, rows = prepare(ppi_net)
    n, nnz = csr.shape[0], len(indices)
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError("ecc: GPU entry point (the CPU form is the reference's own loop)")
    t = {k: torch.from_numpy(v).to(dev) for k, v in
         (("ptr", indptr), ("col", indices), ("mirror", mirror), ("deg", deg), ("order", order))}
    out = torch.empty(max(nnz, 1), dtype=torch.float64, device=dev)
    call("pg_ecc", ptr(t["ptr"]), ptr(t["col"]), ptr(t["mirror"]), ptr(t["deg"]), ptr(t["order"]), n, nnz,
         float(epsilon), ptr(out), _lib.stream_handle(dev))
    vals = out[:nnz].cpu().numpy()
    keep = rows != indices
    return coo_matrix((vals[keep], (rows[keep], indices[keep].astype(np.int64))), shape=csr.shape)
