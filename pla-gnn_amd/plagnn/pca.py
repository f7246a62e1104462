"""GPU drop-in for the PCA front end: ``pca(mat, components)`` of
code/data_preprocess.py:475-487, called on the ECC and GCN*PPI matrices at 528-546.

The reference densifies a sparse N x N matrix (4.6 GB float64 at N = 24 041) and runs
scikit-learn 1.1.1's ``PCA(n_components, random_state=42).fit_transform``, which takes the
randomized-SVD path there. Here the same algorithm runs on the device without ever forming
the dense or the centred matrix:

* the test matrix is the same: ``RandomState(42).normal(size=(N, k + 10))`` (host, float64);
* every product with the centred matrix ``Xc = X - 1 mean^T`` is the sparse SpMM plus a
  rank-1 term, ``pg_csr_spmm_f64`` (HIP): ``Xc Q = X Q - 1 (mean^T Q)``,
  ``Xc^T Q = X^T Q - mean (1^T Q)`` (the transposed CSR);
* the power iterations (7 when k < 0.1 N) are normalised by CholeskyQR2 where scikit-learn
  uses a pivoted LU: both keep the span of ``Xc^(2i+1) Omega``, so the subspace — and the
  singular triplets computed from it — are the same up to rounding;
* ``Q = orth(Xc Q)``, ``B = Q^T Xc``, ``svd(B)`` (taken from the (k+10)^2 triangular factor
  of ``Xc^T Q``), ``U = Q Uhat``, scikit-learn 1.1.1's u-based ``svd_flip`` (README.md:30
  pins 1.1.1), output ``U[:, :k] * S[:k]``.
The Gram / Cholesky / triangular solves and the rank-1 vectors are dense torch float64 on
the device and the (k+10)^2 SVD is host LAPACK (plumbing); the products with the N x N
matrix are the HIP kernel.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib
from ._lib import call, ptr


def _csr(m: sp.csr_matrix, dev):
    m = m.tocsr()
    m.sum_duplicates()
    m.sort_indices()
    return (torch.from_numpy(m.indptr.astype(np.int32)).to(dev),
            torch.from_numpy(m.indices.astype(np.int32)).to(dev),
            torch.from_numpy(m.data.astype(np.float64)).to(dev))


def _spmm(csr, n_rows: int, X: torch.Tensor, u=None, v=None) -> torch.Tensor:
    p, c, w = csr
    Y = torch.empty(n_rows, X.shape[1], dtype=torch.float64, device=X.device)
    call("pg_csr_spmm_f64", n_rows, ptr(p), ptr(c), ptr(w), ptr(X), X.stride(0), X.shape[1], ptr(u), ptr(v),
         ptr(Y), Y.stride(0), _lib.stream_handle(X.device))
    return Y


def _orth(Y: torch.Tensor):
    """Orthonormal basis of Y's columns and R with Y = Q R: CholeskyQR2 (two Gram /
    Cholesky / triangular-solve passes, GEMM-shaped), falling back to Householder QR when a
    Gram matrix is not numerically positive definite."""
    R = torch.eye(Y.shape[1], dtype=Y.dtype, device=Y.device)
    for _ in range(2):
        L, info = torch.linalg.cholesky_ex(Y.t() @ Y)
        if int(info.item()) != 0:
            Q, R2 = torch.linalg.qr(Y)
            return Q.contiguous(), R2 @ R
        Y = torch.linalg.solve_triangular(L, Y.t(), upper=False).t()
        R = L.t() @ R
    return Y.contiguous(), R


def pca(mat, components: int, random_state: int = 42, n_oversamples: int = 10,
        device: str = "cuda") -> np.ndarray:
    """``PCA(n_components=components, random_state=42).fit_transform(mat)`` (scikit-learn
    1.1.1, randomized path) for a sparse or dense N x D matrix with N >= D; float64 out."""
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError("plagnn.pca runs on a HIP device")
    A = sp.csr_matrix(mat, dtype=np.float64)
    n, d = A.shape
    k = int(components)
    if not (max(n, d) > 500 and 1 <= k < 0.8 * min(n, d)):
        raise ValueError("pca: scikit-learn would take the full-SVD path for this shape/k (not built)")
    if n < d:
        raise ValueError("pca: N < D (scikit-learn's transposed randomized SVD) is not built")
    size = k + n_oversamples
    if size > 512:
        raise ValueError("pca: components + oversamples must be <= 512")
    n_iter = 7 if k < 0.1 * min(n, d) else 4
    mean = torch.from_numpy(np.asarray(A.sum(axis=0)).ravel() / n).to(dev)
    ones = None
    fwd, bwd = _csr(A, dev), _csr(A.T, dev)
    Q = torch.from_numpy(np.random.RandomState(random_state).normal(size=(d, size))).to(dev)

    def xc(Qm):  # Xc Q: rows n
        return _spmm(fwd, n, Qm, ones, (mean @ Qm).contiguous())

    def xct(Qm):  # Xc^T Q: rows d
        return _spmm(bwd, d, Qm, mean, Qm.sum(0).contiguous())

    for _ in range(n_iter):
        Q = _orth(xc(Q))[0]
        Q = _orth(xct(Q))[0]
    Q = _orth(xc(Q))[0]
    # B = Q^T Xc = Z^T with Z = Xc^T Q = Qz Rz, so B = Rz^T Qz^T and svd(B) = svd(Rz^T) with
    # the right factor rotated: U_hat and S come from the small (k+10)^2 factor (host LAPACK)
    _, Rz = _orth(xct(Q))
    Uh, s_np, _ = np.linalg.svd(Rz.t().cpu().numpy(), full_matrices=False)
    s = torch.from_numpy(s_np).to(dev)
    U = Q @ torch.from_numpy(Uh).to(dev)
    idx = U.abs().argmax(0)
    U = U * torch.sign(U[idx, torch.arange(U.shape[1], device=dev)])
    return (U[:, :k] * s[:k]).cpu().numpy()
