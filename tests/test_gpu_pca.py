"""GPU parity of the PCA front end (plagnn.pca.pca, HIP pg_csr_spmm_f64 products) against
the CPU restatement of scikit-learn 1.1.1's randomized PCA (oracle.pca_randomized) and the
reference's own pca() output (tests/golden/pca.npz).

Bars (float64): every output column within 1e-8 of its magnitude against the oracle (same
test matrix, same u-based signs; QR instead of LU normalisation keeps the same subspace up
to rounding) and, up to sign, against the golden fixture (scikit-learn 1.7.2 flips by V).
"""
import os

import numpy as np
import pytest
import torch
from scipy.sparse import coo_matrix, random as sprandom

pytestmark = pytest.mark.gpu
DEV = "cuda"
HERE = os.path.dirname(os.path.abspath(__file__))


def _cols_close(a, b, rtol):
    scale = np.abs(b).max(axis=0)
    return np.abs(a - b).max(axis=0) <= rtol * scale


def test_pca_matches_reference_golden_and_oracle(oracle_mod):
    from plagnn.pca import pca

    z = np.load(os.path.join(HERE, "golden", "pca.npz"))
    n, nc = int(z["n"]), int(z["nc"])
    m = coo_matrix((z["val"], (z["row"], z["col"])), shape=(n, n))
    got = pca(m, nc)
    ora = oracle_mod.pca_randomized(m, nc)
    assert np.all(_cols_close(got, ora, 1e-8))
    s = np.sign(np.sum(got * z["out"], axis=0))
    assert np.all(_cols_close(got * s, z["out"], 1e-8))
    idx = np.abs(got).argmax(axis=0)
    assert np.all(got[idx, np.arange(nc)] > 0)  # scikit-learn 1.1.1's u-based svd_flip


@pytest.mark.parametrize("n,nc,density,seed", [(3000, 60, 0.004, 1), (1200, 400, 0.01, 2)])
def test_pca_random_sparse(oracle_mod, n, nc, density, seed):
    """A general sparse matrix (not symmetric, negative values, empty rows / columns) and
    a case with n_iter = 4 (k >= 0.1 N) and k + 10 > 384 columns (four column chunks)."""
    from plagnn.pca import pca

    m = sprandom(n, n, density=density, random_state=seed, format="coo",
                 data_rvs=np.random.default_rng(seed).standard_normal)
    m = m.tocsr()
    m[:7] = 0  # empty rows
    m.eliminate_zeros()
    got = pca(m, nc)
    ora = oracle_mod.pca_randomized(m, nc)
    # near-degenerate trailing components can rotate with rounding: compare the well
    # separated leading ones per column, and the whole subspace by projection
    sv = np.linalg.norm(ora, axis=0)
    gap = np.minimum(np.abs(np.diff(np.r_[np.inf, sv])), np.abs(np.diff(np.r_[sv, 0.0]))) / sv[0]
    sep = gap > 1e-4
    assert sep[:5].all()
    assert np.all(_cols_close(got[:, sep], ora[:, sep], 1e-7))
    qa, _ = np.linalg.qr(got)
    qb, _ = np.linalg.qr(ora)
    assert np.linalg.norm(qa @ (qa.T @ qb) - qb) <= 1e-6 * np.sqrt(nc)
