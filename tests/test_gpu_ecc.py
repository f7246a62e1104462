"""§8f rank 2: edge clustering coefficient on the GPU (pg_ecc) vs the reference's own
outputs (tests/golden/ecc.npz, made by running code/data_preprocess.py:175-214) and vs
the C oracle on power-law graphs with hubs. Bit-exact (integer counts, one f64 division)."""
import os

import numpy as np
import pytest
from scipy.sparse import coo_matrix

from conftest import ROOT

pytestmark = pytest.mark.gpu
GOLD = os.path.join(ROOT, "tests", "golden", "ecc.npz")


def _sym_powerlaw(n, m, seed):
    rng = np.random.default_rng(seed)
    w = rng.pareto(1.1, n) + 1.0
    p = w / w.sum()
    s = rng.choice(n, m, p=p)
    d = rng.choice(n, m, p=p)
    keep = s != d
    r = np.concatenate([s[keep], d[keep]])
    c = np.concatenate([d[keep], s[keep]])
    a = coo_matrix((np.ones(len(r), np.int64), (r, c)), shape=(n, n)).tocsr()
    a.data[:] = 1  # duplicates collapse to one edge, as in the PPI build
    return a.tocoo()


@pytest.mark.parametrize("case", ["tri", "rand30"])
def test_ecc_matches_reference_golden(case):
    from plagnn import ecc

    d = np.load(GOLD)
    adj = d[f"{case}_adj"]
    r, c = np.nonzero(adj)
    m = coo_matrix((np.ones(len(r), np.int64), (r, c)), shape=adj.shape)
    got = ecc.edge_clustering_coefficients(m).toarray()
    np.testing.assert_array_equal(got, d[f"{case}_ecc"])


@pytest.mark.parametrize("n,m,eps", [(500, 4000, 0.0), (3000, 60000, 0.5)])
def test_ecc_matches_oracle_powerlaw(oracle_mod, n, m, eps):
    from plagnn import ecc

    a = _sym_powerlaw(n, m, seed=n)
    ref = oracle_mod.edge_clustering_coefficients(a, epsilon=eps)
    got = ecc.edge_clustering_coefficients(a, epsilon=eps)
    np.testing.assert_array_equal(got.toarray(), ref.toarray())
    # same entry set (explicit zeros included), both directions
    assert got.nnz == ref.nnz
