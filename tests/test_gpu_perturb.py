"""§8f rank 4: topology perturbation on the GPU (pg_perturb_*) vs the reference's own
outputs (tests/golden/perturb.npz: construct_gcn_matrix + modify_network_topology run on
a synthetic GEO-style CSV, code/data_preprocess.py:128-172, 217-257), vs the dense numpy
restatement (np.corrcoef / np.mean / np.std verbatim) and, at the full PPI size, vs the
streaming C oracle. The output adjacency is bit-exact (integer entries, identical
order); diff's mean / std agree to 1e-13 relative (compensated vs numpy's pairwise sums)."""
import os

import numpy as np
import pytest
from scipy.sparse import coo_matrix

from conftest import ROOT

pytestmark = pytest.mark.gpu
GOLD = os.path.join(ROOT, "tests", "golden", "perturb.npz")


def _case(d, name):
    n = d[f"{name}_expr_normal"].shape[0]
    ppi = coo_matrix((d[f"{name}_ppi_val"], (d[f"{name}_ppi_row"], d[f"{name}_ppi_col"])), shape=(n, n))
    return ppi, d[f"{name}_expr_normal"], d[f"{name}_expr_inter"], float(d[f"{name}_thr"])


def _assert_same_coo(got, row, col, val):
    np.testing.assert_array_equal(got.row, row)
    np.testing.assert_array_equal(got.col, col)
    np.testing.assert_array_equal(got.data, val)
    assert got.data.dtype == np.int64


@pytest.mark.parametrize("name", ["small", "mid"])
def test_perturb_matches_reference_golden(name):
    from plagnn import perturb

    d = np.load(GOLD)
    ppi, en, ei, thr = _case(d, name)
    got, st = perturb.modify_network_topology_expr(ppi, en, ei, thr, return_stats=True)
    _assert_same_coo(got, d[f"{name}_out_row"], d[f"{name}_out_col"], d[f"{name}_out_val"])
    np.testing.assert_allclose([st.mean, st.std], d[f"{name}_mean_std"], rtol=1e-13, atol=1e-16)


def test_perturb_sd_matches_numpy_cov_diagonal():
    from plagnn import perturb

    rng = np.random.default_rng(3)
    x = rng.lognormal(1.0, 1.0, (5000, 3))
    x[rng.random(5000) < 0.3] = 0.0
    sd = perturb.pcc_sd(x)
    ref = np.sqrt(np.diag(np.cov(x[:400])))  # diag of the OpenBLAS product
    np.testing.assert_array_equal(sd[:400], ref)


def _synthetic(n, S, p_edge, seed, dup=False):
    rng = np.random.default_rng(seed)
    en = rng.lognormal(1.0, 1.0, (n, S))
    ei = en * rng.lognormal(0.0, 0.5, (n, S))
    en[rng.random(n) < 0.25] = 0.0  # zero rows: NaN correlations -> 0
    ei[rng.random(n) < 0.25] = 0.0
    ei[5] = ei[4]  # identical rows: correlation exactly 1 (clip path)
    m = int(p_edge * n * n / 2)
    r, c = rng.integers(0, n, m), rng.integers(0, n, m)
    keep = r != c
    r, c = r[keep], c[keep]
    rr, cc = np.concatenate([r, c]), np.concatenate([c, r])
    a = coo_matrix((np.ones(len(rr), np.int64), (rr, cc)), shape=(n, n)).tocsr()
    if not dup:
        a.data[:] = 1
    return a.tocoo(), en, ei


@pytest.mark.parametrize("n,S,thr,dup", [(1500, 3, 1.0, False), (777, 5, 0.8, True), (64, 2, 0.5, False)])
def test_perturb_matches_numpy_oracle(oracle_mod, n, S, thr, dup):
    from plagnn import perturb

    ppi, en, ei = _synthetic(n, S, 0.02, seed=n + S, dup=dup)
    ref, (mean, std) = oracle_mod.modify_network_topology(ppi, oracle_mod.pcc_matrix(en),
                                                          oracle_mod.pcc_matrix(ei), thr)
    got, st = perturb.modify_network_topology_expr(ppi, en, ei, thr, return_stats=True)
    np.testing.assert_allclose([st.mean, st.std], [mean, std], rtol=1e-13, atol=1e-16)
    _assert_same_coo(got, ref.row, ref.col, ref.data)
    assert st.removed > 0 and st.added > 0


def test_perturb_full_ppi_size_vs_stream_oracle(oracle_mod):
    """N = 24 041 (the PPI size): thresholds from the GPU agree with the streaming C
    oracle's over all 578 M pairs; rows sampled across the matrix are bit-exact."""
    from plagnn import perturb

    n = 24041
    ppi, en, ei = _synthetic(n, 3, 50.0 / n, seed=11)
    got, st = perturb.modify_network_topology_expr(ppi, en, ei, 2.2, return_stats=True)
    ps = oracle_mod.PerturbStream(ppi, en, ei)
    nn = float(n) * float(n)
    mean = ps.row_sum(False, 0.0, 0, n) / nn
    assert abs(st.mean - mean) <= 1e-13 * abs(mean) + 1e-16
    gcsr = got.tocsr()
    for r0 in (0, 7919, n - 40):
        r, c, v = ps.rows(st.lo_thr, st.hi_thr, r0, r0 + 40)
        sub = gcsr[r0:r0 + 40].tocoo()
        np.testing.assert_array_equal(sub.row + r0, r)
        np.testing.assert_array_equal(sub.col, c)
        np.testing.assert_array_equal(sub.data, v)
    assert st.removed > 0 and st.added > 0
