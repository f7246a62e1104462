"""The oracle itself: known-answer tests for the DGL 0.8.2 semantics it restates, and the
golden vectors produced by the reference's own functions (tests/golden/gen_golden.py)."""
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_csc_is_stable_by_edge_id(oracle_mod):
    # dst 0 receives edges 3, 1, 0 (ids) -> listed in id order 0, 1, 3; self-loop (id E+v) last
    src = [5, 2, 9, 7, 1]
    dst = [0, 0, 1, 0, 1]
    g = oracle_mod.OracleGraph(src, dst, 10)
    assert list(g.indptr[:3]) == [0, 4, 7]
    assert list(g.indices[0:4]) == [5, 2, 7, 0]
    assert list(g.eids[0:4]) == [0, 1, 3, 5]
    assert list(g.indices[4:7]) == [9, 1, 1]


def test_triangle_pendant_max(oracle_mod):
    # triangle 0-1-2 + pendant 0-3, symmetric, self-loops appended
    r = [0, 1, 0, 2, 1, 2, 0, 3]
    c = [1, 0, 2, 0, 2, 1, 3, 0]
    g = oracle_mod.OracleGraph(r, c, 4)
    X = np.array([[1.0, 0.0], [3.0, -1.0], [2.0, 5.0], [0.5, 7.0]], np.float32)
    out, argx, _ = oracle_mod.spmm_max(g, X)
    # node 0 in-neighbours: 1, 2, 3 (edge order) then itself
    np.testing.assert_array_equal(out[0], [3.0, 7.0])
    np.testing.assert_array_equal(argx[0], [1, 3])
    np.testing.assert_array_equal(out[3], [1.0, 7.0])
    np.testing.assert_array_equal(argx[3], [0, 3])


def test_ties_first_in_edge_order_wins(oracle_mod):
    # all-zero messages: argmax = first in-edge (edge order), not the self-loop
    src = [3, 1, 2]
    dst = [0, 0, 0]
    g = oracle_mod.OracleGraph(src, dst, 4)
    out, argx, _ = oracle_mod.spmm_max(g, np.zeros((4, 3), np.float32))
    np.testing.assert_array_equal(out[0], 0.0)
    np.testing.assert_array_equal(argx[0], [3, 3, 3])
    # exact positive tie between nodes 1 and 2 -> node 1 (edge id 1 before 2)
    X = np.zeros((4, 1), np.float32)
    X[1] = X[2] = 4.0
    out, argx, _ = oracle_mod.spmm_max(g, X)
    assert out[0, 0] == 4.0 and argx[0, 0] == 1


def test_duplicate_self_loop_and_backward_accumulates(oracle_mod):
    # explicit self-loop 0->0 (PPI_inter diagonal) + DGL's appended loop: two entries
    src = [0, 1, 1]
    dst = [0, 0, 2]
    g = oracle_mod.OracleGraph(src, dst, 3)
    X = np.array([[2.0], [1.0], [0.0]], np.float32)
    out, argx, arge = oracle_mod.spmm_max(g, X)
    assert out[0, 0] == 2.0 and argx[0, 0] == 0 and arge[0, 0] == 0  # first of the two loops
    # node 1 is the argmax of nodes 1 and 2: its gradient accumulates both
    dZ = np.array([[1.0], [10.0], [100.0]], np.float32)
    dX = oracle_mod.spmm_max_bwd(g, argx, arge, dZ)
    np.testing.assert_array_equal(dX[:, 0], [1.0, 110.0, 0.0])


def test_inf_masked_to_zero_and_zero_in_degree(oracle_mod):
    g = oracle_mod.OracleGraph([0], [1], 3, self_loop=False)
    X = np.array([[-np.inf], [1.0], [2.0]], np.float32)
    out, _, _ = oracle_mod.spmm_max(g, X)
    assert out[1, 0] == 0.0  # max = -inf -> 0 (replace_inf_with_zero)
    assert out[0, 0] == 0.0 and out[2, 0] == 0.0  # no in-edges -> 0


def test_weighted_max_and_sum_mean(oracle_mod):
    src = [1, 2, 3]
    dst = [0, 0, 0]
    w = np.array([2.0, -1.0, 0.5], np.float32)
    g = oracle_mod.OracleGraph(src, dst, 4, edge_weight=w)
    X = np.array([[0.0], [1.0], [-3.0], [8.0]], np.float32)
    out, argx, _ = oracle_mod.spmm_max(g, X, use_weight=True)
    assert out[0, 0] == 4.0 and argx[0, 0] == 3  # max(2, 3, 4, 0 (self, w=1))
    s = oracle_mod.spmm_sum(g, X, use_weight=True)
    assert s[0, 0] == 2.0 + 3.0 + 4.0 + 0.0
    m = oracle_mod.spmm_sum(g, X, mean=True)
    assert m[0, 0] == pytest.approx((1.0 - 3.0 + 8.0 + 0.0) / 4)


def test_multi_loss_matches_reference_golden(oracle_mod):
    d = np.load(os.path.join(GOLD, "multi_loss.npz"))
    w = oracle_mod.weight_cal(d["loc"])
    np.testing.assert_array_equal(w, d["weight"])
    inp = torch.tensor(d["probs"], requires_grad=True)
    loss = oracle_mod.multi_loss(inp, torch.tensor(d["target"]), w)
    loss.backward()
    assert loss.item() == d["loss"]
    np.testing.assert_array_equal(inp.grad.numpy(), d["grad"])


def test_adam_torch110_matches_torch_adam(oracle_mod):
    torch.manual_seed(0)
    p0 = torch.randn(1000)
    p_ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([p_ref], lr=5e-3)
    p = p0.clone()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    for step in range(1, 6):
        g = torch.randn(1000)
        p_ref.grad = g.clone()
        opt.step()
        oracle_mod.adam_step_torch110([p], [g], [m], [v], step, 5e-3)
    torch.testing.assert_close(p, p_ref.detach(), rtol=1e-6, atol=1e-7)


def test_ecc_golden_present():
    d = np.load(os.path.join(GOLD, "ecc.npz"))
    e = d["tri_ecc"]
    assert e[0, 1] == 1.0 and e[1, 2] == 1.0 and e[0, 3] == 0.0


@pytest.mark.parametrize("case", ["tri", "rand30"])
def test_ecc_oracle_matches_reference_golden(oracle_mod, case):
    """The C restatement of code/data_preprocess.py:175-214 reproduces the reference's
    own output (fixture made by running the reference function) bit for bit."""
    from scipy.sparse import coo_matrix

    d = np.load(os.path.join(GOLD, "ecc.npz"))
    adj = d[f"{case}_adj"]
    r, c = np.nonzero(adj)
    m = coo_matrix((np.ones(len(r), np.int64), (r, c)), shape=adj.shape)
    np.testing.assert_array_equal(oracle_mod.edge_clustering_coefficients(m).toarray(), d[f"{case}_ecc"])


@pytest.mark.parametrize("alpha", [0.1, 0.3])
def test_eval_oracle_matches_reference_golden(oracle_mod, alpha):
    """protein_loc_correction / performances_record restatements (code/train.py:19-86)
    vs the reference's own outputs on the committed fixture."""
    d = np.load(os.path.join(GOLD, "eval.npz"))
    pred = oracle_mod.protein_loc_correction(torch.from_numpy(d["proba"]), alpha)
    np.testing.assert_array_equal(pred.numpy(), d[f"pred_{alpha}"])
    perf = np.array(oracle_mod.performances_record(torch.from_numpy(d["true"]), pred), np.float64)
    np.testing.assert_array_equal(perf, d[f"perf_{alpha}"])


# ---------------------------------------------------------------- §8f: topology perturbation
def _perturb_case(d, name):
    from scipy.sparse import coo_matrix

    n = d[f"{name}_expr_normal"].shape[0]
    ppi = coo_matrix((d[f"{name}_ppi_val"], (d[f"{name}_ppi_row"], d[f"{name}_ppi_col"])), shape=(n, n))
    out = coo_matrix((d[f"{name}_out_val"], (d[f"{name}_out_row"], d[f"{name}_out_col"])), shape=(n, n))
    return ppi, d[f"{name}_expr_normal"], d[f"{name}_expr_inter"], float(d[f"{name}_thr"]), out


@pytest.mark.parametrize("name", ["small", "mid"])
def test_perturb_numpy_oracle_matches_reference_golden(oracle_mod, name):
    d = np.load(os.path.join(GOLD, "perturb.npz"))
    ppi, en, ei, thr, ref = _perturb_case(d, name)
    pn, pi = oracle_mod.pcc_matrix(en), oracle_mod.pcc_matrix(ei)
    if d[f"{name}_pcc_normal"].size:
        np.testing.assert_array_equal(pn, d[f"{name}_pcc_normal"])
    got, (mean, std) = oracle_mod.modify_network_topology(ppi, pn, pi, thr)
    np.testing.assert_array_equal(got.row, ref.row)
    np.testing.assert_array_equal(got.col, ref.col)
    np.testing.assert_array_equal(got.data, ref.data)
    np.testing.assert_array_equal([mean, std], d[f"{name}_mean_std"])
    assert got.nnz != len(d[f"{name}_ppi_row"])  # the threshold fires in both fixtures


@pytest.mark.parametrize("name", ["small", "mid"])
def test_perturb_stream_oracle_matches_reference_golden(oracle_mod, name):
    d = np.load(os.path.join(GOLD, "perturb.npz"))
    ppi, en, ei, thr, ref = _perturb_case(d, name)
    ps = oracle_mod.PerturbStream(ppi, en, ei)
    mean, std, lo, hi = ps.stats(thr)
    # compensated sums vs numpy's pairwise sums: a few ulp apart
    np.testing.assert_allclose([mean, std], d[f"{name}_mean_std"], rtol=1e-13, atol=1e-16)
    r, c, v = ps.rows(lo, hi, 0, ps.n)
    np.testing.assert_array_equal(r, ref.row)
    np.testing.assert_array_equal(c, ref.col)
    np.testing.assert_array_equal(v, ref.data)


def _align_cols(a, g):
    """a's columns sign-matched to g's (scikit-learn 1.7.2 flips by V, 1.1.1 by U)."""
    s = np.sign(np.sum(a * g, axis=0))
    s[s == 0] = 1
    return a * s


def test_pca_oracle_matches_reference_golden(oracle_mod):
    """The randomized-PCA restatement (scikit-learn 1.1.1's algorithm) against the reference's
    own pca() (code/data_preprocess.py:475-487) on its own ECC matrix (tests/golden/pca.npz):
    every column within 1e-9 of its magnitude up to sign; the restatement's signs follow
    1.1.1's u-based svd_flip (largest |entry| of each column positive)."""
    import os

    from scipy.sparse import coo_matrix

    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "pca.npz"))
    n, nc = int(z["n"]), int(z["nc"])
    m = coo_matrix((z["val"], (z["row"], z["col"])), shape=(n, n))
    got = oracle_mod.pca_randomized(m, nc)
    gold = z["out"]
    assert got.shape == gold.shape == (n, nc)
    a = _align_cols(got, gold)
    scale = np.abs(gold).max(axis=0)
    assert np.all(np.abs(a - gold).max(axis=0) <= 1e-9 * scale)
    idx = np.abs(got).argmax(axis=0)
    assert np.all(got[idx, np.arange(nc)] > 0)


def test_parallel_oracle_step_equals_serial(oracle_mod):
    """The CPU baseline's form of the oracle (OpenMP rows forward, torch scatter_add_
    backward, as DGL's CPU backend runs them) computes the same step: the forward is a
    selection (bit-exact), the backward sums the same terms."""
    from conftest import random_graph

    src, dst = random_graph(300, 3000, seed=5, self_loop=False)
    dims = [20, 16, 12, 8, 6, 12]
    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.standard_normal((300, dims[0])).astype(np.float32))
    labels = torch.from_numpy((rng.random((300, 12)) < 0.3).astype(np.float32))
    w = np.linspace(0.5, 2.0, 12)
    ew = rng.random(len(src)).astype(np.float32)
    p = oracle_mod.init_params(dims, seed=4)
    for weight in (None, ew):
        og = oracle_mod.OracleGraph(src, dst, 300, edge_weight=weight)
        a = oracle_mod.train_step(og, x, labels, list(range(0, 300, 2)), w, p, use_weight=weight is not None)
        b = oracle_mod.train_step(og, x, labels, list(range(0, 300, 2)), w, p, use_weight=weight is not None,
                                  parallel=True)
        assert torch.equal(a[0], b[0])
        for k in a[2]:
            torch.testing.assert_close(a[2][k], b[2][k], rtol=1e-5, atol=1e-7)


def test_rowwise_loc_correction_equals_vectorised(oracle_mod):
    rng = np.random.default_rng(0)
    proba = torch.from_numpy(rng.random((500, 12)).astype(np.float32))
    for alpha in (0.1, 0.5):
        assert torch.equal(oracle_mod.protein_loc_correction(proba, alpha),
                           oracle_mod.protein_loc_correction(proba, alpha, rowwise=True))


def test_decision_alignment(oracle_mod):
    """spmm_max_align takes another computation's winner only when the two candidates lie
    within BAND_ULPS x 2^-24 of their running-error scale; _act takes another
    computation's sign only at pre-activations that small against their own scale. Both
    count the differing decisions outside the band as hard."""
    src = np.array([1, 2, 3], np.int64)
    dst = np.array([0, 0, 0], np.int64)
    og = oracle_mod.OracleGraph(src, dst, 4, self_loop=False)
    X = np.array([[0.0, 0.0], [1.0, 5.0], [1.0 - 1e-7, 4.0], [0.5, 5.0]], np.float32)
    S = np.abs(X).astype(np.float64)
    band = 64 * oracle_mod.U32  # 3.8e-6 of the candidates' scale
    out, ax, ae = oracle_mod.spmm_max(og, X)
    assert ax[0].tolist() == [1, 1]
    hint = np.full((4, 2), -1, np.int32)
    hint[0] = [1, 1]  # positions: edge 1->0 is 0, 2->0 is 1, 3->0 is 2
    n, hard, _ = oracle_mod.spmm_max_align(og, X, False, hint, S, band, out, ax, ae)
    assert (n, hard) == (1, 1) and ax[0].tolist() == [2, 1] and out[0, 0] == np.float32(1.0 - 1e-7)
    hint[0] = [2, 2]
    n, hard, _ = oracle_mod.spmm_max_align(og, X, False, hint, S, band, out, ax, ae)
    assert (n, hard) == (1, 1) and ax[0].tolist() == [2, 3]  # 0.5 is far from the max; the tie at 5.0 is taken
    # a candidate 1e-7 below a maximum of scale 1e-3 is NOT a rounding tie
    X2 = X.copy()
    X2[1, 0], X2[2, 0], X2[3, 0] = 1e-3, 1e-3 - 1e-7, 0.0
    out, ax, ae = oracle_mod.spmm_max(og, X2)
    hint[0] = [1, -1]
    n, hard, _ = oracle_mod.spmm_max_align(og, X2, False, hint, np.abs(X2).astype(np.float64), band, out, ax, ae)
    assert (n, hard) == (0, 1) and ax[0, 0] == 1
    pre = torch.tensor([1e-9, -1e-9, 1.0, -1.0])
    signs = {"s": torch.tensor([False, True, False, True])}
    y = oracle_mod._act(pre, 0.01, "s", signs, torch.ones(4, dtype=torch.float64))
    assert signs["_flips"] == 2 and signs["_hard_flips"] == 2
    torch.testing.assert_close(y, torch.tensor([1e-11, -1e-9, 1.0, -0.01]), rtol=1e-6, atol=0)
    signs = {"s": torch.tensor([False, True, True, False])}
    oracle_mod._act(pre, 0.01, "s", signs, torch.full((4,), 1e-6, dtype=torch.float64))  # 1e-9 is 0.017 ulp of 1e0,
    assert signs["_flips"] == 0 and signs["_hard_flips"] == 2                          # 16.7 k ulp of 1e-6
