"""CPU-side tests: the C-ABI library loads and exports every declared symbol, the host
graph builder matches the oracle's CSC, the CPU-device backend matches the oracle, and
the dgl shim exposes the API surface the reference uses."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, hub_graph, random_graph


def _declared_symbols():
    h = open(os.path.join(ROOT, "include", "plagnn.h")).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|size_t|const char\*)\s+(pg_[a-z0-9_]+)\(", h, re.M)))


def test_library_exports_every_declared_symbol():
    from plagnn import _lib

    L = _lib.lib()
    declared = _declared_symbols()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(L, name), name
    assert set(declared) == set(_lib.SIGNATURES), "ctypes signatures out of sync with header"
    assert L.pg_version() == 13


def test_error_reporting():
    from plagnn import _lib

    with pytest.raises(_lib.PlagnnError, match="out of range"):
        import plagnn

        plagnn.CSRGraph(np.array([0, 5]), np.array([1, 1]), 3)


@pytest.mark.parametrize("seed", [0, 1])
def test_csr_build_matches_oracle(oracle_mod, seed):
    import plagnn

    src, dst = random_graph(300, 2000, seed)
    g = plagnn.CSRGraph(src, dst, 300)
    og = oracle_mod.OracleGraph(src, dst, 300, self_loop=False)
    np.testing.assert_array_equal(g.fwd.ptr, og.indptr)
    np.testing.assert_array_equal(g.fwd.col, og.indices)
    np.testing.assert_array_equal(g.eid, og.eids)
    # transpose: rows = sources, destinations ascending, slots point back
    for u in range(0, 300, 37):
        t0, t1 = g.bwd.ptr[u], g.bwd.ptr[u + 1]
        dsts = g.bwd.col[t0:t1]
        assert np.all(np.diff(dsts) >= 0)
        assert np.all(g.fwd.col[g.bwd.eslot[t0:t1]] == u)


def test_schedule_covers_rows_longest_first():
    import plagnn

    src, dst = hub_graph(200, 1000)
    g = plagnn.CSRGraph(src, dst, 200, chunk=64)
    it = g.fwd.items.reshape(-1, 4)[: g.fwd.n_items]
    lens = it[:, 2] - it[:, 1]
    assert np.all(np.diff(lens) <= 0)
    cover = np.zeros(g.num_edges, np.int32)
    for r, k0, k1, _ in it:
        assert g.fwd.ptr[r] <= k0 <= k1 <= g.fwd.ptr[r + 1]
        cover[k0:k1] += 1
    assert np.all(cover == 1)
    assert g.fwd.n_merges >= 1 and g.fwd.max_deg > 1000
    # split rows: every row past the chunk once, with its slot run, longest first
    ms = g.fwd.merges.reshape(-1, 4)[: g.fwd.n_merges]
    deg = np.diff(g.fwd.ptr)
    assert sorted(ms[:, 0].tolist()) == np.flatnonzero(deg > 64).tolist()
    assert np.all(np.diff(ms[:, 2]) <= 0)
    assert np.all(ms[:, 2] == (deg[ms[:, 0]] + 63) // 64)


def test_pad2d_group_rejects_bad_parts():
    """pg_pad2d_group validates every part before launching anything (no GPU needed)."""
    import ctypes

    from plagnn import _lib

    L = _lib.lib()
    src = np.zeros((2, 3), np.float32)
    dst = np.zeros((4, 4), np.float32)
    good = dict(src=src.ctypes.data, lds=3, rows=2, cols=3, dst=dst.ctypes.data, ldd=4, drows=4, dcols=4)
    for bad in (dict(drows=-1, rows=0), dict(rows=5), dict(cols=5), dict(ldd=3), dict(lds=2), dict(dst=None)):
        part = _lib.PgPad2d(**{**good, **bad})
        assert L.pg_pad2d_group(ctypes.byref(part), 1, None) != 0, bad
    assert L.pg_pad2d_group(None, _lib.PG_PAD2D_MAX + 1, None) != 0
    assert L.pg_pad2d_group(None, 0, None) == 0  # nothing to do


@pytest.mark.parametrize("F", [1, 5, 64, 130])
@pytest.mark.parametrize("weighted", [False, True])
def test_cpu_backend_max_bitexact(oracle_mod, F, weighted):
    import plagnn
    from plagnn import ops

    src, dst = hub_graph(120, 400, seed=F)
    n = 120
    rng = np.random.default_rng(F)
    w = rng.standard_normal(len(src)).astype(np.float32) if weighted else None
    g = plagnn.CSRGraph(src, dst, n)
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False, edge_weight=w)
    X = rng.standard_normal((n, F)).astype(np.float32)
    X[rng.random((n, F)) < 0.3] = 0.0  # ties at zero, as after relu
    dg = g.on("cpu")
    ews = dg.edge_weight_slots(None if w is None else torch.from_numpy(w))
    out, argpos = ops.spmm_max(dg, torch.from_numpy(X), ews)
    ref, argx, arge = oracle_mod.spmm_max(og, X, use_weight=weighted)
    np.testing.assert_array_equal(out.numpy(), ref)
    np.testing.assert_array_equal(ops.argpos_to_src(dg, argpos).numpy(), argx)
    dZ = rng.standard_normal((n, F)).astype(np.float32)
    dX = ops.spmm_max_backward(dg, argpos, torch.from_numpy(dZ), ews)
    np.testing.assert_array_equal(dX.numpy(), oracle_mod.spmm_max_bwd(og, argx, arge, dZ, weighted))


def test_cpu_backend_sum_mean(oracle_mod):
    import plagnn
    from plagnn import ops

    src, dst = random_graph(80, 500, 3)
    g = plagnn.CSRGraph(src, dst, 80)
    og = oracle_mod.OracleGraph(src, dst, 80, self_loop=False)
    X = np.random.default_rng(3).standard_normal((80, 7)).astype(np.float32)
    dg = g.on("cpu")
    for mean in (False, True):
        out = ops.spmm_sum(dg, torch.from_numpy(X), mean=mean)
        np.testing.assert_array_equal(out.numpy(), oracle_mod.spmm_sum(og, X, mean=mean))
    # transposed with mean = backward of mean aggregation; check against autograd of a dense op
    A = np.zeros((80, 80), np.float64)
    for s, d in zip(src, dst):
        A[d, s] += 1
    deg = A.sum(1, keepdims=True)
    dZ = np.random.default_rng(4).standard_normal((80, 7))
    expect = (A / np.maximum(deg, 1)).T @ dZ
    got = ops.spmm_sum(dg, torch.from_numpy(dZ.astype(np.float32)), mean=True, transpose=True)
    np.testing.assert_allclose(got.numpy(), expect, rtol=1e-5, atol=1e-5)


def test_dgl_shim_surface_like_utils_create_graph():
    """The exact call sequence of code/utils.py:28-51 and train.py:145-146."""
    import dgl
    from scipy.sparse import coo_matrix

    n = 40
    rng = np.random.default_rng(0)
    r = rng.integers(0, n, 100)
    c = rng.integers(0, n, 100)
    ppi = coo_matrix((np.ones(100), (r, c)), shape=(n, n))
    g = dgl.graph((list(ppi.row), list(ppi.col)), num_nodes=n)
    g = dgl.add_self_loop(g)
    assert g.num_nodes() == n and g.num_edges() == 100 + n
    s, d = g.edges()
    assert torch.equal(s[100:], torch.arange(n)) and torch.equal(d[100:], torch.arange(n))
    loc = coo_matrix((np.ones(5), ([0, 1, 2, 3, 4], [0, 1, 2, 3, 4])), shape=(n, 12))
    g.nodes[list(range(n))].data["loc"] = torch.from_numpy(loc.toarray().astype(np.float32))
    feat = torch.tensor(np.hstack((rng.random((n, 3)), rng.random((n, 6)))), dtype=torch.float)
    g.nodes[list(range(n))].data["feat"] = feat
    assert g.ndata["feat"].shape == (n, 9) and g.ndata["loc"].shape == (n, 12)
    g2 = g.to("cpu")
    assert torch.equal(g2.ndata["feat"], feat)
    dgl.seed(70)


def test_update_all_builtins_match_oracle(oracle_mod):
    import dgl
    import dgl.function as fn

    src, dst = random_graph(60, 300, 5, self_loop=False)
    g = dgl.add_self_loop(dgl.graph((src, dst), num_nodes=60))
    og = oracle_mod.OracleGraph(src, dst, 60)
    X = np.random.default_rng(5).standard_normal((60, 4)).astype(np.float32)
    g.ndata["h"] = torch.from_numpy(X)
    g.update_all(fn.copy_u("h", "m"), fn.max("m", "neigh"))
    np.testing.assert_array_equal(g.ndata["neigh"].numpy(), oracle_mod.spmm_max(og, X)[0])
    g.update_all(fn.copy_u("h", "m"), fn.mean("m", "neigh"))
    np.testing.assert_array_equal(g.ndata["neigh"].numpy(), oracle_mod.spmm_sum(og, X, mean=True))


def test_gnn32_cpu_forward_backward_matches_oracle(oracle_mod):
    import dgl
    from plagnn.model import GNN32

    n = 90
    src, dst = random_graph(n, 600, 8, self_loop=False)
    g = dgl.add_self_loop(dgl.graph((src, dst), num_nodes=n))
    og = oracle_mod.OracleGraph(src, dst, n)
    torch.manual_seed(1)
    model = GNN32(13, 16, 12, 10, 8, 12)
    x = torch.randn(n, 13)
    labels = (torch.rand(n, 12) < 0.3).float()
    idx = list(range(0, n, 2))
    w = oracle_mod.weight_cal(labels.numpy().astype(np.float64))
    w[~np.isfinite(w)] = 1.0
    logits = model(g, x)
    loss = oracle_mod.multi_loss(logits[idx], labels[idx], w)
    loss.backward()
    p = {k: v.detach() for k, v in model.state_dict().items()}
    ref_logits, ref_loss, ref_grads = oracle_mod.train_step(og, x, labels, idx, w, p)
    torch.testing.assert_close(logits.detach(), ref_logits, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(loss.detach(), ref_loss, rtol=1e-5, atol=1e-6)
    for name, prm in model.named_parameters():
        torch.testing.assert_close(prm.grad, ref_grads[name], rtol=1e-4, atol=1e-5, msg=name)


def test_workload_generators():
    """cfg3's ±3 % perturbation and cfg4's synthetic intervention expression (host side)."""
    from plagnn import data, workload

    ds = data.make_dataset("s0", n=3000, seed=70)
    r, c = data.random_perturbation(ds, seed=1)
    assert np.all(r != c)
    key = np.sort(r * ds.n + c)
    assert np.array_equal(key, np.sort(c * ds.n + r)) and len(np.unique(key)) == len(key)
    old = set((ds.row.astype(np.int64) * ds.n + ds.col).tolist())
    changed = len(set(key.tolist()) ^ old) / len(old)
    assert 0.03 < changed < 0.09, changed
    for gse in data.GSE_THRESHOLDS:
        inter = data.intervention_expression(ds, gse)
        diff = np.nonzero(np.any(inter != ds.expr, axis=1))[0]
        assert len(diff) == 2 and np.all(ds.expr[diff].sum(1) > 0)
    assert workload.CFG4_VARIANTS[0] == "normal" and len(workload.CFG4_VARIANTS) == 4
