"""GPU parity of the HIP kernels, called through the C-ABI, against the oracle.

Bars: the max aggregation and its argmax are bit-exact (selection, integer positions);
the max backward is bit-exact on rows that are not split across work items (same
ascending-destination summation order as the oracle's sequential scatter_add_) and
within 1e-6 relative of it on split rows, which are bit-exact against the schedule's own
piecewise order (`_piecewise_max_bwd`); sums / GEMMs within the fp32 tolerances stated per
test.
"""
import numpy as np
import pytest
import torch

from conftest import hub_graph, random_graph

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _graph(src, dst, n, chunk=256, bwd_trans=None):
    import plagnn

    return plagnn.CSRGraph(src, dst, n, chunk=chunk, bwd_trans=bwd_trans)


@pytest.mark.parametrize("F", [1, 3, 63, 64, 65, 128, 256, 300, 400, 503, 504, 512, 1100])
def test_spmm_max_fwd_bitexact(oracle_mod, F):
    from plagnn import ops

    n = 500
    src, dst = hub_graph(n, 1500, seed=F)  # one in-hub (split rows) + one out-hub
    g = _graph(src, dst, n)
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False)
    rng = np.random.default_rng(F)
    X = rng.standard_normal((n, F)).astype(np.float32)
    X[rng.random((n, F)) < 0.4] = 0.0  # ties at zero (post-relu)
    X[7] = X[11]  # exact positive ties between nodes
    dg = g.on(DEV)
    out, argpos = ops.spmm_max(dg, torch.from_numpy(X).to(DEV))
    ref, argx, arge = oracle_mod.spmm_max(og, X)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(ops.argpos_to_src(dg, argpos).cpu().numpy(), argx)


@pytest.mark.parametrize("F", [64, 65, 256])
def test_spmm_max_fwd_special_values(oracle_mod, F):
    """-inf / +inf / NaN entries: strict > never selects NaN or -inf, and a +-inf result is
    stored as 0 (DGL replace_inf_with_zero). A feature with no winner (all inputs -inf or
    NaN) records "none" (-1 from argpos_to_src) where DGL leaves argX at its initial 0;
    unreachable on the reference path (self-loops and relu outputs >= 0)."""
    from plagnn import ops

    n = 300
    src, dst = hub_graph(n, 900, seed=7 + F)
    g = _graph(src, dst, n)
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False)
    rng = np.random.default_rng(F)
    X = rng.standard_normal((n, F)).astype(np.float32)
    r = rng.random((n, F))
    X[r < 0.1] = -np.inf
    X[(r >= 0.1) & (r < 0.15)] = np.nan
    X[(r >= 0.15) & (r < 0.17)] = np.inf
    X[:, 0] = -np.inf  # a column no row can win
    dg = g.on(DEV)
    out, argpos = ops.spmm_max(dg, torch.from_numpy(X).to(DEV))
    ref, argx, _ = oracle_mod.spmm_max(og, X)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    got = ops.argpos_to_src(dg, argpos).cpu().numpy()
    won = got >= 0
    np.testing.assert_array_equal(got[won], argx[won])
    assert np.all(argx[~won] == 0) and np.all(ref[~won] == 0)
    assert np.all(~won[:, 0]) and won.mean() > 0.5


@pytest.mark.parametrize("F", [256, 512, 1100])
@pytest.mark.parametrize("weighted", [False, True])
def test_spmm_max_fwd_ties_across_split_rows(oracle_mod, F, weighted):
    """Few distinct values, so most maxima are ties, on a graph whose hub rows are taken
    whole by one workgroup per slice (F = 256 / 512: the sliced kernel, runs combined in
    order) or split into chunks and merged (F = 1100: the whole-row kernel): the earliest
    maximal edge must win everywhere, as in one sequential pass."""
    from plagnn import ops

    n = 600
    src, dst = hub_graph(n, 3000, seed=F)
    rng = np.random.default_rng(F + 1)
    w = rng.choice(np.array([0.5, 1.0, 2.0], np.float32), len(src)) if weighted else None
    g = _graph(src, dst, n)
    assert g.fwd.n_merges >= 1
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False, edge_weight=w)
    X = rng.integers(0, 4, (n, F)).astype(np.float32)
    dg = g.on(DEV)
    ews = dg.edge_weight_slots(None if w is None else torch.from_numpy(w))
    out, argpos = ops.spmm_max(dg, torch.from_numpy(X).to(DEV), ews)
    ref, argx, _ = oracle_mod.spmm_max(og, X, use_weight=weighted)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    got = ops.argpos_to_src(dg, argpos).cpu().numpy()
    won = got >= 0
    np.testing.assert_array_equal(got[won], argx[won])
    assert np.all(ref[~won] == 0)


@pytest.mark.parametrize("F", [300, 1100])
@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("chunk", [4, 64])
def test_spmm_max_fwd_whole_row_split_rows_race(oracle_mod, F, weighted, chunk):
    """The whole-row forward (widths whose slices do not share out over the XCDs) combines
    split rows inside the launch: with chunk = 4 almost every row is cut into pieces that
    race for the last ticket. Bit-exact maxima and argmax against the oracle (ties at zero and
    few distinct values: the earliest maximal edge wins), twice in a row (tickets restart)."""
    from plagnn import ops

    n = 700
    src, dst = hub_graph(n, 2000, seed=F + chunk)
    rng = np.random.default_rng(F + 7)
    w = rng.choice(np.array([0.5, 1.0, 2.0], np.float32), len(src)) if weighted else None
    g = _graph(src, dst, n, chunk=chunk)
    assert g.fwd.n_merges >= (500 if chunk == 4 else 1)
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False, edge_weight=w)
    X = rng.integers(0, 4, (n, F)).astype(np.float32)
    X[rng.random((n, F)) < 0.3] = 0.0
    dg = g.on(DEV)
    ews = dg.edge_weight_slots(None if w is None else torch.from_numpy(w))
    Xd = torch.from_numpy(X).to(DEV)
    out, argpos = ops.spmm_max(dg, Xd, ews)
    out2, argpos2 = ops.spmm_max(dg, Xd, ews)
    torch.cuda.synchronize()
    assert torch.equal(out, out2) and torch.equal(argpos, argpos2)
    ref, argx, _ = oracle_mod.spmm_max(og, X, use_weight=weighted)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    got = ops.argpos_to_src(dg, argpos).cpu().numpy()
    won = got >= 0
    np.testing.assert_array_equal(got[won], argx[won])
    assert np.all(ref[~won] == 0)


@pytest.mark.parametrize("F", [4, 65, 256, 503])
@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("trans", [False, True])
def test_spmm_max_bwd(oracle_mod, F, weighted, trans):
    """trans: list descriptors at the transposed indices (the default on large graphs)."""
    from plagnn import ops

    n = 400
    src, dst = hub_graph(n, 1200, seed=F + 1)
    rng = np.random.default_rng(F)
    w = rng.uniform(-1, 2, len(src)).astype(np.float32) if weighted else None
    g = _graph(src, dst, n, bwd_trans=trans)
    assert g.bwd_trans == trans
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False, edge_weight=w)
    X = rng.standard_normal((n, F)).astype(np.float32)
    X[rng.random((n, F)) < 0.4] = 0.0
    dZ = rng.standard_normal((n, F)).astype(np.float32)
    dg = g.on(DEV)
    ews = dg.edge_weight_slots(None if w is None else torch.from_numpy(w))
    out, argpos = ops.spmm_max(dg, torch.from_numpy(X).to(DEV), ews)
    ref, argx, arge = oracle_mod.spmm_max(og, X, use_weight=weighted)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    dX_ref = oracle_mod.spmm_max_bwd(og, argx, arge, dZ, use_weight=weighted)
    dX = ops.spmm_max_backward(dg, argpos, torch.from_numpy(dZ).to(DEV), ews).cpu().numpy()
    split_rows = set(g.bwd.merges.reshape(-1, 4)[: g.bwd.n_merges, 0].tolist())
    exact = np.array([u not in split_rows for u in range(n)])
    np.testing.assert_array_equal(dX[exact], dX_ref[exact])
    # split rows: a different summation grouping, bounded by the error scale sum |terms|
    mag = np.abs(oracle_mod.spmm_max_bwd(og, argx, arge, np.abs(dZ), use_weight=False))
    if weighted:
        mag = mag * np.abs(w).max()
    assert np.all(np.abs(dX - dX_ref) <= 1e-5 * mag + 1e-6)
    # fused relu' mask
    mask = torch.from_numpy(X).to(DEV)
    dXm = ops.spmm_max_backward(dg, argpos, torch.from_numpy(dZ).to(DEV), ews, mask=mask).cpu().numpy()
    np.testing.assert_array_equal(dXm, np.where(X > 0, dX, 0.0))
    # DGL scatter form (atomics: the fp32 summation order varies run to run, as in DGL)
    dXs = ops.spmm_max_backward_scatter(dg, argpos, torch.from_numpy(dZ).to(DEV), ews).cpu().numpy()
    np.testing.assert_allclose(dXs, dX_ref, rtol=1e-4, atol=1e-4)


def _piecewise_max_bwd(g, argpos, dZ, ew_slots):
    """dX of the max backward exactly as its schedule sums it: every out-CSR row longer than
    the schedule's chunk is cut into pieces of `chunk` edges, each piece summed in
    ascending destination order in f32 from +0, and the pieces' sums added in piece order
    from +0 (sum_merge_kernel's order, and the in-pull combine's); a shorter row is one
    piece. The contributions are the pack's records: w * dZ[v, f] (f32 product) where the
    argmax position of (v, f) is the edge's in-CSR position."""
    fptr, bptr, bcol, bslot, c = g.fwd.ptr, g.bwd.ptr, g.bwd.col, g.bwd.eslot, g.bwd.chunk
    n, F = dZ.shape
    ap = argpos.astype(np.int64)
    if argpos.dtype == np.int16:  # u16 records ("none" = 0xFFFF matches no position)
        ap &= 0xFFFF
    dX = np.zeros((n, F), np.float32)
    for u in range(len(bptr) - 1):
        b, e = int(bptr[u]), int(bptr[u + 1])
        pieces = [(b, e)] if e - b <= c else [(k, min(e, k + c)) for k in range(b, e, c)]
        tot = np.zeros(F, np.float32)
        for k0, k1 in pieces:
            acc = np.zeros(F, np.float32)
            for t in range(k0, k1):
                v, s = int(bcol[t]), int(bslot[t])
                hit = ap[v] == s - int(fptr[v])
                val = dZ[v] if ew_slots is None else np.float32(ew_slots[s]) * dZ[v]
                acc[hit] += val[hit]
            tot = acc if len(pieces) == 1 else tot + acc
        dX[u] = tot
    return dX


@pytest.mark.parametrize("F", [4, 64, 256, 503, 504])
@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("chunk_bwd,trans", [(4, False), (4, True), (64, False), (512, True)])
def test_spmm_max_bwd_split_rows_bitexact(oracle_mod, F, weighted, chunk_bwd, trans):
    """Every row bit-exact, split rows included, against the schedule's own summation order
    (`_piecewise_max_bwd`). chunk_bwd = 4 splits almost every source row, so thousands of
    pieces race for the in-pull combine's tickets (F % 4 == 0; F = 503 takes the separate
    merge launch); two calls in a row must agree (the tickets restart at zero every call)."""
    import plagnn
    from plagnn import ops

    n = 700
    src, dst = hub_graph(n, 1500, seed=F + chunk_bwd)
    rng = np.random.default_rng(F + 3)
    w = rng.uniform(-1, 2, len(src)).astype(np.float32) if weighted else None
    g = plagnn.CSRGraph(src, dst, n, chunk=256, chunk_bwd=chunk_bwd, bwd_trans=trans)
    assert g.bwd.n_merges >= (300 if chunk_bwd == 4 else 1)
    X = rng.standard_normal((n, F)).astype(np.float32)
    X[rng.random((n, F)) < 0.4] = 0.0
    dZ = rng.standard_normal((n, F)).astype(np.float32)
    dg = g.on(DEV)
    ews = dg.edge_weight_slots(None if w is None else torch.from_numpy(w))
    out, argpos = ops.spmm_max(dg, torch.from_numpy(X).to(DEV), ews)
    dZd = torch.from_numpy(dZ).to(DEV)
    dX = ops.spmm_max_backward(dg, argpos, dZd, ews)
    dX2 = ops.spmm_max_backward(dg, argpos, dZd, ews)
    torch.cuda.synchronize()
    assert torch.equal(dX, dX2)
    ref = _piecewise_max_bwd(g, argpos.cpu().numpy(), dZ, None if ews is None else ews.cpu().numpy())
    np.testing.assert_array_equal(dX.cpu().numpy(), ref)
    # the fused relu' mask on the combined rows
    dXm = ops.spmm_max_backward(dg, argpos, dZd, ews, mask=torch.from_numpy(X).to(DEV)).cpu().numpy()
    np.testing.assert_array_equal(dXm, np.where(X > 0, ref, 0.0))


@pytest.mark.parametrize("F", [64, 256, 504])
@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("chunk_bwd", [4, 64])
def test_spmm_max_bwd_bf16_split_rows_bitexact(F, weighted, chunk_bwd):
    """bf16 storage (cfg5's records: 4-B {bf16 dout, f} unweighted, 8-B {w * dout, f}
    weighted): every row bit-exact against the schedule's piecewise f32 sums of the bf16
    upstream gradient, rounded once to bf16 at the end."""
    import plagnn
    from plagnn import ops

    n = 700
    src, dst = hub_graph(n, 1500, seed=F + chunk_bwd + 1)
    rng = np.random.default_rng(F + 11)
    w = rng.uniform(-1, 2, len(src)).astype(np.float32) if weighted else None
    g = plagnn.CSRGraph(src, dst, n, chunk=256, chunk_bwd=chunk_bwd)
    X = rng.standard_normal((n, F)).astype(np.float32)
    X[rng.random((n, F)) < 0.4] = 0.0
    Xb = torch.from_numpy(X).to(DEV).to(torch.bfloat16)
    dZb = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(DEV).to(torch.bfloat16)
    dg = g.on(DEV)
    ews = dg.edge_weight_slots(None if w is None else torch.from_numpy(w))
    out, argpos = ops.spmm_max(dg, Xb, ews)
    dX = ops.spmm_max_backward(dg, argpos, dZb, ews)
    dX2 = ops.spmm_max_backward(dg, argpos, dZb, ews)
    torch.cuda.synchronize()
    assert dX.dtype == torch.bfloat16 and torch.equal(dX, dX2)
    ref = _piecewise_max_bwd(g, argpos.cpu().numpy(), dZb.float().cpu().numpy(),
                             None if ews is None else ews.cpu().numpy())
    np.testing.assert_array_equal(dX.float().cpu().numpy(),
                                  torch.from_numpy(ref).to(torch.bfloat16).float().numpy())


def test_spmm_max_int32_positions(oracle_mod):
    """A row of >= 65535 entries forces int32 argmax positions."""
    from plagnn import _lib, ops

    n = 70
    deg = 70000
    rng = np.random.default_rng(0)
    src = np.concatenate([rng.integers(0, n, deg), np.arange(n)]).astype(np.int64)
    dst = np.concatenate([np.zeros(deg, np.int64), np.arange(n)])
    g = _graph(src, dst, n)
    assert g.arg_kind == _lib.PG_ARG_I32
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False)
    X = rng.standard_normal((n, 8)).astype(np.float32)
    dg = g.on(DEV)
    out, argpos = ops.spmm_max(dg, torch.from_numpy(X).to(DEV))
    ref, argx, arge = oracle_mod.spmm_max(og, X)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(ops.argpos_to_src(dg, argpos).cpu().numpy(), argx)


def test_spmm_empty_rows_and_edges():
    from plagnn import ops

    n = 10
    src = np.array([1, 2], np.int64)
    dst = np.array([0, 0], np.int64)
    g = _graph(src, dst, n)  # rows 1..9 have no in-edges
    dg = g.on(DEV)
    X = torch.arange(n * 4, dtype=torch.float32, device=DEV).reshape(n, 4)
    out, argpos = ops.spmm_max(dg, X)
    o = out.cpu()
    assert torch.equal(o[0], X[2].cpu()) and torch.all(o[1:] == 0)
    assert torch.all(ops.argpos_to_src(dg, argpos)[1:] == -1)
    dX = ops.spmm_max_backward(dg, argpos, torch.ones(n, 4, device=DEV)).cpu()
    assert torch.equal(dX[2], torch.ones(4)) and dX[1].sum() == 0 and dX[0].sum() == 0


@pytest.mark.parametrize("trans", [False, True])
@pytest.mark.parametrize("dead", [False, True])
@pytest.mark.parametrize("F", [4, 256])
def test_spmm_max_bwd_sources_without_out_edges(oracle_mod, F, dead, trans):
    """The highest-numbered nodes send no edges (their transposed rows are empty at the end
    of the entry range), and a graph with no edges at all: every dx row is still written
    (zeros for the empty ones), with and without dead-none records."""
    from plagnn import ops

    n, n_src = 300, 240
    rng = np.random.default_rng(F + dead)
    src = rng.integers(0, n_src, 2000).astype(np.int64)
    dst = rng.integers(0, n, 2000).astype(np.int64)
    g = _graph(src, dst, n, bwd_trans=trans)
    assert np.all(g.out_degrees()[n_src:] == 0) and np.any(g.in_degrees()[n_src:] > 0)
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False)
    X = np.maximum(rng.standard_normal((n, F)), 0).astype(np.float32)
    dZ = rng.standard_normal((n, F)).astype(np.float32)
    dg = g.on(DEV)
    Xd = torch.from_numpy(X).to(DEV)
    _, argpos = ops.spmm_max(dg, Xd, dead_none=dead)
    _, argx, arge = oracle_mod.spmm_max(og, X)
    ref = np.where(X > 0, oracle_mod.spmm_max_bwd(og, argx, arge, dZ), 0.0)
    dx = torch.full((n, F), float("nan"), device=DEV)
    ops.spmm_max_backward(dg, argpos, torch.from_numpy(dZ).to(DEV), mask=Xd, dx=dx, dead_none=dead)
    np.testing.assert_array_equal(dx.cpu().numpy(), ref)
    assert np.all(dx.cpu().numpy()[n_src:] == 0)
    # no edges at all
    e = np.zeros(0, np.int64)
    g0 = _graph(e, e, 7, bwd_trans=trans)
    dg0 = g0.on(DEV)
    X0 = torch.rand(7, F, device=DEV)
    out0, arg0 = ops.spmm_max(dg0, X0, dead_none=dead)
    assert torch.all(out0 == 0)
    dx0 = torch.full((7, F), float("nan"), device=DEV)
    ops.spmm_max_backward(dg0, arg0, torch.rand(7, F, device=DEV), mask=X0, dx=dx0, dead_none=dead)
    assert torch.all(dx0 == 0)


@pytest.mark.parametrize("trans", [False, True])
@pytest.mark.parametrize("F", [65, 256])
def test_spmm_max_bwd_hub_past_lds_histogram(oracle_mod, F, trans):
    """A destination with 6 000 in-edges (u16 records; past the 4 096-entry LDS histogram of
    the count and place passes, whose list counters are then global integer atomics) and a
    source with 6 000 out-edges: bit-exact on unsplit rows."""
    from plagnn import ops

    n = 3000
    src, dst = hub_graph(n, 6000, seed=F)
    g = _graph(src, dst, n, bwd_trans=trans)
    assert g.in_degrees().max() > 4096 and g.arg_kind == 16
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False)
    rng = np.random.default_rng(F)
    X = np.maximum(rng.standard_normal((n, F)), 0).astype(np.float32)
    dZ = rng.standard_normal((n, F)).astype(np.float32)
    dg = g.on(DEV)
    Xd = torch.from_numpy(X).to(DEV)
    _, argx, arge = oracle_mod.spmm_max(og, X)
    dX_ref = oracle_mod.spmm_max_bwd(og, argx, arge, dZ)
    split_rows = set(g.bwd.merges.reshape(-1, 4)[: g.bwd.n_merges, 0].tolist())
    exact = np.array([u not in split_rows for u in range(n)])
    mag = np.abs(oracle_mod.spmm_max_bwd(og, argx, arge, np.abs(dZ)))
    for dead in (False, True):
        _, argpos = ops.spmm_max(dg, Xd, dead_none=dead)
        dX = ops.spmm_max_backward(dg, argpos, torch.from_numpy(dZ).to(DEV), mask=Xd,
                                   dead_none=dead).cpu().numpy()
        ref = np.where(X > 0, dX_ref, 0.0)
        np.testing.assert_array_equal(dX[exact], ref[exact])
        assert np.all(np.abs(dX - ref) <= 1e-5 * mag + 1e-6)


@pytest.mark.parametrize("F", [128, 512])
@pytest.mark.parametrize("dead", [False, True])
def test_spmm_max_bwd_wide_items_split_rows(oracle_mod, F, dead):
    """The large-graph backward schedule (graph.default_chunk_bwd above 65 536 nodes: 512
    out-edges per item) on a graph small enough for the oracle: sources with 700 / 1 500 /
    3 000 out-edges are split into 2 / 3 / 6 items whose partials go through sum_merge;
    bit-exact on unsplit rows, split rows within the summation-order bound."""
    import plagnn
    from plagnn import ops

    n = 2500
    rng = np.random.default_rng(F + dead)
    srcs, dsts = [rng.integers(0, n, 8 * n)], [rng.integers(0, n, 8 * n)]
    for u, d in ((3, 700), (5, 1500), (9, 3000)):
        srcs.append(np.full(d, u))
        dsts.append(rng.integers(0, n, d))
    src = np.concatenate(srcs + [np.arange(n)]).astype(np.int64)
    dst = np.concatenate(dsts + [np.arange(n)]).astype(np.int64)
    g = plagnn.CSRGraph(src, dst, n, chunk=256, chunk_bwd=512, bwd_trans=dead)  # both placements
    assert g.bwd.chunk == 512 and g.bwd.n_merges >= 3
    split_rows = set(g.bwd.merges.reshape(-1, 4)[: g.bwd.n_merges, 0].tolist())
    assert {3, 5, 9} <= split_rows
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False)
    X = np.maximum(rng.standard_normal((n, F)), 0).astype(np.float32)
    dZ = rng.standard_normal((n, F)).astype(np.float32)
    dg = g.on(DEV)
    Xd = torch.from_numpy(X).to(DEV)
    _, argx, arge = oracle_mod.spmm_max(og, X)
    ref = np.where(X > 0, oracle_mod.spmm_max_bwd(og, argx, arge, dZ), 0.0)
    mag = np.abs(oracle_mod.spmm_max_bwd(og, argx, arge, np.abs(dZ)))
    _, argpos = ops.spmm_max(dg, Xd, dead_none=dead)
    dX = ops.spmm_max_backward(dg, argpos, torch.from_numpy(dZ).to(DEV), mask=Xd, dead_none=dead).cpu().numpy()
    exact = np.array([u not in split_rows for u in range(n)])
    np.testing.assert_array_equal(dX[exact], ref[exact])
    assert np.all(np.abs(dX - ref) <= 1e-5 * mag + 1e-6)
    assert np.abs(dX[[3, 5, 9]]).sum() > 0


@pytest.mark.parametrize("mean", [False, True])
@pytest.mark.parametrize("weighted", [False, True])
def test_spmm_sum_fwd_bwd(oracle_mod, mean, weighted):
    from plagnn import ops

    n, F = 300, 70
    src, dst = hub_graph(n, 800, seed=3)
    rng = np.random.default_rng(2)
    w = rng.uniform(0, 1, len(src)).astype(np.float32) if weighted else None
    g = _graph(src, dst, n)
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False, edge_weight=w)
    X = rng.standard_normal((n, F)).astype(np.float32)
    dg = g.on(DEV)
    ews = dg.edge_weight_slots(None if w is None else torch.from_numpy(w))
    Xd = torch.from_numpy(X).to(DEV).requires_grad_(True)
    out = ops.SumAggregate.apply(Xd, dg, ews, mean)
    ref = oracle_mod.spmm_sum(og, X, mean=mean, use_weight=weighted)
    # hub rows are summed in 256-entry partials (fp32 reassociation)
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref, rtol=1e-4, atol=1e-4)
    # backward against the dense adjacency (float64)
    A = np.zeros((n, n))
    for k, (s, d) in enumerate(zip(src, dst)):
        A[d, s] += 1.0 if w is None else w[k]
    if mean:
        A = A / np.maximum(np.bincount(dst, minlength=n), 1)[:, None]
    dZ = rng.standard_normal((n, F)).astype(np.float32)
    out.backward(torch.from_numpy(dZ).to(DEV))
    np.testing.assert_allclose(Xd.grad.cpu().numpy(), A.T @ dZ, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("shape", [(300, 200, 100), (1000, 503, 503), (37, 12, 2000), (256, 504, 24041)])
def test_gemm_f32(ta, tb, shape):
    from plagnn import ops

    M, N, K = shape
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((N, K) if tb else (K, N), generator=g)
    ref = (A.double().t() if ta else A.double()) @ (B.double().t() if tb else B.double())
    C = ops.gemm(A.to(DEV), B.to(DEV), transa=ta, transb=tb).cpu().double()
    tol = 2e-6 * (K ** 0.5) * 4
    assert (C - ref).abs().max().item() <= tol * max(1.0, ref.abs().max().item()), (C - ref).abs().max()


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(20004, 508, 1000), (20004, 252, 500)], ids=["x3_128x128", "x3_128x64"])
def test_gemm_f32_x3_tiles(ta, tb, M, N, K):
    """The unsplit 128 x 128 and 128 x 64 three-piece tiles (csrc/gemm.hip pick_tile_x3:
    >= 512 tiles of 128 x 128, else >= 512 of 128 x 64) in every transpose combination, on
    ragged extents: M and N not multiples of the tile, K not a multiple of the 16-k step.
    Error bound per output: 1e-6 of sum_k |a b| (the f32 level, as
    test_gemm_f32_is_f32_accurate)."""
    from plagnn import ops

    g = torch.Generator().manual_seed(M + 3 * N + K + 7 * ta + 11 * tb)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((N, K) if tb else (K, N), generator=g)
    a64 = A.double().t() if ta else A.double()
    b64 = B.double().t() if tb else B.double()
    C = ops.gemm(A.to(DEV), B.to(DEV), transa=ta, transb=tb).cpu().double()
    err = ((C - a64 @ b64).abs() / (a64.abs() @ b64.abs())).max().item()
    assert err <= 1e-6, err


def test_gemm_f32_non_finite_contract():
    """include/plagnn.h (pg_gemm_f32): the three-piece path takes finite operands with
    |x| < 3.39e38; an Inf operand, or a finite one that rounds to Inf in bf16, gives NaN in
    the outputs it feeds, and leaves every other output exact to the f32 level."""
    from plagnn import ops

    M, N, K = 3000, 504, 504
    g = torch.Generator().manual_seed(5)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g)
    A[7, 3] = float("inf")
    A[11, 100] = 3.4e38  # rounds to Inf in bf16
    C = ops.gemm(A.to(DEV), B.to(DEV), transa=False, transb=True).cpu().double()
    assert torch.isnan(C[7]).all() and torch.isnan(C[11]).all()
    ok = torch.ones(M, dtype=torch.bool)
    ok[[7, 11]] = False
    a64, b64 = A[ok].double(), B.double().t()
    err = ((C[ok] - a64 @ b64).abs() / (a64.abs() @ b64.abs())).max().item()
    assert err <= 1e-6, err


@pytest.mark.parametrize("ta,tb,M,N,K", [(False, True, 3000, 504, 504), (False, False, 3000, 512, 256),
                                         (True, False, 256, 1008, 24041), (True, True, 136, 200, 1000)])
def test_gemm_f32_is_f32_accurate(ta, tb, M, N, K):
    """The f32 GEMM (three-piece bf16 products on the aligned path, gemm_x3.hip; the f32
    MFMA chain elsewhere) has f32 accuracy: the error of every output, relative to the sum
    of |a b| over its products, stays at the float32 level (measured 1.5e-8 .. 4.8e-7; a
    two-piece split, 2^-17 per product, would be ~1e-6 .. 8e-6)."""
    from plagnn import ops

    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((N, K) if tb else (K, N), generator=g)
    a64 = A.double().t() if ta else A.double()
    b64 = B.double().t() if tb else B.double()
    ref = a64 @ b64
    scale = a64.abs() @ b64.abs()
    C = ops.gemm(A.to(DEV), B.to(DEV), transa=ta, transb=tb).cpu().double()
    err = (C - ref).abs()
    assert float((err / scale).max()) <= 1e-6
    assert float(err.norm() / ref.norm()) <= 2e-6


def test_gemm_epilogue_and_beta():
    from plagnn import _lib, ops

    torch.manual_seed(0)
    A = torch.randn(200, 64)
    B = torch.randn(48, 64)
    bias = torch.randn(48)
    C0 = torch.randn(200, 48)
    Cd = C0.to(DEV)
    ops.gemm(A.to(DEV), B.to(DEV), transb=True, out=Cd, beta=1.0, bias=bias.to(DEV),
             act=_lib.PG_ACT_LEAKY)
    ref = torch.nn.functional.leaky_relu(A.double() @ B.double().t() + C0.double() + bias.double())
    torch.testing.assert_close(Cd.cpu().double(), ref, rtol=1e-5, atol=1e-5)
    # strided (padded) output view, relu
    buf = torch.zeros(200, 52, device=DEV)
    ops.gemm(A.to(DEV), B.to(DEV), transb=True, out=buf[:, :48], bias=bias.to(DEV), act=_lib.PG_ACT_RELU)
    torch.testing.assert_close(buf[:, :48].cpu().double(), torch.relu(A.double() @ B.double().t() + bias.double()),
                               rtol=1e-5, atol=1e-5)
    assert torch.all(buf[:, 48:] == 0)


def test_col_sum_act_bwd():
    from plagnn import _lib, ops

    torch.manual_seed(0)
    x = torch.randn(24041, 100)
    s = ops.col_sum(x.to(DEV)).cpu()
    torch.testing.assert_close(s.double(), x.double().sum(0), rtol=1e-5, atol=1e-3)
    y = torch.randn(300, 40)
    dy = torch.randn(300, 40)
    yd, dyd = y.to(DEV), dy.to(DEV)
    _lib.call("pg_act_bwd", dyd.data_ptr(), 40, yd.data_ptr(), 40, 300, 40, _lib.PG_ACT_LEAKY, 0.01,
              _lib.stream_handle(yd.device))
    ref = torch.where(y > 0, dy, dy * 0.01)
    torch.testing.assert_close(dyd.cpu(), ref, rtol=0, atol=0)


def test_sigmoid_multi_loss_matches_oracle_on_golden_inputs(oracle_mod):
    """Loss and d loss / d z of the fused kernel vs the oracle's multi_loss (code/train.py:
    89-108) on logits re-derived from the golden fixture's probabilities. The pinning to
    the reference's own output is transitive: the oracle matches the golden loss itself in
    tests/test_oracle.py::test_multi_loss_matches_reference_golden."""
    import os

    from plagnn import _lib

    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "multi_loss.npz"))
    probs = np.clip(d["probs"].astype(np.float64), 1e-6, 1 - 1e-6)
    z = np.log(probs / (1 - probs)).astype(np.float32)  # logits whose sigmoid ~ probs
    p32 = torch.sigmoid(torch.from_numpy(z))
    target = d["target"]
    w = d["weight"]
    n, C = z.shape
    # oracle: multi_loss on sigmoid(z) through autograd
    zt = torch.from_numpy(z).requires_grad_(True)
    ref = oracle_mod.multi_loss(torch.sigmoid(zt), torch.from_numpy(target), w)
    ref.backward()
    cw = np.empty(2 * C, np.float32)
    cw[0::2] = w.astype(np.float32)
    cw[1::2] = (w + 1.0).astype(np.float32)
    zd = torch.from_numpy(z).to(DEV)
    lab = torch.from_numpy(target).to(DEV)
    cwd = torch.from_numpy(cw).to(DEV)
    idx = torch.arange(n, dtype=torch.int32, device=DEV)
    prob = torch.empty(n, C, device=DEV)
    loss = torch.empty(1, device=DEV)
    dz = torch.empty(n, C, device=DEV)
    L = _lib.lib()
    ws = torch.empty(L.pg_sigmoid_multi_loss_workspace(n, C), dtype=torch.uint8, device=DEV)
    _lib.call("pg_sigmoid_multi_loss", zd.data_ptr(), C, n, C, lab.data_ptr(), C, cwd.data_ptr(),
              idx.data_ptr(), n, prob.data_ptr(), C, loss.data_ptr(), dz.data_ptr(), C, ws.data_ptr(),
              ws.numel(), _lib.stream_handle(zd.device))
    torch.testing.assert_close(prob.cpu(), p32, rtol=1e-6, atol=1e-7)
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item())
    torch.testing.assert_close(dz.cpu(), zt.grad, rtol=1e-5, atol=1e-8)


def test_adam_matches_oracle_and_torch(oracle_mod):
    from plagnn import _lib

    torch.manual_seed(0)
    n = 100_003
    p0 = torch.randn(n)
    p_ref = p0.clone()
    m_ref, v_ref = torch.zeros(n), torch.zeros(n)
    pd, md, vd = p0.to(DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    st = torch.zeros(4, device=DEV)
    s = _lib.stream_handle(pd.device)
    for step in range(1, 8):
        g = torch.randn(n)
        gd = g.to(DEV)
        _lib.call("pg_adam_prepare", st.data_ptr(), 5e-5, 0.9, 0.999, s)
        _lib.call("pg_adam_apply", pd.data_ptr(), gd.data_ptr(), md.data_ptr(), vd.data_ptr(), n,
                  st.data_ptr(), 0.9, 0.999, 1e-8, 0.0, s)
        oracle_mod.adam_step_torch110([p_ref], [g], [m_ref], [v_ref], step, 5e-5)
    torch.testing.assert_close(pd.cpu(), p_ref, rtol=1e-6, atol=1e-9)
    assert st[0].item() == 7.0


def test_gemm_fused_activation_backward():
    """dact epilogue: (A @ B + beta*C) * act'(Y) with Y an activation output."""
    from plagnn import _lib, ops

    torch.manual_seed(1)
    A = torch.randn(300, 96)
    B = torch.randn(96, 40)
    Y = torch.randn(300, 40)
    C0 = torch.randn(300, 40)
    for act, slope in ((_lib.PG_ACT_LEAKY, 0.01), (_lib.PG_ACT_RELU, 0.0)):
        Cd = C0.to(DEV)
        ops.gemm(A.to(DEV), B.to(DEV), out=Cd, beta=1.0, act=act, dact=Y.to(DEV))
        full = A.double() @ B.double() + C0.double()
        ref = torch.where(Y > 0, full, full * slope)
        torch.testing.assert_close(Cd.cpu().double(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("F,weighted", [(256, False), (512, True), (64, False)])
def test_spmm_max_bwd_skip_zero_maxima_is_exact(F, weighted):
    """fwd_out = the forward's output: entries whose maximum is 0 are skipped (their winner is
    relu-masked or weighted 0), and dx is bitwise unchanged — hub rows and dead features
    (all-zero columns, whose ties all sit at position 0) included; the same with records
    made by the forward with PG_ARG_DEAD_NONE (what TrainEngine runs)."""
    from plagnn import ops

    n = 800
    src, dst = hub_graph(n, 3000, seed=F)
    g = _graph(src, dst, n)
    dg = g.on(DEV)
    gen = torch.Generator().manual_seed(F + 1)
    P = torch.relu(torch.randn(n, F, generator=gen))
    P[:, ::3] = 0.0  # dead features
    P = P.to(DEV)
    ew = dg.edge_weight_slots(torch.rand(g.num_edges, generator=gen)) if weighted else None
    if weighted:
        ew[::7] = 0.0  # zero weights: max 0 with a live winner
    out, arg = ops.spmm_max(dg, P, ew)
    dZ = torch.randn(n, F, generator=gen).to(DEV)
    a = ops.spmm_max_backward(dg, arg, dZ, ew, mask=P)
    b = ops.spmm_max_backward(dg, arg, dZ, ew, mask=P, fwd_out=out)
    assert torch.equal(a, b)
    # PG_ARG_DEAD_NONE records: the same maxima, "none" where the maximum is 0, and the
    # backward bitwise the same without fwd_out
    out_d, arg_d = ops.spmm_max(dg, P, ew, dead_none=True)
    assert torch.equal(out_d, out)
    none = torch.full_like(arg, -1)
    assert torch.equal(arg_d, torch.where(out == 0, none, arg))
    assert torch.equal(ops.spmm_max_backward(dg, arg_d, dZ, ew, mask=P, dead_none=True), a)
    bf = P.to(torch.bfloat16)
    outb, argb = ops.spmm_max(dg, bf, ew)
    dZb = dZ.to(torch.bfloat16)
    ab = ops.spmm_max_backward(dg, argb, dZb, ew, mask=bf)
    assert torch.equal(ab, ops.spmm_max_backward(dg, argb, dZb, ew, mask=bf, fwd_out=outb))
    _, argb_d = ops.spmm_max(dg, bf, ew, dead_none=True)
    assert torch.equal(ops.spmm_max_backward(dg, argb_d, dZb, ew, mask=bf, dead_none=True), ab)


@pytest.mark.parametrize("M,N,K,ta", [(256, 1024, 24041, True), (100, 256, 24041, True),
                                      (97, 260, 9000, False), (512, 512, 6000, True)])
def test_gemm_split_k_and_row_sums_accuracy(M, N, K, ta):
    """Split-K products within float32 bounds of a float64 reference, deterministic (two
    calls bitwise equal), beta = 1 accumulating onto C; the row sums (bias gradients) are
    accumulated in float64 inside the kernel, so even a sum whose terms cancel (zero-mean
    rows) lands within a few float32 roundings of the exact value."""
    from plagnn import ops

    gen = torch.Generator().manual_seed(M + N)
    A = (torch.randn(K, M, generator=gen) if ta else torch.randn(M, K, generator=gen)).to(DEV)
    B = torch.randn(K, N, generator=gen).to(DEV)
    sk = ops._split_k(M, N, K)
    assert sk > 1
    rs_a, rs_b = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    c1 = ops.gemm(A, B, transa=ta, split_k=sk, rowsum=rs_a)
    c2 = ops.gemm(A, B, transa=ta, split_k=sk, rowsum=rs_b)
    assert torch.equal(c1, c2) and torch.equal(rs_a, rs_b)
    a64 = (A.t() if ta else A).double()
    ref = a64 @ B.double()
    err = (c1.double() - ref).abs().max().item()
    assert err <= 2e-6 * (a64.abs() @ B.double().abs()).max().item()
    rs64 = a64.sum(1)
    # one float32 rounding per slice partial (|partial| ~ ||row||_2 / sqrt(sk)), not one per term
    bound = 2e-7 * sk ** 0.5 * a64.pow(2).sum(1).sqrt() + 2e-7 * rs64.abs()
    assert torch.all((rs_a.double() - rs64).abs() <= bound)
    C = torch.randn(M, N, generator=gen).to(DEV)
    C0 = C.clone()
    ops.gemm(A, B, transa=ta, out=C, beta=1.0, split_k=sk)
    torch.testing.assert_close(C, C0 + c1, rtol=1e-5, atol=1e-4)


def test_gemm_split_k_deferred_batch_reduce_is_bitwise():
    """pg_gemm_f32_partials + one pg_gemm_splitk_reduce_batch over several products equals
    each product's own pg_gemm_f32 (split-K with its reduce launch) bitwise, row sums and
    beta = 1 included (TrainEngine defers every weight gradient's combine to one launch)."""
    import ctypes

    from plagnn import _lib, ops
    from plagnn._lib import call, ptr

    gen = torch.Generator().manual_seed(11)
    shapes = [(256, 1024, 24041), (100, 256, 24041), (12, 100, 24041), (97, 260, 9000)]
    jobs, refs, outs, keep = [], [], [], []
    for i, (M, N, K) in enumerate(shapes):
        A = torch.randn(K, M, generator=gen).to(DEV)
        B = torch.randn(K, N, generator=gen).to(DEV)
        sk = ops._split_k(M, N, K)
        beta = float(i % 2)
        C0 = torch.randn(M, N, generator=gen).to(DEV)
        ref, rs_ref = C0.clone(), torch.empty(M, device=DEV)
        ops.gemm(A, B, transa=True, out=ref, beta=beta, split_k=sk, rowsum=rs_ref)
        C, rs = C0.clone(), torch.empty(M, device=DEV)
        ws = torch.empty(int(_lib.lib().pg_gemm_f32_workspace(M, N, K, sk)), dtype=torch.uint8, device=DEV)
        used = ctypes.c_int(0)
        call("pg_gemm_f32_partials", 1, 0, M, N, K, ptr(A), A.stride(0), ptr(B), B.stride(0),
             _lib.epilogue(rowsum=rs), sk, ptr(ws), ws.numel(), ctypes.byref(used), _lib.stream_handle(A.device))
        assert used.value > 1
        j = _lib.PgSplitkJob()
        j.ws, j.split_k, j.M, j.N, j.alpha, j.beta = ptr(ws), used.value, M, N, 1.0, beta
        j.C, j.ldc, j.rowsum = ptr(C), C.stride(0), ptr(rs)
        jobs.append(j)
        refs.append((ref, rs_ref))
        outs.append((C, rs))
        keep += [A, B, ws]
    arr = (_lib.PgSplitkJob * len(jobs))(*jobs)
    call("pg_gemm_splitk_reduce_batch", arr, len(jobs), _lib.stream_handle(torch.device(DEV)))
    torch.cuda.synchronize()
    for (ref, rs_ref), (C, rs) in zip(refs, outs):
        assert torch.equal(C, ref)
        assert torch.equal(rs, rs_ref)


def _group_parts(specs, gen):
    """pg_gemm_part_t array + the tensors behind it; spec = (ta, tb, M, N, K, beta, rowsum,
    misalign): misalign offsets A by one float (the grouped kernel does not take it)."""
    from plagnn import _lib
    from plagnn._lib import ptr

    parts = (_lib.PgGemmPart * len(specs))()
    keep = []
    for q, (ta, tb, M, N, K, beta, want_rs, mis) in zip(parts, specs):
        a = torch.randn(K * M + 1, generator=gen).to(DEV)
        A = (a[1:] if mis else a[:-1]).view(*((K, M) if ta else (M, K)))
        B = torch.randn(*((N, K) if tb else (K, N)), generator=gen).to(DEV)
        C = torch.randn(M, N, generator=gen).to(DEV)
        rs = torch.full((M,), float("nan"), device=DEV) if want_rs else None
        q.transa, q.transb, q.M, q.N, q.K = int(ta), int(tb), M, N, K
        q.A, q.lda, q.B, q.ldb = ptr(A), A.stride(0), ptr(B), B.stride(0)
        q.beta, q.C, q.ldc, q.rowsum = beta, ptr(C), C.stride(0), ptr(rs)
        keep.append((ta, tb, A, B, C, C.clone(), rs, beta))
    return parts, keep


# the cfg2 step's weight gradients (TrainEngine groups them), one with beta = 1, and ragged
_CFG2_WGRADS = [(True, False, 256, 1008, 24041, 0.0, True, False), (True, False, 504, 504, 24041, 0.0, True, False),
                (True, False, 256, 512, 24041, 1.0, True, False), (True, False, 256, 256, 24041, 0.0, True, False),
                (True, False, 100, 256, 24041, 0.0, True, False), (True, False, 12, 100, 24041, 0.0, True, False),
                (True, False, 0, 64, 24041, 0.0, False, False), (True, False, 132, 20, 999, 1.0, False, False)]


@pytest.mark.parametrize("case", ["grouped", "misaligned", "mixed"])
def test_gemm_f32_group(case):
    """pg_gemm_f32_group against float64: every part's product within float32 bounds, beta
    = 1 accumulating, row sums, an empty part, a ragged short-K part; deterministic (two
    calls bitwise equal). `misaligned` / `mixed` (a part on another transposition) take the
    one-by-one path, which must give the same contract."""
    from plagnn import _lib
    from plagnn._lib import call, ptr

    specs = list(_CFG2_WGRADS)
    if case == "misaligned":
        specs[3] = specs[3][:7] + (True,)
    elif case == "mixed":
        specs[-1] = (False, True, 132, 20, 999, 1.0, False, False)
    gen = torch.Generator().manual_seed(5)
    parts, keep = _group_parts(specs, gen)
    n = len(specs)
    ws = torch.empty(int(_lib.lib().pg_gemm_f32_group_workspace(parts, n)), dtype=torch.uint8, device=DEV)
    st = _lib.stream_handle(torch.device(DEV))
    call("pg_gemm_f32_group", parts, n, ptr(ws), ws.numel(), st)
    first = [(C.clone(), None if rs is None else rs.clone()) for (_, _, _, _, C, _, rs, _) in keep]
    for (_, _, _, _, C, C0, _, _) in keep:
        C.copy_(C0)
    call("pg_gemm_f32_group", parts, n, ptr(ws), ws.numel(), st)
    torch.cuda.synchronize()
    for (ta, tb, A, B, C, C0, rs, beta), (c1, r1) in zip(keep, first):
        assert torch.equal(C, c1) and (rs is None or torch.equal(rs, r1))
        a64 = (A.t() if ta else A).double()
        b64 = (B.t() if tb else B).double()
        if a64.shape[0] == 0:
            continue
        ref = a64 @ b64 + beta * C0.double()
        scale = (a64.abs() @ b64.abs()).max().item() + beta * C0.abs().max().item()
        assert (C.double() - ref).abs().max().item() <= 2e-6 * scale
        if rs is not None:
            rs64 = a64.sum(1)
            bound = 2e-7 * 256 ** 0.5 * a64.pow(2).sum(1).sqrt() + 2e-7 * rs64.abs()
            assert torch.all((rs.double() - rs64).abs() <= bound)


def test_gemm_f32_group_bad_args():
    from plagnn import _lib

    gen = torch.Generator().manual_seed(6)
    parts, keep = _group_parts(_CFG2_WGRADS[:2], gen)
    L = _lib.lib()
    ws = torch.empty(int(L.pg_gemm_f32_group_workspace(parts, 2)), dtype=torch.uint8, device=DEV)
    assert L.pg_gemm_f32_group(parts, 2, ws.data_ptr(), ws.numel() - 256, None) == -3
    parts[1].beta = 0.5
    assert L.pg_gemm_f32_group(parts, 2, ws.data_ptr(), ws.numel(), None) == -1
    assert L.pg_gemm_f32_group(parts, 17, ws.data_ptr(), ws.numel(), None) == -1
    parts[1].beta = 0.0
    parts[0].C = None  # a part with outputs needs C
    assert L.pg_gemm_f32_group(parts, 2, ws.data_ptr(), ws.numel(), None) == -1


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(1, 4, 4), (33, 12, 20), (129, 132, 100), (64, 4, 1000), (4, 260, 36)])
def test_gemm_f32_edge_shapes_with_epilogue(ta, tb, M, N, K):
    """Small and ragged shapes through pg_gemm_f32 (the three-piece path wherever the
    operands are 16-B aligned with 4-multiple extents): partial K tiles, tiles past M / N,
    beta = 1, bias and leaky_relu, against float64."""
    from plagnn import _lib, ops

    g = torch.Generator().manual_seed(M * 131 + N * 7 + K)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((N, K) if tb else (K, N), generator=g)
    bias = torch.randn(N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    Cd = C0.to(DEV)
    ops.gemm(A.to(DEV), B.to(DEV), transa=ta, transb=tb, out=Cd, beta=1.0, bias=bias.to(DEV),
             act=_lib.PG_ACT_LEAKY)
    a64 = A.double().t() if ta else A.double()
    b64 = B.double().t() if tb else B.double()
    ref = torch.nn.functional.leaky_relu(a64 @ b64 + C0.double() + bias.double(), 0.01)
    scale = (a64.abs() @ b64.abs()) + C0.double().abs() + bias.double().abs()
    err = (Cd.cpu().double() - ref).abs()
    assert float((err / scale).max()) <= 2e-6


@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("M,N,K1,K2", [(24041, 256, 256, 256), (1000, 300, 300, 400), (777, 200, 400, 300),
                                      (300, 104, 4, 60), (513, 64, 100, 28)])
def test_gemm_f32_cat_equals_concatenated(tb, M, N, K1, K2):
    """pg_gemm_f32_cat ([A1 | A2] op([B1 ; B2]) over two K pieces, the split at any multiple
    of 4, K steps straddling it included) equals pg_gemm_f32 on the concatenated operands
    bit for bit (the same tile and k order), with and without bias + leaky_relu."""
    from plagnn import _lib, ops

    g = torch.Generator(device="cpu").manual_seed(M + N + K1)
    A1 = torch.randn(M, K1, generator=g).to(DEV)
    A2 = torch.randn(M, K2, generator=g).to(DEV)
    B1 = torch.randn(*((N, K1) if tb else (K1, N)), generator=g).to(DEV)
    B2 = torch.randn(*((N, K2) if tb else (K2, N)), generator=g).to(DEV)
    bias = torch.randn(N, generator=g).to(DEV)
    A = torch.cat([A1, A2], 1)
    B = torch.cat([B1, B2], 1 if tb else 0)
    for kw in ({}, {"bias": bias, "act": _lib.PG_ACT_LEAKY}):
        got = ops.gemm_cat(A1, A2, B1, B2, transb=tb, **kw)
        assert got is not None
        want = ops.gemm(A, B, transb=tb, **kw)
        assert torch.equal(got, want), float((got - want).abs().max())


@pytest.mark.gpu
def test_pad2d_group_matches_torch():
    """pg_pad2d_group: zero-padded copies of several operands in one launch (the drop-in
    SAGEConv's weight images), including strided destinations and an empty part."""
    from plagnn import ops

    torch.manual_seed(3)
    srcs = [torch.randn(503, 503, device=DEV), torch.randn(1, 503, device=DEV), torch.randn(256, 503, device=DEV),
            torch.randn(256, 503, device=DEV), torch.randn(0, 7, device=DEV)]
    W = torch.full((512, 512), 7.0, device=DEV)
    b = torch.full((1, 512), 7.0, device=DEV)
    Wcat = torch.full((256, 1024), 7.0, device=DEV)
    E = torch.full((3, 9), 7.0, device=DEV)
    ops.pad2d_group([(srcs[0], W), (srcs[1], b), (srcs[2], Wcat[:, :512]), (srcs[3], Wcat[:, 512:]), (srcs[4], E)])
    want = [torch.nn.functional.pad(srcs[0], (0, 9, 0, 9)), torch.nn.functional.pad(srcs[1], (0, 9)),
            torch.cat([torch.nn.functional.pad(srcs[2], (0, 9)), torch.nn.functional.pad(srcs[3], (0, 9))], 1),
            torch.zeros(3, 9, device=DEV)]
    for got, ref in zip([W, b, Wcat, E], want):
        assert torch.equal(got, ref)
