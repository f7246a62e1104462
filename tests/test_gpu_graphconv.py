"""BASELINE configs[0] ("2-layer GraphConv hidden=64") and the SAGEConv 'mean' / 'gcn'
aggregators on the GPU: the shim's layers (dgl.nn.pytorch.GraphConv / SAGEConv, whose
aggregations run on pg_spmm_sum through plagnn.ops.SumAggregate) against the oracle's
restatement of DGL 0.8.2 (oracle.graph_conv / oracle.sage_mean: degree norms with
clamp(min=1), the product order by in_feats > out_feats, lin_before_mp). The reference
itself only runs SAGEConv 'pool' (code/model.py:13-15), so these are reference-unpinned.

Bars: a layer's output and gradients within 1e-5 of each tensor's magnitude (float32
reassociation: hub rows are summed in 256-entry partials); the whole cfg1 step at
N = 24,041 with the full-size bars of test_gpu_fullsize (decision-aligned leaky_relu,
1e-4 of each tensor's magnitude, float64 judgement past it).
"""
import numpy as np
import pytest
import torch

from conftest import hub_graph

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, tol, name):
    a = a.detach().cpu().double()
    b = b.detach().cpu().double()
    scale = max(b.abs().max().item(), 1e-12)
    err = (a - b).abs().max().item()
    assert err <= tol * scale, f"{name}: max err {err:.3e} vs scale {scale:.3e}"


def _layer_case(n=500, hub=700, seed=5, weighted=False):
    import dgl

    src, dst = hub_graph(n, hub, seed=seed)  # self-loops appended: every in-degree >= 1
    rng = np.random.default_rng(seed)
    w = rng.uniform(0.1, 1.0, len(src)).astype(np.float32) if weighted else None
    g = dgl.graph((torch.from_numpy(src), torch.from_numpy(dst)), num_nodes=n).to(DEV)
    return src, dst, w, g, rng


@pytest.mark.parametrize("weighted", [False, True], ids=["copy_u", "u_mul_e"])
@pytest.mark.parametrize("norm", ["both", "left", "right", "none"])
@pytest.mark.parametrize("fin,fout", [(40, 16), (16, 40)], ids=["w_first", "aggregate_first"])
def test_graphconv_layer_matches_oracle(oracle_mod, fin, fout, norm, weighted):
    from dgl.nn.pytorch import GraphConv

    n = 500
    src, dst, w, g, rng = _layer_case(n, weighted=weighted)
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False, edge_weight=w)
    conv = GraphConv(fin, fout, norm=norm).to(DEV)
    W = torch.from_numpy(rng.standard_normal((fin, fout)).astype(np.float32) * 0.3)
    b = torch.from_numpy(rng.standard_normal(fout).astype(np.float32) * 0.1)
    with torch.no_grad():
        conv.weight.copy_(W)
        conv.bias.copy_(b)
    x = torch.from_numpy(rng.standard_normal((n, fin)).astype(np.float32))
    xd = x.to(DEV, copy=True).requires_grad_(True)
    ew = None if w is None else torch.from_numpy(w).to(DEV)
    y = conv(g, xd, edge_weight=ew)
    dZ = torch.from_numpy(rng.standard_normal((n, fout)).astype(np.float32))
    y.backward(dZ.to(DEV))

    xo, Wo, bo = (t.clone().requires_grad_(True) for t in (x, W, b))
    yo = oracle_mod.graph_conv(og, xo, Wo, bo, norm=norm, use_weight=weighted)
    yo.backward(dZ)
    _close(y, yo, 1e-5, "out")
    _close(xd.grad, xo.grad, 1e-5, "d feat")
    _close(conv.weight.grad, Wo.grad, 1e-5, "d weight")
    _close(conv.bias.grad, bo.grad, 1e-5, "d bias")


def test_graphconv_rejects_zero_in_degree():
    import dgl
    import plagnn
    from dgl.nn.pytorch import GraphConv

    g = dgl.graph((torch.tensor([0, 1]), torch.tensor([1, 2])), num_nodes=3).to(DEV)
    with pytest.raises(plagnn.PlagnnError):
        GraphConv(4, 2).to(DEV)(g, torch.ones(3, 4, device=DEV))


@pytest.mark.parametrize("weighted", [False, True], ids=["copy_u", "u_mul_e"])
@pytest.mark.parametrize("aggr", ["mean", "gcn"])
@pytest.mark.parametrize("fin,fout", [(40, 16), (16, 40)], ids=["lin_before_mp", "lin_after_mp"])
def test_sage_mean_gcn_layer_matches_oracle(oracle_mod, aggr, fin, fout, weighted):
    from dgl.nn.pytorch import SAGEConv

    n = 500
    src, dst, w, g, rng = _layer_case(n, seed=7, weighted=weighted)
    og = oracle_mod.OracleGraph(src, dst, n, self_loop=False, edge_weight=w)
    conv = SAGEConv(fin, fout, aggr).to(DEV)
    p = {"fc_neigh.weight": torch.from_numpy(rng.standard_normal((fout, fin)).astype(np.float32) * 0.3),
         "bias": torch.from_numpy(rng.standard_normal(fout).astype(np.float32) * 0.1)}
    if aggr == "mean":
        p["fc_self.weight"] = torch.from_numpy(rng.standard_normal((fout, fin)).astype(np.float32) * 0.3)
    conv.load_state_dict(p)
    x = torch.from_numpy(rng.standard_normal((n, fin)).astype(np.float32))
    xd = x.to(DEV, copy=True).requires_grad_(True)
    ew = None if w is None else torch.from_numpy(w).to(DEV)
    y = conv(g, xd, edge_weight=ew)
    dZ = torch.from_numpy(rng.standard_normal((n, fout)).astype(np.float32))
    y.backward(dZ.to(DEV))

    po = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    xo = x.clone().requires_grad_(True)
    yo = oracle_mod.sage_mean(og, xo, po, "", aggr, use_weight=weighted)
    yo.backward(dZ)
    _close(y, yo, 1e-5, "out")
    _close(xd.grad, xo.grad, 1e-5, "d feat")
    sd = dict(conv.named_parameters())
    for k in p:
        _close(sd[k].grad, po[k].grad, 1e-5, "d " + k)


@pytest.mark.parametrize("conv", ["graphconv", "mean"])
def test_cfg1_full_size_step_matches_oracle(oracle_mod, conv):
    """cfg1 at N = 24,041 (S0): GNN(dims = [503, 64, 64, 100, 12], conv) on the shim
    (cuda), one training step — forward, multi_loss on the train rows (code/train.py:
    89-108, 203), backward — against oracle.train_step on the same parameters, with the
    leaky_relu decisions aligned inside the rounding band."""
    import dgl
    from plagnn import workload
    from plagnn.model import GNN
    from plagnn.train import multi_loss
    from test_gpu_fullsize import _check_signs, _close_judged, _oracle_graph, _Yardstick

    wl = workload.build("cfg1", device=DEV)
    assert wl.conv == "graphconv"
    dims = wl.dims
    sd = oracle_mod.init_params(dims, seed=6, conv=conv)
    torch.manual_seed(0)
    model = GNN(dims, conv=conv).to(DEV)
    model.load_state_dict(sd)
    src, dst, _ = wl.edges_without_loops()
    g = dgl.add_self_loop(dgl.graph((torch.from_numpy(src), torch.from_numpy(dst)), num_nodes=wl.n)).to(DEV)
    x = torch.from_numpy(wl.ds.feat)
    labels = torch.from_numpy(wl.ds.loc.astype(np.float32))
    signs = {}

    def rec(name):
        def hook(_m, _inp, out):
            signs[name] = (out.detach() > 0).cpu()
        return hook

    for i in range(len(dims) - 3):
        getattr(model, f"conv{i + 1}").register_forward_hook(rec(f"conv{i + 1}.out"))
    model.liner1.register_forward_hook(rec("liner1"))
    logits = model(g, x.to(DEV))
    tr = torch.as_tensor(wl.train_index, device=DEV)
    loss = multi_loss(logits[tr], labels.to(DEV)[tr], wl.class_weight)
    loss.backward()
    grads = {k: v.grad.cpu() for k, v in model.named_parameters()}

    og = _oracle_graph(oracle_mod, wl)
    ref_logits, ref_loss, ref_grads = oracle_mod.train_step(og, x, labels, wl.train_index, wl.class_weight, sd,
                                                            signs=signs)
    _check_signs(signs)
    s64 = {k: v for k, v in signs.items() if not k.startswith("_")}
    exact = _Yardstick(lambda: oracle_mod.train_step(og, x, labels, wl.train_index, wl.class_weight, sd,
                                                     dtype=torch.float64, signs=s64))
    _close_judged(logits, ref_logits, lambda: exact.get()[0], name="logits")
    assert abs(loss.item() - ref_loss.item()) <= 1e-4 * abs(ref_loss.item())
    assert set(grads) == set(ref_grads)
    for k, v in ref_grads.items():
        _close_judged(grads[k], v, lambda k=k: exact.get()[2][k], name="grad " + k)
