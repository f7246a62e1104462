"""The drop-in SAGEConv's cached [H | M] buffer must never serve a stale H.

SagePool keeps the padded [H | M] buffer of an input that takes no gradient (the features,
the same tensor every epoch) between calls. Under torch.no_grad() every layer input is
such a tensor, and a freed layer output's memory is handed to the next same-size
allocation, which starts at the same version counter: the cache must key on the tensor
object itself, not on its address. The model runs twice under no_grad with the weights
changed in between (cuda), against the CPU composition of the same model
(code/model.py:19-31 forward, as an inference after an optimizer step would run it).
"""
import copy

import numpy as np
import pytest
import torch

from conftest import random_graph


def _pair(seed=0):
    import dgl
    from plagnn.model import GNN32

    n = 1500
    src, dst = random_graph(n, 12 * n, seed=seed, self_loop=False)
    g = dgl.add_self_loop(dgl.graph((list(src), list(dst)), num_nodes=n))
    torch.manual_seed(seed)
    feats = torch.randn(n, 503).clamp_min(0)
    model = GNN32(503, 64, 48, 40, 16, 12)
    return g, feats, model


@pytest.mark.gpu
def test_no_grad_forward_after_weight_change_matches_cpu():
    g, feats, model = _pair()
    gpu = copy.deepcopy(model).to("cuda")
    gg, fg = g.to("cuda"), feats.to("cuda")
    rng = torch.Generator().manual_seed(7)
    with torch.no_grad():
        for it in range(3):
            want = model(g, feats)
            got = gpu(gg, fg).cpu()
            err = float((got - want).abs().max())
            print(f"  no_grad forward {it}: max abs err {err:.2e}")
            assert err <= 1e-5, (it, err)
            # change every parameter in place (an optimizer step), identically on both
            for (_, p), (_, q) in zip(model.named_parameters(), gpu.named_parameters()):
                d = 0.05 * torch.randn(p.shape, generator=rng)
                p.add_(d)
                q.add_(d.to("cuda"))


@pytest.mark.gpu
def test_hm_cache_rejects_new_tensor_at_same_address():
    """The cache directly: a new tensor that reuses a freed input's memory (same address,
    same version) gets its own H, not the freed one's."""
    from plagnn import ops

    n, F = 256, 64
    a = torch.full((n, F), 1.0, device="cuda")
    hm1, _ = ops._hm_buffer(a, F, keep=False)
    assert float(hm1[:, :F].min()) == 1.0
    addr = a.data_ptr()
    del a, hm1
    b = torch.full((n, F), 2.0, device="cuda")
    if b.data_ptr() != addr:
        pytest.skip("allocator did not reuse the block")
    hm2, _ = ops._hm_buffer(b, F, keep=False)
    assert float(hm2[:, :F].min()) == 2.0 and float(hm2[:, :F].max()) == 2.0
