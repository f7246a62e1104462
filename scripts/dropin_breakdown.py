"""Where the drop-in epoch's time goes (code/train.py:197-207 on the dgl shim): the whole
epoch and its pieces, each timed over `reps` back-to-back iterations (one sync at the end),
so host dispatch and device time both show. Usage: python scripts/dropin_breakdown.py [cfg]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dgl  # noqa: E402
from plagnn import workload  # noqa: E402
from plagnn.model import GNN  # noqa: E402
from plagnn.train import multi_loss  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
dev = torch.device("cuda")
wl = workload.build(cfg, device=dev)
src, dst, _ = wl.edges_without_loops()
g = dgl.add_self_loop(dgl.graph((torch.from_numpy(src), torch.from_numpy(dst)), num_nodes=wl.n)).to(dev)
x = torch.from_numpy(wl.ds.feat).to(dev)
labels = torch.from_numpy(wl.ds.loc.astype(np.float32)).to(dev)
tr = torch.as_tensor(wl.train_index, device=dev)
va = torch.as_tensor(wl.val_index, device=dev)
torch.manual_seed(0)
model = GNN(wl.dims).to(dev)
opt = torch.optim.Adam(model.parameters(), lr=5e-5)
w = wl.class_weight


def timed(name, fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name:28s} {(t2 - t0) / reps * 1e3:8.3f} ms/iter  (host issue {(t1 - t0) / reps * 1e3:8.3f} ms)")


def epoch():
    opt.zero_grad()
    logits = model(g, x)
    loss = multi_loss(logits[tr], labels[tr], w)
    loss.backward()
    opt.step()
    multi_loss(logits[va], labels[va], w)


def fwd_only():
    with torch.no_grad():
        model(g, x)


def fwd_bwd():
    logits = model(g, x)
    logits.sum().backward()


logits0 = model(g, x).detach()


def loss_only():
    lg = logits0.clone().requires_grad_(True)
    loss = multi_loss(lg[tr], labels[tr], w)
    loss.backward()
    multi_loss(lg.detach()[va], labels[va], w)


def adam_only():
    opt.step()


for p in model.parameters():
    p.grad = torch.zeros_like(p)
timed("epoch (train.py:197-207)", epoch)
timed("forward (no grad)", fwd_only)
timed("forward + backward", fwd_bwd)
timed("multi_loss train+val fwd/bwd", loss_only)
timed("Adam.step", adam_only)
