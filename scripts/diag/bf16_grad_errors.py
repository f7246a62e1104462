"""Diagnostic: per-tensor gradient error of the bf16 engine vs the fp32 engine (same
parameters), relative to each tensor's max magnitude, for a few problem sizes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import plagnn  # noqa: E402
from test_gpu_engine import _problem  # noqa: E402

for n, e, dims in ((600, 6000, (503, 64, 48, 32, 16, 12)), (4000, 80000, (503, 64, 48, 32, 16, 12)),
                   (4000, 80000, (503, 256, 256, 256, 100, 12))):
    src, dst, x, labels, w, tr, va, model = _problem(n=n, e=e, dims=dims)
    loops = np.arange(n)
    cg = plagnn.CSRGraph(np.concatenate([src, loops]), np.concatenate([dst, loops]), n)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    a = plagnn.TrainEngine(cg, x, labels, dims, w, tr, va, device="cuda", params=sd)
    b = plagnn.TrainEngineBF16(cg, x, labels, dims, w, tr, va, device="cuda", params=sd)
    for eng in (a, b):
        eng.forward()
        eng.backward()
    torch.cuda.synchronize()
    ga, gb = a.grads(), b.grads()
    print(f"n={n} dims={dims} loss f32 {a.losses()} bf16 {b.losses()}")
    for k in ga:
        s = ga[k].abs().max().item()
        err = (ga[k] - gb[k]).abs().max().item()
        rel = (ga[k] - gb[k]).norm().item() / max(ga[k].norm().item(), 1e-30)
        print(f"  {k:28s} max-err/max {err / max(s, 1e-30):.4f}  rel-L2 {rel:.4f}")

# (2) the layer-1 weight gradients recomputed in float64 from the bf16 engine's OWN stored
# operands (dY, dP, H): isolates the GEMM from the propagation of rounding
n, e, dims = 600, 6000, (503, 64, 48, 32, 16, 12)
src, dst, x, labels, w, tr, va, model = _problem(n=n, e=e, dims=dims)
loops = np.arange(n)
cg = plagnn.CSRGraph(np.concatenate([src, loops]), np.concatenate([dst, loops]), n)
sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
b = plagnn.TrainEngineBF16(cg, x, labels, dims, w, tr, va, device="cuda", params=sd)
b.forward()
b.backward()
torch.cuda.synchronize()
Fi, Fo = b.pd[0], b.pd[1]
dY = b.DYP[0][:, :Fo].double()
dP = b.DYP[0][:, Fo:].double()
HM = b.HM[0].double()
ref_cat = dY.t() @ HM
ref_pool = dP.t() @ HM[:, :Fi]
for name, got, ref in (("Wcat", b.G["conv1.Wcat"], ref_cat), ("Wpool", b.G["conv1.Wpool"], ref_pool)):
    err = (got.double() - ref).abs().max().item()
    print(f"GEMM check {name}: max err {err:.3e} vs max {ref.abs().max().item():.3e}")
# (3) inputs exactly representable in bf16: the fp32 engine sees the same features
xb = x.to(torch.bfloat16).float()
a = plagnn.TrainEngine(cg, xb, labels, dims, w, tr, va, device="cuda", params=sd)
c = plagnn.TrainEngineBF16(cg, xb, labels, dims, w, tr, va, device="cuda", params=sd)
for eng in (a, c):
    eng.forward()
    eng.backward()
torch.cuda.synchronize()
ga, gc = a.grads(), c.grads()
for k in ("conv1.fc_pool.weight", "conv1.fc_self.weight", "conv1.fc_neigh.weight"):
    rel = (ga[k] - gc[k]).norm().item() / ga[k].norm().item()
    print(f"  bf16-exact inputs: {k:24s} rel-L2 {rel:.4f}")
