"""Diagnostic: the upstream gradient dM of each max aggregation (and dP) in the engine, in the
float32 oracle and in the float64 oracle (both aligned to the engine's decisions): how far
each float32 computation is from float64, per layer. Usage:
  python scripts/diag/dm_error.py [config]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from oracle import oracle as om  # noqa: E402
import plagnn  # noqa: E402
from plagnn import workload  # noqa: E402
from test_gpu_fullsize import _engine_signs  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
wl = workload.build(cfg, device="cuda")
x = torch.from_numpy(wl.ds.feat)
labels = torch.from_numpy(wl.ds.loc.astype(np.float32))
sd = oracle.init_params(wl.dims, seed=2)
eng = plagnn.TrainEngine(wl.graph(), x, labels, wl.dims, wl.class_weight, wl.train_index, wl.val_index,
                         device="cuda", edge_weight=wl.edge_weight, params=sd)
eng.forward()
eng.backward()
torch.cuda.synchronize()
signs = _engine_signs(eng)
src, dst, w = wl.edges_without_loops()
og = oracle.OracleGraph(src, dst, wl.n, edge_weight=w)

captured = []
fwd_args = []
orig = om._MaxAggregate.backward
orig_f = om._MaxAggregate.forward


def fhook(ctx, P, g, use_weight, parallel=False, align=None):
    r = orig_f(ctx, P, g, use_weight, parallel, align)
    fwd_args.append((ctx.argx.copy(), ctx.arge.copy(), r.detach().clone()))
    return r


om._MaxAggregate.forward = staticmethod(fhook)


def hook(ctx, dZ):
    captured.append(dZ.detach().clone())
    r = orig(ctx, dZ)
    captured.append(r[0].detach().clone())
    return r


om._MaxAggregate.backward = staticmethod(hook)
s32 = {k: v for k, v in signs.items()}
r32 = oracle.train_step(og, x, labels, wl.train_index, wl.class_weight, sd, use_weight=w is not None, signs=s32)
c32 = captured[:]
f32a = fwd_args[:]
captured.clear()
s64 = {k: v for k, v in signs.items() if not k.startswith("_")}
r64 = oracle.train_step(og, x, labels, wl.train_index, wl.class_weight, sd, use_weight=w is not None, signs=s64,
                        dtype=torch.float64)
c64 = captured[:]
L = eng.L
for i in range(L):
    l = L - 1 - i  # backward order: top layer first
    F, Fi = eng.dims[l], eng.pd[l]
    dm_e = eng.dHM[l][:, Fi:Fi + F].double().cpu()
    dm_o, dm_t = c32[2 * i].double(), c64[2 * i]
    P = eng.Pl[l][:, :F].cpu().double()
    dp_e = eng.dP[l][:, :F].double().cpu()
    dp_o, dp_t = c32[2 * i + 1].double() * (P > 0), c64[2 * i + 1] * (P > 0)
    sc = dm_t.abs().max().item()
    print(f"layer {l + 1}: dM max err engine {(dm_e - dm_t).abs().max().item() / sc:.2e}, oracle32 "
          f"{(dm_o - dm_t).abs().max().item() / sc:.2e} (of max |dM|); rms engine "
          f"{((dm_e - dm_t) ** 2).mean().sqrt().item() / sc:.2e}, oracle32 {((dm_o - dm_t) ** 2).mean().sqrt().item() / sc:.2e}")
    b_e, b_o, b_t = dp_e.sum(0), dp_o.sum(0), dp_t.sum(0)
    cond = (dp_t.abs().sum(0) / b_t.abs().clamp_min(1e-30)).max().item()
    print(f"   bias_pool: engine err {(b_e - b_t).abs().max().item():.3e}, oracle32 {(b_o - b_t).abs().max().item():.3e}, "
          f"scale {b_t.abs().max().item():.3e}, max sum|terms|/|sum| {cond:.2e}")
from plagnn import ops  # noqa: E402
for l in range(L):
    F, Fi = eng.dims[l], eng.pd[l]
    ax_e = ops.argpos_to_src(eng.dg, eng.arg[l][:, :F].contiguous()).cpu().numpy()
    ax_o, ae_o, m_o = f32a[l]
    m_e = eng.HM[l][:, Fi:Fi + F].cpu().numpy()
    diff = ax_e != ax_o
    mv = np.abs(m_e - m_o.numpy())
    print(f"fwd layer {l + 1}: winners differing {diff.sum()}, M differing {(mv > 0).sum()}, "
          f"max |M diff| {mv.max():.3e} (max |M| {np.abs(m_o.numpy()).max():.3e})")
    if diff.sum():
        idx = np.argwhere(diff)[:5]
        for v, f in idx:
            print(f"   ({v},{f}) engine src {ax_e[v, f]} oracle src {ax_o[v, f]} M_e {m_e[v, f]:.6e} M_o {m_o[v, f]:.6e}")
g32, g64 = r32[2], r64[2]
ge = eng.grads()
for k in ge:
    if k.endswith("bias"):
        t = g64[k].double()
        print(f"{k}: engine {(ge[k].cpu().double() - t).abs().max().item():.3e} oracle32 "
              f"{(g32[k].double() - t).abs().max().item():.3e} scale {t.abs().max().item():.3e}")
