"""Generate the golden fixtures in tests/golden/ from the reference's OWN functions.

Run in the build container only (it reads /root/reference; the GPU box never runs it):
    python tests/golden/gen_golden.py

The reference's train.py cannot be imported as a module here (it imports dgl and reads
../data/generate_materials/label_list.json at import time, code/train.py:12, 128-129), so
the dgl-free functions below are taken from it by AST (function definitions only) and
executed in a namespace holding torch / numpy:
    protein_loc_correction   code/train.py:19-40
    performances_record      code/train.py:43-86
    multi_loss               code/train.py:89-108
    weight_cal               code/train.py:111-126
data_preprocess.py imports cleanly (pandas/scipy/sklearn/tqdm), so
    edge_clustering_coefficients  code/data_preprocess.py:175-214
is called directly. Only the produced input/output arrays are committed (no source).
"""
from __future__ import annotations

import ast
import os
import sys

import numpy as np
import torch

REF = "/root/reference/code"
HERE = os.path.dirname(os.path.abspath(__file__))


def _train_functions():
    src = open(os.path.join(REF, "train.py")).read()
    tree = ast.parse(src)
    wanted = {"protein_loc_correction", "performances_record", "multi_loss", "weight_cal"}
    mod = ast.Module(body=[n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in wanted],
                     type_ignores=[])
    ns = {"torch": torch, "np": np}
    exec(compile(mod, os.path.join(REF, "train.py"), "exec"), ns)
    return ns


def gen_loss(ns):
    rng = np.random.default_rng(1234)
    n, C = 97, 12
    loc = (rng.random((200, C)) < 0.2).astype(np.float64)
    loc[rng.random(200) < 0.4] = 0.0
    w = ns["weight_cal"](loc)
    probs = rng.random((n, C)).astype(np.float32)
    probs[0, :4] = [0.0, 1.0, 1e-12, 1 - 1e-8]  # exercise both clamps
    target = (rng.random((n, C)) < 0.3).astype(np.float32)
    inp = torch.tensor(probs, requires_grad=True)
    loss = ns["multi_loss"](inp, torch.tensor(target), w)
    loss.backward()
    np.savez(os.path.join(HERE, "multi_loss.npz"), loc=loc, weight=w, probs=probs, target=target,
             loss=np.float32(loss.item()), grad=inp.grad.numpy())


def gen_eval(ns):
    rng = np.random.default_rng(99)
    n, C = 64, 12
    proba = torch.tensor(rng.random((n, C)).astype(np.float32))
    true = torch.tensor((rng.random((n, C)) < 0.25).astype(np.float32))
    true[true.sum(1) == 0, 0] = 1.0  # performances_record divides by |true|
    out = {"proba": proba.numpy(), "true": true.numpy()}
    for alpha in (0.1, 0.3):
        pred = ns["protein_loc_correction"](proba, alpha)
        aim, cov, acc = ns["performances_record"](true, pred)
        out[f"pred_{alpha}"] = pred.numpy()
        out[f"perf_{alpha}"] = np.array([aim, cov, acc], np.float64)
    np.savez(os.path.join(HERE, "eval.npz"), **out)


def gen_ecc():
    sys.path.insert(0, REF)
    import data_preprocess as dp  # noqa: E402
    from scipy.sparse import coo_matrix

    cases = {}
    # triangle {0,1,2} + pendant 0-3 (SURVEY.md §4 probe)
    r = [0, 1, 0, 2, 1, 2, 0, 3]
    c = [1, 0, 2, 0, 2, 1, 3, 0]
    cases["tri"] = coo_matrix((np.ones(len(r), int), (r, c)), shape=(4, 4))
    rng = np.random.default_rng(7)
    n = 30
    a = rng.random((n, n)) < 0.15
    a = np.triu(a, 1)
    a = a | a.T
    rr, cc = np.nonzero(a)
    cases["rand30"] = coo_matrix((np.ones(len(rr), int), (rr, cc)), shape=(n, n))
    out = {}
    for k, m in cases.items():
        e = dp.edge_clustering_coefficients(m).toarray()
        out[f"{k}_adj"] = m.toarray().astype(np.int8)
        out[f"{k}_ecc"] = e
    np.savez(os.path.join(HERE, "ecc.npz"), **out)


if __name__ == "__main__":
    ns = _train_functions()
    gen_loss(ns)
    gen_eval(ns)
    gen_ecc()
    print("golden fixtures written to", HERE)
