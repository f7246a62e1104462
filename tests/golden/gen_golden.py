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
is called directly, and so are
    construct_gcn_matrix          code/data_preprocess.py:128-172 (on a synthetic GEO-style CSV)
    modify_network_topology       code/data_preprocess.py:217-257
Only the produced input/output arrays are committed (no source).
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


def gen_perturb():
    """Reference end to end: a GEO-style expression CSV (duplicate ids averaged, ids not in
    the PPI dropped, PPI proteins missing from the CSV zero-filled) -> construct_gcn_matrix
    for both states -> modify_network_topology. Stored: the expression matrices it returns
    (our drop-in's input), the PPI, and the perturbed PPI; plus diff's mean / std."""
    import tempfile

    import pandas as pd
    from scipy.sparse import coo_matrix

    sys.path.insert(0, REF)
    import data_preprocess as dp  # noqa: E402

    out = {}
    for name, n, p_edge, thr, seed in (("small", 60, 0.12, 1.0, 5), ("mid", 400, 0.05, 1.5, 6)):
        rng = np.random.default_rng(seed)
        ids = [f"P{i:05d}" for i in range(n)]
        normal = ["GSM1", "GSM2", "GSM3"]
        inter = ["GSM4", "GSM5", "GSM6"]
        rows = []
        for i, pid in enumerate(ids):
            if rng.random() < 0.2:
                continue  # protein absent from the expression set -> zero row
            for _ in range(1 + int(rng.random() < 0.15)):  # some ids measured twice
                rows.append([pid] + list(rng.lognormal(1.0, 1.0, 6)))
        rows.append(["XNOTPPI"] + list(rng.lognormal(1.0, 1.0, 6)))  # not in the PPI
        df = pd.DataFrame(rows, columns=["uniprot_id"] + normal + inter)
        with tempfile.TemporaryDirectory() as td:
            csv = os.path.join(td, "expr.csv")
            df.to_csv(csv, index=False)
            gcn_n, expr_n = dp.construct_gcn_matrix(csv, normal, ids)
            gcn_i, expr_i = dp.construct_gcn_matrix(csv, inter, ids)
        a = np.triu(rng.random((n, n)) < p_edge, 1)
        a = a | a.T
        r, c = np.nonzero(a)
        data = np.ones(len(r), np.int64)
        if name == "small":  # one duplicated edge: value 2 after tocsr(), untouched by both rules
            r, c, data = np.append(r, r[0]), np.append(c, c[0]), np.append(data, 1)
        ppi = coo_matrix((data, (r, c)), shape=(n, n))
        res = dp.modify_network_topology(ppi, gcn_n, gcn_i, thr).tocoo()
        diff = gcn_i.tocsr() - gcn_n.tocsr()
        diff = diff.toarray()
        out[f"{name}_expr_normal"] = np.asarray(expr_n, np.float64)
        out[f"{name}_expr_inter"] = np.asarray(expr_i, np.float64)
        out[f"{name}_ppi_row"], out[f"{name}_ppi_col"], out[f"{name}_ppi_val"] = ppi.row, ppi.col, ppi.data
        out[f"{name}_thr"] = np.float64(thr)
        out[f"{name}_out_row"], out[f"{name}_out_col"] = res.row, res.col
        out[f"{name}_out_val"] = np.asarray(res.data, np.int64)
        out[f"{name}_mean_std"] = np.array([np.mean(diff), np.std(diff)])
        out[f"{name}_pcc_normal"] = gcn_n.toarray() if n <= 60 else np.zeros(0)
    np.savez_compressed(os.path.join(HERE, "perturb.npz"), **out)


def gen_pca():
    """The reference's own pca() (code/data_preprocess.py:475-487) on an ECC matrix made by its
    own edge_clustering_coefficients (175-214), as at 528-530. scikit-learn here is 1.7.2
    (the reference pins 1.1.1): the randomized SVD it runs is the same algorithm (Gaussian
    test matrix from RandomState(42), 7 LU-normalised power iterations, QR, SVD of the
    projection), but 1.7.2's PCA flips signs by V (u_based_decision=False) where 1.1.1 flips
    by U; the fixture therefore pins the columns up to sign, and the stored u-based sign is
    1.1.1's rule applied to these columns."""
    from scipy.sparse import coo_matrix

    sys.path.insert(0, REF)
    import data_preprocess as dp  # noqa: E402

    rng = np.random.default_rng(2023)
    n, nc = 800, 30
    a = np.triu(rng.random((n, n)) < 0.02, 1)
    a = a | a.T
    r, c = np.nonzero(a)
    ppi = coo_matrix((np.ones(len(r), np.int64), (r, c)), shape=(n, n))
    ecc = dp.edge_clustering_coefficients(ppi).tocoo()
    feat = dp.pca(ecc.toarray(), nc)
    np.savez_compressed(os.path.join(HERE, "pca.npz"), n=np.int64(n), nc=np.int64(nc), row=ecc.row,
                        col=ecc.col, val=ecc.data.astype(np.float64), out=feat)


if __name__ == "__main__":
    only = sys.argv[1:]
    if not only or "train" in only:
        ns = _train_functions()
        gen_loss(ns)
        gen_eval(ns)
    if not only or "ecc" in only:
        gen_ecc()
    if not only or "perturb" in only:
        gen_perturb()
    if not only or "pca" in only:
        gen_pca()
    print("golden fixtures written to", HERE)
