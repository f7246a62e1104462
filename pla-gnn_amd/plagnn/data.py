"""Synthetic stand-ins for the PLA-GNN inputs, in the reference's formats.

The reference's real inputs (BioGRID PPI, GEO expression, UniProt labels) are downloads
that are not in /root/reference (``data/PPI.7z`` is a missing blob), so every benchmark
and test here runs on seeded synthetic data with the same shapes and storage formats:

  PPI_*.npz            scipy COO, int ones, symmetric, no diagonal   (data_preprocess.py:106-110)
  ECC_*_pca.npy        N x 250 float64                                (data_preprocess.py:528-546)
  GCN_*_pca.npy        N x 250 float64
  expr_*.npy           N x 3 float64                                  (data_preprocess.py:166-172)
  loc_matrix.npz       COO float64 N x 12                             (data_preprocess.py:433-447)
  protein_ppi.json     N protein ids                                  (main_normal.py:62)
  label_list.json      [[id, [GO ids]], ...]                          (train.py:128-129)
  label_with_loc_list.json  row ids with at least one location        (train.py:154-155)

Graph models: S0 = Chung-Lu power law (mean degree 50, exponent 2.1, degree cap 5000);
RMAT (a, b, c, d) = (0.57, 0.19, 0.19, 0.05) for the x16 scale config.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

N_PPI = 24041      # code/main.py:40, code/performance.py:99
N_CLASSES = 12     # code/train.py:179
N_PCA = 250        # data_preprocess.py:530
GO_IDS = ["GO:0005576", "GO:0005634", "GO:0005737", "GO:0005739", "GO:0005783", "GO:0005794",
          "GO:0005886", "GO:0005773", "GO:0005777", "GO:0005856", "GO:0005829", "GO:0005730"]


def _symmetrize_unique(a: np.ndarray, b: np.ndarray, n: int):
    keep = a != b
    a, b = a[keep], b[keep]
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    key = np.unique(lo.astype(np.int64) * n + hi)
    lo, hi = key // n, key % n
    return lo, hi


def chung_lu(n: int, mean_deg: float = 50.0, gamma: float = 2.1, max_deg: int = 5000,
             seed: int = 70):
    """Undirected power-law graph; returns (row, col) of the symmetric directed edge list
    (each undirected edge twice, no self-loops), in a shuffled order."""
    rng = np.random.default_rng(seed)
    w = (np.arange(n) + 1.0) ** (-1.0 / (gamma - 1.0))
    for _ in range(4):
        w = w / w.mean() * mean_deg
        w = np.minimum(w, max_deg)
    p = w / w.sum()
    target = n * mean_deg / 2.0
    m = int(target * 1.05)
    lo = hi = np.zeros(0, np.int64)
    for _ in range(6):
        a = rng.choice(n, m, p=p)
        b = rng.choice(n, m, p=p)
        lo, hi = _symmetrize_unique(np.concatenate([a, lo]), np.concatenate([b, hi]), n)
        if len(lo) >= target:
            break
        m = int((target - len(lo)) * 1.3) + 1
    if len(lo) > target:
        sel = rng.choice(len(lo), int(target), replace=False)
        lo, hi = lo[sel], hi[sel]
    perm = rng.permutation(n)  # hubs are not all low ids
    lo, hi = perm[lo], perm[hi]
    row = np.concatenate([lo, hi])
    col = np.concatenate([hi, lo])
    order = rng.permutation(len(row))  # BioGRID set-iteration order is arbitrary
    return row[order].astype(np.int32), col[order].astype(np.int32)


def rmat(n: int, mean_deg: float = 50.0, abcd=(0.57, 0.19, 0.19, 0.05), seed: int = 70):
    """Undirected RMAT graph restricted to n nodes (symmetric, no self-loops)."""
    rng = np.random.default_rng(seed)
    levels = int(np.ceil(np.log2(n)))
    target = n * mean_deg / 2.0
    a, b, c, _ = abcd
    lo = hi = np.zeros(0, np.int64)
    m = int(target * 1.25)
    for _ in range(6):
        u = np.zeros(m, np.int64)
        v = np.zeros(m, np.int64)
        for _lv in range(levels):
            r = rng.random(m)
            bit_u = (r >= a + b).astype(np.int64)               # quadrants c, d
            bit_v = (((r >= a) & (r < a + b)) | (r >= a + b + c)).astype(np.int64)  # b, d
            u = (u << 1) | bit_u
            v = (v << 1) | bit_v
        keep = (u < n) & (v < n)
        lo, hi = _symmetrize_unique(np.concatenate([u[keep], lo]), np.concatenate([v[keep], hi]), n)
        if len(lo) >= target:
            break
        m = int((target - len(lo)) * 1.6) + 1
    if len(lo) > target:
        sel = rng.choice(len(lo), int(target), replace=False)
        lo, hi = lo[sel], hi[sel]
    perm = rng.permutation(n)
    lo, hi = perm[lo], perm[hi]
    row = np.concatenate([lo, hi])
    col = np.concatenate([hi, lo])
    order = rng.permutation(len(row))
    return row[order].astype(np.int32), col[order].astype(np.int32)


def features(n: int, seed: int = 70):
    """expr (N x 3, lognormal, 30 % rows zero), gcn_pca and ecc_pca (N x 250, PCA-like
    spectra), all float64 like the reference's .npy artefacts."""
    rng = np.random.default_rng(seed + 1)
    expr = rng.lognormal(1.0, 1.0, size=(n, 3))
    expr[rng.random(n) < 0.3] = 0.0
    sig = 1.0 / np.sqrt(np.arange(1, N_PCA + 1))
    gcn = rng.standard_normal((n, N_PCA)) * sig
    ecc = rng.standard_normal((n, N_PCA)) * sig * 0.5
    return expr, gcn, ecc


def labels(n: int, seed: int = 70, labelled_frac: float = 0.5):
    """loc matrix (N x 12 {0,1}) with ~labelled_frac rows labelled (1-3 locations)."""
    rng = np.random.default_rng(seed + 2)
    loc = np.zeros((n, N_CLASSES), np.float64)
    lab = rng.random(n) < labelled_frac
    prior = np.linspace(2.0, 0.5, N_CLASSES)
    prior /= prior.sum()
    for i in np.nonzero(lab)[0]:
        k = 1 + int(rng.random() < 0.35) + int(rng.random() < 0.1)
        loc[i, rng.choice(N_CLASSES, k, replace=False, p=prior)] = 1.0
    return loc


@dataclass
class Dataset:
    n: int
    row: np.ndarray
    col: np.ndarray
    expr: np.ndarray
    gcn: np.ndarray
    ecc: np.ndarray
    loc: np.ndarray

    @property
    def feat(self) -> np.ndarray:
        """hstack(expr, gcn, ecc) as float32: code/utils.py:47-48."""
        return np.hstack((self.expr, np.hstack((self.gcn, self.ecc)))).astype(np.float32)

    @property
    def labelled(self) -> np.ndarray:
        return np.nonzero(self.loc.sum(1) > 0)[0]

    def edges_with_self_loops(self):
        """COO src/dst of dgl.add_self_loop(dgl.graph((row, col), N)) (utils.py:44-45)."""
        loops = np.arange(self.n)
        return (np.concatenate([self.row.astype(np.int64), loops]),
                np.concatenate([self.col.astype(np.int64), loops]))


def make_dataset(kind: str = "s0", n: Optional[int] = None, seed: int = 70,
                 mean_deg: float = 50.0) -> Dataset:
    if kind == "s0":
        n = N_PPI if n is None else n
        row, col = chung_lu(n, mean_deg=mean_deg, max_deg=min(5000, max(8, n // 4)), seed=seed)
    elif kind == "rmat":
        n = 16 * N_PPI if n is None else n
        row, col = rmat(n, mean_deg=mean_deg, seed=seed)
    else:
        raise ValueError(kind)
    expr, gcn, ecc = features(n, seed)
    return Dataset(n, row, col, expr, gcn, ecc, labels(n, seed))


def random_perturbation(ds: Dataset, seed: int, frac: float = 0.03):
    """SURVEY.md §8d cfg3 topology: about `frac` of the undirected edges removed and as many
    random ones added (the size of a ΔPCC-style change, code/data_preprocess.py:217-257).
    Returns the symmetric (row, col) int64 edge list, no self-loops, no duplicates."""
    rng = np.random.default_rng(seed)
    n = ds.n
    r, c = ds.row.astype(np.int64), ds.col.astype(np.int64)
    up = r < c
    ur, uc = r[up], c[up]
    keep = rng.random(len(ur)) >= frac
    na = int((~keep).sum())
    ar, ac = rng.integers(0, n, na), rng.integers(0, n, na)
    lo, hi = _symmetrize_unique(np.concatenate([ur[keep], ar]), np.concatenate([uc[keep], ac]), n)
    return np.concatenate([lo, hi]), np.concatenate([hi, lo])


# The three drug datasets of the reference and their ΔPCC thresholds
# (code/data_preprocess.py:498, 511, 520); main_inter.py trains on <GSE>/PPI_inter.npz.
GSE_THRESHOLDS = {"GSE30931": 2.75, "GSE27182": 2.99, "GSE74572": 2.91}


def intervention_expression(ds: Dataset, gse: str, n_genes: int = 2) -> np.ndarray:
    """Synthetic 'intervention' expression for one dataset: the normal expression with
    `n_genes` expressed genes (seeded by the GSE number) rescaled per sample by
    exp(N(0, 1)). With the reference's thresholds every such gene moves about 0.3 N
    correlation pairs past mean ± thr·std, so two genes change about 2-3 % of S0's edges
    (measured on the reference's own operations at N = 3 000)."""
    rng = np.random.default_rng(int(gse[3:]))
    expressed = np.nonzero(ds.expr.sum(1) > 0)[0]
    genes = rng.choice(expressed, n_genes, replace=False)
    inter = ds.expr.copy()
    inter[genes] *= np.exp(rng.standard_normal((n_genes, ds.expr.shape[1])))
    return inter


def write_reference_layout(ds: Dataset, root: str, gse: str = "GSE30931") -> None:
    """Write ds under root/data/generate_materials/ exactly where main_normal.py /
    main_inter.py / train.py read (code/main_normal.py:57-63, code/train.py:128, 151, 154)."""
    from scipy import sparse

    gm = os.path.join(root, "data", "generate_materials")
    gd = os.path.join(gm, f"{gse}_data")
    os.makedirs(gd, exist_ok=True)
    ppi = sparse.coo_matrix((np.ones(len(ds.row), np.int64), (ds.row, ds.col)), shape=(ds.n, ds.n))
    sparse.save_npz(os.path.join(gm, "PPI_normal.npz"), ppi)
    sparse.save_npz(os.path.join(gd, "PPI_inter.npz"), ppi)
    np.save(os.path.join(gm, "ECC_normal_pca.npy"), ds.ecc)
    for name in ("GCN_normal_pca", "GCN_inter_pca"):
        np.save(os.path.join(gd, name + ".npy"), ds.gcn)
    np.save(os.path.join(gd, "ECC_inter_pca.npy"), ds.ecc)
    for name in ("expr_normal", "expr_inter"):
        np.save(os.path.join(gd, name + ".npy"), ds.expr)
    sparse.save_npz(os.path.join(gm, "loc_matrix.npz"), sparse.coo_matrix(ds.loc))
    ids = [f"P{i:05d}" for i in range(ds.n)]
    with open(os.path.join(gm, "protein_ppi.json"), "w") as f:
        json.dump(ids, f)
    label_list = [[ids[i], [GO_IDS[c] for c in np.nonzero(ds.loc[i])[0]]] for i in range(ds.n)]
    with open(os.path.join(gm, "label_list.json"), "w") as f:
        json.dump(label_list, f)
    with open(os.path.join(gm, "label_with_loc_list.json"), "w") as f:
        json.dump([int(i) for i in ds.labelled], f)
    os.makedirs(os.path.join(root, "data", "log"), exist_ok=True)
