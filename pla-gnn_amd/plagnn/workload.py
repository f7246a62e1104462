"""The benchmark workloads of BASELINE.json `configs`, built the same way
for bench.py and the full-size parity tests.

  cfg1   S0, 2 GraphConv layers of hidden 64 (BASELINE configs[0]; dgl GraphConv, norm
         'both'), then the reference's MLP head: not a configuration of the reference
         (its layers are SAGEConv 'pool'), reference-unpinned
  cfg2   S0 PPI stand-in (N = 24 041, mean degree 50), SAGE-pool 503 -> 256 x 3, fp32
  ref    S0, the reference's own dims GNN32(503, 400, 300, 200, 100, 12) (code/train.py:179)
  cfg3   GSE30931's PPI_inter of S0 (pg_perturb with the dataset's threshold,
         code/data_preprocess.py:217-257, 498), ECC of that graph (pg_ecc,
         code/data_preprocess.py:175-214) as u_mul_e edge weights, hidden 512, fp32
  cfg4   the perturbation replicas of main_inter.py: rank r trains variant r % 4 —
         0 the normal graph, 1-3 <GSE>/PPI_inter for GSE30931 / GSE27182 / GSE74572, each
         built by pg_perturb (modify_network_topology, code/data_preprocess.py:217-257)
         with that dataset's threshold — and the gradients are averaged over ranks
  cfg5   RMAT x16 (N = 384 656), hidden 512, bf16 storage with f32 accumulation

Every rank draws the same synthetic base data (seed 70, code/main_normal.py:11) and the
same initial parameters; only the graph differs between cfg4's variants. The training
rows are round 1, fold 1 of the reference's KFold loop (code/train.py:162-178).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from . import data
from .graph import CSRGraph
from .train import FOLD_SEEDS, fold_splits, weight_cal

CONFIGS = {
    # name: (graph kind, dims, bf16, description)
    "cfg1": ("s0", [503, 64, 64, 100, 12], False,
             "S0 PPI stand-in, 2x GraphConv (norm both) hidden 64 + MLP 64 -> 100 -> 12, fp32"),
    "cfg2": ("s0", [503, 256, 256, 256, 100, 12], False,
             "S0 PPI stand-in (N=24041, mean deg 50), 3x SAGE-pool hidden 256, fp32"),
    "ref": ("s0", [503, 400, 300, 200, 100, 12], False,
            "S0 PPI stand-in, reference dims GNN32(503,400,300,200,100,12), fp32"),
    "cfg3": ("s0", [503, 512, 512, 512, 100, 12], False,
             "GSE30931 PPI_inter of S0 (pg_perturb, thr 2.75), ECC_inter edge weights (pg_ecc, u_mul_e max), "
             "hidden 512, fp32"),
    "cfg4": ("s0", [503, 400, 300, 200, 100, 12], False,
             "normal S0 + PPI_inter replicas of GSE30931/GSE27182/GSE74572 (pg_perturb, the reference "
             "thresholds), one graph per rank (rank % 4), reference dims, grad all-reduce"),
    "cfg5": ("rmat", [503, 512, 512, 512, 100, 12], True,
             "RMAT x16 PPI (N=384656, a,b,c,d=.57,.19,.19,.05, mean deg 50), hidden 512, bf16 storage, "
             "f32 accumulate"),
    "cfg5-f32": ("rmat", [503, 512, 512, 512, 100, 12], False,
                 "RMAT x16 PPI (N=384656, a,b,c,d=.57,.19,.19,.05, mean deg 50), hidden 512, fp32"),
}
CFG4_VARIANTS = ["normal"] + list(data.GSE_THRESHOLDS)
CONV = {"cfg1": "graphconv"}  # the graph layer of each config (default: SAGEConv 'pool')


@dataclass
class Workload:
    name: str
    dims: List[int]
    bf16: bool
    desc: str
    ds: data.Dataset
    src: np.ndarray            # COO with DGL's self-loops appended (edge ids E..E+N-1)
    dst: np.ndarray
    edge_weight: Optional[torch.Tensor]  # per edge id (self-loops 1.0), or None
    variant: str
    train_index: List[int]
    val_index: List[int]
    class_weight: np.ndarray
    conv: str = "pool"

    def graph(self) -> CSRGraph:
        return CSRGraph(self.src, self.dst, self.ds.n)

    @property
    def n(self) -> int:
        return self.ds.n

    def edges_without_loops(self):
        """(src, dst, weight) before add_self_loop — the oracle appends the loops itself."""
        e = len(self.src) - self.ds.n
        w = None if self.edge_weight is None else self.edge_weight.numpy()[:e]
        return self.src[:e], self.dst[:e], w


def _with_loops(row, col, n, w=None):
    loops = np.arange(n, dtype=np.int64)
    src = np.concatenate([np.asarray(row, np.int64), loops])
    dst = np.concatenate([np.asarray(col, np.int64), loops])
    ew = None
    if w is not None:
        ew = torch.from_numpy(np.concatenate([np.asarray(w, np.float32), np.ones(n, np.float32)]))
    return src, dst, ew


def ecc_weights(row, col, n, device="cuda") -> np.ndarray:
    """ECC of the (symmetric) graph at every directed edge, float32 (pg_ecc)."""
    from scipy.sparse import coo_matrix

    from . import ecc

    a = coo_matrix((np.ones(len(row), np.int64), (row, col)), shape=(n, n))
    e = ecc.edge_clustering_coefficients(a, device=device).tocsr()
    return np.asarray(e[row, col]).ravel().astype(np.float32)


def perturbed_graph(ds: data.Dataset, gse: str, device="cuda"):
    """<GSE>/PPI_inter of the synthetic dataset: pg_perturb with the dataset's threshold on
    the normal and the synthetic intervention expression (data.intervention_expression)."""
    from scipy.sparse import coo_matrix

    from . import perturb

    ppi = coo_matrix((np.ones(len(ds.row), np.int64), (ds.row, ds.col)), shape=(ds.n, ds.n))
    inter = data.intervention_expression(ds, gse)
    res = perturb.modify_network_topology_expr(ppi, ds.expr, inter, data.GSE_THRESHOLDS[gse], device=device)
    return res.row.astype(np.int64), res.col.astype(np.int64)


def fold_job(label, job: int):
    """The reference's training job `job` of its rounds x folds loop (code/train.py:162-178,
    10 folds): round job // 10 (KFold seed FOLD_SEEDS[round]), fold job % 10."""
    rnd, fold = divmod(int(job), 10)
    splits = fold_splits(label, 10, FOLD_SEEDS[rnd % len(FOLD_SEEDS)])
    for _ in range(fold):
        next(splits)
    return next(splits)


def build(name: str, rank: int = 0, device="cuda", n: Optional[int] = None, job: int = 0) -> Workload:
    """The workload of BASELINE config `name` for `rank` (n overrides the node count, for
    reduced-size parity cases of the same construction; job selects the (round, fold) of
    the train / val rows, fold_job; 0 = round 1, fold 1)."""
    kind, dims, bf16, desc = CONFIGS[name]
    ds = data.make_dataset(kind, n=n, seed=70)
    label = [int(i) for i in ds.labelled]
    train_idx, val_idx = fold_job(label, job)
    w = weight_cal(ds.loc)
    variant = "normal"
    ew = None
    if name == "cfg3":
        row, col = perturbed_graph(ds, "GSE30931", device)
        src, dst, ew = _with_loops(row, col, ds.n, ecc_weights(row, col, ds.n, device))
        variant = "GSE30931+ecc"
    elif name == "cfg4":
        variant = CFG4_VARIANTS[rank % len(CFG4_VARIANTS)]
        if variant == "normal":
            src, dst = ds.edges_with_self_loops()
        else:
            row, col = perturbed_graph(ds, variant, device)
            src, dst, _ = _with_loops(row, col, ds.n)
    else:
        src, dst = ds.edges_with_self_loops()
    return Workload(name, list(dims), bf16, desc, ds, src, dst, ew, variant, train_idx, val_idx, w,
                    CONV.get(name, "pool"))
