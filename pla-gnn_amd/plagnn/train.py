"""Host-side mirror of code/train.py's training-loop helpers (same names, arguments and
results), used by TrainEngine callers and the benchmark.

  weight_cal(loc_mat)            code/train.py:111-126
  multi_loss(input, target, w)   code/train.py:89-108 (autograd form, for the drop-in path;
                                 the engine uses the fused pg_sigmoid_multi_loss kernel)
  fold_splits(label, fold_num)   code/train.py:162-178: KFold(n_splits, shuffle, random_state
                                 = fseed) over the labelled-node list, mapped to node ids
"""
from __future__ import annotations

from typing import Iterator, List, Sequence, Tuple

import numpy as np
import torch

FOLD_SEEDS = [12, 22, 32, 42, 52, 62, 72, 82, 92, 100]  # code/train.py:162


def weight_cal(loc_mat: np.ndarray) -> np.ndarray:
    class_num = loc_mat.sum(axis=0)
    sample_num = int((loc_mat.sum(axis=1) != 0).sum())
    return (sample_num - class_num) / class_num


def multi_loss(input: torch.Tensor, target: torch.Tensor, i_weight) -> torch.Tensor:
    loss = 0
    for i in range(len(i_weight)):
        x = input[:, i]
        t = target[:, i]
        s = (t * torch.log(torch.clamp(x, 1e-9, 10.)) * i_weight[i]
             + (1 - t) * torch.log(torch.clamp(1 - x, 1e-9, 10.))) / (i_weight[i] + 1) * 2
        loss += -s.sum() / len(input)
    return loss


def fold_splits(label: Sequence[int], fold_num: int, fseed: int
                ) -> Iterator[Tuple[List[int], List[int]]]:
    from sklearn.model_selection import KFold

    kfold = KFold(n_splits=fold_num, random_state=fseed, shuffle=True)
    for train_idx, val_idx in kfold.split(label):
        yield [label[i] for i in train_idx], [label[i] for i in val_idx]


def loc_correction_per_row(loc_proba: torch.Tensor, alpha: float) -> torch.Tensor:
    """code/train.py:19-39 as the reference runs it on the logits' own device: the column
    min/max scaling and the row normalisation there, then ITS per-row Python loop (36-38)
    filling a CPU matrix one row at a time (each row's mask comes back from the device: the
    transfer torch 1.10 made implicitly is explicit here). Same result as
    plagnn.loc_eval.protein_loc_correction; this is the cost a drop-in user pays."""
    min_p = loc_proba.min(dim=0).values
    max_p = loc_proba.max(dim=0).values
    new_p = (loc_proba - min_p) / (max_p - min_p)
    new_p = new_p / new_p.sum(dim=1).reshape(-1, 1)
    loc_pred = torch.zeros(loc_proba.shape)
    rmax = new_p.max(dim=1).values
    thresholds = rmax - (rmax - new_p.min(dim=1).values) * alpha
    for row in range(len(loc_proba)):
        loc_pred[row][(new_p[row] > thresholds[row]).cpu()] = 1.
    return loc_pred.double()


def performances_per_row(loc_true: torch.Tensor, loc_pred: torch.Tensor):
    """code/train.py:42-86 as the reference runs it: both matrices to the host (52-53), then
    its per-row loop of small tensor operations with float32 running sums (60-78)."""
    t = loc_true.clone().detach().long().cpu()
    p = loc_pred.clone().detach().long().cpu()
    ones = torch.ones(t.shape[1], dtype=torch.long)
    aim = cov = acc = 0.
    for i in range(len(t)):
        t[i] = torch.eq(ones, t[i])
        p[i] = torch.eq(ones, p[i])
        both = (t[i] & p[i]).sum().float()
        pred = p[i].sum().float()
        either = (t[i] | p[i]).sum().float()
        if pred != 0:
            aim = aim + both / pred
        cov = cov + both / t[i].sum().float()
        acc = acc + both / either
    n = len(t)
    return float(aim / n), float(cov / n), float(acc / n)
