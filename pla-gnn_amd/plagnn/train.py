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
