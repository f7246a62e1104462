"""Per-epoch evaluation on the GPU: drop-ins for the reference's
``protein_loc_correction(loc_proba, alpha)`` and ``performances_record(loc_true,
loc_pred)`` (code/train.py:19-86), which run as Python loops over the rows with a host
copy every epoch (train.py:210-214). Same inputs and outputs; the work is three HIP
kernels (``pg_loc_correction``, ``pg_loc_performance``)."""
from __future__ import annotations

from typing import Tuple

import torch

from . import _lib
from ._lib import call, ptr


def _ws(n: int, C: int, device) -> torch.Tensor:
    return torch.empty(int(_lib.lib().pg_loc_eval_workspace(n, C)), dtype=torch.uint8, device=device)


def protein_loc_correction(loc_proba: torch.Tensor, alpha: float) -> torch.Tensor:
    """Location prediction matrix (float64, 0/1) of code/train.py:19-39."""
    if loc_proba.device.type != "cuda":
        raise ValueError("protein_loc_correction: GPU entry point")
    p = loc_proba.detach().to(torch.float32).contiguous()
    n, C = p.shape
    pred = torch.empty(n, C, dtype=torch.float64, device=p.device)
    call("pg_loc_correction", ptr(p), C, n, C, float(alpha), ptr(pred), C, ptr(_ws(n, C, p.device)),
         int(_lib.lib().pg_loc_eval_workspace(n, C)), _lib.stream_handle(p.device))
    return pred


def performances_record(loc_true: torch.Tensor, loc_pred: torch.Tensor) -> Tuple[float, float, float]:
    """(aim, coverage, accuracy) of code/train.py:42-86."""
    t = loc_true.detach().to(torch.float32).contiguous()
    pr = loc_pred.detach().to(device=t.device, dtype=torch.float64).contiguous()
    n, C = t.shape
    out = torch.empty(3, dtype=torch.float64, device=t.device)
    call("pg_loc_performance", ptr(t), C, ptr(pr), C, n, C, ptr(out), ptr(_ws(n, C, t.device)),
         int(_lib.lib().pg_loc_eval_workspace(n, C)), _lib.stream_handle(t.device))
    a, c, r = out.cpu().tolist()
    return a, c, r
