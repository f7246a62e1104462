"""§8f rank 3: per-epoch evaluation on the GPU vs the reference's own outputs
(tests/golden/eval.npz, made by running code/train.py:19-86) and vs the oracle at the
full S0 size (N = 24,041 rows)."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(ROOT, "tests", "golden", "eval.npz")


@pytest.mark.parametrize("alpha", [0.1, 0.3])
def test_eval_matches_reference_golden(alpha):
    from plagnn import loc_eval

    d = np.load(GOLD)
    pred = loc_eval.protein_loc_correction(torch.from_numpy(d["proba"]).to(DEV), alpha)
    np.testing.assert_array_equal(pred.cpu().numpy(), d[f"pred_{alpha}"])
    perf = np.array(loc_eval.performances_record(torch.from_numpy(d["true"]).to(DEV), pred), np.float64)
    np.testing.assert_array_equal(perf, d[f"perf_{alpha}"])


@pytest.mark.parametrize("alpha", [0.0, 0.2, 0.5])
def test_eval_matches_oracle_full_size(oracle_mod, alpha):
    from plagnn import loc_eval

    rng = np.random.default_rng(5)
    n, C = 24041, 12
    proba = torch.from_numpy(rng.random((n, C)).astype(np.float32))
    true = torch.from_numpy((rng.random((n, C)) < 0.2).astype(np.float32))
    true[true.sum(1) == 0, 3] = 1.0
    pred = loc_eval.protein_loc_correction(proba.to(DEV), alpha)
    ref = oracle_mod.protein_loc_correction(proba, alpha)
    np.testing.assert_array_equal(pred.cpu().numpy(), ref.numpy())
    got = loc_eval.performances_record(true.to(DEV), pred)
    exp = oracle_mod.performances_record(true, ref)
    np.testing.assert_array_equal(np.array(got), np.array(exp))
