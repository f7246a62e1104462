"""Generate tests/golden/dropin_cli.npz: what the reference's OWN, unmodified entry script
computes, to pin the drop-in path's composition on the GPU.

Run in the build container only (it reads /root/reference; the GPU box never runs it):
    python tests/golden/gen_dropin.py

The unmodified code/main_normal.py (which runs code/train.py, code/model.py and
code/utils.py) is executed from a scratch copy outside the repository, on this
repository's `dgl` package with `-d cpu` (the CPU device: the library's OpenMP message
passing, torch-CPU dense algebra), on a seeded synthetic dataset written in the
reference's artefact formats (plagnn.data.write_reference_layout). Seed 70
(main_normal.py:11-16), the reference's KFold rounds (train.py:162-178), GNN32 at the
reference dims (train.py:179), Adam lr 5e-5 (main_normal.py:26), multi_loss (train.py:
89-108). Only outputs are stored: every epoch's train / val loss of every (round, fold)
from its fig_data_<round>.json (train.py:351-357) and the final logits of three
(round, fold) pairs ({round}_{fold}_loc_logits.npy, train.py:289); and, from a second run
with -e 1 and -e 2 (the same models: -e does not change what the torch RNG draws), the
same pairs' logits of the first and second epoch, i.e. the forward at the initial
parameters and after one Adam step. No source is stored.
tests/test_gpu_dropin_cli.py replays the same seeds and folds through the shim on cuda.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

REF = "/root/reference/code"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(ROOT, "pla-gnn_amd")

N, MEAN_DEG, SEED = 1500, 12.0, 70
EPOCHS, FOLDS = 3, 2
LOGITS = [(1, 1), (1, 2), (10, 2)]


def main():
    sys.path.insert(0, PKG)
    from plagnn import data

    ds = data.make_dataset("s0", n=N, mean_deg=MEAN_DEG, seed=SEED)
    with tempfile.TemporaryDirectory() as tmp:
        code = os.path.join(tmp, "code")
        os.makedirs(code)
        for f in ("main_normal.py", "train.py", "model.py", "utils.py"):
            shutil.copy(os.path.join(REF, f), os.path.join(code, f))
        data.write_reference_layout(ds, tmp, gse="GSE30931")
        env = dict(os.environ, PYTHONPATH=PKG + os.pathsep + os.environ.get("PYTHONPATH", ""), MPLBACKEND="Agg")
        log = os.path.join(tmp, "data", "log", "GSE30931", "normal")

        def cli(epochs):
            shutil.rmtree(log, ignore_errors=True)
            r = subprocess.run([sys.executable, "main_normal.py", "-data", "GSE30931", "-d", "cpu", "-e", str(epochs),
                                "-f", str(FOLDS)], cwd=code, env=env, capture_output=True, text=True, timeout=3600)
            if r.returncode != 0:
                raise SystemExit(r.stderr[-4000:])

        cli(1)
        first = {p: np.load(os.path.join(log, f"{p[0]}_{p[1]}_loc_logits.npy")).astype(np.float32) for p in LOGITS}
        cli(2)  # the forward after ONE Adam step
        second = {p: np.load(os.path.join(log, f"{p[0]}_{p[1]}_loc_logits.npy")).astype(np.float32) for p in LOGITS}
        cli(EPOCHS)
        tl = np.zeros((10, FOLDS, EPOCHS), np.float64)
        vl = np.zeros((10, FOLDS, EPOCHS), np.float64)
        for rnd in range(1, 11):
            with open(os.path.join(log, f"fig_data_{rnd}.json")) as f:
                fig = json.load(f)
            (alpha,) = fig["train"].keys()
            for fold in range(1, FOLDS + 1):
                tl[rnd - 1, fold - 1] = fig["train"][alpha][str(fold)]["loss"]
                vl[rnd - 1, fold - 1] = fig["validation"][alpha][str(fold)]["loss"]
        out = {"n": N, "mean_deg": MEAN_DEG, "seed": SEED, "epochs": EPOCHS, "folds": FOLDS,
               "train_loss": tl, "val_loss": vl, "logits_at": np.array(LOGITS, np.int64)}
        for rnd, fold in LOGITS:
            out[f"logits_{rnd}_{fold}"] = np.load(os.path.join(log, f"{rnd}_{fold}_loc_logits.npy")).astype(np.float32)
            out[f"logits0_{rnd}_{fold}"] = first[(rnd, fold)]
            out[f"logits1_{rnd}_{fold}"] = second[(rnd, fold)]
    np.savez_compressed(os.path.join(HERE, "dropin_cli.npz"), **out)
    print("wrote dropin_cli.npz:", {k: getattr(v, "shape", v) for k, v in out.items()})


if __name__ == "__main__":
    main()
