"""§8f rows measured on the S0 stand-in: edge clustering coefficient (pg_ecc) and the
per-epoch evaluation (pg_loc_correction + pg_loc_performance), each against its CPU
restatement in oracle/ (the reference's own algorithms) on the same host. Prints one JSON
line per row. Usage (GPU box): python scripts/bench_f8.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402
from scipy.sparse import coo_matrix  # noqa: E402

import oracle  # noqa: E402  (CPU baseline leg only)
from plagnn import _lib, data, ecc, loc_eval  # noqa: E402
from plagnn._lib import call, ptr  # noqa: E402


def hip_time(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps / 1e3


def main():
    ds = data.make_dataset("s0", seed=70)
    src, dst = ds.row.astype(np.int64), ds.col.astype(np.int64)  # symmetric, no diagonal (the PPI form)
    n = ds.n
    adj = coo_matrix((np.ones(len(src), np.int64), (src, dst)), shape=(n, n))
    csr, indptr, indices, mirror, deg, order, rows = ecc.prepare(adj)
    nnz = len(indices)
    dev = torch.device("cuda")
    t = {k: torch.from_numpy(v).to(dev) for k, v in
         (("ptr", indptr), ("col", indices), ("mirror", mirror), ("deg", deg), ("order", order))}
    out = torch.empty(nnz, dtype=torch.float64, device=dev)
    st = _lib.stream_handle(dev)

    def run():
        call("pg_ecc", ptr(t["ptr"]), ptr(t["col"]), ptr(t["mirror"]), ptr(t["deg"]), ptr(t["order"]), n, nnz,
             0.0, ptr(out), st)
    sec = hip_time(run)
    tests = float(np.minimum(np.diff(indptr)[rows], np.diff(indptr)[indices]).sum()) / 2  # bit tests
    t0 = time.perf_counter()
    ref = oracle.edge_clustering_coefficients(adj)
    cpu = time.perf_counter() - t0
    got = ecc.edge_clustering_coefficients(adj)
    exact = bool(np.array_equal(got.toarray(), ref.toarray()))
    print(json.dumps({"row": "8f-2 edge clustering coefficient", "n": n, "stored_edges": nnz,
                      "gpu_ms": round(sec * 1e3, 3), "edges_per_s": round(nnz / sec, 1),
                      "bit_tests_per_s": round(tests / sec, 1),
                      "cpu_baseline": {"ms": round(cpu * 1e3, 1), "edges_per_s": round(nnz / cpu, 1), "cores": 1,
                                       "kind": "port", "sample": "oracle/ecc_oracle.c on the same graph"},
                      "bit_exact_vs_oracle": exact}))

    rng = np.random.default_rng(3)
    C = 12
    proba = torch.from_numpy(rng.random((n, C)).astype(np.float32))
    true = torch.from_numpy(ds.loc.astype(np.float32))
    lab = torch.from_numpy(np.asarray(ds.labelled, np.int64))
    pd_, td = proba.to(dev), true[lab].to(dev)

    def ev():
        pred = loc_eval.protein_loc_correction(pd_, 0.1)
        return loc_eval.performances_record(td, pred[lab.to(dev)])
    sec = hip_time(ev, reps=5)
    t0 = time.perf_counter()
    pred_ref = oracle.protein_loc_correction(proba, 0.1)
    perf_ref = oracle.performances_record(true[lab], pred_ref[lab])
    cpu = time.perf_counter() - t0
    print(json.dumps({"row": "8f-3 per-epoch eval (protein_loc_correction + performances_record)",
                      "rows": n, "labelled": int(len(lab)), "gpu_ms": round(sec * 1e3, 3),
                      "cpu_baseline": {"ms": round(cpu * 1e3, 1), "cores": 1, "kind": "port",
                                       "sample": "oracle torch-CPU restatement, per-row Python loop as train.py:60-78"},
                      "matches_oracle": list(ev()) == list(perf_ref)}))


if __name__ == "__main__":
    main()
