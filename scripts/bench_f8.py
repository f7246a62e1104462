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
from plagnn import _lib, data, ecc, loc_eval, perturb  # noqa: E402
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

    # 8f-4: topology perturbation (normal vs intervention expression, N x 3 like the GEO sets)
    en = ds.expr
    ei = en * np.random.default_rng(4).lognormal(0.0, 0.5, en.shape)
    ei[np.random.default_rng(5).random(n) < 0.05] = 0.0
    thr = 2.2
    perturb.modify_network_topology_expr(adj, en, ei, thr)  # warm-up (module load, first launch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    got, pst = perturb.modify_network_topology_expr(adj, en, ei, thr, return_stats=True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # the four device passes alone (sd, sum, sum of squares, count, fill), HIP events
    xn, xi = perturb._centred(en), perturb._centred(ei)
    tx, ti = torch.from_numpy(xn).to(dev), torch.from_numpy(xi).to(dev)
    sdn, sdi = torch.empty(n, dtype=torch.float64, device=dev), torch.empty(n, dtype=torch.float64, device=dev)
    wsp = torch.empty(int(_lib.lib().pg_perturb_workspace(n)), dtype=torch.uint8, device=dev)
    tot = torch.zeros(2, dtype=torch.float64, device=dev)
    pc = adj.tocsr()
    pc.sort_indices()
    tp, tc = torch.from_numpy(pc.indptr.astype(np.int32)).to(dev), torch.from_numpy(pc.indices.astype(np.int32)).to(dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(np.diff(got.tocsr().indptr), out=offs[1:])
    to = torch.from_numpy(offs).to(dev)
    oc = torch.empty(max(got.nnz, 1), dtype=torch.int32, device=dev)
    ov = torch.empty(max(got.nnz, 1), dtype=torch.int64, device=dev)
    base = (ptr(tx), ptr(ti), ptr(sdn), ptr(sdi), n, 3, 0.5)

    def passes():
        call("pg_perturb_prepare", ptr(tx), ptr(ti), n, 3, 0.5, ptr(sdn), ptr(sdi), st)
        call("pg_perturb_sum", *base, 0, 0.0, ptr(tot[0:1]), ptr(wsp), wsp.numel(), st)
        call("pg_perturb_sum", *base, 1, pst.mean, ptr(tot[1:2]), ptr(wsp), wsp.numel(), st)
        call("pg_perturb_count", *base, ptr(tp), ptr(tc), 0, pst.lo_thr, pst.hi_thr, ptr(cnt), st)
        call("pg_perturb_fill", *base, ptr(tp), ptr(tc), 0, pst.lo_thr, pst.hi_thr, ptr(to), ptr(oc), ptr(ov), st)
    ksec = hip_time(passes, reps=3)
    # CPU: the streaming C restatement, 1 core, on a row sample (all four passes over
    # those rows x all columns), scaled to N rows
    ps = oracle.PerturbStream(adj, en, ei)
    rs = 300
    t0 = time.perf_counter()
    ps.row_sum(False, 0.0, 0, rs)
    ps.row_sum(True, pst.mean, 0, rs)
    r_, c_, v_ = ps.rows(pst.lo_thr, pst.hi_thr, 0, rs)
    cpu_rows = time.perf_counter() - t0
    cpu_full = cpu_rows * n / rs
    sub = got.tocsr()[0:rs].tocoo()
    exact = bool(np.array_equal(sub.row, r_) and np.array_equal(sub.col, c_) and np.array_equal(sub.data, v_))
    pairs = float(n) * n
    print(json.dumps({"row": "8f-4 topology perturbation (corrcoef x2 + modify_network_topology)", "n": n,
                      "samples": 3, "thr": thr, "edges_in": int(adj.nnz), "edges_out": int(got.nnz),
                      "removed": pst.removed, "added": pst.added,
                      "gpu_kernels_ms": round(ksec * 1e3, 3), "gpu_call_ms": round(wall * 1e3, 1),
                      "pairs_per_s": round(pairs / ksec, 1),
                      "cpu_baseline": {"ms": round(cpu_full * 1e3, 1), "pairs_per_s": round(pairs / cpu_full, 1),
                                       "cores": 1, "kind": "port",
                                       "sample": f"oracle/perturb_oracle.c (streaming restatement) over {rs} of {n} "
                                                 f"rows x all columns, scaled to {n} rows"},
                      "bit_exact_vs_oracle_sample_rows": exact}))

    # 8f-4b: the PCA front end on the S0 ECC matrix (data_preprocess.py:528-530: pca(ecc, 250))
    from plagnn.pca import pca as pca_gpu

    eccm = got_ecc = ecc.edge_clustering_coefficients(adj)
    pca_gpu(eccm, 250)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    feat = pca_gpu(eccm, 250)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # CPU: the oracle restatement = the reference's path (dense N x N float64, LU-normalised
    # randomized SVD as scikit-learn 1.1.1), whole, on the host's BLAS threads
    t0 = time.perf_counter()
    ref = oracle.pca_randomized(eccm, 250)
    cpu = time.perf_counter() - t0
    sv = np.linalg.norm(ref, axis=0)
    gap = np.minimum(np.abs(np.diff(np.r_[np.inf, sv])), np.abs(np.diff(np.r_[sv, 0.0]))) / sv[0]
    sep = gap > 1e-4
    err = np.abs(feat - ref).max(axis=0) / np.abs(ref).max(axis=0)
    print(json.dumps({"row": "8f-4b PCA front end (pca(ecc, 250), scikit-learn 1.1.1 randomized path)",
                      "n": n, "nnz": int(eccm.nnz), "components": 250, "gpu_call_ms": round(wall * 1e3, 1),
                      "separated_components": int(sep.sum()),
                      "max_rel_err_separated_vs_oracle": float(err[sep].max()) if sep.any() else None,
                      "max_rel_err_all_vs_oracle": float(err.max()),
                      "cpu_baseline": {"ms": round(cpu * 1e3, 1), "cores": int(os.environ.get("OMP_NUM_THREADS", "0") or 0),
                                       "kind": "port",
                                       "sample": "oracle.pca_randomized: the whole dense float64 randomized PCA "
                                                 "(numpy/scipy BLAS + LAPACK) on the same matrix"}}))


if __name__ == "__main__":
    main()
