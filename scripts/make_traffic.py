"""Build profiles/pmc_traffic.json from rocprofv3 --pmc passes over bench.py
(scripts/pmc_round.sh): HBM-side bytes per engine launch for each kernel group, with the
gfx950 corrections of MI355X_MICROARCH.md (FETCH_SIZE counts half of a wide coalesced
read: x2; WRITE_SIZE exact; both in KB). Infinity-Cache hits are counted by these
counters (they are L2-miss / fabric requests), so for tables that fit the 256 MiB MALL
this is fabric traffic, an upper bound on true HBM bytes.

Usage: python scripts/make_traffic.py gpurun_out/pmc cfg2 [--launches gemm_f32=23,...]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

GROUPS = {
    "gemm_f32_kernel": "gemm_f32", "gemm_dma_kernel": "gemm_f32", "splitk_reduce_kernel": "gemm_f32",
    "splitk_reduce_batch_kernel": "gemm_f32",
    "gemm_bf16_kernel": "gemm_f32", "head_kernel": "head", "head_final_kernel": "head",
    "max_fwd_kernel": "spmm_max_fwd", "max_merge_kernel": "spmm_max_fwd",
    "group_pack_kernel": "spmm_max_bwd", "max_bwd_pull_kernel": "spmm_max_bwd",
    "max_bwd_kernel": "spmm_max_bwd", "sum_merge_kernel": "spmm_max_bwd",
    "multi_loss_kernel": "loss", "multi_loss_final_kernel": "loss", "sigmoid_zero_kernel": "loss",
    "adam_apply_kernel": "adam", "adam_prepare_kernel": "adam",
}


def group_of(name):
    n = name.replace("(anonymous namespace)::", "").replace("pg_gemm::", "").replace("void ", "")
    return GROUPS.get(n.split("(")[0].split("<")[0].strip())


def collect(root, counter):
    per_group = defaultdict(float)
    steps = 0
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                g = group_of(r["Kernel_Name"])
                if "adam_apply_kernel" in r["Kernel_Name"]:
                    steps += 1
                if g:
                    per_group[g] += float(r["Counter_Value"])
    return per_group, steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("config")
    ap.add_argument("--launches", default="", help="overrides of the per-step launch counts, e.g. gemm_f32=22")
    ap.add_argument("--gemm-group", default="gemm_f32", help="name of the GEMM group (gemm_bf16 for cfg5)")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    launches = {"gemm_f32": 22.0, "spmm_max_fwd": 3.0, "spmm_max_bwd": 3.0, "head": 1.0, "adam": 1.0}
    launches.update({k: float(v) for k, v in (kv.split("=") for kv in a.launches.split(",") if kv)})
    fetch, s1 = collect(a.root, "FETCH_SIZE")
    write, s2 = collect(a.root, "WRITE_SIZE")
    out = json.load(open(a.out)) if os.path.exists(a.out) else {}
    cfg = {}
    for g in sorted(set(fetch) | set(write)):
        per_step = (2 * fetch.get(g, 0.0) / max(s1, 1) + write.get(g, 0.0) / max(s2, 1)) * 1024
        cfg[g] = per_step / launches.get(g, 1.0)
    if a.gemm_group != "gemm_f32" and "gemm_f32" in cfg:
        cfg[a.gemm_group] = cfg.pop("gemm_f32")
    out[a.config] = cfg
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(cfg, indent=1))


if __name__ == "__main__":
    main()
