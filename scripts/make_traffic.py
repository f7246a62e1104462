"""Build profiles/pmc_traffic.json from rocprofv3 --pmc passes over bench.py
(scripts/pmc_traffic.sh): HBM-side bytes per launch of each kernel group, with the gfx950
corrections of MI355X_MICROARCH.md "HBM" (FETCH_SIZE counts half of a wide coalesced read:
x2; WRITE_SIZE exact; both in KB): bytes = 2 FETCH_SIZE + WRITE_SIZE, summed over every
dispatch of the group in the headline process and divided by the STEPS that process ran
(head dispatches / 2: head_kernel + head_final_kernel once per step, in the timing graphs
too), so a library call made of several dispatches (the grouped weight gradients:
partials + combine) is counted whole; bench.py divides by the group's library calls per
step for "per call" figures. Infinity-Cache hits are counted by these
counters (L2 memory-side requests), so for tables that fit the 256 MiB MALL this is fabric
traffic, an upper bound on true HBM bytes. Groups: scripts/prof_groups.py's.

Usage: python scripts/make_traffic.py <pmc root> <config> [--gemm-group gemm_bf16]
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_groups import group_of  # noqa: E402


def collect(root, counter, key=None):
    """{group: [bytes, dispatches]} of the process with the most dispatches of `counter`
    (key: the grouping function, default the kernel group)."""
    key = key or group_of
    per_file = []
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        acc = defaultdict(lambda: [0.0, 0])
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                a = acc[key(r["Kernel_Name"])]
                a[0] += float(r["Counter_Value"]) * 1024.0
                a[1] += 1
        per_file.append(acc)
    return max(per_file, key=lambda a: sum(v[1] for v in a.values())) if per_file else {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("config")
    ap.add_argument("--gemm-group", default="gemm_f32", help="name of the GEMM group (gemm_bf16 for cfg5)")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "pmc_traffic.json"))
    ap.add_argument("--by-kernel", action="store_true", help="also print bytes per dispatch of each kernel")
    a = ap.parse_args()
    fetch = collect(os.path.join(a.root, "fetch"), "FETCH_SIZE")
    write = collect(os.path.join(a.root, "write"), "WRITE_SIZE")
    if a.by_kernel:
        short = lambda n: n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]  # noqa: E731
        fk = collect(os.path.join(a.root, "fetch"), "FETCH_SIZE", short)
        wk = collect(os.path.join(a.root, "write"), "WRITE_SIZE", short)
        for k in sorted(fk):
            f, w = fk[k], wk.get(k, [0.0, 1])
            print(f"{k:70s} n={f[1]:5d} fetch2x {2 * f[0] / f[1] / 1e6:9.2f} MB  write {w[0] / max(w[1], 1) / 1e6:9.2f} MB")
    out = json.load(open(a.out)) if os.path.exists(a.out) else {}
    steps_f = fetch.get("head", [0.0, 0])[1] / 2
    steps_w = write.get("head", [0.0, 0])[1] / 2
    if steps_f <= 0 or steps_w <= 0:
        raise SystemExit("no head dispatches in the counter files: cannot count steps")
    per_step = {}
    for g in sorted(set(fetch) | set(write)):
        if g == "other":
            continue
        f = fetch.get(g, [0.0, 0])
        w = write.get(g, [0.0, 0])
        per_step[a.gemm_group if g == "gemm" else g] = round(2.0 * f[0] / steps_f + w[0] / steps_w)
    cfg = {"bytes_per_step": per_step, "steps": [steps_f, steps_w],
           "dispatches_per_step": {a.gemm_group if g == "gemm" else g: round(v[1] / steps_f, 2)
                                   for g, v in fetch.items() if g != "other"}}
    out[a.config] = cfg
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(cfg, indent=1))


if __name__ == "__main__":
    main()
