"""Summarise rocprofv3 --pmc csv passes (gpurun_out/pmc/<pass>/**/counter_collection.csv)
per kernel symbol: mean counter value per dispatch. Applies the gfx950 corrections of
MI355X_MICROARCH.md: FETCH_SIZE reports half of a wide coalesced read (x2), sizes in KB.
Usage: python scripts/pmc_summary.py gpurun_out/pmc [--json out.json]"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json")
    a = ap.parse_args()
    agg = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(a.root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                key = short(r["Kernel_Name"])
                agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
                agg[key]["_grid"].append(float(r.get("Grid_Size", 0) or 0))
    out = {}
    for k, cs in agg.items():
        row = {}
        for c, vals in cs.items():
            if c.startswith("_"):
                continue
            row[c] = sum(vals) / len(vals)
        if "FETCH_SIZE" in row:
            row["HBM_READ_BYTES_corrected"] = row["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in row:
            row["HBM_WRITE_BYTES"] = row["WRITE_SIZE"] * 1024
        if "SQ_VALU_MFMA_BUSY_CYCLES" in row and "GRBM_GUI_ACTIVE" in row and row["GRBM_GUI_ACTIVE"]:
            # busy cycles summed over SIMDs (4 per CU, 256 CUs); GUI_ACTIVE summed over 8 XCDs
            row["mfma_util"] = row["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * row["GRBM_GUI_ACTIVE"] / 8)
        if "TCC_HIT_sum" in row and "TCC_MISS_sum" in row:
            t = row["TCC_HIT_sum"] + row["TCC_MISS_sum"]
            row["l2_hit_rate"] = row["TCC_HIT_sum"] / t if t else 0.0
        out[k] = row
    for k in sorted(out):
        r = out[k]
        parts = [f"{c}={v:.4g}" for c, v in sorted(r.items())]
        print(f"{k[:90]}\n    " + "  ".join(parts))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
