"""Per-kernel summary of the counter passes that scripts/probes/spmm_pmc.sh leaves in
gpurun_out/sppmc_<i>/ (SQ passes: wave cycles split into waiting / issue-stalled / active,
instructions per wave, clock; cache passes: L2 hit rate, fabric bytes and L1->L2 reads per
launch). SQ_WAVE_CYCLES and SQ_WAIT_* count quad-cycles (MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name)[:48]


def main():
    base = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out")
    for d in sorted(glob.glob(os.path.join(base, "sppmc_*"))):
        if not os.path.isdir(d):
            continue
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        launches = collections.defaultdict(set)
        dur = collections.defaultdict(list)
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                k = short(r["Kernel_Name"])
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                launches[k].add(r["Dispatch_Id"])
        for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        print(f"== {os.path.basename(d)}")
        for k in sorted(agg):
            n = max(1, len(launches[k]))
            a = {c: v / n for c, v in agg[k].items()}
            us = sum(dur[k]) / max(1, len(dur[k])) / 1e3 if dur[k] else float("nan")
            s = f"{k:48s} {us:7.1f} us "
            if "SQ_WAVE_CYCLES" in a:
                wc, w = a["SQ_WAVE_CYCLES"], max(1.0, a["SQ_WAVES"])
                s += (f"waves {w:.0f} wait {a['SQ_WAIT_ANY'] / wc:.2f} stall {a['SQ_WAIT_INST_ANY'] / wc:.2f} "
                      f"active {a['SQ_ACTIVE_INST_ANY'] / wc:.2f} vmem/wave {a['SQ_INSTS_VMEM_RD'] / w:.0f} "
                      f"valu/wave {a['SQ_INSTS_VALU'] / w:.0f}")
            elif "GRBM_GUI_ACTIVE" in a:
                s += f"clock {a['GRBM_GUI_ACTIVE'] / 8 / us / 1e3:.2f} GHz"
            if "TCC_HIT_sum" in a:
                h, m = a["TCC_HIT_sum"], a["TCC_MISS_sum"]
                s += f"L2 hit {h / max(1.0, h + m):.2f} req {a['TCC_REQ_sum'] / 1e6:.2f} M"
            if "FETCH_SIZE" in a:
                s += f"fetch {a['FETCH_SIZE'] / 1e3:.1f} MB L1->L2 reads {a.get('TCP_TCC_READ_REQ_sum', 0) / 1e6:.2f} M"
            print(s)


if __name__ == "__main__":
    main()
