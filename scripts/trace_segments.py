"""Per-segment kernel averages of a scripts/bwd_bench.py rocprofv3 kernel trace: one segment
per benchmarked (chunk, graph, F) case, split at the max_fwd_kernel launch that opens it.
python scripts/trace_segments.py <kernel_trace.csv> <label,label,...>"""
import collections
import csv
import re
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    labels = sys.argv[2].split(",") if len(sys.argv) > 2 else []
    seg, out = -1, collections.OrderedDict()
    for r in rows:
        n = re.sub(r"\(anonymous namespace\)::|void ", "", r["Kernel_Name"]).split("(")[0]
        if n.startswith("max_fwd_kernel"):
            seg += 1
        if seg < 0 or not re.search(r"bwd_|sum_merge|max_bwd|group_pack", n):
            continue
        lab = labels[seg] if seg < len(labels) else str(seg)
        out.setdefault((lab, n[:64]), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = collections.OrderedDict()
    for (lab, n), v in out.items():
        print(f"{lab:14s} {sum(v) / len(v):9.1f} us x{len(v):3d} {n}")
        tot[lab] = tot.get(lab, 0.0) + sum(v) / len(v)
    for lab, t in tot.items():
        print(f"{lab:14s} total {t:9.1f} us")


if __name__ == "__main__":
    main()
