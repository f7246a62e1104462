"""Average duration per (kernel, grid size) from a rocprofv3 kernel_trace.csv, for the
kernels whose name matches the pattern (default: the max backward's passes)."""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"bwd_|sum_merge|max_fwd|max_merge")
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if not pat.search(n):
            continue
        short = re.sub(r"\(anonymous namespace\)::|void ", "", n).split("(")[0]
        d[(short, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (k, grid), v in sorted(d.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        print(f"{sum(v) / len(v):9.1f} us  x{len(v):3d}  blocks {grid // 256:>7}  {k}")


if __name__ == "__main__":
    main()
