"""Summarise gemm_stamp_probe outputs: K-loop vs outside-loop shader clocks per block."""
import csv
import glob
import statistics as S
import sys

for f in sorted(glob.glob((sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps") + "/*.csv")):
    try:
        ks = [list(map(int, l.split())) for l in open(f + ".ksteps") if l.strip()]
    except OSError:
        continue
    rows = list(csv.DictReader(open(f)))[: len(ks)]
    tot = [sum(k) for k in ks]
    clk = [int(r["clocks"]) for r in rows]
    mid = [x for k in ks for x in k[1:-2]] or [0]
    print(f"{f.split('/')[-1]:40} steps {len(ks[0]) + 1:3} loop {S.median(tot):9.0f} block {S.median(clk):9.0f} "
          f"outside {S.median([c - t for c, t in zip(clk, tot)]):8.0f} step {S.median(mid):6.0f} "
          f"last {S.median([k[-1] for k in ks]):6.0f}")
