#!/bin/bash
# rocprofv3 kernel stats of the drop-in model's forward + backward (dropin_kernels.py):
# gpurun_out/dk/ (per-kernel totals over 20+ reps)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/dk -o dk \
   -- python3 $R/scripts/probes/dropin_kernels.py > $R/gpurun_out/dk.out 2>&1) || { tail -5 $R/gpurun_out/dk.out; exit 1; }
tail -2 $R/gpurun_out/dk.out
python3 - <<'PY'
import csv, glob, re
f = glob.glob("gpurun_out/dk/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
    n = re.sub(r"\(anonymous namespace\)::|void ", "", r["Name"]).split("(")[0][:70]
    print(f"{float(r['TotalDurationNs'])/1e3:10.1f} us {int(r['Calls']):6d} calls {float(r['AverageNs'])/1e3:8.1f} us avg  {n}")
print("total", tot / 1e3)
PY
