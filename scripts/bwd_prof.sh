#!/bin/bash
# rocprofv3 kernel stats of scripts/bwd_bench.py (per-pass split of the max backward).
#   TAG=x bash scripts/bwd_prof.sh [s0|rmat|all]
cd $GRAFT_REPO_ROOT
TAG=${TAG:-bwd}
OUT=gpurun_out/prof_$TAG
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$OUT -o run -- python3 $GRAFT_REPO_ROOT/scripts/bwd_bench.py ${1:-all} ${REPS:-20} > $GRAFT_REPO_ROOT/$OUT.txt 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; cat $OUT.txt | grep -v amdgpu.ids
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print(f\"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>5}  {r['Name'][:110]}\")
"
exit $rc
