#!/bin/bash
# Copy the judged summaries of a scripts/prof_bench.sh + scripts/pmc_traffic.sh session from
# gpurun_out/ into profiles/<round>/ (and profiles/pmc_traffic.json).
#   ROUND=r03 TAG=r03 bash scripts/collect_profiles.sh
set -eu
ROUND=${ROUND:-r03}; TAG=${TAG:-$ROUND}
SRC=gpurun_out/prof_$TAG; DST=profiles/$ROUND
mkdir -p $DST
rm -f $DST/rocprof_kernel_stats_*.csv
cp gpurun_out/prof_$TAG.json $DST/bench_default_under_rocprof.json
cp $SRC.groups.json $DST/rocprof_groups_default_bench.json
cp $SRC.groups.txt $DST/rocprof_groups_default_bench.txt
HEAD=$(python3 -c "import json;print(json.loads(open('gpurun_out/prof_$TAG.json').read().splitlines()[-1])['pid'])")
# only the processes of the last profiled run (gpurun_out/ keeps earlier runs' files too)
PIDS=$(sed -n 's/^# process \([0-9]*\).*/\1/p' $SRC.groups.txt)
for pid in $PIDS; do
  f=$SRC/${pid}_kernel_stats.csv
  [ -f $f ] || continue
  if [ "$pid" = "$HEAD" ]; then cp $f $DST/rocprof_kernel_stats_cfg2_headline.csv
  else cp $f $DST/rocprof_kernel_stats_child_${pid}.csv; fi
done
for c in cfg2 cfg5; do
  if [ -d gpurun_out/pmc_$c ]; then
    G=gemm_f32; [ $c = cfg5 ] && G=gemm_bf16
    python3 scripts/make_traffic.py gpurun_out/pmc_$c $c --gemm-group $G --by-kernel > $DST/pmc_traffic_by_kernel_$c.txt
  elif [ -f gpurun_out/pmc_traffic_$c.json ]; then  # pruned on the box (scripts/round_profiles.sh)
    cp gpurun_out/pmc_traffic_by_kernel_$c.txt $DST/pmc_traffic_by_kernel_$c.txt
    python3 -c "
import json, os
p = 'profiles/pmc_traffic.json'
d = json.load(open(p)) if os.path.exists(p) else {}
d.update(json.load(open('gpurun_out/pmc_traffic_$c.json')))
json.dump(d, open(p, 'w'), indent=1)"
  fi
done
ls $DST
