#!/bin/bash
# A/B of bench flag sets on one box: FLAGS="base|--separate-l1-head" (| separated, "base" =
# none), REPS alternations per config; per-launch-site breakdown of the last one.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
IFS='|' read -ra FL <<< "${FLAGS:-base}"
for r in $(seq 1 ${REPS:-2}); do
for C in ${CONFIGS:-cfg2}; do
for i in "${!FL[@]}"; do
  F="${FL[$i]}"; [ "$F" = base ] && F=""
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-legs --sub-configs= --dump-breakdown gpurun_out/abf_${C}_$i.json $F ${BENCH_ARGS:-} > gpurun_out/abf_${C}_${i}_line.json 2> gpurun_out/abf_${C}_$i.err || { echo "$C [$F] failed"; tail -5 gpurun_out/abf_${C}_$i.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/abf_${C}_${i}_line.json'))
print('$r $C [${FL[$i]}]', d['ms_per_step'], d['step_distribution']['median_ms'], d['roofline']['frac'], d['kernels_ms_per_step'])
"
done; done; done
