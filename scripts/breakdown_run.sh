#!/bin/bash
# Per-launch-site breakdown of the default bench (cfg2) and cfg5: gpurun_out/bd_<cfg>.json
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for C in ${CONFIGS:-cfg2 cfg5}; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-legs --sub-configs= --dump-breakdown gpurun_out/bd_$C.json ${BENCH_ARGS:-} > gpurun_out/bd_${C}_line.json 2> gpurun_out/bd_${C}.err || exit $?
  python3 scripts/show_breakdown.py gpurun_out/bd_$C.json
done
