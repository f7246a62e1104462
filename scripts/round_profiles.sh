#!/bin/bash
# The round's judged profiles, made on the GPU box and pruned to their summaries (gpurun
# merges back at most 64 MiB): PMC traffic of cfg2 and cfg5 (scripts/pmc_traffic.sh ->
# gpurun_out/pmc_traffic.json + per-kernel tables), then the rocprofv3 kernel trace of the
# default bench command (scripts/prof_bench.sh -> groups summary + kernel stats csvs).
# Copy them into profiles/<round>/ afterwards with scripts/collect_profiles.sh.
#   TAG=r05 bash scripts/round_profiles.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05}
for c in cfg2 cfg5; do
  CONFIG=$c bash scripts/pmc_traffic.sh > gpurun_out/pmc_$c.log 2>&1 || { tail -5 gpurun_out/pmc_$c.log; exit 1; }
  G=gemm_f32; [ $c = cfg5 ] && G=gemm_bf16
  python3 scripts/make_traffic.py gpurun_out/pmc_$c $c --gemm-group $G --by-kernel \
      --out gpurun_out/pmc_traffic_$c.json > gpurun_out/pmc_traffic_by_kernel_$c.txt || exit 1
  rm -rf gpurun_out/pmc_$c
  echo "pmc $c ok"
done
TAG=$TAG bash scripts/prof_bench.sh > gpurun_out/prof_$TAG.log 2>&1; rc=$?
tail -8 gpurun_out/prof_$TAG.log
# keep the stats csvs, drop the traces
find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -delete
find gpurun_out/prof_$TAG -name "*agent_info.csv" -delete
exit $rc
