#!/bin/bash
# A/B of a `make variant` GEMM library (V) against the product build on the cfg2 step:
# GEMM tests on the product build, then bench.py (no sub-configs / legs / CPU baseline) for
# each library, alternating, and the per-group times.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_gemm_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab_gemm_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base $V; do
    if [ "$v" = "base" ]; then unset PLAGNN_LIB; else export PLAGNN_LIB=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$v.so; fi
    timeout -k 10 300 python -u bench.py --config ${CONFIG:-cfg2} --sub-configs= --no-cpu-baseline --no-legs --steps 30 > gpurun_out/ab_gemm_${v}_$rep.json 2> gpurun_out/ab_gemm_${v}_$rep.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_gemm_${v}_$rep.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/ab_gemm_${v}_$rep.json').read().splitlines()[-1])
print('$v', d['ms_per_step'], d['kernels_ms_per_step'], d['roofline']['achieved'])"
  done
done
