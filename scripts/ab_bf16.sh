#!/bin/bash
# bf16 GEMM tests on the product build, then per-shape times (scripts/gemm_bf16_bench.py)
# for the product build and the `make variant` libraries named in VARS.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bf16_tests.log 2>&1
rc=$?; tail -2 gpurun_out/bf16_tests.log; [ $rc -eq 0 ] || exit $rc
for v in base ${VARS}; do
  if [ "$v" = "base" ]; then unset PLAGNN_LIB; else export PLAGNN_LIB=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python -u scripts/gemm_bf16_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
