#!/bin/bash
# GEMM tests (f32 + bf16) on the current build, then graph-replayed GEMM group times per
# config for the runs in RUNS ("lib:group" pairs: lib = base (the current build) or a
# libplagnn_<lib>.so variant, group = TrainEngine.GROUP_WGRAD), alternated twice
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_bf16.py -k "${TESTK:-gemm}" > gpurun_out/epi_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/epi_tests.log; exit 1; }
  tail -1 gpurun_out/epi_tests.log
fi
for cfg in ${CONFIGS:-cfg2 cfg5}; do
  for r in 1 2; do
    for run in ${RUNS:-prev:1 base:1}; do
      v=${run%%:*}; g=${run##*:}
      if [ "$v" = "base" ]; then unset PLAGNN_LIB; else export PLAGNN_LIB=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$v.so; fi
      CONFIG=$cfg PG_GROUP_WGRAD=$g PG_GROUPS=gemm timeout -k 10 300 python -u scripts/group_ab.py $v >> gpurun_out/epi_ab.jsonl 2> gpurun_out/epi_ab.err || { echo "group_ab failed"; tail -5 gpurun_out/epi_ab.err; exit 1; }
      tail -1 gpurun_out/epi_ab.jsonl | cut -c1-150
    done
  done
done
