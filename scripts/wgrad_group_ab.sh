#!/bin/bash
# Grouped weight gradients: the new GPU tests, then per-group step times with
# TrainEngine.GROUP_WGRAD 0 / 1 alternated across processes (CONFIGS, default cfg2 ref)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_kernels.py} -k "${TESTK:-group or split_k}" > gpurun_out/wg_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/wg_tests.log; exit 1; }
tail -1 gpurun_out/wg_tests.log
for cfg in ${CONFIGS:-cfg2 ref}; do
  for r in 1 2; do
    for g in 0 1; do
      CONFIG=$cfg PG_GROUP_WGRAD=$g timeout -k 10 240 python -u scripts/group_ab.py base >> gpurun_out/wg_ab.jsonl 2> gpurun_out/wg_ab.err || { echo "group_ab failed"; tail -5 gpurun_out/wg_ab.err; exit 1; }
      tail -1 gpurun_out/wg_ab.jsonl | cut -c1-200
    done
  done
done
