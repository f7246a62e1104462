#!/bin/bash
# Engine-level GPU tests (engine, full-size, dist) then the in-engine A/B of LIBS.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_engine.py tests/test_gpu_fullsize.py ${EXTRA_TESTS:-} > gpurun_out/engine_tests.log 2>&1
rc=$?; echo "engine tests rc=$rc: $(tail -1 gpurun_out/engine_tests.log)"
[ $rc -eq 0 ] || { tail -30 gpurun_out/engine_tests.log; exit $rc; }
LIBS="${LIBS:-base}" CONFIGS="${CONFIGS:-cfg2}" bash scripts/engine_ab.sh
