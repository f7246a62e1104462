#!/bin/bash
# A/B of `make variant` libraries: GEMM-group kernel tests on each variant (PLAGNN_LIB), then
# the in-engine per-group times (scripts/engine_ab.sh).
#   LIBS="base gw" CONFIGS="cfg2 ref" TESTK=group bash scripts/ab_lib.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for V in $(echo ${LIBS:-base} | tr ' ' '\n' | sort -u); do
  L=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$V.so; [ $V = base ] && L=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn.so
  PLAGNN_LIB=$L timeout -k 10 300 python -u -m pytest -x -q \
    --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "${TESTK:-gemm}" > gpurun_out/abt_$V.log 2>&1
  rc=$?; echo "tests $V rc=$rc: $(tail -1 gpurun_out/abt_$V.log)"
  [ $rc -eq 0 ] || exit $rc
done
LIBS="${LIBS:-base}" CONFIGS="${CONFIGS:-cfg2}" bash scripts/engine_ab.sh
