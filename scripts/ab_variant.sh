#!/bin/bash
# A/B of one `make variant` library against the product build: the GPU tests on the variant
# (TESTS, default all), the SpMM micro-benchmark, rocprofv3 summaries of a short bench run.
# V=<variant name> -> gpurun_out/ab_tests_<V>.log, spmm_var.txt, prof_ab.txt
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
PLAGNN_LIB=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$V.so timeout -k 10 400 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests_$V.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests_$V.log; [ $rc -eq 0 ] || exit $rc
VARS=$V bash scripts/spmm_variants.sh || exit 1
LIBS="base $V" bash scripts/prof_ab.sh
