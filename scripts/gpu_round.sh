#!/bin/bash
# One GPU session: parity tests, then (only if no crash) a short bench and a kernel-trace
# profile. Every GPU step has its own time limit; a crash/timeout (exit >= 2 from pytest,
# anything non-zero from the others) ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-20}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ge 2 ]; then echo "pytest crashed/timed out; stopping"; exit $rc; fi
if [ "${GEMM_BENCH:-0}" = "1" ]; then
  for cfg in "" ${GEMM_VARIANTS:-"PLAGNN_GEMM_TILE=128x128" "PLAGNN_GEMM_TILE=64x64" "PLAGNN_GEMM_TILE=128x64" "PLAGNN_GEMM_TILE=64x128"}; do
    echo "== $cfg" >> gpurun_out/gemm_bench.txt
    env $cfg timeout -k 10 300 python scripts/gemm_bench.py --no-torch --dims 512,256,256,256,100,12 >> gpurun_out/gemm_bench.txt 2>&1
    rcg=$?; if [ $rcg -ne 0 ]; then echo "gemm_bench rc=$rcg"; tail gpurun_out/gemm_bench.txt; exit $rcg; fi
  done
  grep -v amdgpu.ids gpurun_out/gemm_bench.txt
fi
if [ "${SPMM_BENCH:-0}" = "1" ]; then
  for cfg in "" "PLAGNN_SPMM_FTILE=256" "PLAGNN_BWD_PATH=direct"; do
    env $cfg timeout -k 10 300 python scripts/spmm_bench.py >> gpurun_out/spmm_bench.txt 2>&1
    rcs=$?; if [ $rcs -ne 0 ]; then echo "spmm_bench rc=$rcs"; cat gpurun_out/spmm_bench.txt; exit $rcs; fi
  done
  cat gpurun_out/spmm_bench.txt | grep -v amdgpu.ids
fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc2=$?
echo "bench rc=$rc2"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
if [ $rc2 -ne 0 ]; then exit $rc2; fi
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps $STEPS --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err
  rc3=$?; cd $GRAFT_REPO_ROOT
  echo "rocprof rc=$rc3"; tail -3 gpurun_out/prof.err
  exit $rc3
fi
exit $rc
