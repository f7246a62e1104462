#!/bin/bash
# Round-2 GPU check: the given test files first (verbose), then the whole -m gpu suite,
# smoke() and the default bench line. Every GPU step has its own limit; the chain stops
# at the first failure.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -40
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${SMOKE:-1}" = "1" ]; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "${PROFILE:-0}" = "1" ]; then
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-legs ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err
  rc=$?; cd $GRAFT_REPO_ROOT; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof.err
fi
exit $rc
