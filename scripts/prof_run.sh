#!/bin/bash
# rocprofv3 kernel-trace of the default bench command (no CPU baseline, no legs):
# gpurun_out/prof/ + gpurun_out/prof_bench.json; summaries via scripts/prof_summary.py.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-legs ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err
rc=$?; cd $GRAFT_REPO_ROOT; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof.err
exit $rc
