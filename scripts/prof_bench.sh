#!/bin/bash
# rocprofv3 kernel trace (+ --stats) of the bench command (default: exactly the driver's
# `python bench.py`), one csv set per process (-o %pid%), then the per-group summary that
# checks the line's roofline against the profiler (scripts/prof_groups.py).
#   TAG=r03_cfg2 BENCH_ARGS="" bash scripts/prof_bench.sh
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03}
OUT=gpurun_out/prof_$TAG
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$OUT -o %pid% -- python3 $GRAFT_REPO_ROOT/bench.py ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/$OUT.json 2> $GRAFT_REPO_ROOT/$OUT.err
rc=$?; cd $GRAFT_REPO_ROOT; echo "rocprof rc=$rc"; tail -3 $OUT.err
[ $rc -eq 0 ] && python3 scripts/prof_groups.py $OUT --bench $OUT.json --json $OUT.groups.json > $OUT.groups.txt; cat $OUT.groups.txt
exit $rc
