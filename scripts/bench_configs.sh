#!/bin/bash
# One bench.py line per BASELINE config on one GPU (gpurun_out/bench_<cfg>.json); stops at
# the first failure. CONFIGS / BENCH_ARGS override.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in ${CONFIGS:-ref cfg3 cfg4 cfg5}; do
  timeout -k 10 500 python bench.py --config $c ${BENCH_ARGS:-} > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  rc=$?; echo "bench $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_$c.err; exit $rc; fi
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_$c.json')); print(d['config']['workload'][:60], d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('cpu_baseline') and d['cpu_baseline']['ms_per_step'])"
done
