#!/bin/bash
# GPU tests, smoke(), then every bench config once: gpurun_out/bench_<cfg>.json
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/pt_all.log 2>&1 || { tail -5 gpurun_out/pt_all.log; exit 1; }
tail -1 gpurun_out/pt_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for cfg in ${CFGS:-cfg2 ref cfg3 cfg5}; do
  extra=""; [ "$cfg" != "cfg2" ] && extra="--no-cpu-baseline"
  timeout -k 10 600 python bench.py --config $cfg --steps ${STEPS:-30} --warmup 5 $extra > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { tail -3 gpurun_out/bench_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_$cfg.json')); print('$cfg', d['ms_per_step'], d['value'], d['roofline']['achieved'], d['kernels_ms_per_step'])"
done
