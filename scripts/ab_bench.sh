#!/bin/bash
# A/B of engine knobs on the bench: one short bench.py run per setting in $AB (space-separated
# "VAR=value" groups, "base" = no override). Output: gpurun_out/ab.txt.
set -u
mkdir -p gpurun_out
for cfg in ${AB:-base}; do
  env_args=""; [ "$cfg" != "base" ] && env_args="${cfg//,/ }"
  echo "== $cfg" >> gpurun_out/ab.txt
  env $env_args timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_one.json 2>> gpurun_out/ab.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print(d['ms_per_step'], d['kernels_ms_per_step'])" >> gpurun_out/ab.txt
done
cat gpurun_out/ab.txt
