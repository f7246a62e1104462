#!/bin/bash
# Whole-step bench per library variant: gpurun_out/bab_<v>.json (the shipped library = base).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in ${LIBS:-base}; do
  if [ "$v" = "base" ]; then unset PLAGNN_LIB; else export PLAGNN_LIB=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs ${BENCH_ARGS:-} > gpurun_out/bab_$v.json 2> gpurun_out/bab_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/bab_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bab_$v.json')); print('$v', d['ms_per_step'], d['kernels_ms_per_step'], d['roofline']['achieved'])"
done
