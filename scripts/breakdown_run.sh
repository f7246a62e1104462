#!/bin/bash
# Per-launch-site breakdown of bench configs (CONFIGS, default cfg2 cfg5) for library
# builds (LIBS="base v1 ..." -> plagnn/libplagnn[_V].so) and environment settings
# (ENVS="A=0 A=1", each one run): gpurun_out/bd_<cfg>_<lib>[_<env>].json
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for C in ${CONFIGS:-cfg2 cfg5}; do
for V in ${LIBS:-base}; do
for E in ${ENVS:-NONE=1}; do
  if [ $V = base ]; then L=$PWD/pla-gnn_amd/plagnn/libplagnn.so; else L=$PWD/pla-gnn_amd/plagnn/libplagnn_$V.so; fi
  T=${C}_$V; [ "$E" = NONE=1 ] || T=${T}_${E//=/}
  env $E PLAGNN_LIB=$L timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-legs --sub-configs= --dump-breakdown gpurun_out/bd_$T.json ${BENCH_ARGS:-} > gpurun_out/bd_${T}_line.json 2> gpurun_out/bd_$T.err || exit $?
  echo "== $C $V $E $(python3 -c "import json;d=json.load(open('gpurun_out/bd_${T}_line.json'));print(d['ms_per_step'], d['kernels_ms_per_step'])")"
  python3 scripts/show_breakdown.py gpurun_out/bd_$T.json | grep -E "${SHOW:-spmm}"
done
done
done
