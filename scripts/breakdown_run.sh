#!/bin/bash
# Per-launch-site breakdown of bench configs (CONFIGS, default cfg2 cfg5) for library
# builds (LIBS="base v1 ..." -> plagnn/libplagnn[_V].so): gpurun_out/bd_<cfg>_<lib>.json
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for C in ${CONFIGS:-cfg2 cfg5}; do
for V in ${LIBS:-base}; do
  if [ $V = base ]; then L=$PWD/pla-gnn_amd/plagnn/libplagnn.so; else L=$PWD/pla-gnn_amd/plagnn/libplagnn_$V.so; fi
  PLAGNN_LIB=$L timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-legs --sub-configs= --dump-breakdown gpurun_out/bd_${C}_$V.json ${BENCH_ARGS:-} > gpurun_out/bd_${C}_${V}_line.json 2> gpurun_out/bd_${C}_$V.err || exit $?
  echo "== $C $V $(python3 -c "import json;print(json.load(open('gpurun_out/bd_${C}_${V}_line.json'))['ms_per_step'])")"
  python3 scripts/show_breakdown.py gpurun_out/bd_${C}_$V.json | grep -v "^gemm"
done
done
