#!/bin/bash
# In-engine A/B of library builds (LIBS="base v1 ..." -> plagnn/libplagnn[_V].so): the
# default bench line without legs per build, its per-group times (kernels_ms_per_step).
#   LIBS="base dense" CONFIGS="cfg2 cfg5" bash scripts/engine_ab.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for C in ${CONFIGS:-cfg2}; do
for V in ${LIBS:-base}; do
  if [ $V = base ]; then L=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn.so; else L=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$V.so; fi
  PLAGNN_LIB=$L timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-legs --sub-configs= ${BENCH_ARGS:-} > gpurun_out/eab_${C}_$V.json 2> gpurun_out/eab_${C}_$V.err
  rc=$?
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/eab_${C}_$V.json'))
print('$C $V', d['ms_per_step'], d['kernels_ms_per_step'])
" || { echo "$C $V rc=$rc"; tail -3 gpurun_out/eab_${C}_$V.err; }
  [ $rc -eq 0 ] || exit $rc
done
done
