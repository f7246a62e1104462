#!/bin/bash
# Kernel time of the fused MLP head per build (LIBS: base + phase-skip probe variants), one
# rocprofv3 kernel trace each over scripts/probes/mlp_head_one.py.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/mlph_ph && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for L in ${LIBS:-base}; do
  if [ $L = base ]; then P=$R/pla-gnn_amd/plagnn/libplagnn.so; else P=$R/pla-gnn_amd/plagnn/libplagnn_$L.so; fi
  (cd /tmp && PLAGNN_LIB=$P timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/mlph_ph/$L -o run -- python3 $R/scripts/probes/mlp_head_one.py 40 > $R/gpurun_out/mlph_ph/$L.out 2>&1) || { echo "$L failed"; tail -3 $R/gpurun_out/mlph_ph/$L.out; exit 1; }
  f=$(find gpurun_out/mlph_ph/$L -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'mlp_l1' in r['Name'] or 'l1_split' in r['Name'] or 'head_final' in r['Name']:
        print('$L', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')"
done
