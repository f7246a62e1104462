#!/bin/bash
# The fused MLP head alone: kernel trace, then SQ counter passes (one per pass).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/mlph && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/mlph/trace -o run -- python3 $R/scripts/probes/mlp_head_one.py 30 > $R/gpurun_out/mlph/trace.out 2>&1) || { echo trace failed; tail -5 $R/gpurun_out/mlph/trace.out; exit 1; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/mlph/p$i -o run --pmc $P -- python3 $R/scripts/probes/mlp_head_one.py 10 > $R/gpurun_out/mlph/p$i.out 2>&1) || { echo "pass $i failed"; tail -5 $R/gpurun_out/mlph/p$i.out; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/mlph | grep -A2 -E "mlp_l1|head_final"
find gpurun_out/mlph/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} python3 -c "
import csv,sys
for r in csv.DictReader(open('{}')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'])"
