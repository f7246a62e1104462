#!/bin/bash
# SQ counters of the grouped weight-gradient kernel (scripts/probes/group_one.py) for each
# library in LIBS: one rocprofv3 --pmc pass per counter set, kernel trace only.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/rocprof_counters.txt 2>&1) || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for v in ${LIBS:-base}; do
  if [ "$v" = "base" ]; then unset PLAGNN_LIB; else export PLAGNN_LIB=$R/pla-gnn_amd/plagnn/libplagnn_$v.so; fi
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/grpmc_${v}_$i -o run \
       --pmc $P -- python3 $R/scripts/probes/group_one.py 20 ${GARGS:-} > $R/gpurun_out/grpmc_${v}_$i.out 2>&1) \
       || { echo "pmc $v pass $i failed"; tail -5 $R/gpurun_out/grpmc_${v}_$i.out; exit 1; }
    echo "pmc $v pass $i ok"
  done
done
