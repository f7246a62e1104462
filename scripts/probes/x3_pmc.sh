#!/bin/bash
# SQ counters of the three-piece GEMM: the grouped weight gradients (group_one.py) and one
# short-K forward product (gemm_one.py, fwd.pool.l2: 24041 x 256 x 256, B transposed).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/x3pmc_g$i -o run \
     --pmc $P -- python3 $R/scripts/probes/group_one.py 20 > $R/gpurun_out/x3pmc_g$i.out 2>&1) \
     || { echo "group pass $i failed"; tail -5 $R/gpurun_out/x3pmc_g$i.out; exit 1; }
  (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/x3pmc_f$i -o run \
     --pmc $P -- python3 $R/scripts/gemm_one.py 24041 256 256 0 1 20 > $R/gpurun_out/x3pmc_f$i.out 2>&1) \
     || { echo "fwd pass $i failed"; tail -5 $R/gpurun_out/x3pmc_f$i.out; exit 1; }
  echo "pass $i ok"
done
