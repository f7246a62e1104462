#!/bin/bash
# SQ / TA / TCP counters of the max aggregation kernels on S0 (scripts/probes/spmm_one.py).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/rocprof_counters.txt 2>&1) || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"
# L2 passes (SPMM_PASSES=cache): hit / miss / requests, then fabric fetch bytes and L1->L2 reads
C1="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"
C2="FETCH_SIZE TCP_TCC_READ_REQ_sum"
if [ "${SPMM_PASSES:-sq}" = cache ]; then set -- "$C1" "$C2"; else set -- "$P1" "$P2"; fi
i=0
for P in "$@"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/sppmc_$i -o run \
     --pmc $P -- python3 $R/scripts/probes/spmm_one.py 256 20 bwd > $R/gpurun_out/sppmc_$i.out 2>&1) \
     || { echo "pass $i failed"; tail -5 $R/gpurun_out/sppmc_$i.out; exit 1; }
  echo "pass $i ok"
done
