#!/bin/bash
# LDS counters of the three-piece GEMM on two cfg2 shapes (fwd.cat.l2: 24041 x 256 x 512,
# 128 x 64 tiles; fwd.pool.l1: 24041 x 504 x 504, 128 x 128 tiles), B transposed: is the
# kernel bound by LDS bandwidth / bank conflicts? PLAGNN_LIB selects a variant build.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/x3lds && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  for S in "24041 256 512 0 1" "24041 504 504 0 1"; do
    T=$(echo $S | tr ' ' _)
    (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/x3lds/p${i}_$T -o run \
       --pmc $P -- python3 $R/scripts/gemm_one.py $S 20 > $R/gpurun_out/x3lds/p${i}_$T.out 2>&1) \
       || { echo "pass $i $S failed"; tail -5 $R/gpurun_out/x3lds/p${i}_$T.out; exit 1; }
  done
  echo "pass $i ok"
done
python3 scripts/pmc_summary.py gpurun_out/x3lds
