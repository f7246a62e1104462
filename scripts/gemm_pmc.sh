#!/bin/bash
# SQ counters of the f32 GEMM kernels on one shape, per library variant in LIBS:
# gpurun_out/gpmc_<v>/ (kernel-trace + one --pmc pass each).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
SHAPE=${SHAPE:-"24041 504 504 0 1"}
for v in ${LIBS:-base}; do
  if [ "$v" = "base" ]; then unset PLAGNN_LIB; else export PLAGNN_LIB=$R/pla-gnn_amd/plagnn/libplagnn_$v.so; fi
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/gpmc_$v -o run \
     --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE \
     -- python3 $R/scripts/gemm_one.py $SHAPE 20 > $R/gpurun_out/gpmc_$v.out 2>&1) || { echo "pmc $v failed"; tail -5 gpurun_out/gpmc_$v.out; exit 1; }
  echo "pmc $v ok"
done
