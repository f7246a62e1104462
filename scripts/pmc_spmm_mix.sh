#!/bin/bash
# Instruction-mix / wait PMC passes over a short bench run (one group per rocprofv3 run,
# kernel-trace only): where the SpMM pack/pull/forward waves spend their cycles.
# Output: gpurun_out/pmcmix/<pass>/ ; summary: scripts/pmc_summary.py-style per-kernel sums.
set -u
mkdir -p gpurun_out/pmcmix
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ARGS="--steps 2 --warmup 2 --no-cpu-baseline --no-legs --breakdown-reps 1"
run_pass() {
  name=$1; shift
  cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmcmix/$name -o run --pmc "$@" -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmcmix/$name.out 2> $R/gpurun_out/pmcmix/$name.err
  rc=$?; cd $R
  echo "pass $name rc=$rc"
  return $rc
}
run_pass a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU || exit $?
run_pass b SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_WAVES SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT || exit $?
