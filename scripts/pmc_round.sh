#!/bin/bash
# PMC counter passes (one counter group per rocprofv3 run, kernel-trace only, as the
# MI355X guide prescribes) over a short bench.py run. Output: gpurun_out/pmc/<pass>/.
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ARGS=${PMC_BENCH_ARGS:-"--steps 2 --warmup 2 --no-cpu-baseline --no-legs --breakdown-reps 1"}
run_pass() {
  name=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmc/$name -o run --pmc "$@" -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/$name.out 2> $R/gpurun_out/pmc/$name.err
  rc=$?; cd $R
  echo "pass $name rc=$rc"
  return $rc
}
run_pass sq SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE || exit $?
run_pass fetch FETCH_SIZE || exit $?
run_pass write WRITE_SIZE || exit $?
run_pass tcc TCC_HIT_sum TCC_MISS_sum || exit $?
