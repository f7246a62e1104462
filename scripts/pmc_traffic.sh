#!/bin/bash
# HBM traffic per launch (profiles/pmc_traffic.json): two PMC passes, one counter each
# (FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2: one pass cannot hold both), kernel trace
# only, over a short eager bench run (plain dispatches), then scripts/make_traffic.py.
#   CONFIG=cfg2 bash scripts/pmc_traffic.sh
set -u
R=$GRAFT_REPO_ROOT
CONFIG=${CONFIG:-cfg2}
OUT=$R/gpurun_out/pmc_$CONFIG
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--config $CONFIG --eager --steps 3 --warmup 2 --no-cpu-baseline --no-legs --sub-configs= --breakdown-reps 1"
for c in FETCH_SIZE WRITE_SIZE; do
  d=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/$d -o %pid% -- python3 $R/bench.py $ARGS > $OUT/$d.out 2> $OUT/$d.err
  rc=$?; cd $R; echo "pass $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
GG=gemm_f32; [ $CONFIG = cfg5 ] && GG=gemm_bf16
python3 scripts/make_traffic.py $OUT $CONFIG --gemm-group $GG --by-kernel
