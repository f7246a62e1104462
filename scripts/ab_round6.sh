#!/bin/bash
# Round-6 A/B on one box: GPU tests of variant V (TESTS / KEXPR), then REPS alternations of
# the engine line (no legs) for the product build and each variant in LIBS, per config, with
# the per-launch-site breakdown of the last alternation (gpurun_out/ab6_<cfg>_<lib>.json).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
if [ -n "${V:-}" ]; then
  PLAGNN_LIB=$PWD/pla-gnn_amd/plagnn/libplagnn_$V.so timeout -k 10 ${TT:-400} python -u -m pytest ${TESTS:-tests/test_gpu_kernels.py} -m gpu -x -q --timeout 200 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > gpurun_out/ab6_tests_$V.log 2>&1
  rc=$?; grep -E "passed|failed|Error|assert" gpurun_out/ab6_tests_$V.log | tail -8; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${REPS:-2}); do
for C in ${CONFIGS:-cfg2}; do
for L in ${LIBS:-base}; do
  if [ $L = base ]; then P=$PWD/pla-gnn_amd/plagnn/libplagnn.so; else P=$PWD/pla-gnn_amd/plagnn/libplagnn_$L.so; fi
  PLAGNN_LIB=$P timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-legs --sub-configs= --dump-breakdown gpurun_out/ab6_${C}_$L.json ${BENCH_ARGS:-} > gpurun_out/ab6_${C}_${L}_line.json 2> gpurun_out/ab6_${C}_$L.err || { echo "$C $L failed"; tail -5 gpurun_out/ab6_${C}_$L.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/ab6_${C}_${L}_line.json'))
print('$r $C $L', d['ms_per_step'], d['step_distribution']['median_ms'], d['kernels_ms_per_step'])
"
done; done; done
