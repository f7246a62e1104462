#!/bin/bash
# The whole GPU test suite, then the default bench line without the CPU baseline and the
# sub-configs (the drop-in and epoch-with-eval legs included).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py ${BENCH_ARGS:---sub-configs= --no-cpu-baseline} > gpurun_out/bench_line.json 2> gpurun_out/bench_line.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_line.err; exit $rc; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_line.json'))
print(d['ms_per_step'], d['step_distribution']['median_ms'], d['kernels_ms_per_step'])
print('roofline', d['roofline']['achieved'], d['roofline']['frac'])
print('dropin', {k: v for k, v in (d.get('dropin') or {}).items() if k != 'what'})
print('epoch_with_eval_ms', d.get('epoch_with_eval_ms'), 'dropin ref eval', d.get('dropin_epoch_with_reference_eval_ms'))
"
