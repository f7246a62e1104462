#!/bin/bash
# In-engine sweep of the backward's out-CSR chunk (bench.py --chunk-bwd) for one config.
#   CONFIG=cfg5 CHUNKS="128 256 512" bash scripts/chunk_ab.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for c in ${CHUNKS:-64 128}; do
  timeout -k 10 300 python bench.py --config ${CONFIG:-cfg2} --no-cpu-baseline --no-legs --sub-configs= --chunk-bwd $c > gpurun_out/chunk_${CONFIG:-cfg2}_$c.json 2> gpurun_out/chunk_${CONFIG:-cfg2}_$c.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/chunk_${CONFIG:-cfg2}_$c.json') if l.startswith('{')][-1])
print('${CONFIG:-cfg2} chunk $c', d['ms_per_step'], d['kernels_ms_per_step'])"
done
