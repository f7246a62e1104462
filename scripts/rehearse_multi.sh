#!/bin/bash
# Rehearsal of bench.py's N-rank flow on a one-GPU box: torch.distributed.run with N ranks
# sharing the GPU over gloo (the driver's 8-GPU runs use nccl = RCCL, one GPU per rank).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PLAGNN_BENCH_BACKEND=gloo
# RUNS: config:mode pairs (mode auto = replicas, dp for cfg4)
for run in ${RUNS:-cfg2:auto cfg2:dp cfg4:auto}; do
  cfg=${run%%:*}; mode=${run##*:}
  n=${NR:-2}; [ "$cfg" = "cfg4" ] && n=4
  tag=${cfg}_$mode
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 500)) bench.py --gpus $n --steps 10 --warmup 3 --config $cfg --mode $mode \
    --sub-configs= --no-cpu-baseline --no-legs > gpurun_out/rehearse_$tag.json 2> gpurun_out/rehearse_$tag.err
  rc=$?; echo "$tag n=$n rc=$rc"; cat gpurun_out/rehearse_$tag.json; grep -v amdgpu.ids gpurun_out/rehearse_$tag.err | tail -3
  [ $rc -eq 0 ] || exit $rc
done
