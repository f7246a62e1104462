#!/bin/bash
# A/B of the split-K combine placement (batched at the end of the backward vs right after
# each weight gradient) on the graph-replayed GEMM group: CONFIG=cfg2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for v in 0 1; do
  PG_REDUCE_INLINE=$v PG_GROUPS=gemm timeout -k 10 300 python -u scripts/group_ab.py base >> gpurun_out/ab_inline.jsonl 2> gpurun_out/ab_inline.err || { tail -5 gpurun_out/ab_inline.err; exit 1; }
  tail -1 gpurun_out/ab_inline.jsonl
done; done
