#!/bin/bash
# A/B of `make variant` libraries on the graph-replayed group times of one config, the
# variants alternated across processes: VARS="inslot" CONFIG=cfg2 -> gpurun_out/group_ab.jsonl
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do
  for v in base $VARS; do
    if [ "$v" = "base" ]; then unset PLAGNN_LIB; else export PLAGNN_LIB=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$v.so; fi
    timeout -k 10 240 python -u scripts/group_ab.py $v >> gpurun_out/group_ab.jsonl 2> gpurun_out/group_ab_$v.err || { echo "group_ab $v failed"; tail -5 gpurun_out/group_ab_$v.err; exit 1; }
    tail -1 gpurun_out/group_ab.jsonl
  done
done
