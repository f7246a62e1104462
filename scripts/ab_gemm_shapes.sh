#!/bin/bash
# Per-shape GEMM times (scripts/gemm_bench.py, cfg2 shapes) for the product build and the
# `make variant` libraries named in VARS.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in base ${VARS}; do
  if [ "$v" = "base" ]; then unset PLAGNN_LIB; else export PLAGNN_LIB=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$v.so; fi
  echo "== $v"
  timeout -k 10 300 python -u scripts/gemm_bench.py --no-torch ${GB_ARGS:-} || exit 1
done
