#!/bin/bash
# A/B of the f32 GEMM paths on the cfg2 step shapes: timing and error against float64 for
# the shipped library and each variant in LIBS (plagnn/libplagnn_<v>.so).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in base ${LIBS:-algo1}; do
  if [ "$v" = "base" ]; then unset PLAGNN_LIB; else export PLAGNN_LIB=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$v.so; fi
  echo "== $v" >> gpurun_out/x3_ab.txt
  timeout -k 10 300 python scripts/gemm_bench.py --no-torch --err ${GB_ARGS:-} >> gpurun_out/x3_ab.txt 2>&1 || { echo "gemm_bench $v failed"; tail -5 gpurun_out/x3_ab.txt; exit 1; }
done
cat gpurun_out/x3_ab.txt
