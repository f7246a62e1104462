#!/bin/bash
# SpMM micro-benchmark over library variants (make variant V=... VSRC=spmm): gpurun_out/spmm_var.txt
set -u
mkdir -p gpurun_out
for v in "" ${VARS:-}; do
  lib=$PWD/pla-gnn_amd/plagnn/libplagnn${v:+_$v}.so
  echo "== variant '$v'" >> gpurun_out/spmm_var.txt
  PLAGNN_LIB=$lib timeout -k 10 200 python scripts/spmm_bench.py ${SB_ARGS:-} >> gpurun_out/spmm_var.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/spmm_var.txt
