mkdir -p gpurun_out
for v in "" ${VARS:-pipe}; do
  lib=$PWD/pla-gnn_amd/plagnn/libplagnn${v:+_$v}.so
  echo "== variant '$v'" >> gpurun_out/gemm_var.txt
  PLAGNN_LIB=$lib timeout -k 10 200 python scripts/gemm_bench.py --no-torch ${GB_ARGS:---dims 512,256,256,256,100,12} >> gpurun_out/gemm_var.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/gemm_var.txt
