mkdir -p gpurun_out
for cfg in "X=1" "PLAGNN_GEMM_TILE=128x128" "PLAGNN_GEMM_TILE=64x64" "PLAGNN_GEMM_TILE=128x64" "PLAGNN_GEMM_TILE=64x128"; do
  echo "== $cfg" >> gpurun_out/gemm_bench.txt
  env $cfg timeout -k 10 300 python scripts/gemm_bench.py --no-torch --dims 512,256,256,256,100,12 >> gpurun_out/gemm_bench.txt 2>&1 || exit 1
done
