cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "gemm" > gpurun_out/t_gemm.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/t_gemm.log
LIBS="base w1 base w1" CONFIGS="cfg2 ref" bash scripts/engine_ab.sh
