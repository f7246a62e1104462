cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
echo rc=$?; tail -3 gpurun_out/pytest_gpu_final.log; cat gpurun_out/smoke_final.log | tail -2; cat gpurun_out/bench_final.json
