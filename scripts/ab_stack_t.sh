cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine_bf16.py tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bf16" > gpurun_out/t_st.log 2>&1 || { tail -20 gpurun_out/t_st.log; exit 1; }
tail -1 gpurun_out/t_st.log
for r in 1 2; do for v in 0 1; do
  PG_STACK_T=$v CONFIG=cfg5 PG_GROUPS=gemm ROUNDS=2 timeout -k 10 300 python -u scripts/group_ab.py base >> gpurun_out/ab_stack.jsonl 2> gpurun_out/ab_stack.err || { tail -5 gpurun_out/ab_stack.err; exit 1; }
  tail -1 gpurun_out/ab_stack.jsonl
done; done
