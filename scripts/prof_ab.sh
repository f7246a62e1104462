#!/bin/bash
# rocprofv3 kernel-trace summaries of a short bench run per library variant:
# LIBS="base nolong ..." -> gpurun_out/prof_<v>/  + gpurun_out/prof_ab.txt (by-symbol top kernels)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${LIBS:-base}; do
  if [ "$v" = "base" ]; then unset PLAGNN_LIB; else export PLAGNN_LIB=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$v.so; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-legs ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/gpurun_out/prof_$v.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_$v.err) || { echo "rocprof $v failed"; tail -3 gpurun_out/prof_$v.err; exit 1; }
  echo "== $v" >> gpurun_out/prof_ab.txt
  python3 scripts/prof_summary.py gpurun_out/prof_$v/run_results.db --by-symbol --top ${TOP:-14} | cut -c1-170 >> gpurun_out/prof_ab.txt
done
cat gpurun_out/prof_ab.txt
