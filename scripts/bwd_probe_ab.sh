#!/bin/bash
# Per-pass kernel times of scripts/bwd_bench.py under rocprofv3 for several library builds
# (LIBS="base sp1 ..." -> plagnn/libplagnn[_V].so), one profile each.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for V in ${LIBS:-base}; do
  if [ $V = base ]; then L=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn.so; else L=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$V.so; fi
  OUT=gpurun_out/probe_$V; rm -rf $OUT; mkdir -p $OUT
  cd /tmp && PLAGNN_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/$OUT -o run -- python3 $GRAFT_REPO_ROOT/scripts/bwd_bench.py ${WHICH:-s0} ${REPS:-20} ${CHUNKS:-128} > $GRAFT_REPO_ROOT/$OUT.txt 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; echo "== $V rc=$rc"; grep "us/call" $OUT.txt
  [ $rc -eq 0 ] || exit $rc
  python3 scripts/trace_groups.py $OUT/run_kernel_trace.csv
done
