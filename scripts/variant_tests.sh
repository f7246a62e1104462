#!/bin/bash
# GPU tests of one `make variant` library (V=<name>, TESTS / KEXPR select), then the group
# A/B against the product build (scripts/group_ab.sh).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
PLAGNN_LIB=$GRAFT_REPO_ROOT/pla-gnn_amd/plagnn/libplagnn_$V.so timeout -k 10 500 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 200 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > gpurun_out/vt_$V.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" gpurun_out/vt_$V.log | tail -8; [ $rc -eq 0 ] || exit $rc
if [ "${AB:-1}" = "1" ]; then VARS="$V" bash scripts/group_ab.sh; fi
