#!/bin/bash
# overlap_probe.py under HIP graph-execution settings / library builds: gpurun_out/ovle_<n>.txt
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() { n=$1; shift; env "$@" timeout -k 10 200 python scripts/probes/overlap_probe.py > gpurun_out/ovle_$n.txt 2>&1 || exit $?; echo "== $n $*"; grep " us" gpurun_out/ovle_$n.txt; }
run graph OVL=1
run eager OVL_EAGER=1
