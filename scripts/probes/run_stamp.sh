# per-workgroup GEMM timelines at steady clocks (WARM launches first)
set -e
mkdir -p gpurun_out/stamps
W=${WARM:-500}
for shape in "0 1 24041 256 1008 fwdcat" "0 0 24041 1008 256 dgradcat" "0 0 4096 4096 4096 square"; do
  set -- $shape
  for p in ${PROBES:-gemm_stamp_probe}; do
    WARM=$W timeout -k 5 60 ./scripts/probes/$p $1 $2 $3 $4 $5 gpurun_out/stamps/$6_$p.csv
  done
done
