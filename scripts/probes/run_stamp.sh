# per-workgroup GEMM timelines at steady clocks (WARM launches first)
set -e
mkdir -p gpurun_out/stamps
W=${WARM:-500}
for shape in "0 1 24041 256 1024 fwdcat" "0 1 24041 512 512 fwdpool" "0 0 24041 1024 256 dgradcat" "0 0 24041 512 256 dgradcat2"; do
  set -- $shape
  WARM=$W timeout -k 5 60 ./scripts/probes/gemm_stamp_probe $1 $2 $3 $4 $5 gpurun_out/stamps/$6.csv
done
