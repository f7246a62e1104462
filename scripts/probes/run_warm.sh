bash scripts/probes/run_stamp.sh && for w in 5 100; do timeout -k 10 300 python bench.py --steps 20 --warmup $w --no-cpu-baseline > gpurun_out/bench_w$w.json 2>/dev/null || exit 1; done
