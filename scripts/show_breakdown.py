"""Print a bench.py --dump-breakdown file: per launch site ms, and TFLOP/s (gemm) or GB/s."""
import json
import sys

bd = json.load(open(sys.argv[1]))
tot = sum(r["ms"] for r in bd.values())
for k, r in sorted(bd.items(), key=lambda kv: -kv[1]["ms"]):
    rate = ""
    if r["work"]:
        rate = (f"{r['work'] / r['ms'] / 1e9:8.1f} TF" if k.startswith("gemm")
                else f"{r['work'] / r['ms'] / 1e6:8.1f} GB/s")
    print(f"{k:28} {r['ms'] * 1e3:8.1f} us {100 * r['ms'] / tot:5.1f}% {rate}")
print(f"{'total':28} {tot * 1e3:8.1f} us")
