"""Per-kernel VGPR/AGPR/occupancy/scratch/LDS from hipcc -Rpass-analysis (gfx950).
Usage: [RU_FLAGS=-DX=1] python scripts/resource_usage.py pla-gnn_amd/csrc/spmm.hip [filter]"""
import os
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                      "-ffp-contract=off", "-c", src, "-o", "/dev/null",
                      "-Rpass-analysis=kernel-resource-usage"] + os.environ.get("RU_FLAGS", "").split(), capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        name = subprocess.run(["c++filt"], input=t.split(":", 1)[1].strip(), capture_output=True,
                              text=True).stdout.strip()
        cur = {"name": name}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt in r["name"]:
        print(f"vgpr {r.get('VGPRs'):>4} agpr {r.get('AGPRs'):>3} occ {r.get('Occupancy [waves/SIMD]'):>2} "
              f"scr {r.get('ScratchSize [bytes/lane]'):>4} lds {r.get('LDS Size [bytes/block]'):>6}  "
              f"{r['name'][:150]}")
