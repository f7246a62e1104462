"""Register / LDS / occupancy summary of every kernel in a HIP source (hipcc remarks).
Usage: python scripts/kres.py csrc/file.hip [extra hipcc flags...] [--grep SUBSTR]"""
import re
import subprocess
import sys

args = sys.argv[1:]
pat = None
if "--grep" in args:
    i = args.index("--grep")
    pat = args[i + 1]
    del args[i:i + 2]
src, extra = args[0], args[1:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-c", src,
       "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?(?:\[[^\]]*\])?):\s*(\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
for r in rows:
    if pat and pat not in r["name"]:
        continue
    print(f"v{r.get('VGPRs', '?'):>4} a{r.get('AGPRs', '?'):>4} spill{r.get('VGPRs Spill', '?'):>3} "
          f"occ{r.get('Occupancy [waves/SIMD]', '?'):>2} lds{r.get('LDS Size [bytes/block]', '?'):>7}  {r['name'][:110]}")
