"""The cfg2 step's grouped weight gradients (pg_gemm_f32_group: 8 parts, K = 24 041) on
random operands, repeated, for rocprofv3 counter passes (scripts/probes/group_pmc.sh).
Usage: python scripts/probes/group_one.py [reps] [--dims 512,256,256,256,104,12]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import torch  # noqa: E402

from plagnn import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dims = [512, 256, 256, 256, 104, 12]
if "--dims" in sys.argv:
    dims = [int(x) for x in sys.argv[sys.argv.index("--dims") + 1].split(",")]
N, L = 24041, len(dims) - 3
dev = "cuda"
torch.manual_seed(0)
parts = []
# the engine's order: liner2, liner1, then cat / pool of the layers from the top down
dz = torch.randn(N, dims[-1] + (-dims[-1]) % 4, device=dev)
a4 = torch.randn(N, dims[-2], device=dev)
a3 = torch.randn(N, dims[-3], device=dev)
da4 = torch.randn(N, dims[-2], device=dev)
parts.append((dz, a4, torch.empty(dz.shape[1], dims[-2], device=dev), True, False, 0.0,
              torch.empty(dz.shape[1], device=dev)))
parts.append((da4, a3, torch.empty(dims[-2], dims[-3], device=dev), True, False, 0.0, torch.empty(dims[-2], device=dev)))
for l in reversed(range(L)):
    Fi, Fo = dims[l], dims[l + 1]
    dyp = torch.randn(N, Fo + Fi, device=dev)
    hm = torch.randn(N, 2 * Fi, device=dev)
    parts.append((dyp[:, :Fo], hm, torch.empty(Fo, 2 * Fi, device=dev), True, False, 0.0, torch.empty(Fo, device=dev)))
    parts.append((dyp[:, Fo:], hm[:, :Fi], torch.empty(Fi, Fi, device=dev), True, False, 0.0, torch.empty(Fi, device=dev)))
for _ in range(reps):
    ops.gemm_group(parts)
torch.cuda.synchronize()
print("ok", len(parts), "parts")
