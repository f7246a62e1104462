"""Kernel list of the drop-in model's forward + backward (bench.py's dropin_device_time
loop), for rocprofv3 --kernel-trace --stats. Usage (GPU box):
  rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/dk -o dk -- python3 scripts/probes/dropin_kernels.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pla-gnn_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402
from plagnn import workload  # noqa: E402

wl = workload.build("cfg2", device="cuda")
print(bench.dropin_device_time(wl, wl.dims, torch.device("cuda"), reps=20))
