"""Floors for config 5's bias-gradient column sum (4992 x 256 fp32, 5.1 MB): minitorch's
add_reduce against torch.sum(dim=0) and a plain device copy of the same tensor, HIP events around
200 calls each. Run under rocprofv3 --kernel-trace --stats for per-kernel durations.
usage: python scripts/reduce_floor.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llmsys-project-flashattn_amd"))
import numpy as np
import torch

import minitorch


def timed(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1e3, 2)


backend = minitorch.TensorBackend(minitorch.HipKernelOps)
rng = np.random.default_rng(0)
out = {}
for rows, cols in [(4992, 256), (4992, 1024), (4992, 10000), (128, 9984)]:
    x = rng.standard_normal((rows, cols)).astype(np.float32)
    a = minitorch.tensor_from_numpy(x, backend)
    t = torch.from_numpy(x).cuda()
    d = torch.empty_like(t)
    out[f"{rows}x{cols}"] = {
        "minitorch_us": timed(lambda: backend.add_reduce(a, 0)),
        "torch_sum_us": timed(lambda: torch.sum(t, 0)),
        "copy_us": timed(lambda: d.copy_(t)),
    }
print(json.dumps(out))
