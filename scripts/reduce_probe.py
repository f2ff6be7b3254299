"""Column-reduction timing at config 5's shapes (the bias gradients of the linears and the LM
head): backend.add_reduce(a, 0) on [rows, cols] fp32 device tensors, HIP events around 200
calls each. Run it under rocprofv3 --kernel-trace --stats to split the reduce and fold kernels.
usage: python scripts/reduce_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llmsys-project-flashattn_amd"))
import numpy as np
import torch

import minitorch

backend = minitorch.TensorBackend(minitorch.HipKernelOps)
out = {}
rng = np.random.default_rng(0)
for rows, cols in [(4992, 256), (4992, 1024), (4992, 10000), (128, 9984), (39, 256)]:
    a = minitorch.tensor_from_numpy(rng.standard_normal((rows, cols)).astype(np.float32), backend)
    r = backend.add_reduce(a, 0)
    ref = a.to_numpy().astype(np.float64).sum(0)
    err = float(np.abs(r.to_numpy().reshape(-1) - ref).max())
    for _ in range(10):
        backend.add_reduce(a, 0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        backend.add_reduce(a, 0)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 200 * 1e3
    out[f"{rows}x{cols}"] = {"us": round(us, 2), "GB/s": round(rows * cols * 4 / us / 1e3, 1), "max_err": err}
print(json.dumps(out))
