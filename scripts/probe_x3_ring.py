"""Round 6: error of the fp32 split ring backward, X3 form (knob 0) against the fp32-MFMA form
(knob 65), each against a float64 torch reference of the same inputs (a checker on the GPU):
max |err| / max |ref| and the mean signed error / mean |ref| (bias) of dQ, dK, dV.
usage: MT_DIAG=1 python scripts/probe_x3_ring.py"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip
_hip.use_library(os.path.join(os.path.dirname(_hip.LIB_PATH), "diag", "libminitorch_hip_diag.so"))
g = torch.Generator(device="cuda").manual_seed(3)
for shape, causal in [((8, 16, 1024, 64), False), ((2, 16, 1024, 64), False), ((2, 16, 1024, 64), True), ((8, 16, 1024, 32), False)]:
    q, k, v, do = (torch.randn(shape, device="cuda", generator=g) for _ in range(4))
    o, m, l = _hip.flash_fwd(q, k, v, causal)
    q64, k64, v64 = (t.double().requires_grad_() for t in (q, k, v))
    s = q64 @ k64.transpose(-1, -2) / shape[-1] ** 0.5
    if causal:
        s = s.masked_fill(torch.ones(shape[2], shape[2], device="cuda", dtype=torch.bool).triu(1), float("-inf"))
    o64 = torch.softmax(s, -1) @ v64
    ref = torch.autograd.grad(o64, (q64, k64, v64), do.double())
    for kn in ("0", "65"):
        os.environ["MT_KNOB"] = kn
        got = _hip.flash_bwd(q, k, v, o, do, m, l, causal)
        torch.cuda.synchronize()
        msg = []
        for name, a, r in zip(("dq", "dk", "dv"), got, ref):
            e = a.double() - r
            msg.append(f"{name} max {float(e.abs().max() / r.abs().max()):.2e} bias {float(e.mean() / r.abs().mean()):+.1e}"
                       f" bias_signed {float((e * r.sign()).mean() / r.abs().mean()):+.1e}")
        print(f"{shape} causal={causal} knob {kn}: " + " | ".join(msg), flush=True)
