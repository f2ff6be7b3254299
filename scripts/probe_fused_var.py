"""Diagnostics: the fused backward's dQ hand-off forms (MT_KNOB, diagnostics build) agree: dQ
bit for bit across the forms that compute every partial (0, 8, 16, 32, 40: the partials are
the same products, summed in key-block order), dK / dV bit for bit unless the walk is rotated
(32, 40: the query steps summed in another order), all within the oracle bounds on 2 heads.
usage: MT_DIAG=1 python scripts/probe_fused_var.py [causal]"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
import torch
from minitorch import _hip

_hip.use_library(os.path.join(os.path.dirname(_hip.LIB_PATH), "diag", "libminitorch_hip_diag.so"))
causal = len(sys.argv) > 1 and sys.argv[1] == "causal"
g = torch.Generator(device="cuda").manual_seed(9)
B, H, N, d = 8, 16, 4096, 64
q, k, v, do = (torch.randn((B, H, N, d), device="cuda", generator=g).to(torch.bfloat16) for _ in range(4))
o, m, l = _hip.flash_fwd(q, k, v, causal)
res = {}
for knob in (16, 0, 8, 32, 40):
    os.environ["MT_KNOB"] = str(knob)
    _hip.set_policy(120)
    res[knob] = _hip.flash_bwd(q, k, v, o, do, m, l, causal)
    torch.cuda.synchronize()
_hip.set_policy(0)
os.environ.pop("MT_KNOB")
ref = res[16]
for knob, gr in res.items():
    same = [bool(torch.equal(a, b)) for a, b in zip(gr, ref)]
    diff = [float((a.float() - b.float()).abs().max()) for a, b in zip(gr, ref)]
    print(f"knob {knob}: equal to the round-3 form (dq, dk, dv) {same}, max |diff| {diff}")
from test_flash_gpu import _grad_check
for knob in (0, 32):
    _grad_check(q, k, v, do, res[knob], causal, [(0, 0), (7, 15)], f"knob {knob}")
    print(f"knob {knob}: oracle bounds ok on 2 heads")
