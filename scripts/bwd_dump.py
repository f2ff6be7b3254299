"""Backward outputs of the library MT_HIP_LIB names, saved for a bitwise comparison of two
builds (separate processes: one library per process). usage: python scripts/bwd_dump.py OUT.pt
[cmp OTHER.pt]: with cmp, prints the max |difference| per tensor against OTHER."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip
out = {}
g = torch.Generator(device="cuda").manual_seed(11)
for shape, causal in [((8, 16, 4096, 64), False), ((8, 16, 4096, 64), True), ((2, 3, 1000, 64), True),
                      ((1, 2, 4001, 64), False)]:
    q, k, v, do = (torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16) for _ in range(4))
    o, m, l = _hip.flash_fwd(q, k, v, causal)
    dq, dk, dv = _hip.flash_bwd(q, k, v, o, do, m, l, causal)
    out[f"{shape}{causal}"] = [t.cpu() for t in (dq, dk, dv)]
torch.save(out, sys.argv[1])
if len(sys.argv) > 3 and sys.argv[2] == "cmp":
    other = torch.load(sys.argv[3], weights_only=True)
    for key, ts in out.items():
        d = [float((a.float() - b.float()).abs().max()) for a, b in zip(ts, other[key])]
        print(key, "max|d| dq %.3e dk %.3e dv %.3e" % tuple(d), flush=True)
