"""Finite-output check of the bf16 forward (O, m, l) and backward (dQ, dK, dV) over ragged and
causal shapes, product library; prints the NaN/inf counts per tensor and where they sit."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip
g = torch.Generator(device="cuda").manual_seed(5)
for shape, causal in [((2, 3, 1000, 64), True), ((2, 3, 1000, 64), False), ((2, 3, 1024, 64), True),
                      ((4, 64, 129, 64), True), ((1, 64, 4001, 64), True), ((2, 3, 1000, 128), True)]:
    q, k, v, do = (torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16) for _ in range(4))
    o, m, l = _hip.flash_fwd(q, k, v, causal)
    dq, dk, dv = _hip.flash_bwd(q, k, v, o, do, m, l, causal)
    torch.cuda.synchronize()
    out = []
    for name, t in (("o", o), ("m", m), ("l", l), ("dq", dq), ("dk", dk), ("dv", dv)):
        bad = ~torch.isfinite(t.float())
        n = int(bad.sum())
        where = ""
        if n:
            idx = bad.nonzero()
            where = f" first {idx[0].tolist()} rows {sorted(set(idx[:, 2].tolist()))[:8]}"
        out.append(f"{name}:{n}{where}")
    print(shape, "causal" if causal else "", " ".join(out), flush=True)
