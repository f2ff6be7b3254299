"""Probe (GPU box): the default fused bf16 backward (policy 0) against the split kernels
(policy 121) on every head of a shape: per head the max |dQ/dK/dV difference|, and for the
worst heads the rows and key blocks where dQ differs most.
usage: python scripts/probe_fused_dq.py [causal] [B,H,N,d]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch

from minitorch import _hip

causal = "causal" in sys.argv[1:]
shape = next((a for a in sys.argv[1:] if "," in a), "8,16,4096,64")
B, H, N, d = (int(x) for x in shape.split(","))
g = torch.Generator(device="cuda").manual_seed(3)
q, k, v, do = (torch.randn((B, H, N, d), device="cuda", generator=g).to(torch.bfloat16) for _ in range(4))
o, m, l = _hip.flash_fwd(q, k, v, causal)
res = {}
for pol in (0, 121, 0):
    _hip.set_policy(pol)
    out = _hip.flash_bwd(q, k, v, o, do, m, l, causal)
    torch.cuda.synchronize()
    if pol in res:
        for a, b2, n in zip(res[pol], out, "qkv"):
            print(f"policy {pol} repeat: d{n} bitwise equal: {torch.equal(a, b2)}")
    res[pol] = out
_hip.set_policy(0)
f, s = res[0], res[121]
worst = []
for n, a, b2 in zip("qkv", f, s):
    diff = (a.float() - b2.float()).abs()
    ref = b2.float().abs().amax(dim=(2, 3))
    per_head = diff.amax(dim=(2, 3))
    print(f"d{n}: max diff {per_head.max().item():.3e}; heads with diff > 4e-3: "
          f"{int((per_head > 4e-3).sum())} of {B * H}; max |d{n}| {ref.max().item():.3e}")
    if n == "q":
        top = torch.topk(per_head.flatten(), 4)
        for val, idx in zip(top.values.tolist(), top.indices.tolist()):
            b, h = divmod(idx, H)
            rows = diff[b, h].amax(dim=1)
            r = int(rows.argmax())
            print(f"  head ({b},{h}) max {val:.3e} at query row {r} (step {r // 64}, key block of "
                  f"the diagonal {r // 256}); rows > 4e-3: {torch.nonzero(rows > 4e-3).flatten().tolist()[:40]}")
            print(f"    fused {f[0][b, h, r, :8].float().tolist()}")
            print(f"    split {s[0][b, h, r, :8].float().tolist()}")
