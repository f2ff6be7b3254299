"""Probe (GPU box, diagnostics library): forward outputs under MT_KNOB values against knob 0
(same kernel family, another schedule) and, on one head, against the C oracle.
usage: MT_KNOBS=0,4 python scripts/probe_knob_fwd.py B,H,N,d [causal] [iters]   (DTYPE=fp32: fp32 I/O)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llmsys-project-flashattn_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from minitorch import _hip

_hip.use_library(os.path.join(os.path.dirname(_hip.LIB_PATH), "diag", "libminitorch_hip_diag.so"))
B, H, N, d = (int(x) for x in sys.argv[1].split(","))
causal = "causal" in sys.argv[2:]
iters = int(sys.argv[-1]) if sys.argv[-1].isdigit() else 0
g = torch.Generator(device="cuda").manual_seed(5)
dt = torch.float32 if os.environ.get("DTYPE") == "fp32" else torch.bfloat16
q, k, v = (torch.randn((B, H, N, d), device="cuda", generator=g).to(dt) for _ in range(3))
outs = {}
for kn in os.environ.get("MT_KNOBS", "0").split(","):
    os.environ["MT_KNOB"] = kn
    o, m, l = _hip.flash_fwd(q, k, v, causal)
    for _ in range(iters):
        _hip.flash_fwd(q, k, v, causal, out=o, m=m, l=l)
    torch.cuda.synchronize()
    outs[kn] = (o.float(), m + torch.log(l))
base = outs[next(iter(outs))]
for kn, (o, lse) in outs.items():
    print(f"knob {kn}: max |O - O(knob0)| {(o - base[0]).abs().max().item():.3e}, "
          f"max |lse - lse(knob0)| {(lse - base[1]).abs().max().item():.3e}")
if not iters:
    from oracle import cref
    for (b, h) in ((0, 0), (B - 1, H - 1)):
        qs, ks, vs = (t[b, h].float().cpu().numpy() for t in (q, k, v))
        o_ref = cref.attn_fwd(qs[None], ks[None], vs[None], causal)[0][0]
        for kn, (o, _) in outs.items():
            print(f"head ({b},{h}) knob {kn}: max |O - oracle| {np.abs(o[b, h].cpu().numpy() - o_ref).max():.3e}")
    for kn, (o, lse) in outs.items():  # every head (DTYPE=fp32: the fp32 bound is 1e-5)
        qs, ks, vs = (t.float().cpu().numpy().reshape(B * H, N, d) for t in (q, k, v))
        o_ref, m_ref, l_ref = cref.attn_fwd(qs, ks, vs, causal)
        err = np.abs(o.cpu().numpy().reshape(B * H, N, d) - o_ref).max()
        lerr = np.abs(lse.cpu().numpy().reshape(B * H, N) - (m_ref + np.log(l_ref))).max()
        print(f"all heads knob {kn}: max |O - oracle| {err:.3e}, max |lse - oracle| {lerr:.3e}")
