"""Probe (GPU box): where the C3 causal dQ of one head leaves the tests/bounds.py bound. Prints
the worst elements with their error, bound, reference value and the bound's terms.
usage: python scripts/probe_dq_bound.py b h [causal]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llmsys-project-flashattn_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch

from minitorch import _hip
from oracle import cref
from bounds import grad_bounds, head_terms

b0, h0 = int(sys.argv[1]), int(sys.argv[2])
causal = "causal" in sys.argv[3:]
B, H, N, d = 8, 16, 4096, 64
g = torch.Generator(device="cuda").manual_seed(3)
q, k, v, do = (torch.randn((B, H, N, d), device="cuda", generator=g).to(torch.bfloat16) for _ in range(4))
o, m, l = _hip.flash_fwd(q, k, v, causal)
dq, dk, dv = _hip.flash_bwd(q, k, v, o, do, m, l, causal)
torch.cuda.synchronize()
f = lambda t: t[b0, h0].float().cpu().numpy()
qs, ks, vs, dos = f(q), f(k), f(v), f(do)
o_ref, m_ref, l_ref = cref.attn_fwd(qs[None], ks[None], vs[None], causal)
g_ref = cref.attn_bwd(qs[None], ks[None], vs[None], dos[None], m_ref, l_ref, causal)
bnd = grad_bounds(qs, ks, vs, dos, causal)
P, absdS, E, sc = head_terms(qs, ks, vs, dos, causal)
# the kernel's own lse against the oracle's
lse_k = f(m.unsqueeze(-1))[:, 0] + np.log(f(l.unsqueeze(-1))[:, 0])
lse_r = m_ref[0] + np.log(l_ref[0])
print(f"lse: max |kernel - oracle| {np.abs(lse_k - lse_r).max():.3e}")
o_err = np.abs(f(o) - o_ref[0])
print(f"O: max err {o_err.max():.3e}")
for name, got, ref, bd in zip(("dq", "dk", "dv"), (dq, dk, dv), g_ref, bnd):
    err = np.abs(f(got) - ref[0])
    ratio = err / bd
    flat = np.argsort(ratio.ravel())[::-1][:6]
    print(f"{name}: max err {err.max():.3e}, max ratio {ratio.max():.3f}")
    for idx in flat:
        i, t = divmod(int(idx), d)
        print(f"   row {i} col {t}: err {err[i, t]:.3e} bound {bd[i, t]:.3e} ratio {ratio[i, t]:.2f} "
              f"ref {ref[0][i, t]:.4f} got {f(got)[i, t]:.4f} keys {int((P[i] > 0).sum())} "
              f"maxP {P[i].max():.3f} sum|dS| {absdS[i].sum():.3e} O err row {o_err[i].max():.2e}")
