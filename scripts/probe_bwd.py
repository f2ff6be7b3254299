"""Probe: bf16 d=64 backward error per (N, B, H, policy) against the oracle, with the
rows of the worst dK error (debug aid, GPU box)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llmsys-project-flashattn_amd")]
import numpy as np, torch
from minitorch import _hip
from oracle import attention as A

def run(B, H, N, causal, pol):
    rng = np.random.default_rng(11)
    q, k, v, do = (A.bf16_round(rng.standard_normal((B, H, N, 64)).astype(np.float32)) for _ in range(4))
    t = [torch.from_numpy(x).cuda().bfloat16() for x in (q, k, v, do)]
    _hip.set_policy(pol)
    o, m, l = _hip.flash_fwd(t[0], t[1], t[2], causal)
    g = _hip.flash_bwd(t[0], t[1], t[2], o, t[3], m, l, causal)
    torch.cuda.synchronize()
    _hip.set_policy(0)
    ro, rm, rl = A.attention_fwd(q, k, v, causal)
    refs = A.attention_bwd(q, k, v, ro, do, rm, rl, causal)
    out = []
    for name, got, ref in zip(("dq", "dk", "dv"), g, refs):
        e = np.abs(got.float().cpu().numpy() - ref)
        bh, row = np.unravel_index(e.max(axis=-1).reshape(B * H, N).argmax(), (B * H, N))
        out.append(f"{name} {e.max():.3g} @bh{bh} row{row}")
    bad_rows = np.where(np.abs(g[1].float().cpu().numpy() - refs[1]).max(-1).reshape(B * H, N) > 0.05)
    print(f"B{B} H{H} N{N} causal={causal} pol={pol}: " + ", ".join(out),
          f"bad dk rows: {sorted(set(bad_rows[1].tolist()))[:8]}..{len(bad_rows[1])} heads {sorted(set(bad_rows[0].tolist()))}", flush=True)

for (B, H, N) in [(1, 1, 64), (2, 3, 192)]:
    for pol in (0, 40, 42, 43, 62, 66):
        run(B, H, N, False, pol)
