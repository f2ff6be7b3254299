"""Accuracy of the fp32 kernels' X3 forms (bf16 MFMA in three pieces per operand) against the
v_mfma_f32_32x32x2_f32 forms (MT_KNOB 65) and the C oracle: per output, the max error over
max|ref| and the signed bias mean((got - ref) * sign(ref)) / mean|ref| (a rounding mode that
is not round-to-nearest in a long accumulation shows up as a nonzero bias).
usage: python scripts/probe_x3_bias.py B,H,N,d [causal]   (diagnostics library)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llmsys-project-flashattn_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from minitorch import _hip
from oracle import cref

_hip.use_library(os.path.join(os.path.dirname(_hip.LIB_PATH), "diag", "libminitorch_hip_diag.so"))
B, H, N, d = (int(x) for x in sys.argv[1].split(","))
causal = "causal" in sys.argv[2:]
g = torch.Generator(device="cuda").manual_seed(3)
q, k, v, do = (torch.randn((B, H, N, d), device="cuda", generator=g) for _ in range(4))
heads = [(0, 0), (B - 1, H - 1), (B // 2, H // 2)]
qs, ks, vs, dos = (np.stack([t[b, h].cpu().numpy() for (b, h) in heads]) for t in (q, k, v, do))
o_ref, m_ref, l_ref = cref.attn_fwd(qs, ks, vs, causal)
g_ref = cref.attn_bwd(qs, ks, vs, dos, m_ref, l_ref, causal)
for kn in ("0", "65"):
    os.environ["MT_KNOB"] = kn
    o, m, l = _hip.flash_fwd(q, k, v, causal)
    grads = _hip.flash_bwd(q, k, v, o, do, m, l, causal)
    torch.cuda.synchronize()
    for name, got, ref in zip(("O", "dQ", "dK", "dV"), (o,) + tuple(grads), (o_ref,) + tuple(g_ref)):
        gs = np.stack([got[b, h].cpu().numpy() for (b, h) in heads]).astype(np.float64)
        r = ref.astype(np.float64)
        err = np.abs(gs - r).max() / np.abs(r).max()
        bias = ((gs - r) * np.sign(r)).mean() / np.abs(r).mean()
        print(f"knob {kn:>2} {name}: max err / max|ref| {err:.3e}  bias {bias:+.3e}", flush=True)
