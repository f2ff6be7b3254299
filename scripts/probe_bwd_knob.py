"""Bitwise comparison of backward forms (diagnostics build, MT_KNOB arms) against the default
form on the same inputs. usage: MT_DIAG=1 python scripts/probe_bwd_knob.py KNOB[,KNOB..]
HEAD_DIM=128 runs the shapes at d = 128. Prints, per shape and arm, the max |difference| of dQ, dK, dV from knob 0."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip
_hip.use_library(os.path.join(os.path.dirname(_hip.LIB_PATH), "diag", "libminitorch_hip_diag.so"))
knobs = sys.argv[1].split(",")
g = torch.Generator(device="cuda").manual_seed(5)
D = int(os.environ.get("HEAD_DIM", "64"))  # HEAD_DIM=128: the same shapes at d = 128
for shape, causal in [((8, 16, 4096, D), False), ((8, 16, 4096, D), True), ((2, 3, 1000, D), False),
                      ((2, 3, 1000, D), True), ((1, 2, 8192, D), True), ((3, 2, 320, D), False)]:
    q, k, v, do = (torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16) for _ in range(4))
    o, m, l = _hip.flash_fwd(q, k, v, causal)
    os.environ["MT_KNOB"] = "0"
    ref = [t.clone() for t in _hip.flash_bwd(q, k, v, o, do, m, l, causal)]
    for kn in knobs:
        os.environ["MT_KNOB"] = kn
        got = _hip.flash_bwd(q, k, v, o, do, m, l, causal)
        torch.cuda.synchronize()
        d = [float((a.float() - b.float()).abs().max()) for a, b in zip(got, ref)]
        print(f"{shape} causal={causal} knob {kn}: max|d| dq {d[0]:.3e} dk {d[1]:.3e} dv {d[2]:.3e}", flush=True)
