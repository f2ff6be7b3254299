"""Error probe of a forward variant against a torch fp32 reference (diagnostics, GPU box).
usage: MT_DIAG=1 [OUT32=1] python scripts/probe_fq.py POL KNOB [causal]   (OUT32: fp32 output)
Runs the default (policy 0) and POL with MT_KNOB=KNOB on randn inputs and on range cases
(a K value past the fp16 range, rows whose scores are all far below zero, a 150x spike) and
prints max-abs O error and max LSE error of each, plus whether the two agree."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip
_DIAG = os.path.join(os.path.dirname(_hip.LIB_PATH), "diag", "libminitorch_hip_diag.so")
if os.environ.get("MT_DIAG") == "1":
    _hip.use_library(_DIAG)
pol, knob = int(sys.argv[1]), sys.argv[2]
causal = len(sys.argv) > 3 and sys.argv[3] == "causal"


def ref(q, k, v):
    s = torch.einsum("bhqd,bhkd->bhqk", q.float(), k.float()) / q.shape[-1] ** 0.5
    if causal:
        n = q.shape[2]
        s = s.masked_fill(torch.ones(n, n, device=q.device, dtype=torch.bool).triu(1), float("-inf"))
    lse = torch.logsumexp(s, -1)
    return torch.einsum("bhqk,bhkd->bhqd", torch.exp(s - lse[..., None]), v.float()), lse


def run(q, k, v, p, kn):
    os.environ["MT_KNOB"] = kn
    _hip.set_policy(p)
    o, m, l = _hip.flash_fwd(q, k, v, causal, out_dtype=torch.float32 if os.environ.get("OUT32") == "1" else None)
    torch.cuda.synchronize()
    return o.float(), m + torch.log(l)


g = torch.Generator(device="cuda").manual_seed(1)
cases = []
for shape in [(2, 4, 1024, 64), (8, 16, 4096, 64), (1, 8, 2048, 64), (2, 2, 256, 64)]:
    q, k, v = (torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16) for _ in range(3))
    cases.append((f"randn {shape}", q, k, v))
shape = (2, 4, 1024, 64)
q, k, v = (torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16) for _ in range(3))
k2 = k.clone(); k2[0, 1, 700, 5] = 70000.0; q2 = q.clone(); q2[0, 1, :, 5] = 1e-6
cases.append(("K past fp16 range (q tiny there)", q2, k2, v))
q3 = q.clone(); q3[1, 2] = 3.0; k3 = k.clone(); k3[1, 2] = -abs(k3[1, 2]) - 2.0
cases.append(("all scores far below zero in one head", q3, k3, v))
q4 = q.clone(); q4[0, 0, 100] *= 150.0
cases.append(("150x spike row", q4, k, v))
q5 = q * 12.0
cases.append(("12x logits", q5, k, v))
for name, q, k, v in cases:
    o_ref, lse_ref = ref(q, k, v)
    o0, l0 = run(q, k, v, 0, "0")
    o1, l1 = run(q, k, v, pol, knob)
    e0 = (o0 - o_ref).abs().max().item(); e1 = (o1 - o_ref).abs().max().item()
    f0 = (l0 - lse_ref).abs().nan_to_num(1e9).max().item(); f1 = (l1 - lse_ref).abs().nan_to_num(1e9).max().item()
    print(f"{name:40s} default O {e0:.3e} lse {f0:.3e} | variant O {e1:.3e} lse {f1:.3e} | "
          f"nonfinite {int((~torch.isfinite(o1)).sum())}", flush=True)
