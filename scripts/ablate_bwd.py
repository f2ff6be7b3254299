"""Interleaved in-process A/B timing of backward kernel policies (diagnostics).
usage: python scripts/ablate_bwd.py p1,p2,... [causal]   (SHAPE=B,H,N,d, DTYPE=fp32)
ENVAB=NAME:v1,v2,...: the arms are values of the environment knob NAME (policy p1)"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip
# diagnostics build (make DIAG=1): the product library rejects the ablation policies
_DIAG = os.path.join(os.path.dirname(_hip.LIB_PATH), "diag", "libminitorch_hip_diag.so")
if os.environ.get("MT_DIAG") == "1":  # only when asked: the diag build can be stale
    assert os.path.exists(_DIAG), "make -C llmsys-project-flashattn_amd DIAG=1"
    _hip.use_library(_DIAG)
pols = [int(x) for x in sys.argv[1].split(",")]
env_name, env_vals = None, None
if os.environ.get("ENVAB"):
    env_name, vals = os.environ["ENVAB"].split(":")
    env_vals = vals.split(",")
arms = env_vals if env_vals else pols
causal = len(sys.argv) > 2 and sys.argv[2] == "causal"
B, H, N, d = (int(x) for x in os.environ.get("SHAPE", "8,16,4096,64").split(","))
dt = torch.float32 if os.environ.get("DTYPE") == "fp32" else torch.bfloat16
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v, do = (torch.randn((B, H, N, d), device="cuda", generator=g).to(dt) for _ in range(4))
o, m, l = _hip.flash_fwd(q, k, v, causal)
ws = torch.empty(_hip.lib().mt_flash_attn_bwd_workspace_bytes(B, H, N, d) // 4, device="cuda")
dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
flops = 2.5 * 4.0 * B * H * N * N * d / (2 if causal else 1)
res = {p: [] for p in arms}
for rnd in range(int(os.environ.get("ROUNDS", "5"))):
    for p in arms:
        if env_vals:
            os.environ[env_name] = p
            _hip.set_policy(pols[0])
        else:
            _hip.set_policy(p)
        for _ in range(2):
            _hip.flash_bwd(q, k, v, o, do, m, l, causal, dq=dq, dk=dk, dv=dv, workspace=ws)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); e0.record()
        for _ in range(5):
            _hip.flash_bwd(q, k, v, o, do, m, l, causal, dq=dq, dk=dk, dv=dv, workspace=ws)
        e1.record(); torch.cuda.synchronize()
        res[p].append(e0.elapsed_time(e1) / 5)
_hip.set_policy(0)
print(f"shape {(B, H, N, d)} {dt} causal={causal}")
for p in arms:
    t = sorted(res[p]); med = t[len(t) // 2]
    print(f"bwd {(env_name + '=' + p) if env_vals else 'policy %3d' % p}: median {med:.4f} ms  min {t[0]:.4f}  -> {flops / med / 1e9:.1f} TF/s (FA-2 convention)")
