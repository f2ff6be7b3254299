"""Interleaved in-process A/B timing of forward-kernel policies (diagnostics).
usage: python scripts/ablate.py p1,p2,... [causal]
ENVAB=NAME:v1,v2,...: the arms are values of the environment knob NAME (policy p1)"""
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip
# diagnostics build (make DIAG=1): the product library rejects the ablation policies
_DIAG = os.path.join(os.path.dirname(_hip.LIB_PATH), "diag", "libminitorch_hip_diag.so")
if os.environ.get("MT_DIAG") == "1":  # only when asked: the diag build can be stale
    assert os.path.exists(_DIAG), "make -C llmsys-project-flashattn_amd DIAG=1"
    _hip.use_library(_DIAG)
pols = [int(x) for x in sys.argv[1].split(",")]
env_name, env_vals = None, []
if os.environ.get("ENVAB"):
    env_name, vals = os.environ["ENVAB"].split(":")
    env_vals = vals.split(",")
arms = env_vals if env_vals else pols
causal = len(sys.argv) > 2 and sys.argv[2] == "causal"
B, H, N, d = (int(x) for x in os.environ.get("SHAPE", "8,16,4096,64").split(","))
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((B, H, N, d), device="cuda", generator=g).to(torch.bfloat16) for _ in range(3))
o = torch.empty_like(q, dtype=torch.float32 if os.environ.get("OUT") == "f32" else q.dtype)  # OUT=f32: fp32 output
m = torch.empty((B, H, N), device="cuda"); l = torch.empty_like(m)
res = {p: [] for p in arms}
flops = 4.0 * B * H * N * N * d / (2 if causal else 1)
for rnd in range(int(os.environ.get("ROUNDS", "5"))):
    for p in arms:
        if env_name:
            os.environ[env_name] = p
            _hip.set_policy(pols[0])
        else:
            _hip.set_policy(p)
        for _ in range(3): _hip.flash_fwd(q, k, v, causal, out=o, m=m, l=l)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); e0.record()
        for _ in range(10): _hip.flash_fwd(q, k, v, causal, out=o, m=m, l=l)
        e1.record(); torch.cuda.synchronize()
        res[p].append(e0.elapsed_time(e1) / 10)
for p in arms:
    t = sorted(res[p]); med = t[len(t) // 2]
    print(f"{env_name + '=' + p if env_name else 'policy %3d' % p}: median {med:.4f} ms  min {t[0]:.4f}  -> {flops / med / 1e9:.1f} TF/s")
