"""Interleaved in-process A/B timing of forward-kernel policies (diagnostics, GPU box).
usage: python scripts/ab_fwd.py POL[,POL...] [causal] [B,H,N,d] [rounds]   (DTYPE=fp32 for fp32 I/O,
OUT32=1 for the bf16 kernels' fp32 output)
MT_DIAG=1: the diagnostics library; ENVAB=NAME:v1,v2,..: the arms are values of an environment
knob (e.g. MT_KNOB, read per launch by the diagnostics build) under policy POL"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip
_DIAG = os.path.join(os.path.dirname(_hip.LIB_PATH), "diag", "libminitorch_hip_diag.so")
if os.environ.get("MT_DIAG") == "1":
    assert os.path.exists(_DIAG), "make -C llmsys-project-flashattn_amd DIAG=1"
    _hip.use_library(_DIAG)
# an arm is POL or POL:KNOB (the policy with MT_KNOB=KNOB, read per launch by the diagnostics build)
pols = [x for x in sys.argv[1].split(",")]
env_name, env_vals = None, None
if os.environ.get("ENVAB"):
    env_name, _v = os.environ["ENVAB"].split(":")
    env_vals = _v.split(",")
arms = env_vals if env_vals else pols
causal = len(sys.argv) > 2 and sys.argv[2] == "causal"
B, H, N, d = (int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "8,16,4096,64").split(","))
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 7
g = torch.Generator(device="cuda").manual_seed(0)
dt = torch.float32 if os.environ.get("DTYPE") == "fp32" else torch.bfloat16
q, k, v = (torch.randn((B, H, N, d), device="cuda", generator=g).to(dt) for _ in range(3))
# OUT32=1: the bf16 kernels' fp32 output (MT_BF16_F32OUT)
o = torch.empty_like(q, dtype=torch.float32 if os.environ.get("OUT32") == "1" else q.dtype)
m = torch.empty((B, H, N), device="cuda"); l = torch.empty_like(m)
flops = 4.0 * B * H * N * N * d / (2 if causal else 1)
t0 = time.time()
while time.time() - t0 < 0.5:  # clock ramp
    _hip.flash_fwd(q, k, v, causal, out=o, m=m, l=l); torch.cuda.synchronize()
res = {p: [] for p in arms}
reps = max(int(os.environ.get("REPS", "3")), int(2e12 / flops))
for rnd in range(rounds):
    for p in arms:
        if env_vals:
            os.environ[env_name] = p
            _hip.set_policy(int(pols[0]))
        else:
            pol, _, knob = p.partition(":")
            if knob:
                os.environ["MT_KNOB"] = knob
            else:
                os.environ.pop("MT_KNOB", None)
            _hip.set_policy(int(pol))
        for _ in range(2): _hip.flash_fwd(q, k, v, causal, out=o, m=m, l=l)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); e0.record()
        for _ in range(reps): _hip.flash_fwd(q, k, v, causal, out=o, m=m, l=l)
        e1.record(); torch.cuda.synchronize()
        res[p].append(e0.elapsed_time(e1) / reps)
_hip.set_policy(0)
print(f"shape {(B, H, N, d)} {dt} causal={causal} reps={reps} rounds={rounds}")
for p in arms:
    t = sorted(res[p]); med = t[len(t) // 2]
    print(f"{(env_name + '=' + p) if env_vals else 'policy %6s' % p}: median {med:.4f} ms  min {t[0]:.4f}  -> {flops / med / 1e9:.1f} TF/s", flush=True)
