"""Is the forward power-bound? (diagnostics, GPU box) Interleaved timing of one kernel policy
on the same shape with inputs that differ only in bit activity: randn, randn x 2^-8 (the
same exponent spread, small magnitudes), all zeros, and a constant. A loop whose cycles do
not depend on data (the forward's) runs at equal wall time on all of them unless the chip
lowers its clock for the busier data (MI355X_MICROARCH 'DVFS give-back' item 1).
usage: [MT_DIAG=1] [PROBE_BWD=1] [PROBE_SHAPE=B,H,N,d] python scripts/power_probe.py POL [KNOB] [causal]
PROBE_BWD=1 times the backward (on the forward's own O, m, l of each arm) instead."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip
if os.environ.get("MT_DIAG") == "1":
    _hip.use_library(os.path.join(os.path.dirname(_hip.LIB_PATH), "diag", "libminitorch_hip_diag.so"))
pol = int(sys.argv[1]) if len(sys.argv) > 1 else 0
if len(sys.argv) > 2:
    os.environ["MT_KNOB"] = sys.argv[2]
causal = len(sys.argv) > 3 and sys.argv[3] == "causal"
_hip.set_policy(pol)
B, H, N, d = (int(x) for x in os.environ.get("PROBE_SHAPE", "8,16,4096,64").split(","))
bwd = os.environ.get("PROBE_BWD") == "1"
g = torch.Generator(device="cuda").manual_seed(0)
base = [torch.randn((B, H, N, d), device="cuda", generator=g) for _ in range(3)]
arms = {
    "randn": [t.to(torch.bfloat16) for t in base],
    "randn/256": [(t / 256).to(torch.bfloat16) for t in base],
    "zeros": [torch.zeros((B, H, N, d), device="cuda", dtype=torch.bfloat16) for _ in range(3)],
    "const0.5": [torch.full((B, H, N, d), 0.5, device="cuda", dtype=torch.bfloat16) for _ in range(3)],
}
o = torch.empty((B, H, N, d), device="cuda", dtype=torch.bfloat16)
m = torch.empty((B, H, N), device="cuda"); l = torch.empty_like(m)
flops = 4.0 * B * H * N * N * d / (2 if causal else 1) * (2.5 if bwd else 1.0)
if bwd:  # per arm: its own forward outputs and dO = its V (same bit activity)
    saved = {}
    for a, (q, k, v) in arms.items():
        oa, ma, la = _hip.flash_fwd(q, k, v, causal)
        saved[a] = (oa, ma, la, v.clone(), torch.empty_like(q), torch.empty_like(q), torch.empty_like(q))
    ws = torch.empty(_hip.lib().mt_flash_attn_bwd_workspace_bytes(B, H, N, d) // 4 + 64, device="cuda")

def call(a):
    q, k, v = arms[a]
    if not bwd:
        _hip.flash_fwd(q, k, v, causal, out=o, m=m, l=l)
        return
    oa, ma, la, do, dq, dk, dv = saved[a]
    _hip.flash_bwd(q, k, v, oa, do, ma, la, causal, dq=dq, dk=dk, dv=dv, workspace=ws)

reps = 50 if bwd else 200
t0 = time.time()
while time.time() - t0 < 1.0:
    call("randn"); torch.cuda.synchronize()
res = {a: [] for a in arms}
for rnd in range(5):
    for a in arms:
        for _ in range(reps // 10): call(a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); e0.record()
        for _ in range(reps): call(a)
        e1.record(); torch.cuda.synchronize()
        res[a].append(e0.elapsed_time(e1) / reps)
print(f"{'backward' if bwd else 'forward'} {(B, H, N, d)} policy {pol} knob {os.environ.get('MT_KNOB')} causal={causal}")
for a in arms:
    t = sorted(res[a]); med = t[len(t) // 2]
    print(f"  {a:10s} median {med:.4f} ms -> {flops / med / 1e9:.1f} TF/s", flush=True)
