"""Is the forward power-bound? (diagnostics, GPU box) Interleaved timing of one kernel policy
on the same shape with inputs that differ only in bit activity: randn, randn x 2^-8 (the
same exponent spread, small magnitudes), all zeros, and a constant. A loop whose cycles do
not depend on data (the forward's) runs at equal wall time on all of them unless the chip
lowers its clock for the busier data (MI355X_MICROARCH 'DVFS give-back' item 1).
usage: [MT_DIAG=1] python scripts/power_probe.py POL [KNOB] [causal]"""
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
B, H, N, d = 8, 16, 4096, 64
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
flops = 4.0 * B * H * N * N * d / (2 if causal else 1)
t0 = time.time()
while time.time() - t0 < 1.0:
    _hip.flash_fwd(*arms["randn"], causal, out=o, m=m, l=l); torch.cuda.synchronize()
res = {a: [] for a in arms}
for rnd in range(5):
    for a, (q, k, v) in arms.items():
        for _ in range(20): _hip.flash_fwd(q, k, v, causal, out=o, m=m, l=l)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); e0.record()
        for _ in range(200): _hip.flash_fwd(q, k, v, causal, out=o, m=m, l=l)
        e1.record(); torch.cuda.synchronize()
        res[a].append(e0.elapsed_time(e1) / 200)
print(f"policy {pol} knob {os.environ.get('MT_KNOB')} causal={causal}")
for a in arms:
    t = sorted(res[a]); med = t[len(t) // 2]
    print(f"  {a:10s} median {med:.4f} ms -> {flops / med / 1e9:.1f} TF/s", flush=True)
