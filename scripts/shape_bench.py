"""Forward timing for arbitrary (B,H,N,d) shapes and policies (diagnostics).
usage: python scripts/shape_bench.py B H N d [causal] [policies]
OUT=both: each policy with the bf16 O and with the fp32 O (MT_BF16_F32OUT), interleaved."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip
B, H, N, d = (int(x) for x in sys.argv[1:5])
causal = len(sys.argv) > 5 and sys.argv[5] == "causal"
pols = [int(x) for x in sys.argv[6].split(",")] if len(sys.argv) > 6 else [0]
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((B, H, N, d), device="cuda", generator=g).to(torch.bfloat16) for _ in range(3))
o = torch.empty_like(q); o32 = torch.empty_like(q, dtype=torch.float32); m = torch.empty((B, H, N), device="cuda"); l = torch.empty_like(m)
flops = 4.0 * B * H * N * N * d / (2 if causal else 1)
# untimed clock ramp (~0.3 s of kernels) so the first policy is not measured on a cold GPU
import time
_hip.set_policy(pols[0])
t_ramp = time.perf_counter()
while time.perf_counter() - t_ramp < 0.3:
    _hip.flash_fwd(q, k, v, causal, out=o, m=m, l=l)
    torch.cuda.synchronize()
outs = [("bf16 O", o), ("fp32 O", o32)] if os.environ.get("OUT") == "both" else [("", o)]
for rnd in range(int(os.environ.get("ROUNDS", "1"))):
  for p in pols:
    for tag, ot in outs:
        _hip.set_policy(p)
        for _ in range(2): _hip.flash_fwd(q, k, v, causal, out=ot, m=m, l=l)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); e0.record()
        reps = 5
        for _ in range(reps): _hip.flash_fwd(q, k, v, causal, out=ot, m=m, l=l)
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"({B},{H},{N},{d}) causal={causal} policy {p} {tag}: {ms:.3f} ms  {flops / ms / 1e9:.1f} TF/s")
_hip.set_policy(0)
