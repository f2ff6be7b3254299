"""Forward kernel time against grid rounds (diagnostics, GPU box, run under rocprofv3
--kernel-trace): C3-like shapes (B,16,4096,64) for B = 1, 2, 4, 8, 16, each launched 200 times,
so the per-launch fixed cost (prologue / epilogue / ramp) can be fitted from the trace.
usage: rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 scripts/round_fit.py"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip

g = torch.Generator(device="cuda").manual_seed(0)
for B in (1, 2, 4, 8, 16):
    q, k, v = (torch.randn((B, 16, 4096, 64), device="cuda", generator=g).to(torch.bfloat16)
               for _ in range(3))
    o = torch.empty_like(q); m = torch.empty((B, 16, 4096), device="cuda"); l = torch.empty_like(m)
    for _ in range(200):
        _hip.flash_fwd(q, k, v, False, out=o, m=m, l=l)
    torch.cuda.synchronize()
    print("B", B, "done", flush=True)
