"""bf16 forward and backward time at (8,16,4096,d) for head dims outside the d = 64 / 128
kernels (d = 32, 48, 96) beside d = 64 and 128: which kernels the product dispatches there and
their TFLOP/s. usage: python scripts/headdim_bench.py [d,d,...]"""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip
ds = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [32, 48, 64, 96, 128]
out = {}
for d in ds:
    B, H, N = 8, 16, 4096
    g = torch.Generator(device="cuda").manual_seed(d)
    q, k, v, do = (torch.randn((B, H, N, d), device="cuda", generator=g).to(torch.bfloat16) for _ in range(4))
    for causal in (False, True):
        o, m, l = _hip.flash_fwd(q, k, v, causal)
        ws = torch.empty(_hip.lib().mt_flash_attn_bwd_workspace_bytes(B, H, N, d) // 4, device="cuda")
        def fwd():
            _hip.flash_fwd(q, k, v, causal, out=o, m=m, l=l)
        def bwd():
            _hip.flash_bwd(q, k, v, o, do, m, l, causal, workspace=ws)
        res = {}
        for name, fn, mult in (("fwd", fwd, 4.0), ("bwd", bwd, 10.0)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            res[name + "_ms"] = round(ms, 3)
            res[name + "_tflops"] = round(mult * B * H * N * N * d / (2 if causal else 1) / ms / 1e9, 1)
        out[f"d={d}{' causal' if causal else ''}"] = res
        print(json.dumps({f"d={d}{' causal' if causal else ''}": res}), flush=True)
