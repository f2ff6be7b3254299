"""Config-2 fp32 forward + backward on the HIP path (rocprofv3 PMC target, GPU box)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llmsys-project-flashattn_amd")]
import torch
from minitorch import _hip
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v, do = (torch.randn((8, 16, 1024, 64), device="cuda", generator=g) for _ in range(4))
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    o, m, l = _hip.flash_fwd(q, k, v, False)
    _hip.flash_bwd(q, k, v, o, do, m, l, False)
torch.cuda.synchronize()
print("ok")
