"""Which HIP runtime the process binds when the library loads before / after torch (GPU box)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
order = sys.argv[1] if len(sys.argv) > 1 else "lib-first"
def maps():
    m = open("/proc/self/maps").read()
    return sorted(set(l.split()[-1] for l in m.splitlines() if "amdhip" in l or "hsa-runtime" in l))
if order == "lib-first":
    from minitorch import _hip
    _hip.lib()
    print("after lib:", maps())
import torch
print("after torch import:", maps())
x = torch.randn((1, 1, 128, 64), device="cuda").to(torch.bfloat16)
print("after torch cuda:", maps(), torch.version.hip)
from minitorch import _hip
o, m, l = _hip.flash_fwd(x, x, x, False)
torch.cuda.synchronize()
print("flash ok", float(o.float().abs().sum()))
