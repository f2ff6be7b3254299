import sys, os, numpy as np, torch
sys.path.insert(0, "llmsys-project-flashattn_amd")
from minitorch import _hip
rng = np.random.default_rng(3)
n = 4096
f = np.float32
m0 = (rng.standard_normal(n) * 0.01).astype(np.float32)
g = (rng.standard_normal(n) * 0.01).astype(np.float32)
p = np.zeros(n, np.float32); v = np.zeros(n, np.float32)
dp, dg, dm, dv = (torch.from_numpy(x.copy()).cuda() for x in (p, g, m0, v))
_hip.adam_step([dp.data_ptr()], [dg.data_ptr()], [dm.data_ptr()], [dv.data_ptr()], [n], 0.9, 0.999, 1e-8, 1e-3)
torch.cuda.synchronize()
gm = dm.cpu().numpy()
nm = m0 * f(0.9) + g * f(1 - 0.9)
fm = (m0.astype(np.float64) * np.float64(f(0.9)) + (g * f(1 - 0.9)).astype(np.float64)).astype(np.float32)
bad = np.nonzero(gm != nm)[0]
print("mismatches vs numpy", len(bad), "vs fma-emulation", int((gm != fm).sum()))
for i in bad[:5]:
    print(i, repr(m0[i]), repr(g[i]), "gpu", repr(gm[i]), "np", repr(nm[i]), "fma", repr(fm[i]))
