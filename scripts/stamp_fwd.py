"""Where the d = 64 forward's tile loop spends its cycles: the diagnostics build's stamped v6
(policy 144 = the default 140 with s_memtime stamps at the phase boundaries of the bulk loop,
each followed by an lgkmcnt(0)), C3 (8,16,4096,64) bf16. Per wave the kernel sums the cycles
of [DMA issue, P1 QK_A, P2 PV_B, P3 QK_B, P4 PV_A, vmcnt(0), barrier] over its tiles; this
prints the per-tile mean of each segment (median over waves), the shares, and the same for
waves 0-3 and 4-7 (the SIMD partners). The stamps perturb the schedule (each drains the LDS
reads in flight): read the shares, not the length. Writes JSON with --json FILE.
usage: MT_DIAG=1 python scripts/stamp_fwd.py [--json FILE]"""
import json
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import ctypes
import numpy as np
import torch
from minitorch import _hip

_hip.use_library(os.path.join(os.path.dirname(_hip.LIB_PATH), "diag", "libminitorch_hip_diag.so"))
lib = _hip.lib()
lib.mt_diag_set_debug_buffer.argtypes = [ctypes.c_void_p]
B, H, N, d = 8, 16, 4096, 64
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((B, H, N, d), device="cuda", generator=g).to(torch.bfloat16) for _ in range(3))
nblk = (N // 512) * B * H
dbg = torch.zeros(nblk * 8 * 8, dtype=torch.int64, device="cuda")
lib.mt_diag_set_debug_buffer(ctypes.c_void_p(dbg.data_ptr()))
o = torch.empty_like(q)
m = torch.empty((B, H, N), device="cuda"); l = torch.empty_like(m)
res = {}
for pol in (140, 144):
    _hip.set_policy(pol)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:  # steady clock
        for _ in range(20):
            _hip.flash_fwd(q, k, v, False, out=o, m=m, l=l)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        _hip.flash_fwd(q, k, v, False, out=o, m=m, l=l)
    e1.record(); torch.cuda.synchronize()
    res[pol] = e0.elapsed_time(e1) / 50
_hip.set_policy(0)
a = dbg.view(nblk, 8, 8).cpu().numpy().astype(np.float64)
tiles = a[:, :, 7] .clip(min=1)
per_tile = a[:, :, :7] / tiles[:, :, None]
names = ["dma_issue", "P1_qk_A", "P2_pv_B", "P3_qk_B", "P4_pv_A", "vmcnt0", "barrier"]
out = {"shape": [B, H, N, d], "ms_default_140": res[140], "ms_stamped_144": res[144],
       "note": "cycles per tile per wave (s_memtime ticks), median over waves; stamps perturb: read shares"}
for tag, sel in (("all", slice(0, 8)), ("waves0-3", slice(0, 4)), ("waves4-7", slice(4, 8))):
    med = np.median(per_tile[:, sel, :].reshape(-1, 7), axis=0)
    tot = med.sum()
    out[tag] = {n: {"cycles": round(float(c), 1), "share": round(float(c / tot), 4)} for n, c in zip(names, med)}
    out[tag]["total_cycles_per_tile"] = round(float(tot), 1)
print(f"default 140: {res[140]:.4f} ms, stamped 144: {res[144]:.4f} ms")
for tag in ("all", "waves0-3", "waves4-7"):
    print(tag, "total/tile", out[tag]["total_cycles_per_tile"],
          " ".join(f"{n}={out[tag][n]['cycles']:.0f}({100 * out[tag][n]['share']:.1f}%)" for n in names))
if "--json" in sys.argv:
    json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
