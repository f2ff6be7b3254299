"""Same-process interleaved A/B of the bf16 backward across library builds, through the bare
C ABI (each .so with its own ctypes handle; e.g. the product library beside an A/B build from
scripts/build_abl.sh). usage: python scripts/bwd_lib_ab.py LIB.so [LIB.so ...]
(SHAPE=B,H,N,d, CAUSAL=1, ROUNDS=n, REPS=n). Times prep + pass [+ reduce] per call."""
import ctypes
import os
import sys

import torch

libs = sys.argv[1:]
B, H, N, d = (int(x) for x in os.environ.get("SHAPE", "8,16,4096,64").split(","))
causal = int(os.environ.get("CAUSAL", "0"))
vp, i64 = ctypes.c_void_p, ctypes.c_int64
handles = []
for p in libs:
    L = ctypes.CDLL(os.path.abspath(p), mode=ctypes.RTLD_LOCAL)
    L.mt_flash_attn_bwd_workspace_bytes.restype = i64
    L.mt_flash_attn_bwd_workspace_bytes.argtypes = [i64] * 4
    L.mt_flash_attn_fwd.argtypes = [ctypes.c_int, ctypes.c_int] + [vp] * 6 + [i64] * 4 + [vp] * 5
    L.mt_flash_attn_bwd_v3.argtypes = [ctypes.c_int, ctypes.c_int] + [vp] * 10 + [i64] * 4 + [vp, vp, vp, i64, vp]
    handles.append(L)
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v, do = (torch.randn((B, H, N, d), device="cuda", generator=g).to(torch.bfloat16) for _ in range(4))
o = torch.empty_like(q)
m = torch.empty((B, H, N), device="cuda")
l = torch.empty_like(m)
st = vp(torch.cuda.current_stream().cuda_stream)
assert handles[0].mt_flash_attn_fwd(1, causal, q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                    m.data_ptr(), l.data_ptr(), B, H, N, d, None, None, None, None, st) == 0
wsb = max(L.mt_flash_attn_bwd_workspace_bytes(B, H, N, d) for L in handles)
ws = torch.empty(wsb // 4 + 64, device="cuda")
dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)


def bwd(L):
    assert L.mt_flash_attn_bwd_v3(1, causal, q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                  do.data_ptr(), m.data_ptr(), l.data_ptr(), dq.data_ptr(), dk.data_ptr(),
                                  dv.data_ptr(), B, H, N, d, None, None, ws.data_ptr(), ws.numel() * 4, st) == 0


flops = 2.5 * 4.0 * B * H * N * N * d / (2 if causal else 1)
reps = int(os.environ.get("REPS", "10"))
for L in handles:
    for _ in range(10):
        bwd(L)
torch.cuda.synchronize()
res = [[] for _ in handles]
for _ in range(int(os.environ.get("ROUNDS", "9"))):
    for i, L in enumerate(handles):
        bwd(L)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            bwd(L)
        e1.record()
        torch.cuda.synchronize()
        res[i].append(e0.elapsed_time(e1) / reps)
print(f"bwd shape {(B, H, N, d)} causal={causal} reps={reps}")
for p, t in zip(libs, res):
    t = sorted(t)
    med = t[len(t) // 2]
    print(f"{os.path.basename(p):40s} median {med:.4f} ms  min {t[0]:.4f}  -> {flops / med / 1e9:.1f} TF/s", flush=True)
