"""Same-process interleaved A/B of the bf16 forward across library builds, through the bare
C ABI (each .so loaded with its own ctypes handle: e.g. the product library beside a
timing-only ablation build from scripts/build_abl.sh).
usage: python scripts/fwd_lib_ab.py LIB.so [LIB.so ...]   (SHAPE=B,H,N,d, OUT=f32|bf16,
CAUSAL=1, ROUNDS=n, REPS=n)"""
import ctypes
import os
import sys

import torch

libs = sys.argv[1:]
B, H, N, d = (int(x) for x in os.environ.get("SHAPE", "8,16,4096,64").split(","))
causal = int(os.environ.get("CAUSAL", "0"))
out32 = os.environ.get("OUT", "bf16") == "f32"
vp, i64 = ctypes.c_void_p, ctypes.c_int64
handles = []
for p in libs:
    L = ctypes.CDLL(os.path.abspath(p), mode=ctypes.RTLD_LOCAL)
    L.mt_flash_attn_fwd.argtypes = [ctypes.c_int, ctypes.c_int] + [vp] * 6 + [i64] * 4 + [vp] * 5
    handles.append(L)
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((B, H, N, d), device="cuda", generator=g).to(torch.bfloat16) for _ in range(3))
o = torch.empty(q.shape, dtype=torch.float32 if out32 else torch.bfloat16, device="cuda")
m = torch.empty((B, H, N), device="cuda")
l = torch.empty_like(m)
st = vp(torch.cuda.current_stream().cuda_stream)
dtype = 2 if out32 else 1


def fwd(L):
    assert L.mt_flash_attn_fwd(dtype, causal, q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                               m.data_ptr(), l.data_ptr(), B, H, N, d, None, None, None, None, st) == 0


flops = 4.0 * B * H * N * N * d / (2 if causal else 1)
reps = int(os.environ.get("REPS", "20"))
for L in handles:  # clock ramp
    for _ in range(50):
        fwd(L)
torch.cuda.synchronize()
res = [[] for _ in handles]
for _ in range(int(os.environ.get("ROUNDS", "11"))):
    for i, L in enumerate(handles):
        fwd(L)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fwd(L)
        e1.record()
        torch.cuda.synchronize()
        res[i].append(e0.elapsed_time(e1) / reps)
print(f"shape {(B, H, N, d)} causal={causal} out={'f32' if out32 else 'bf16'} reps={reps}")
for p, t in zip(libs, res):
    t = sorted(t)
    med = t[len(t) // 2]
    print(f"{os.path.basename(p):40s} median {med:.4f} ms  min {t[0]:.4f}  -> {flops / med / 1e9:.1f} TF/s", flush=True)
