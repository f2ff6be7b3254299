"""Backward timing through the bare C ABI of any library build (same-box A/B of builds whose
Python bindings differ, e.g. the round-3 library beside the current one).
usage: python scripts/bwd_lib_time.py LIB.so [causal]   (SHAPE=B,H,N,d; bf16)
Prints the mean backward time (prep + fused pass [+ reduce]) over 5 rounds of 5 calls."""
import ctypes
import os
import sys

import torch

lib_path = sys.argv[1]
causal = len(sys.argv) > 2 and sys.argv[2] == "causal"
B, H, N, d = (int(x) for x in os.environ.get("SHAPE", "8,16,4096,64").split(","))
L = ctypes.CDLL(os.path.abspath(lib_path))
vp, i64 = ctypes.c_void_p, ctypes.c_int64
L.mt_flash_attn_bwd_workspace_bytes.restype = i64
L.mt_flash_attn_bwd_workspace_bytes.argtypes = [i64] * 4
L.mt_flash_attn_fwd.argtypes = [ctypes.c_int, ctypes.c_int] + [vp] * 6 + [i64] * 4 + [vp] * 5
L.mt_flash_attn_bwd.argtypes = [ctypes.c_int, ctypes.c_int] + [vp] * 10 + [i64] * 4 + [vp] * 3
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v, do = (torch.randn((B, H, N, d), device="cuda", generator=g).to(torch.bfloat16) for _ in range(4))
o = torch.empty_like(q)
m = torch.empty((B, H, N), device="cuda")
l = torch.empty_like(m)
st = vp(torch.cuda.current_stream().cuda_stream)
assert L.mt_flash_attn_fwd(1, int(causal), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                           m.data_ptr(), l.data_ptr(), B, H, N, d, None, None, None, None, st) == 0
ws = torch.empty(L.mt_flash_attn_bwd_workspace_bytes(B, H, N, d) // 4 + 64, device="cuda")
dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)


def bwd():
    assert L.mt_flash_attn_bwd(1, int(causal), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                               do.data_ptr(), m.data_ptr(), l.data_ptr(), dq.data_ptr(), dk.data_ptr(),
                               dv.data_ptr(), B, H, N, d, None, ws.data_ptr(), st) == 0


flops = 2.5 * 4.0 * B * H * N * N * d / (2 if causal else 1)
ts = []
for _ in range(3):
    bwd()
for rnd in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(5):
        bwd()
    e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 5)
ms = sorted(ts)[len(ts) // 2]
print(f"{os.path.basename(lib_path)} ({B},{H},{N},{d}) causal={causal}: bwd {ms:.4f} ms "
      f"(median of 5; min {min(ts):.4f}) {flops / ms / 1e9:.1f} TF/s")
