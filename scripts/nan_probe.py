"""Finite-output sweep of the product bf16 forward (O, m, l) and backward (dQ, dK, dV) over ragged,
causal and key-padded shapes at d = 64 and 128, plus a cheap consistency check per shape: the
backward's dV against dV = Pᵀ·dO from a torch fp32 recomputation of P. Prints one line per shape
and a final count of failures; exits 1 if any output is non-finite or dV is off."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import torch
from minitorch import _hip
g = torch.Generator(device="cuda").manual_seed(5)
shapes = []
for d in (48, 64, 96, 128):
    for N in (65, 127, 255, 257, 511, 513, 1000, 1023, 1025, 2049, 4001):
        for causal in (False, True):
            shapes.append(((2, 3, N, d), causal, None))
    shapes.append(((3, 4, 1000, d), False, [1000, 700, 1]))
    shapes.append(((3, 4, 1000, d), True, [999, 513, 64]))
bad_total = 0
for shape, causal, kv in shapes:
    B, H, N, d = shape
    q, k, v, do = (torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16) for _ in range(4))
    kvt = None if kv is None else torch.tensor(kv, dtype=torch.int32, device="cuda")
    o, m, l = _hip.flash_fwd(q, k, v, causal, kv_len=kvt)
    dq, dk, dv = _hip.flash_bwd(q, k, v, o, do, m, l, causal, kv_len=kvt)
    torch.cuda.synchronize()
    out = []
    nbad = 0
    for name, t in (("o", o), ("m", m), ("l", l), ("dq", dq), ("dk", dk), ("dv", dv)):
        b = int((~torch.isfinite(t.float())).sum())
        nbad += b
        if b:
            out.append(f"{name}:{b}")
    # dV = Pᵀ dO in fp32 from the inputs (masked keys have P = 0)
    s = torch.einsum("bhqd,bhkd->bhqk", q.float(), k.float()) / d ** 0.5
    if causal:
        s = s.masked_fill(torch.ones(N, N, device="cuda", dtype=torch.bool).triu(1), float("-inf"))
    if kv is not None:
        s = s.masked_fill(torch.arange(N, device="cuda")[None, None, None, :] >= kvt[:, None, None, None], float("-inf"))
    p = torch.softmax(s, -1).nan_to_num(0.0)
    dv_ref = torch.einsum("bhqk,bhqd->bhkd", p, do.float())
    err = float((dv.float() - dv_ref).abs().max())
    ok_dv = err < 0.05 + 0.02 * float(dv_ref.abs().max())
    if nbad or not ok_dv:
        bad_total += 1
    print(shape, "causal" if causal else "", "kv" if kv else "", "nonfinite:" + (",".join(out) or "0"),
          f"dv_err {err:.3e}", "" if ok_dv else "DV-OFF", flush=True)
print("failures:", bad_total)
sys.exit(1 if bad_total else 0)
