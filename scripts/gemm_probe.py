"""Config 5's LM-head GEMMs through mt_matmul_f32 (rocBLAS sgemm) in each operand layout, and
torch.matmul (hipBLASLt) beside them: C[4992,10000] = X[4992,256] @ W[256,10000] (forward),
dX = dC @ Wᵀ and dW = Xᵀ @ dC (backward). HIP events over 30 calls each; prints JSON (µs,
TF/s) so the layout choice in combine.hip's gemm_rocblas can be made from measurements.
usage: python scripts/gemm_probe.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llmsys-project-flashattn_amd"))
import torch

from minitorch import _hip

lib = _hip.lib()
M, K, N = 4992, 256, 10000
torch.manual_seed(0)
x = torch.randn(M, K, device="cuda")
w = torch.randn(K, N, device="cuda")
dc = torch.randn(M, N, device="cuda")


def mm(c, a, b, m, n, k):
    """c[m,n] = a[m,k] @ b[k,n] with arbitrary 2-D strides (torch views)."""
    s = lambda t: (ctypes.c_int64 * 3)(0, t.stride(0), t.stride(1))  # noqa: E731
    _hip.check(lib.mt_matmul_f32(c.data_ptr(), a.data_ptr(), b.data_ptr(), 1, m, n, k, s(a), s(b), s(c),
                                 _hip.stream_ptr()), "mt_matmul_f32")


def timed(fn, it=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


out = {}
flop = 2.0 * M * N * K
c = torch.empty(M, N, device="cuda")
wt = w.t().contiguous()  # [N, K]: W stored transposed
xt = x.t().contiguous()  # [K, M]
cases = {
    "fwd NN (W [K,N])": lambda: mm(c, x, w, M, N, K),
    "fwd W as [N,K]ᵀ view": lambda: mm(c, x, wt.t(), M, N, K),
    "fwd X as [K,M]ᵀ view": lambda: mm(c, xt.t(), w, M, N, K),
    "fwd both transposed views": lambda: mm(c, xt.t(), wt.t(), M, N, K),
    "fwd torch.matmul": lambda: torch.matmul(x, w, out=c),
}
ref = x @ w
for name, fn in cases.items():
    us = timed(fn)
    fn()
    torch.cuda.synchronize()
    out[name] = {"us": round(us, 1), "TF/s": round(flop / us / 1e6, 1),
                 "max_rel": float(((c - ref).abs().max() / ref.abs().max()).item())}
dx = torch.empty(M, K, device="cuda")
dw = torch.empty(K, N, device="cuda")
cases_b = {
    "dX = dC @ Wᵀ (W view)": lambda: mm(dx, dc, w.t(), M, K, N),
    "dX = dC @ (Wᵀ copy)": lambda: mm(dx, dc, wt, M, K, N),
    "dW = Xᵀ @ dC (X view)": lambda: mm(dw, x.t(), dc, K, N, M),
    "dW = (Xᵀ copy) @ dC": lambda: mm(dw, xt, dc, K, N, M),
    "dX torch": lambda: torch.matmul(dc, w.t(), out=dx),
    "dW torch": lambda: torch.matmul(x.t(), dc, out=dw),
}
for name, fn in cases_b.items():
    us = timed(fn)
    out[name] = {"us": round(us, 1), "TF/s": round(flop / us / 1e6, 1)}
# the 256 x 256 linears (48 + 24 per step): Y = X W, dX = dY Wᵀ, dW = Xᵀ dY
E = 256
x2 = torch.randn(M, E, device="cuda")
w2 = torch.randn(E, E, device="cuda")
dy2 = torch.randn(M, E, device="cuda")
y2 = torch.empty(M, E, device="cuda")
dw2 = torch.empty(E, E, device="cuda")
w2t = w2.t().contiguous()
x2t = x2.t().contiguous()
f2 = 2.0 * M * E * E
cases_s = {
    "lin Y = X W": lambda: mm(y2, x2, w2, M, E, E),
    "lin Y torch": lambda: torch.matmul(x2, w2, out=y2),
    "lin dX = dY Wᵀ (view)": lambda: mm(y2, dy2, w2.t(), M, E, E),
    "lin dX = dY (Wᵀ copy)": lambda: mm(y2, dy2, w2t, M, E, E),
    "lin dX torch": lambda: torch.matmul(dy2, w2.t(), out=y2),
    "lin dW = Xᵀ dY (view)": lambda: mm(dw2, x2.t(), dy2, E, E, M),
    "lin dW = (Xᵀ copy) dY": lambda: mm(dw2, x2t, dy2, E, E, M),
    "lin dW torch": lambda: torch.matmul(x2.t(), dy2, out=dw2),
}
for name, fn in cases_s.items():
    us = timed(fn, 200)
    out[name] = {"us": round(us, 2), "TF/s": round(f2 / us / 1e6, 1)}
# split-K for dX (K = 10000 over S batched slices, then a fixed-order sum of the S partials)


def mmb(c, a, b, batch, m, n, k, sa, sb, sc):
    arr = lambda t: (ctypes.c_int64 * 3)(*t)  # noqa: E731
    _hip.check(lib.mt_matmul_f32(c.data_ptr(), a.data_ptr(), b.data_ptr(), batch, m, n, k, arr(sa), arr(sb),
                                 arr(sc), _hip.stream_ptr()), "mt_matmul_f32")


refdx = dc @ wt
for S in (2, 4, 5, 8, 10):
    ks = N // S
    part = torch.empty(S, M, K, device="cuda")

    def fn(S=S, ks=ks, part=part):
        mmb(part, dc, wt, S, M, K, ks, (ks, N, 1), (ks * K, K, 1), (M * K, K, 1))
        torch.sum(part, 0, out=dx)
    us = timed(fn)
    fn()
    torch.cuda.synchronize()
    out[f"dX split-K S={S}"] = {"us": round(us, 1), "TF/s": round(flop / us / 1e6, 1),
                                "max_rel": float(((dx - refdx).abs().max() / refdx.abs().max()).item())}
# split-K for the linears' dW (256 x 256 over K = 4992)
for S in (2, 4, 8):
    ks = M // S
    part2 = torch.empty(S, E, E, device="cuda")

    def fn2(S=S, ks=ks, part2=part2):
        mmb(part2, x2t, dy2, S, E, E, ks, (ks, M, 1), (ks * E, E, 1), (E * E, E, 1))
        torch.sum(part2, 0, out=dw2)
    out[f"lin dW split-K S={S} (Xᵀ copy)"] = {"us": round(timed(fn2, 200), 2)}

    def fn3(S=S, ks=ks, part2=part2):
        mmb(part2, x2.t(), dy2, S, E, E, ks, (ks * E, 1, E), (ks * E, E, 1), (E * E, E, 1))
        torch.sum(part2, 0, out=dw2)
    out[f"lin dW split-K S={S} (X view)"] = {"us": round(timed(fn3, 200), 2)}
out["preferred_blas"] = str(torch.backends.cuda.preferred_blas_library())
print(json.dumps(out, indent=1))
