"""The X3 fp32 GEMM (mt_set_gemm_backend(2): bf16 MFMA in three pieces per operand) against
rocBLAS (backend 0) on config 5's GEMMs in the operand layouts minitorch hands over: error over
max|ref| against an fp64 torch matmul, and HIP-event time per call.
usage: python scripts/gemm_x3_probe.py
(backend 3: the X3 GEMM on 64x64 tiles only; backend 2: 128x128 tiles where they fill the chip)"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llmsys-project-flashattn_amd"))
import torch

from minitorch import _hip

lib = _hip.lib()


def mm(c, a, b):
    """c[m,n] = a[m,k] @ b[k,n] with arbitrary 2-D strides (torch views)."""
    s = lambda t: (ctypes.c_int64 * 3)(0, t.stride(0), t.stride(1))  # noqa: E731
    M, K = a.shape
    N = b.shape[1]
    _hip.check(lib.mt_matmul_f32(c.data_ptr(), a.data_ptr(), b.data_ptr(), 1, M, N, K, s(a), s(b), s(c),
                                 _hip.stream_ptr()), "mt_matmul_f32")


def timed(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


torch.manual_seed(0)
T, E, V = 4992, 256, 10000
x = torch.randn(T, E, device="cuda")
w = torch.randn(E, E, device="cuda") * 0.05
dy = torch.randn(T, E, device="cuda")
wl = torch.randn(E, V, device="cuda") * 0.05
dc = torch.randn(T, V, device="cuda") * 0.01
cases = {
    "linear fwd  [4992,256]x[256,256]": (x, w),
    "linear dX   dY x Wt (B col-major)": (dy, w.t()),
    "linear dW   Xt x dY (A col-major, K=4992)": (x.t(), dy),
    "lm-head fwd [4992,256]x[256,10000]": (x, wl),
    "lm-head dX  dC x Wt (K=10000)": (dc, wl.t()),
    "lm-head dW  Xt x dC (K=4992)": (x.t(), dc),
    "ragged      [333,77]x[77,45]": (torch.randn(333, 77, device="cuda"), torch.randn(77, 45, device="cuda")),
}
for name, (a, b) in cases.items():
    ref = (a.double() @ b.double())
    out = {}
    for be in (0, 3, 2):
        lib.mt_set_gemm_backend(be)
        c = torch.empty(a.shape[0], b.shape[1], device="cuda")
        mm(c, a, b)
        torch.cuda.synchronize()
        err = float((c.double() - ref).abs().max() / ref.abs().max())
        us = timed(lambda: mm(c, a, b))
        out[be] = (err, us)
    lib.mt_set_gemm_backend(0)
    print(f"{name:44s} rocBLAS {out[0][1]:8.1f} us err {out[0][0]:.2e} | x3-64 {out[3][1]:8.1f} us err "
          f"{out[3][0]:.2e} | x3 {out[2][1]:8.1f} us err {out[2][0]:.2e}", flush=True)
