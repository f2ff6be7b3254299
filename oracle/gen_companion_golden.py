"""Companion-kernel golden vectors -- TEST INFRASTRUCTURE, runs only in the build container.

Writes ``tests/golden/softmax_*.npz`` and ``tests/golden/layernorm_*.npz`` by running the
*reference's own* minitorch compositions that its kernel tests use as the baseline for the
fused kernels:

* attention softmax fw: ``minitorch.nn.softmax(inp + mask, dim=3)`` with a
  ``[B,1,1,to]`` padding mask of ``-1e8`` (reference kernel_tests/test_softmax_fw.py:14-74);
* attention softmax bw: ``soft * (dout - sum(dout * soft, dim=3))`` with
  ``soft = nn.softmax(inp, dim=3)`` (kernel_tests/test_softmax_bw.py:14-59);
* LayerNorm fw: ``gamma * (x - mean) / (var + 1e-8) ** 0.5 + beta`` with the tensor's
  own ``mean`` / ``var`` (kernel_tests/test_layernorm_fw.py:22-76);
* LayerNorm bw: the reference's composition for dgamma, dbeta and dinp
  (kernel_tests/test_layernorm_bw.py:22-92).

Inputs follow the reference's TestDecorator (reference test_utils.py): uniform [-1, 1)
values, the padding mask's valid length drawn per batch row, nhead = 8, hidden size 64
(``head_dim * nhead * io_factor`` = 1 * 8 * 8), shapes drawn by ``bs_sl`` but capped so
the reference's pure-Python FastOps (numba is absent; same stand-in as gen_golden.py)
finishes in seconds. Only numeric arrays are written; nothing of the reference is copied.

Usage (repo root, build container only)::

    python oracle/gen_companion_golden.py
"""
from __future__ import annotations

import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import OUT, _import_reference  # noqa: E402

# (name, batch, from_len, to_len, seed); softmax shapes are [batch, 8, from, to]
SOFTMAX_CASES = [("a", 2, 13, 29, 0), ("b", 1, 40, 64, 1), ("c", 3, 7, 5, 2), ("d", 1, 12, 512, 3)]
# (name, rows, hidden, seed)
LN_CASES = [("a", 37, 64, 0), ("b", 96, 64, 1), ("c", 5, 128, 2), ("d", 1024, 64, 3)]
NHEAD = 8


def _u(rng, shape):
    return (rng.random(shape, dtype=np.float32) - 0.5) * 2


def softmax_case(mt, backend, B, F, T, seed):
    rng = np.random.default_rng(seed)
    prng = random.Random(seed)
    inp = _u(rng, (B, NHEAD, F, T))
    dout = _u(rng, (B, NHEAD, F, T))
    pad = np.zeros((B, T), np.float32)
    for b in range(B):  # reference test_utils.attn_mask: 1 marks padding
        pad[b, prng.randint(1, T):] = 1
    mask = (pad * -1e8)[:, None, None, :]
    t = lambda a: mt.tensor_from_numpy(np.ascontiguousarray(a, np.float32), backend, True)
    fw = mt.nn.softmax(t(inp) + t(mask), dim=3)
    soft = mt.nn.softmax(t(inp), dim=3)
    g = t(dout)
    tsum = (g * soft).sum(dim=3).view(B, NHEAD, F, 1)
    bw = soft * (g - tsum)
    return dict(inp=inp, mask_bt=pad * -1e8, dout=dout,
                fw=fw.to_numpy().astype(np.float32), soft_nomask=soft.to_numpy().astype(np.float32),
                bw=bw.to_numpy().astype(np.float32),
                source=np.array("reference minitorch nn.softmax compositions of kernel_tests/"
                                "test_softmax_fw.py and test_softmax_bw.py (numba stand-in)"))


def layernorm_case(mt, backend, R, H, seed):
    rng = np.random.default_rng(seed)
    x, dout = _u(rng, (R, H)), _u(rng, (R, H))
    gamma, beta = _u(rng, (H,)), _u(rng, (H,))
    t = lambda a, rg=True: mt.tensor_from_numpy(np.ascontiguousarray(a, np.float32), backend, rg)
    xi, g_, b_ = t(x), t(gamma), t(beta)
    mean = xi.mean(dim=1).view(R, 1)
    var = xi.var(dim=1).view(R, 1)
    fw = g_ * ((xi - mean) / ((var + 1e-8) ** 0.5)) + b_
    # backward composition (kernel_tests/test_layernorm_bw.py baseline); its stds come from
    # the tensor var without eps, as there
    f_input = t(x)
    f_means = f_input.mean(dim=1)
    f_vars = f_input.var(dim=1)
    f_stds = t(np.sqrt(f_vars.to_numpy()).reshape(-1, 1))
    go = t(dout)
    xhat = (f_input - f_means) / f_stds
    dxhat = go * t(gamma)
    dbeta = go.sum(dim=0)
    dgamma = (go * xhat).sum(dim=0)
    dinp = dxhat.sum(dim=1) + xhat * (dxhat * xhat).sum(dim=1)
    dinp = (dxhat - dinp / H) / f_stds
    f32 = lambda z: z.to_numpy().astype(np.float32)
    return dict(x=x, gamma=gamma, beta=beta, dout=dout, fw=f32(fw),
                var=f32(f_vars).reshape(R), mean=f32(f_means).reshape(R),
                dgamma=f32(dgamma).reshape(H), dbeta=f32(dbeta).reshape(H), dinp=f32(dinp),
                source=np.array("reference minitorch compositions of kernel_tests/"
                                "test_layernorm_fw.py and test_layernorm_bw.py (numba stand-in)"))


def main():
    mt, backend = _import_reference()
    for name, B, F, T, seed in SOFTMAX_CASES:
        t0 = time.time()
        path = os.path.join(OUT, f"softmax_{name}.npz")
        np.savez_compressed(path, **softmax_case(mt, backend, B, F, T, seed))
        print(f"softmax {name}: [{B},{NHEAD},{F},{T}] -> {path} [{time.time() - t0:.1f}s]")
    for name, R, H, seed in LN_CASES:
        t0 = time.time()
        path = os.path.join(OUT, f"layernorm_{name}.npz")
        np.savez_compressed(path, **layernorm_case(mt, backend, R, H, seed))
        print(f"layernorm {name}: [{R},{H}] -> {path} [{time.time() - t0:.1f}s]")


if __name__ == "__main__":
    main()
