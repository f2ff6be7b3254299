"""Companion kernels (csrc/softmax_layernorm.hip) through the C ABI at the shapes that select
each code path: the register-resident row kernels for every NV (row length a multiple of 4,
1 .. 16 float4 per lane, partial last pieces), the scalar kernels (row length not a multiple
of 4, longer than 4096, or a misaligned base), broadcast and full masks, the future mask, the
fused LayerNorm backward (a wave per row up to hidden 1024, a workgroup per row above; row
counts not a multiple of 4 and larger than the grid) and its scalar form (hidden % 4 != 0). References are float64 NumPy
restatements of the contracts the kernels cite (reference src/softmax_kernel.cu:35-224,
:308-341; src/layernorm_kernel.cu:36-98, :192-368), at the reference kernel tests' tolerances
(kernel_tests/test_softmax_fw.py:14 1e-3, test_softmax_bw.py:14 1e-2/1e-3,
test_layernorm_fw.py:22 1e-2/1e-3, test_layernorm_bw.py:22 1e-3/1e-2)."""
import ctypes
import zlib
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "llmsys-project-flashattn_amd"))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from minitorch import _hip
    return torch, _hip


def _softmax_ref(x, mask, future):
    z = x.astype(np.float64)
    if mask is not None:
        z = z + mask
    if future:
        F, T = x.shape[-2:]
        z = np.where(np.triu(np.ones((F, T)), 1) > 0, -1e8, z)
    e = np.exp(z - z.max(-1, keepdims=True))
    return e / (e.sum(-1, keepdims=True) + 1e-8)


@pytest.mark.parametrize("shape", [(2, 3, 5, 64), (1, 2, 7, 256), (2, 2, 9, 260), (1, 1, 16, 1024),
                                   (1, 2, 3, 2048), (1, 1, 4, 4096), (2, 2, 6, 39), (1, 1, 3, 4100),
                                   (1, 2, 65, 1000)])
@pytest.mark.parametrize("mode", ["none", "padmask", "fullmask", "future"])
def test_softmax_fw_bw(hip, shape, mode):
    torch, _hip = hip
    L, s = _hip.lib(), _hip.stream_ptr()
    rng = np.random.default_rng(zlib.crc32(repr((shape, mode)).encode()))
    B, nh, F, T = shape
    x = (rng.standard_normal(shape) * 3).astype(np.float32)
    mask, ms = None, None
    if mode == "padmask":  # [B, to] additive padding mask, broadcast over heads and rows
        mask = ((rng.random((B, T)) < 0.3) * -1e4).astype(np.float32)
        ms = (ctypes.c_int64 * 4)(T, 0, 0, 1)
    elif mode == "fullmask":  # [B, nh, from, to]
        mask = (rng.standard_normal(shape) * 2).astype(np.float32)
        ms = (ctypes.c_int64 * 4)(nh * F * T, F * T, T, 1)
    xd = torch.from_numpy(x).cuda()
    md = torch.from_numpy(mask).cuda() if mask is not None else None
    out = torch.empty_like(xd)
    _hip.check(L.mt_attn_softmax_fw(out.data_ptr(), xd.data_ptr(), md.data_ptr() if md is not None else None,
                                    B, nh, F, T, ms, int(mode == "future"), s), "softmax_fw")
    torch.cuda.synchronize()
    mref = None if mask is None else (mask[:, None, None, :] if mode == "padmask" else mask)
    y = _softmax_ref(x, mref, mode == "future")
    np.testing.assert_allclose(out.cpu().numpy(), y, atol=1e-3, rtol=1e-3)
    dy = rng.standard_normal(shape).astype(np.float32)
    dyd = torch.from_numpy(dy).cuda()
    dinp = torch.empty_like(xd)
    _hip.check(L.mt_attn_softmax_bw(dinp.data_ptr(), dyd.data_ptr(), out.data_ptr(), B * nh * F, T, s),
               "softmax_bw")
    torch.cuda.synchronize()
    yk = out.cpu().numpy().astype(np.float64)
    dref = yk * (dy - (dy * yk).sum(-1, keepdims=True))
    np.testing.assert_allclose(dinp.cpu().numpy(), dref, atol=1e-2, rtol=1e-3)


def test_softmax_misaligned_base(hip):
    """A row base off 16 B takes the scalar kernel (same results)."""
    torch, _hip = hip
    L, s = _hip.lib(), _hip.stream_ptr()
    rng = np.random.default_rng(5)
    x = rng.standard_normal((1 + 4 * 8 * 256,)).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    out = torch.empty_like(xd)
    _hip.check(L.mt_attn_softmax_fw(out.data_ptr() + 4, xd.data_ptr() + 4, None, 1, 4, 8, 256, None, 0, s),
               "softmax_fw")
    torch.cuda.synchronize()
    y = _softmax_ref(x[1:].reshape(1, 4, 8, 256), None, False)
    np.testing.assert_allclose(out.cpu().numpy()[1:].reshape(1, 4, 8, 256), y, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("rows,H", [(5, 32), (64, 256), (4992, 256), (999, 512), (4103, 1024), (7, 1026), (1500, 2048),
                                    (13, 2048), (6, 4096), (3, 4100), (9, 36)])
def test_layernorm_fw_bw(hip, rows, H):
    torch, _hip = hip
    L, s = _hip.lib(), _hip.stream_ptr()
    rng = np.random.default_rng(rows * 10007 + H)
    x = (rng.standard_normal((rows, H)) * 2 + 0.5).astype(np.float32)
    g = rng.standard_normal(H).astype(np.float32)
    b = rng.standard_normal(H).astype(np.float32)
    xd, gd, bd = (torch.from_numpy(a).cuda() for a in (x, g, b))
    y = torch.empty_like(xd)
    var = torch.empty((rows,), device="cuda")
    mean = torch.empty((rows,), device="cuda")
    _hip.check(L.mt_layernorm_fw(y.data_ptr(), var.data_ptr(), mean.data_ptr(), xd.data_ptr(), gd.data_ptr(),
                                 bd.data_ptr(), rows, H, s), "layernorm_fw")
    torch.cuda.synchronize()
    x64 = x.astype(np.float64)
    mu = x64.mean(-1, keepdims=True)
    v = (x64 * x64).mean(-1, keepdims=True) - mu ** 2 + 1e-8
    xh = (x64 - mu) / np.sqrt(v)
    np.testing.assert_allclose(y.cpu().numpy(), g * xh + b, atol=1e-2, rtol=1e-3)
    np.testing.assert_allclose(mean.cpu().numpy(), mu[:, 0], atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(var.cpu().numpy(), v[:, 0], atol=1e-3, rtol=1e-3)
    dy = rng.standard_normal((rows, H)).astype(np.float32)
    dyd = torch.from_numpy(dy).cuda()
    dx = torch.empty_like(xd)
    dg = torch.empty((1, H), device="cuda")
    db = torch.empty((1, H), device="cuda")
    ws = torch.empty(max(1, L.mt_layernorm_bw_workspace_bytes(rows, H) // 4), device="cuda")
    _hip.check(L.mt_layernorm_bw(dg.data_ptr(), db.data_ptr(), dx.data_ptr(), dyd.data_ptr(), xd.data_ptr(),
                                 gd.data_ptr(), bd.data_ptr(), var.data_ptr(), mean.data_ptr(), rows, H,
                                 ws.data_ptr(), s), "layernorm_bw")
    torch.cuda.synchronize()
    dyg = dy * g
    dxr = (dyg - dyg.mean(-1, keepdims=True) - xh * (dyg * xh).mean(-1, keepdims=True)) / np.sqrt(v)
    np.testing.assert_allclose(dx.cpu().numpy(), dxr, atol=1e-3, rtol=1e-2)
    np.testing.assert_allclose(dg.cpu().numpy()[0], (dy * xh).sum(0), atol=1e-3 * max(1, rows / 64), rtol=1e-2)
    np.testing.assert_allclose(db.cpu().numpy()[0], dy.sum(0), atol=1e-3 * max(1, rows / 64), rtol=1e-2)


def test_layernorm_bw_deterministic(hip):
    """The dγ/dβ partials are summed in a fixed order: two runs are bitwise equal."""
    torch, _hip = hip
    L, s = _hip.lib(), _hip.stream_ptr()
    rows, H = 8191, 512
    g = torch.Generator(device="cuda").manual_seed(9)
    x, dy = (torch.randn((rows, H), device="cuda", generator=g) for _ in range(2))
    gm, bt = (torch.randn((H,), device="cuda", generator=g) for _ in range(2))
    y, var, mean = torch.empty_like(x), torch.empty((rows,), device="cuda"), torch.empty((rows,), device="cuda")
    _hip.check(L.mt_layernorm_fw(y.data_ptr(), var.data_ptr(), mean.data_ptr(), x.data_ptr(), gm.data_ptr(),
                                 bt.data_ptr(), rows, H, s), "layernorm_fw")
    ws = torch.empty(L.mt_layernorm_bw_workspace_bytes(rows, H) // 4, device="cuda")
    res = []
    for _ in range(2):
        dx, dgm, dbt = torch.empty_like(x), torch.empty((1, H), device="cuda"), torch.empty((1, H), device="cuda")
        _hip.check(L.mt_layernorm_bw(dgm.data_ptr(), dbt.data_ptr(), dx.data_ptr(), dy.data_ptr(), x.data_ptr(),
                                     gm.data_ptr(), bt.data_ptr(), var.data_ptr(), mean.data_ptr(), rows, H,
                                     ws.data_ptr(), s), "layernorm_bw")
        torch.cuda.synchronize()
        res.append((dx.clone(), dgm.clone(), dbt.clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)
