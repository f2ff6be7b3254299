"""Key padding (kv_len, mt_flash_attn_*_varlen) on the GPU against the CPU oracle.

The contract is the reference's padding mask (src/softmax_kernel.cu:26-33: attn_mask[B,
to_len], -inf for padding tokens), pinned by the reference-generated fixtures
tests/golden/attn_varlen*.npz (oracle/gen_golden.py; checked in test_flash_gpu.py's golden
test and tests/test_oracle.py). Here: random shapes through every kernel family that takes
kv_len (the fp32 / small-d ring kernels, the generic kernels at d = 128, bf16 d = 64's ring
forward and fused backward), ragged N, a row with no valid key (O = 0, zero gradients) and
a full row, causal or not; then the minitorch MultiHeadAttention on a padded batch, whose
flash, fused-softmax and plain branches must agree.

Tolerances: fp32 1e-5 max-abs (the reference MHA bound); bf16 against the oracle on the same
bf16-rounded inputs under the elementwise bounds of tests/bounds.py.
"""
import numpy as np
import pytest

from oracle import attention as A

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "needs an MI355X"
    return torch


def _dev(torch, a, dtype=None):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda").to(dtype or torch.float32)


def _np(t):
    return t.float().cpu().numpy()


CASES = [  # (B, H, N, d, kv_len)
    (3, 2, 200, 32, (200, 77, 0)),
    (3, 2, 130, 64, (1, 130, 64)),
    (2, 2, 96, 128, (96, 40)),
]


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("B,H,N,d,kv", CASES)
def test_varlen_fp32_vs_oracle(torch_dev, B, H, N, d, kv, causal):
    from minitorch import _hip
    torch = torch_dev
    rng = np.random.default_rng(N + d)
    q, k, v, do = (rng.standard_normal((B, H, N, d)).astype(np.float32) for _ in range(4))
    tq, tk, tv, tdo = (_dev(torch, x) for x in (q, k, v, do))
    o, m, l = _hip.flash_fwd(tq, tk, tv, causal, kv_len=kv)
    dq, dk, dv = _hip.flash_bwd(tq, tk, tv, o, tdo, m, l, causal, kv_len=kv)
    torch.cuda.synchronize()
    o_ref, m_ref, l_ref = A.attention_fwd(q, k, v, causal, kv)
    np.testing.assert_allclose(_np(o), o_ref, atol=1e-5, rtol=0)
    np.testing.assert_allclose(_np(l), l_ref, rtol=1e-5, atol=0)
    refs = A.attention_bwd(q, k, v, o_ref, do, m_ref, l_ref, causal, kv)
    for got, ref, name in zip((dq, dk, dv), refs, ("dq", "dk", "dv")):
        np.testing.assert_allclose(_np(got), ref, atol=1e-5, rtol=0, err_msg=name)
    for b, n in enumerate(kv):  # padding keys: exactly zero dK / dV; an empty row: all zero
        assert not _np(dk[b, :, n:]).any() and not _np(dv[b, :, n:]).any()
        if n == 0:
            assert not _np(o[b]).any() and not _np(dq[b]).any()


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("B,H,N,kv", [(3, 2, 200, (200, 77, 0)), (2, 3, 640, (640, 300)),
                                      (2, 1, 1100, (1, 1023))])
def test_varlen_bf16_d64_vs_oracle(torch_dev, B, H, N, kv, causal, parity_record):
    """bf16 d = 64: the ring forward and the fused backward (dQ in the dK/dV pass), key
    blocks wholly past kv_len skipped, the boundary block masked."""
    from bounds import grad_bounds
    from minitorch import _hip
    torch = torch_dev
    d = 64
    rng = np.random.default_rng(7 * N + B)
    q, k, v, do = (A.bf16_round(rng.standard_normal((B, H, N, d)).astype(np.float32)) for _ in range(4))
    tq, tk, tv, tdo = (_dev(torch, x, torch.bfloat16) for x in (q, k, v, do))
    o, m, l = _hip.flash_fwd(tq, tk, tv, causal, kv_len=kv)
    dq, dk, dv = _hip.flash_bwd(tq, tk, tv, o, tdo, m, l, causal, kv_len=kv)
    torch.cuda.synchronize()
    o_ref, m_ref, l_ref = A.attention_fwd(q, k, v, causal, kv)
    refs = A.attention_bwd(q, k, v, o_ref, do, m_ref, l_ref, causal, kv)
    worst = {}
    for b in range(B):
        for h in range(H):
            p_abs, _, _ = A.attention_fwd(q[b:b + 1, h:h + 1], k[b:b + 1, h:h + 1],
                                          np.abs(v[b:b + 1, h:h + 1]), causal, kv[b:b + 1])
            bnd = 1e-3 + 2.0 ** -7 * p_abs[0, 0]
            err = np.abs(_np(o[b, h]) - o_ref[b, h])
            assert (err <= bnd).all(), f"O (b,h)=({b},{h}) max-abs {err.max():.3e}"
            worst["o"] = max(worst.get("o", 0.0), float(err.max()))
            bnds = grad_bounds(q[b, h], k[b, h], v[b, h], do[b, h], causal, kv=kv[b])
            for got, ref, bd, name in zip((dq, dk, dv), refs, bnds, ("dq", "dk", "dv")):
                e = np.abs(_np(got[b, h]) - ref[b, h])
                assert (e <= bd).all(), f"{name} (b,h)=({b},{h}) max-abs {e.max():.3e}, ratio {(e / bd).max():.3f}"
                worst[name] = max(worst.get(name, 0.0), float(e.max()))
        assert not _np(dk[b, :, kv[b]:]).any() and not _np(dv[b, :, kv[b]:]).any()
    parity_record("test_varlen_bf16_d64_vs_oracle", f"({B},{H},{N},64) kv={kv} causal={causal}",
                  bound="1e-3 + 2^-7 elementwise (tests/bounds.py)", **{f"{n}_max_abs": e for n, e in worst.items()})


def test_varlen_bf16_causal_paired_fused(torch_dev, parity_record):
    """kv_len on the causal fused backward's paired grid (light / heavy key blocks per
    workgroup, taken when ceil(nkb / 2)·B·H >= 256): (4,32,1100,64), 384 paired workgroups,
    rows of every padding kind (full, partial, one key, none); heads of each row against the
    oracle, and zero dK / dV past kv_len everywhere."""
    from bounds import grad_bounds
    from minitorch import _hip
    torch = torch_dev
    B, H, N, d = 4, 32, 1100, 64
    kv = (1100, 700, 1, 0)
    rng = np.random.default_rng(1100)
    q, k, v, do = (A.bf16_round(rng.standard_normal((B, H, N, d)).astype(np.float32)) for _ in range(4))
    tq, tk, tv, tdo = (_dev(torch, x, torch.bfloat16) for x in (q, k, v, do))
    o, m, l = _hip.flash_fwd(tq, tk, tv, True, kv_len=kv)
    dq, dk, dv = _hip.flash_bwd(tq, tk, tv, o, tdo, m, l, True, kv_len=kv)
    torch.cuda.synchronize()
    worst = {}
    for b, h in ((0, 0), (1, 17), (2, 31), (3, 5)):
        sl = (slice(b, b + 1), slice(h, h + 1))
        o_ref, m_ref, l_ref = A.attention_fwd(q[sl], k[sl], v[sl], True, kv[b:b + 1])
        refs = A.attention_bwd(q[sl], k[sl], v[sl], o_ref, do[sl], m_ref, l_ref, True, kv[b:b + 1])
        bnds = grad_bounds(q[b, h], k[b, h], v[b, h], do[b, h], True, kv=kv[b])
        for got, ref, bd, name in zip((dq, dk, dv), refs, bnds, ("dq", "dk", "dv")):
            e = np.abs(_np(got[b, h]) - ref[0, 0])
            assert (e <= bd).all(), f"{name} (b,h)=({b},{h}) max-abs {e.max():.3e}, ratio {(e / bd).max():.3f}"
            worst[name] = max(worst.get(name, 0.0), float(e.max()))
    for b in range(B):
        assert not _np(dk[b, :, kv[b]:]).any() and not _np(dv[b, :, kv[b]:]).any()
    parity_record("test_varlen_bf16_causal_paired_fused", f"({B},{H},{N},64) kv={kv} causal",
                  bound="tests/bounds.py", **{f"{n}_max_abs": e for n, e in worst.items()})


@pytest.mark.parametrize("causal", [False, True])
def test_mha_padded_batch_branches_agree(torch_dev, causal):
    """MultiHeadAttention on a right-padded batch: the flash branch (kv_len in the kernel),
    the fused-softmax branch (the reference's [B, to_len] -inf mask in the HIP softmax) and
    the plain composition give the same output and input gradient."""
    import minitorch
    torch = torch_dev
    backend = minitorch.TensorBackend(minitorch.HipKernelOps)
    B, T, E, H = 4, 37, 64, 4
    kv = [37, 20, 5, 30]
    rng = np.random.default_rng(3)
    x_np = rng.standard_normal((B, T, E)).astype(np.float32)
    g_np = rng.standard_normal((B, T, E)).astype(np.float32)
    outs = {}
    for branch in ("flash", "fused", "plain"):
        mha = minitorch.MultiHeadAttention(E, H, causal=causal, p_dropout=0.0, backend=backend,
                                           use_fused_kernel=branch == "fused",
                                           use_flash_attention=branch == "flash")
        prng = np.random.default_rng(11)  # identical weights in every branch
        for p in mha.parameters():
            p.update(minitorch.tensor_from_numpy(
                (0.1 * prng.standard_normal(p.value.shape)).astype(np.float32), backend=backend))
        x = minitorch.tensor_from_numpy(x_np, backend=backend, requires_grad=True)
        y = mha(x, kv_len=kv)
        y.backward(minitorch.tensor_from_numpy(g_np, backend=backend))
        outs[branch] = (y.to_numpy(), x.grad.to_numpy())
    for branch in ("fused", "plain"):
        np.testing.assert_allclose(outs["flash"][0], outs[branch][0], atol=1e-5, rtol=0, err_msg=branch)
        np.testing.assert_allclose(outs["flash"][1], outs[branch][1], atol=1e-5, rtol=0, err_msg=branch)
