"""The CPU oracle is pinned to the reference's own outputs (golden vectors from the
reference minitorch CPU path, tests/golden/, made by oracle/gen_golden.py)."""
import glob
import os

import numpy as np
import pytest

from oracle import attention as A
from oracle import cref

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "attn_*.npz")))
TOL = 2e-6  # fp32 restatement vs the reference's fp32 composition
RTOL = 1e-6  # fp32 summation order on large sums (dV of a 1-key row sums 80 dO rows)


def test_golden_present():
    assert len(GOLDEN) >= 5


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_numpy_oracle_matches_reference(path):
    z = np.load(path)
    causal = bool(z["causal"])
    kv = z["kv_len"] if "kv_len" in z.files else None  # key-padding fixtures (attn_varlen*)
    o, m, l = A.attention_fwd(z["q"], z["k"], z["v"], causal, kv)
    np.testing.assert_allclose(o, z["o"], atol=TOL, rtol=0)
    dq, dk, dv = A.attention_bwd(z["q"], z["k"], z["v"], o, z["do"], m, l, causal, kv)
    for got, name in ((dq, "dq"), (dk, "dk"), (dv, "dv")):
        np.testing.assert_allclose(got, z[name], atol=TOL, rtol=RTOL, err_msg=name)


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_c_oracle_matches_reference(path):
    z = np.load(path)
    causal = bool(z["causal"])
    kv = z["kv_len"] if "kv_len" in z.files else None
    o, m, l = cref.attn_fwd(z["q"], z["k"], z["v"], causal, kv_len=kv)
    np.testing.assert_allclose(o, z["o"], atol=TOL, rtol=0)
    dq, dk, dv = cref.attn_bwd(z["q"], z["k"], z["v"], z["do"], m, l, causal, kv_len=kv)
    for got, name in ((dq, "dq"), (dk, "dk"), (dv, "dv")):
        np.testing.assert_allclose(got, z[name], atol=TOL, rtol=RTOL, err_msg=name)


def test_m_l_contract():
    """P = exp(s - m) / l reproduces the softmax (reference flashattention_kernel.cu:194)."""
    rng = np.random.default_rng(0)
    q, k, v = (rng.standard_normal((1, 2, 40, 16)).astype(np.float32) for _ in range(3))
    for causal in (False, True):
        o, m, l = A.attention_fwd(q, k, v, causal)
        o2, m2, l2 = cref.attn_fwd(q, k, v, causal)
        np.testing.assert_allclose(m, m2, atol=1e-6)
        np.testing.assert_allclose(l, l2, rtol=1e-5)
        ref = A.attention_ref64(q, k, v, causal)
        np.testing.assert_allclose(o, ref, atol=2e-6)


def test_empty_key_rows_are_zero():
    """kv_len = 0 (no valid key): O = 0, l = 0, zero gradients in both oracles (the kernels'
    contract; the reference softmax is NaN there)."""
    rng = np.random.default_rng(1)
    q, k, v, do = (rng.standard_normal((2, 2, 24, 8)).astype(np.float32) for _ in range(4))
    kv = np.array([0, 7], np.int32)
    for causal in (False, True):
        o, m, l = A.attention_fwd(q, k, v, causal, kv)
        o2, m2, l2 = cref.attn_fwd(q, k, v, causal, kv_len=kv)
        assert np.all(o[0] == 0) and np.all(l[0] == 0) and np.isfinite(o).all()
        np.testing.assert_allclose(o, o2, atol=2e-6)
        g = A.attention_bwd(q, k, v, o, do, m, l, causal, kv)
        g2 = cref.attn_bwd(q, k, v, do, m2, l2, causal, kv_len=kv)
        for a, b in zip(g, g2):
            assert np.all(a[0] == 0) and np.isfinite(a).all()
            np.testing.assert_allclose(a, b, atol=2e-5)
        # keys past kv_len get exactly zero dK, dV
        assert np.all(g[1][1, :, 7:] == 0) and np.all(g[2][1, :, 7:] == 0)


def test_bf16_rounding():
    x = np.array([1.0, 1.00390625, 1.005859375, -3.14159, 65504.0, 1e-30], np.float32)
    r = A.bf16_round(x)
    assert r[0] == 1.0 and r[1] == 1.0  # tie to even
    assert np.all(np.abs(r - x) <= np.abs(x) * 2 ** -8)
    np.testing.assert_array_equal(A.bf16_from_bits(A.bf16_bits(x)), r)


# ---- companion-kernel fixtures (oracle/gen_companion_golden.py: the reference's own
# minitorch compositions from its kernel_tests) -------------------------------------------
def _companion(golden_dir, kind):
    import glob
    paths = sorted(glob.glob(os.path.join(golden_dir, f"{kind}_*.npz")))
    assert paths, f"no {kind} fixtures"
    return [dict(np.load(p)) for p in paths]


def test_softmax_fixtures_match_formula(golden_dir):
    """The reference composition equals the kernel contract (softmax_kernel.cu: exp(x - max)
    over (Σ + 1e-8), mask [B,to] added per row; bw y∘(dy − Σ dy∘y)) in NumPy f64."""
    for f in _companion(golden_dir, "softmax"):
        x = f["inp"].astype(np.float64)
        z = x + f["mask_bt"][:, None, None, :]
        e = np.exp(z - z.max(-1, keepdims=True))
        np.testing.assert_allclose(f["fw"], e / (e.sum(-1, keepdims=True) + 1e-8), atol=1e-6)
        e0 = np.exp(x - x.max(-1, keepdims=True))
        y = e0 / e0.sum(-1, keepdims=True)
        dy = f["dout"].astype(np.float64)
        np.testing.assert_allclose(f["bw"], y * (dy - (dy * y).sum(-1, keepdims=True)), atol=1e-6)


def test_layernorm_fixtures_match_formula(golden_dir):
    for f in _companion(golden_dir, "layernorm"):
        x = f["x"].astype(np.float64)
        mu, var = x.mean(-1, keepdims=True), x.var(-1, keepdims=True)
        xh = (x - mu) / np.sqrt(var + 1e-8)
        np.testing.assert_allclose(f["fw"], f["gamma"] * xh + f["beta"], atol=1e-5)
        np.testing.assert_allclose(f["var"], var[:, 0], atol=1e-6)
        dy = f["dout"].astype(np.float64)
        dyg = dy * f["gamma"]
        dx = (dyg - dyg.mean(-1, keepdims=True) - xh * (dyg * xh).mean(-1, keepdims=True)) / np.sqrt(var)
        np.testing.assert_allclose(f["dinp"], dx, atol=1e-4)
        np.testing.assert_allclose(f["dgamma"], (dy * xh).sum(0), atol=1e-4)
        np.testing.assert_allclose(f["dbeta"], dy.sum(0), atol=1e-4)
