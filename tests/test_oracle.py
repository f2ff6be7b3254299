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


def test_golden_present():
    assert len(GOLDEN) >= 5


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_numpy_oracle_matches_reference(path):
    z = np.load(path)
    causal = bool(z["causal"])
    o, m, l = A.attention_fwd(z["q"], z["k"], z["v"], causal)
    np.testing.assert_allclose(o, z["o"], atol=TOL, rtol=0)
    dq, dk, dv = A.attention_bwd(z["q"], z["k"], z["v"], o, z["do"], m, l, causal)
    for got, name in ((dq, "dq"), (dk, "dk"), (dv, "dv")):
        np.testing.assert_allclose(got, z[name], atol=TOL, rtol=0, err_msg=name)


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_c_oracle_matches_reference(path):
    z = np.load(path)
    causal = bool(z["causal"])
    o, m, l = cref.attn_fwd(z["q"], z["k"], z["v"], causal)
    np.testing.assert_allclose(o, z["o"], atol=TOL, rtol=0)
    dq, dk, dv = cref.attn_bwd(z["q"], z["k"], z["v"], z["do"], m, l, causal)
    for got, name in ((dq, "dq"), (dk, "dk"), (dv, "dv")):
        np.testing.assert_allclose(got, z[name], atol=TOL, rtol=0, err_msg=name)


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


def test_bf16_rounding():
    x = np.array([1.0, 1.00390625, 1.005859375, -3.14159, 65504.0, 1e-30], np.float32)
    r = A.bf16_round(x)
    assert r[0] == 1.0 and r[1] == 1.0  # tie to even
    assert np.all(np.abs(r - x) <= np.abs(x) * 2 ** -8)
    np.testing.assert_array_equal(A.bf16_from_bits(A.bf16_bits(x)), r)
