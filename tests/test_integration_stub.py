"""INTEGRATION.md §3's ctypes stub, exec'd verbatim: the four handles of the reference's
loader block (reference minitorch/cuda_kernel_ops.py:26-29) bound to libminitorch_hip.so,
then the reference's own flash_attention_fw / _bw calling sequence (cuda_kernel_ops.py:
605-758: ndpointer argtypes, 1-D float32 storages, l zeros, m = -inf) on a GPU."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_MINITORCH = os.path.join(ROOT, "llmsys-project-flashattn_amd", "minitorch")


def _stub_source():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 3."):text.index("### Device-pointer API")]
    blocks = re.findall(r"```python\n(.*?)```", sec, flags=re.S)
    assert len(blocks) == 1, "INTEGRATION.md §3 must hold exactly one python stub"
    return blocks[0]


def _exec_stub():
    from minitorch import _hip
    if not os.path.exists(_hip.LIB_PATH):
        pytest.skip("library not built")
    ns = {"__file__": os.path.join(PKG_MINITORCH, "cuda_kernel_ops.py"), "__name__": "stub"}
    exec(compile(_stub_source(), "INTEGRATION.md#3", "exec"), ns)
    return ns


def test_stub_binds_the_reference_handles():
    ns = _exec_stub()
    for name in ("lib", "lib_softmax", "lib_layernorm", "lib_flashattention"):
        assert name in ns, name
    fl = ns["lib_flashattention"]
    assert len(fl.launch_flashattention_forward.argtypes) == 10
    assert len(fl.launch_flashattention_backward.argtypes) == 14
    # the names the reference's method bodies call exist on the handles they use
    for h, fn in (("lib", "tensorMap"), ("lib", "tensorZip"), ("lib", "tensorReduce"),
                  ("lib", "MatrixMultiply"), ("lib_softmax", "launch_attn_softmax"),
                  ("lib_softmax", "launch_attn_softmax_bw"), ("lib_layernorm", "launch_layernorm"),
                  ("lib_layernorm", "launch_layernorm_bw"),
                  ("lib_flashattention", "launch_flashattention_forward_causal"),
                  ("lib_flashattention", "launch_flashattention_backward_causal")):
        assert hasattr(ns[h], fn), (h, fn)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_stub_runs_reference_calling_sequence(causal):
    import ctypes
    from oracle import attention as A
    ns = _exec_stub()
    lf = ns["lib_flashattention"]
    B, nh, N, d = 2, 3, 96, 32
    rng = np.random.default_rng(17)
    q, k, v, do = (rng.standard_normal((B, nh, N, d)).astype(np.float32) for _ in range(4))
    # reference flash_attention_fw: l = zeros, O = zeros, m = full(-inf); the body re-sets
    # the ndpointer argtypes itself before every call (cuda_kernel_ops.py:629-642)
    nd = np.ctypeslib.ndpointer(dtype=np.float32, ndim=1, flags="C_CONTIGUOUS")
    fwd = lf.launch_flashattention_forward_causal if causal else lf.launch_flashattention_forward
    fwd.argtypes = [nd] * 6 + [ctypes.c_int] * 4
    fwd.restype = None
    O = np.zeros(B * nh * N * d, np.float32)
    l = np.zeros(B * nh * N, np.float32)
    m = np.full(B * nh * N, -np.inf, np.float32)
    fwd(q.ravel(), k.ravel(), v.ravel(), O, l, m, B, nh, N, d)
    o_ref, m_ref, l_ref = A.attention_fwd(q, k, v, causal)
    np.testing.assert_allclose(O.reshape(q.shape), o_ref, atol=1e-5)
    bwd = lf.launch_flashattention_backward_causal if causal else lf.launch_flashattention_backward
    bwd.argtypes = [nd] * 10 + [ctypes.c_int] * 4
    bwd.restype = None
    dQ, dK, dV = (np.zeros(B * nh * N * d, np.float32) for _ in range(3))
    bwd(q.ravel(), k.ravel(), v.ravel(), O, dQ, dK, dV, do.ravel(), l, m, B, nh, N, d)
    refs = A.attention_bwd(q, k, v, o_ref, do, m_ref, l_ref, causal)
    for got, ref in zip((dQ, dK, dV), refs):
        np.testing.assert_allclose(got.reshape(q.shape), ref, atol=2e-5)
