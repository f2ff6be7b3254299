"""CPU ORACLE (NumPy) -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module. The shipped operator path (``minitorch.hip_kernel_ops``)
never calls it; it exists to check the HIP kernels.

It restates the reference's *CPU* attention, i.e. what ``MultiHeadAttention``
computes on its plain branch with the ``FastOps`` backend
(reference ``minitorch/modules_transfomer.py:177-193``):

    S = (Q @ Kᵀ) * inv(√d)          MatMul (fast_ops.py:291-350) then Mul(Inv)  (tensor.py:169-170)
    S = S + (-FLT_MAX · triu(1))    causal mask  (modules_transfomer.py:63-71)
    P = exp(S − max) · inv(Σ exp)   nn.softmax   (nn.py:120-122)
    O = P @ V

with fp32 storage between ops and fp64 dot-product accumulation (numba types the
``acc = 0.0`` accumulator of ``_tensor_matrix_multiply`` as float64,
``fast_ops.py:339-345``). ``m``/``l`` are returned with the meaning the
reference's flash contract gives them: ``P = exp(S − m) / l``
(``src/flashattention_kernel.cu:194``), ``m`` the row max of the scaled, masked
logits and ``l = Σ exp(S − m)``.

The backward is the exact gradient of that composition (what the reference's
autodiff produces through Max/Exp/Sum/Inv/Mul, ``tensor_functions.py``), computed
from the recomputed P in fp64:
    dV = Pᵀ dO,  dP = dO Vᵀ,  dS = P ∘ (dP − rowsum(dP ∘ P)),
    dQ = dS K / √d,  dK = dSᵀ Q / √d.

Parity pinned: ``tests/test_oracle.py`` checks these functions against the golden
vectors in ``tests/golden/attn_*.npz``, produced from the reference's own minitorch
CPU path by ``oracle/gen_golden.py``.
"""
from __future__ import annotations

import numpy as np

F32_MAX = np.float32(np.finfo(np.float32).max)


def bf16_round(x: np.ndarray) -> np.ndarray:
    """Round fp32 -> bf16 (round-to-nearest-even) and return the values as fp32."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF
    out = (r << 16).astype(np.uint32).view(np.float32)
    nan = np.isnan(x)
    if nan.any():
        out = out.copy()
        out[nan] = np.nan
    return out


def bf16_bits(x: np.ndarray) -> np.ndarray:
    """fp32 -> raw bf16 bit patterns (uint16), round-to-nearest-even."""
    return (bf16_round(x).view(np.uint32) >> 16).astype(np.uint16)


def bf16_from_bits(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << 16).view(np.float32)


def pad_mask(kv_len, B: int, n_k: int) -> np.ndarray:
    """The key-padding mask of a [B] valid-key-count vector as the reference's fused softmax
    takes it (``src/softmax_kernel.cu:26-33``: ``attn_mask[B, to_len]``, 0 for tokens,
    -inf for padding), shaped (B, 1, 1, n_k) to add to (B, H, N, n_k) logits."""
    kv = np.asarray(kv_len).reshape(B, 1, 1, 1)
    return np.where(np.arange(n_k)[None, None, None, :] < kv, np.float32(0), -np.inf).astype(np.float32)


def _scores(q: np.ndarray, k: np.ndarray, causal: bool, kv_len=None) -> np.ndarray:
    """Scaled (and masked) fp32 logits of one (..., N, d) batch, reference op order.
    kv_len: optional [B] valid keys per batch row of a (B, H, N, d) batch (padding mask)."""
    d = q.shape[-1]
    n_q, n_k = q.shape[-2], k.shape[-2]
    s = (q.astype(np.float64) @ np.swapaxes(k, -1, -2).astype(np.float64)).astype(np.float32)
    inv_sqrt_d = np.float32(1.0 / np.float64(np.float32(d ** 0.5)))
    s = (s * inv_sqrt_d).astype(np.float32)
    if causal:
        mask = np.triu(np.ones((n_q, n_k), dtype=np.float32), 1) * -F32_MAX
        s = (s + mask).astype(np.float32)
    if kv_len is not None:
        s = (s + pad_mask(kv_len, q.shape[0], n_k)).astype(np.float32)
    return s


def attention_fwd(q, k, v, causal=False, kv_len=None):
    """(B,H,N,d) fp32 -> (O, m, l), see module docstring. kv_len: optional [B] key-padding
    lengths (keys >= kv_len[b] masked with -inf, as the reference's [B, to_len] softmax
    mask); a row with no valid key returns O = 0, m = -inf, l = 0 (the reference's softmax
    is NaN there)."""
    q = np.asarray(q, np.float32)
    k = np.asarray(k, np.float32)
    v = np.asarray(v, np.float32)
    s = _scores(q, k, causal, kv_len)
    m = s.max(axis=-1, keepdims=True)
    empty = np.isneginf(m)
    with np.errstate(invalid="ignore", divide="ignore"):
        e = np.exp((s - np.where(empty, 0, m)).astype(np.float32).astype(np.float64)).astype(np.float32)
        l = e.sum(axis=-1, keepdims=True, dtype=np.float32)
        p = np.where(empty, 0, (e * np.float32(1.0) / l)).astype(np.float32)
    o = (p.astype(np.float64) @ v.astype(np.float64)).astype(np.float32)
    return o, m[..., 0].astype(np.float32), l[..., 0].astype(np.float32)


def attention_bwd(q, k, v, o, do, m, l, causal=False, kv_len=None):
    """Exact gradients (dQ, dK, dV) of the composition above, fp64 internally."""
    q64, k64, v64, do64 = (np.asarray(a, np.float64) for a in (q, k, v, do))
    d = q.shape[-1]
    s = _scores(np.asarray(q, np.float32), np.asarray(k, np.float32), causal, kv_len).astype(np.float64)
    m64, l64 = np.asarray(m, np.float64)[..., None], np.asarray(l, np.float64)[..., None]
    with np.errstate(invalid="ignore", divide="ignore"):
        p = np.where(l64 > 0, np.exp(s - m64) / l64, 0.0)
    dv = np.swapaxes(p, -1, -2) @ do64
    dp = do64 @ np.swapaxes(v64, -1, -2)
    delta = (dp * p).sum(axis=-1, keepdims=True)
    ds = p * (dp - delta)
    scale = 1.0 / np.sqrt(d)
    dq = (ds @ k64) * scale
    dk = (np.swapaxes(ds, -1, -2) @ q64) * scale
    return dq.astype(np.float32), dk.astype(np.float32), dv.astype(np.float32)


def attention_ref64(q, k, v, causal=False, do=None):
    """Plain fp64 softmax attention (no reference op order) -- an independent check."""
    q, k, v = (np.asarray(a, np.float64) for a in (q, k, v))
    d, n_q, n_k = q.shape[-1], q.shape[-2], k.shape[-2]
    s = q @ np.swapaxes(k, -1, -2) / np.sqrt(d)
    if causal:
        s = np.where(np.triu(np.ones((n_q, n_k)), 1) > 0, -np.inf, s)
    p = np.exp(s - s.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    o = p @ v
    if do is None:
        return o
    do = np.asarray(do, np.float64)
    dv = np.swapaxes(p, -1, -2) @ do
    dp = do @ np.swapaxes(v, -1, -2)
    ds = p * (dp - (dp * p).sum(-1, keepdims=True))
    return o, ds @ k / np.sqrt(d), np.swapaxes(ds, -1, -2) @ q / np.sqrt(d), dv
