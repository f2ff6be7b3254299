"""Elementwise error bounds for the bf16 kernels against the fp32 oracle (test
infrastructure). A bf16 MFMA kernel rounds its MFMA operands that are computed in the
kernel (P before PV and dVᵀ, dS before dKᵀ and dQ) and its outputs to 8 significant
bits, each a relative error of at most 2^-9; everything else accumulates in fp32. So,
elementwise, with |·| taken before the products:

    |O  - O_ref|  <= atol + r · (P |V|)                    (causal rows average few keys)
    |dV - dV_ref| <= atol + r · (Pᵀ |dO|)
    |dK - dK_ref| <= atol + r · (1/√d) · (|dS|ᵀ |Q|)
    |dQ - dQ_ref| <= atol + r · (1/√d) · (|dS| |K|)

where |dS| = P ∘ (|dP − δ| + Δδ) and Δδ = 2^-8 · rowsum(|dO| ∘ |O|) covers δ = rowsum(dO ∘ O)
being formed from the bf16-rounded O. r = 2^-7 is twice the two roundings (operand +
output) each product sees. dQ gets r_dq = 1.5 · 2^-7, twice three roundings: the fused
backward (csrc/fa_bwd_fused.hip) also rounds each 256-key block's partial sum of dS·K to
bf16 before the ordered sum (|partial| <= Σ over the block of |dS||K|). The products are
formed in fp64 from the same bf16-rounded inputs the kernels read.
"""
import numpy as np

R_BF16 = 2.0 ** -7
R_BF16_DQ = 1.5 * 2.0 ** -7


def head_terms(q, k, v, do, causal, kv=None):
    """fp64 P, |dS| pieces for one head (N, d); kv: valid keys of the head's batch row
    (key padding; a row with none gets P = 0)."""
    q, k, v, do = (np.asarray(a, np.float64) for a in (q, k, v, do))
    N, d = q.shape
    sc = 1.0 / np.sqrt(d)
    S = (q @ k.T) * sc
    if causal:
        S[np.triu_indices(N, 1)] = -np.inf
    if kv is not None:
        S[:, int(kv):] = -np.inf
    mx = S.max(axis=1, keepdims=True)
    S -= np.where(np.isneginf(mx), 0.0, mx)
    P = np.exp(S)
    tot = P.sum(axis=1, keepdims=True)
    P = np.where(tot > 0, P / np.where(tot > 0, tot, 1.0), 0.0)
    O = P @ v
    dP = do @ v.T
    delta = (do * O).sum(axis=1, keepdims=True)
    ddelta = 2.0 ** -8 * (np.abs(do) * np.abs(O)).sum(axis=1, keepdims=True)
    absdS = P * (np.abs(dP - delta) + ddelta)
    return P, absdS, sc


def grad_bounds(q, k, v, do, causal, atol=1e-3, r=R_BF16, kv=None, r_dq=None):
    P, absdS, sc = head_terms(q, k, v, do, causal, kv)
    q, k, do = (np.abs(np.asarray(a, np.float64)) for a in (q, k, do))
    r_dq = r * R_BF16_DQ / R_BF16 if r_dq is None else r_dq
    return (atol + r_dq * sc * (absdS @ k),   # dQ
            atol + r * sc * (absdS.T @ q),    # dK
            atol + r * (P.T @ do))            # dV
