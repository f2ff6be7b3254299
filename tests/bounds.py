"""Elementwise error bounds for the bf16 kernels against the fp32 oracle (test
infrastructure). A bf16 MFMA kernel rounds its MFMA operands that are computed in the
kernel (P before PV and dVᵀ, dS before dKᵀ and dQ) and its outputs to 8 significant
bits, each a relative error of at most 2^-9; everything else accumulates in fp32. So,
elementwise, with |·| taken before the products:

    |O  - O_ref|  <= atol + r · (P |V|)                    (causal rows average few keys)
    |dV - dV_ref| <= atol + r · (Pᵀ |dO|)
    |dK - dK_ref| <= atol + (1/√d) · (r · |dS|ᵀ + (1 + r) · Eᵀ) |Q|
    |dQ - dQ_ref| <= atol + (1/√d) · (r · |dS| + (1 + r) · E) |K|

where |dS| = P ∘ |dP − δ| and E = P ∘ Δδ is the error dS inherits from δ = rowsum(dO ∘ O)
formed from the forward's O: that O is off by at most the forward bound r · (P|V|)
elementwise (its P and output roundings), so Δδ = r · rowsum(|dO| ∘ (P|V|)). Δδ is an
absolute error of dP − δ and enters unscaled; scaling it by r again (the round-2 form)
under-counted it on causal rows with a few keys, where |O| ~ 2.5 and the rounded O moves
δ by ~1e-2 (C3 causal head (1,11), row 3: dQ off by 7.4e-3 against a 3.0e-3 bound,
scripts/probe_dq_bound.py). r = 2^-7 is twice the two roundings (operand + output) each
product sees. dQ gets r_dq = 1.5 · 2^-7, twice three roundings: the fused backward
(csrc/fa_bwd_fused.hip) also rounds each 256-key block's partial sum of dS·K to bf16
before the ordered sum (|partial| <= Σ over the block of |dS||K|). The products are formed
in fp64 from the same bf16-rounded inputs the kernels read.
"""
import numpy as np

R_BF16 = 2.0 ** -7
R_BF16_DQ = 1.5 * 2.0 ** -7


def head_terms(q, k, v, do, causal, kv=None, r=R_BF16):
    """fp64 P, |dS| = P|dP − δ| and E = P·Δδ for one head (N, d); kv: valid keys of the
    head's batch row (key padding; a row with none gets P = 0)."""
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
    ddelta = r * (np.abs(do) * (P @ np.abs(v))).sum(axis=1, keepdims=True)
    return P, P * np.abs(dP - delta), P * ddelta, sc


def grad_bounds(q, k, v, do, causal, atol=1e-3, r=R_BF16, kv=None, r_dq=None):
    P, absdS, E, sc = head_terms(q, k, v, do, causal, kv, r)
    q, k, do = (np.abs(np.asarray(a, np.float64)) for a in (q, k, do))
    r_dq = r * R_BF16_DQ / R_BF16 if r_dq is None else r_dq
    return (atol + sc * ((r_dq * absdS + (1 + r_dq) * E) @ k),   # dQ
            atol + sc * ((r * absdS + (1 + r) * E).T @ q),         # dK
            atol + r * (P.T @ do))                                 # dV


def grad_bounds_torch(q, k, v, do, causal, atol=1e-3, r=R_BF16, r_dq=None):
    """grad_bounds for a batch of heads [n, N, d] as fp64 torch tensors on the device (the
    same arithmetic; used where the NumPy form over every head of a full-size config would
    take minutes of host time). Returns the dQ, dK, dV bounds [n, N, d] as fp64 tensors."""
    import torch
    q, k, v, do = (t.to(torch.float64) for t in (q, k, v, do))
    n, N, d = q.shape
    sc = 1.0 / np.sqrt(d)
    S = torch.matmul(q, k.transpose(1, 2)) * sc
    if causal:
        S.masked_fill_(torch.ones(N, N, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    S -= S.amax(dim=2, keepdim=True)
    P = torch.exp(S)
    P /= P.sum(dim=2, keepdim=True)
    del S
    O = torch.matmul(P, v)
    delta = (do * O).sum(dim=2, keepdim=True)
    ddelta = r * (do.abs() * torch.matmul(P, v.abs())).sum(dim=2, keepdim=True)
    absdS = P * (torch.matmul(do, v.transpose(1, 2)) - delta).abs()
    E = P * ddelta
    r_dq = r * R_BF16_DQ / R_BF16 if r_dq is None else r_dq
    return (atol + sc * torch.matmul(r_dq * absdS + (1 + r_dq) * E, k.abs()),
            atol + sc * torch.matmul((r * absdS + (1 + r) * E).transpose(1, 2), q.abs()),
            atol + r * torch.matmul(P.transpose(1, 2), do.abs()))
