"""Batch x heads sharding of the flash-attention path across the GPUs of one node.

Every (b, h) slice of attention is independent in forward and backward (the reference's
grid is ``(B, nh)``, ``src/flashattention_kernel.cu:300``), so the path shards with no
data-path collective: rank r of W owns the contiguous range of flattened B*H rows
``[r*BH/W, (r+1)*BH/W)``. In the ``[B,H,N,d]`` layout that range is one contiguous block
of Q/K/V/O, so a shard is a view, never a repack. The only exchange is the optional
all-gather of the output shards (RCCL over xGMI; ``backend="nccl"`` is RCCL on ROCm),
which BASELINE config 4 names.

The attention callable is injected (default: the HIP kernels through the C ABI) so the
world_size>1 logic can be exercised with ``gloo`` on CPU by the tests.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence, Tuple


def bh_range(bh: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of the flattened B*H axis owned by ``rank``; the first
    ``bh % world`` ranks take one extra row so any B*H works (C3/C4 divide evenly)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    base, rem = divmod(bh, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard(t, world: int, rank: int):
    """View of this rank's rows of a [B,H,N,d] (or [B,H,N]) tensor, flattened to
    [rows, N(, d)]. ``t`` must be contiguous over (B, H)."""
    B, H = t.shape[:2]
    lo, hi = bh_range(B * H, world, rank)
    return t.reshape((B * H,) + tuple(t.shape[2:]))[lo:hi]


def _hip_fwd(q, k, v, causal):
    from . import _hip
    return _hip.flash_fwd(q, k, v, causal)


def _hip_bwd(q, k, v, o, do, m, l, causal):
    from . import _hip
    return _hip.flash_bwd(q, k, v, o, do, m, l, causal)


def _gather(local, world: int, group, bh: int, rank_sizes: Sequence[int]):
    import torch
    import torch.distributed as dist
    if len(set(rank_sizes)) == 1:
        out = torch.empty((bh,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
        return out
    # ragged split: pad to the largest shard, gather, then drop the padding
    mx = max(rank_sizes)
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]].copy_(local)
    buf = torch.empty((world * mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(buf, pad, group=group)
    return torch.cat([buf[r * mx: r * mx + n] for r, n in enumerate(rank_sizes)])


def sharded_flash_fwd(q, k, v, causal: bool = False, group=None, gather: bool = True,
                      attn: Optional[Callable] = None):
    """Forward over this rank's B*H shard of the global [B,H,N,d] Q/K/V.

    Returns ``(O, m, l)``: with ``gather`` the full [B,H,N,d] / [B,H,N] results on every
    rank (one all-gather per output), otherwise this rank's shard [rows,N,d] / [rows,N]."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    B, H, N, d = q.shape
    fn = attn or _hip_fwd
    qs, ks, vs = (shard(t, world, rank) for t in (q, k, v))
    o, m, l = fn(qs[None], ks[None], vs[None], causal)
    o, m, l = o[0], m[0], l[0]
    if not gather or world == 1:
        return (o.reshape(B, H, N, d), m.reshape(B, H, N), l.reshape(B, H, N)) if world == 1 else (o, m, l)
    sizes = [bh_range(B * H, world, r)[1] - bh_range(B * H, world, r)[0] for r in range(world)]
    outs = [_gather(t, world, group, B * H, sizes) for t in (o, m, l)]
    return outs[0].reshape(B, H, N, d), outs[1].reshape(B, H, N), outs[2].reshape(B, H, N)


def sharded_flash_bwd(q, k, v, o, do, m, l, causal: bool = False, group=None, gather: bool = True,
                      attn_bwd: Optional[Callable] = None):
    """Backward over this rank's B*H shard; every input is the global tensor (or any tensor
    whose shard view is this rank's rows). Returns (dQ, dK, dV), gathered if asked."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    B, H, N, d = q.shape
    fn = attn_bwd or _hip_bwd
    args = [shard(t, world, rank)[None] for t in (q, k, v, o, do, m, l)]
    grads = [g[0] for g in fn(*args, causal)]
    if not gather or world == 1:
        return tuple(g.reshape(B, H, N, d) for g in grads) if world == 1 else tuple(grads)
    sizes = [bh_range(B * H, world, r)[1] - bh_range(B * H, world, r)[0] for r in range(world)]
    return tuple(_gather(g, world, group, B * H, sizes).reshape(B, H, N, d) for g in grads)
