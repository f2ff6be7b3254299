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
    [rows, N(, d)]. ``t`` must be viewable as [B*H, ...] (contiguous over (B, H) with the
    trailing strides kept): a permuted projection view such as the MHA's [B,N,H,dh]
    storage would otherwise be silently copied whole on every rank, so it is refused."""
    B, H = t.shape[:2]
    lo, hi = bh_range(B * H, world, rank)
    try:
        flat = t.view((B * H,) + tuple(t.shape[2:]))
    except RuntimeError as e:
        raise ValueError(
            f"shard(): tensor of shape {tuple(t.shape)} and strides {tuple(t.stride())} is not "
            "contiguous over (B, H); call .contiguous() once before sharding") from e
    return flat[lo:hi]


def _local_or_shard(t, global_ndim: int, world: int, rank: int, rows: int):
    """``t`` as this rank's [rows, ...] block: a global tensor (``global_ndim`` dims) is
    sharded; a rank-local one (one dim fewer, as ``sharded_flash_fwd(gather=False)``
    returns) is taken as it is after a row-count check."""
    if t.dim() == global_ndim:
        return shard(t, world, rank)
    if t.dim() == global_ndim - 1:
        if t.shape[0] != rows:
            raise ValueError(f"rank-local tensor has {t.shape[0]} rows, this rank owns {rows}")
        return t
    raise ValueError(f"expected a {global_ndim}-d global or {global_ndim - 1}-d rank-local tensor, "
                     f"got shape {tuple(t.shape)}")


def _world_rank(group, world: Optional[int], rank: Optional[int],
                gather: bool = False) -> Tuple[int, int]:
    """(world, rank): the process group's, or the explicit pair. An explicit pair with
    ``gather`` must be this process's own group rank: the all-gather puts this process's
    rows in its own group slot, so another rank's rows would land in the wrong place."""
    import torch.distributed as dist
    if world is not None or rank is not None:
        if world is None or rank is None:
            raise ValueError("give both world and rank, or neither")
        if gather and world > 1:
            if not dist_ready() or world != _group_world(group):
                raise ValueError("gather=True needs an initialised process group of that world size")
            if rank != dist.get_rank(group):
                raise ValueError(f"gather=True with an explicit rank {rank} that is not this "
                                 f"process's group rank {dist.get_rank(group)}")
        return world, rank
    if dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


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


def chunk_rows(bh: int, world: int, rank: int, chunks: int, c: int) -> Tuple[int, int]:
    """[lo, hi) of the flattened B*H axis that ``rank`` computes as its chunk ``c`` of the
    chunked (overlapped) forward: block-cyclic, chunk c of every rank together is the
    contiguous range [c*W*Rc, (c+1)*W*Rc), Rc = BH / (W*chunks), so each chunk's
    all-gather lands in place in the global output with no copy."""
    rc = bh // (world * chunks)
    lo = (c * world + rank) * rc
    return lo, lo + rc


def forward_workgroups_per_head(N: int, d: int, causal: bool = False) -> int:
    """Workgroups one head contributes to the grid of the bf16 forward's default form
    (capi_flash.hip fwd_bf16_dispatch): d = 64, 512-query 8-wave workgroups (v6; below one per
    CU the dispatcher falls back to the slower split-keys form); d = 128, 256-query workgroups
    (d128v2); causal, light / heavy pairs of 512-query blocks (v6 causal)."""
    if causal:
        return max(1, (-(-N // 512) + 1) // 2)
    return max(1, -(-N // (512 if d == 64 else 256)))


def occupancy_chunks(B: int, H: int, N: int, d: int, world: int, causal: bool = False,
                     max_chunks: int = 4, cus: int = 256) -> int:
    """Chunks for the overlapped all-gather (``sharded_flash_fwd(chunks=...)``, bench.py's
    end-to-end leg): the largest power of two up to ``max_chunks`` such that each chunk's
    forward still launches at least one workgroup per CU (``cus``, 256 on MI355X) and the
    rank's rows divide evenly. A chunk whose grid leaves CUs idle, or drops the d = 64 forward
    into its split-keys form, runs at a fraction of the kernel's rate, which costs more than
    the overlap hides: C3 (8,16,4096,64) takes 2 chunks at 2 ranks (32 heads x 8 workgroups)
    and none from 4 ranks up (at 8 ranks its 16 heads per rank are below one 8-wave workgroup
    per CU even unchunked); C4 (64,16,16384,128) at 8 ranks (128 heads, 64 workgroups each)
    takes 4."""
    rows = (B * H) // world if world > 0 else 0
    if world <= 0 or (B * H) % world:
        return 1
    per_head = forward_workgroups_per_head(N, d, causal)
    c = 1
    while (c * 2 <= max_chunks and rows % (c * 2) == 0
           and (rows // (c * 2)) * per_head >= cus):
        c *= 2
    return c


def _chunked_gather_fwd(q, k, v, causal, group, world, rank, chunks, fn):
    """The gathered forward with the all-gather of finished chunks overlapping the forward of
    the next: chunk c's three all-gathers are issued asynchronously right after its forward
    launches (the RCCL stream waits for exactly that work), then chunk c + 1's forward is
    launched on the compute stream without waiting; the caller's stream waits for every
    gather at the end. (gloo: the CPU forward and gloo's background gather overlap the same
    way.)"""
    import torch
    import torch.distributed as dist
    B, H, N, d = q.shape
    bh = B * H
    flat = [shard(t, 1, 0) for t in (q, k, v)]  # [BH, N, d] views (refuses non-viewable)
    outs, works = None, []
    for c in range(chunks):
        lo, hi = chunk_rows(bh, world, rank, chunks, c)
        res = fn(*(t[lo:hi][None] for t in flat), causal)
        if outs is None:
            outs = [torch.empty((bh,) + tuple(r.shape[2:]), dtype=r.dtype, device=r.device) for r in res]
        n = world * (hi - lo)
        for r, out in zip(res, outs):
            works.append(dist.all_gather_into_tensor(out[c * n:(c + 1) * n], r[0].contiguous(),
                                                     group=group, async_op=True))
    for w in works:
        w.wait()
    return outs[0].view(B, H, N, d), outs[1].view(B, H, N), outs[2].view(B, H, N)


def sharded_flash_fwd(q, k, v, causal: bool = False, group=None, gather: bool = True,
                      attn: Optional[Callable] = None, world: Optional[int] = None,
                      rank: Optional[int] = None, chunks: int = 1):
    """Forward over this rank's B*H shard of the global [B,H,N,d] Q/K/V.

    Returns ``(O, m, l)``: with ``gather`` the full [B,H,N,d] / [B,H,N] results on every
    rank (one all-gather per output), otherwise this rank's shard [rows,N,d] / [rows,N]
    (at world size 1, the full tensors in their global shape).

    ``chunks`` > 1 (with ``gather``): the rank computes its rows in ``chunks`` pieces and
    all-gathers each piece while the next one computes ("chunk the shard
    and overlap"); the rows are dealt block-cyclically (``chunk_rows``) so every gather lands
    in place. Needs B*H divisible by world*chunks, else the forward runs unchunked;
    ``occupancy_chunks`` picks a count that keeps every chunk's grid at one workgroup per CU.
    Each chunk's forward runs on a smaller grid, where the bf16 dispatcher may pick another
    kernel form (split keys): the gathered O is then within the forward's parity bound of the
    unchunked one, not bit-identical (bit-identical with the CPU attention the tests inject).

    ``world``/``rank`` default to the process group's; giving them explicitly computes that
    rank's shard without any collective (with ``gather``, ``rank`` must be this process's
    group rank) — a single process can then produce every rank's rows of a ragged split."""
    world, rank = _world_rank(group, world, rank, gather)
    if gather and world > 1 and not (dist_ready() and world == _group_world(group)):
        raise ValueError("gather=True needs an initialised process group of that world size")
    B, H, N, d = q.shape
    fn = attn or _hip_fwd
    if gather and world > 1 and chunks > 1 and (B * H) % (world * chunks) == 0:
        return _chunked_gather_fwd(q, k, v, causal, group, world, rank, chunks, fn)
    qs, ks, vs = (shard(t, world, rank) for t in (q, k, v))
    o, m, l = fn(qs[None], ks[None], vs[None], causal)
    o, m, l = o[0], m[0], l[0]
    if world == 1:
        return o.reshape(B, H, N, d), m.reshape(B, H, N), l.reshape(B, H, N)
    if not gather:
        return o, m, l
    sizes = [bh_range(B * H, world, r)[1] - bh_range(B * H, world, r)[0] for r in range(world)]
    outs = [_gather(t, world, group, B * H, sizes) for t in (o, m, l)]
    return outs[0].reshape(B, H, N, d), outs[1].reshape(B, H, N), outs[2].reshape(B, H, N)


def sharded_flash_bwd(q, k, v, o, do, m, l, causal: bool = False, group=None, gather: bool = True,
                      attn_bwd: Optional[Callable] = None, world: Optional[int] = None,
                      rank: Optional[int] = None):
    """Backward over this rank's B*H shard. q, k, v and do are the global [B,H,N,d]
    tensors; o, m and l are either global ([B,H,N,d] / [B,H,N]) or this rank's rows
    ([rows,N,d] / [rows,N], the ``gather=False`` forward's output), so a training step
    that never gathers O feeds its forward straight into the backward. Returns
    (dQ, dK, dV): gathered [B,H,N,d] with ``gather``, else this rank's [rows,N,d]
    (at world size 1, the global shape). ``world``/``rank``: as in sharded_flash_fwd."""
    world, rank = _world_rank(group, world, rank, gather)
    if gather and world > 1 and not (dist_ready() and world == _group_world(group)):
        raise ValueError("gather=True needs an initialised process group of that world size")
    B, H, N, d = q.shape
    lo, hi = bh_range(B * H, world, rank)
    fn = attn_bwd or _hip_bwd
    args = [shard(t, world, rank) for t in (q, k, v)]
    args.append(_local_or_shard(o, 4, world, rank, hi - lo))
    args.append(shard(do, world, rank))
    args += [_local_or_shard(t, 3, world, rank, hi - lo) for t in (m, l)]
    grads = [g[0] for g in fn(*(a[None] for a in args), causal)]
    if world == 1:
        return tuple(g.reshape(B, H, N, d) for g in grads)
    if not gather:
        return tuple(grads)
    sizes = [bh_range(B * H, world, r)[1] - bh_range(B * H, world, r)[0] for r in range(world)]
    return tuple(_gather(g, world, group, B * H, sizes).reshape(B, H, N, d) for g in grads)


def dist_ready() -> bool:
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def _group_world(group) -> int:
    import torch.distributed as dist
    return dist.get_world_size(group)
