"""Data-parallel training step for the minitorch transformer path.

One process per GPU (``torch.distributed``; backend ``"nccl"`` is RCCL over xGMI on
ROCm, ``"gloo"`` in the CPU tests). Each rank runs forward/backward on its shard of the
global batch; the gradients are then averaged with bucketed all-reduces before every
optimizer step, so all replicas stay identical. The reference trains on one GPU
(``project/run_machine_translation.py:195-237``); its loss is a mean over the batch, so
averaging the per-rank mean gradients reproduces the single-process step exactly when the
shards are equal.

Buckets are flat fp32 buffers of up to ``bucket_mb`` MiB (few, large collectives suit
xGMI's point-to-point links; the whole DecoderLM fits one 256 MiB bucket). Device
gradients are all-reduced in place on the GPU; NumPy-backed gradients (CPU backends) are
staged through CPU torch tensors.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from .module import Parameter
from .tensor import Tensor
from .tensor_data import TensorData


def world_and_rank(group=None) -> Tuple[int, int]:
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def shard_rows(x: np.ndarray, world: int, rank: int) -> np.ndarray:
    """Rank's contiguous share of the leading (batch) axis; the batch must divide evenly
    so that the averaged gradient equals the full-batch gradient."""
    n = x.shape[0]
    if n % world:
        raise ValueError(f"global batch {n} does not divide over {world} ranks")
    per = n // world
    return x[rank * per:(rank + 1) * per]


def _flat_torch(t: Tensor):
    """(flat fp32 torch view of t's values, is_device)."""
    import torch
    if not t._tensor.is_dense():
        t = t.contiguous()
    st = t._tensor._storage
    if isinstance(st, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(t._tensor.to_numpy()).reshape(-1)), False
    return st.reshape(-1)[: t._tensor.size].float(), True


def _grads(parameters: Sequence[Parameter]) -> List[Tuple[Parameter, Tensor]]:
    out = []
    for p in parameters:
        g = getattr(p.value, "grad", None) if p.value is not None else None
        if g is not None:
            out.append((p, g))
    return out


def allreduce_gradients(parameters: Sequence[Parameter], group=None, bucket_mb: int = 256) -> None:
    """Average every parameter's ``.grad`` across ranks (SUM all-reduce / world size)."""
    import torch
    import torch.distributed as dist
    world, _ = world_and_rank(group)
    if world == 1:
        return
    pending = _grads(parameters)
    limit = bucket_mb * (1 << 20) // 4
    i = 0
    while i < len(pending):
        bucket, n = [], 0
        while i < len(pending) and (not bucket or n + pending[i][1]._tensor.size <= limit):
            bucket.append(pending[i])
            n += pending[i][1]._tensor.size
            i += 1
        flats = [_flat_torch(g) for _, g in bucket]
        on_dev = flats[0][1]
        buf = torch.cat([f for f, _ in flats])
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        buf /= world
        off = 0
        for (p, g), (f, _) in zip(bucket, flats):
            sz = f.numel()
            piece = buf[off:off + sz]
            off += sz
            storage = piece.clone() if on_dev else piece.numpy().copy()
            p.value.grad = Tensor(TensorData(storage, g.shape), backend=g.backend)


def broadcast_parameters(parameters: Sequence[Parameter], src: int = 0, group=None) -> None:
    """Copy rank ``src``'s parameter values to every rank (identical initialisation)."""
    import torch
    import torch.distributed as dist
    world, _ = world_and_rank(group)
    if world == 1:
        return
    for p in parameters:
        v = p.value
        f, on_dev = _flat_torch(v)
        f = f.clone()
        dist.broadcast(f, src=src, group=group)
        storage = f if on_dev else f.numpy().copy()
        p.update(Tensor(TensorData(storage, v.shape), backend=v.backend))


def train_step(model, optimizer, loss_fn, inputs, targets, group=None) -> float:
    """One data-parallel step: forward + backward on this rank's shard, gradient
    all-reduce, optimizer step. ``loss_fn(model, inputs, targets)`` returns a scalar
    minitorch Tensor (mean over the shard). Returns the loss averaged over ranks."""
    import torch
    import torch.distributed as dist
    optimizer.zero_grad()
    loss = loss_fn(model, inputs, targets)
    loss.backward()
    allreduce_gradients(optimizer.parameters, group=group)
    optimizer.step()
    value = float(loss.item())
    world, _ = world_and_rank(group)
    if world > 1:
        t = torch.tensor([value], dtype=torch.float64)
        if dist.get_backend(group) == "nccl":
            t = t.cuda()
        dist.all_reduce(t, group=group)
        value = float(t[0]) / world
    return value
