"""World-size-2 ``gloo`` tests of the B*H sharding + output all-gather (minitorch/shard.py)
on CPU. The per-shard attention is the CPU oracle here (test infrastructure); on the GPU
box the same code calls the HIP kernels with backend "nccl" (RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from minitorch.shard import bh_range, shard


def test_bh_range_partition():
    for bh in (1, 3, 7, 128, 1024):
        for world in (1, 2, 3, 4, 8):
            spans = [bh_range(bh, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == bh
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1
    t = torch.arange(2 * 3 * 4 * 5, dtype=torch.float32).reshape(2, 3, 4, 5)
    s = shard(t, 2, 1)
    assert s.shape == (3, 4, 5) and s.data_ptr() == t.reshape(6, 4, 5)[3].data_ptr()


def test_shard_refuses_permuted_view():
    t = torch.zeros(2, 5, 3, 4).permute(0, 2, 1, 3)  # [B,H,N,d] view of [B,N,H,d] storage
    with pytest.raises(ValueError, match="not contiguous over"):
        shard(t, 2, 0)


def test_explicit_rank_ragged_no_collective():
    """One process computes every rank's rows of a ragged 3-way split (B*H = 4) with
    explicit world/rank, feeds each rank-local forward into the backward, and the pieces
    concatenate to the unsharded oracle result."""
    from minitorch.shard import sharded_flash_bwd, sharded_flash_fwd
    g = torch.Generator().manual_seed(3)
    shape = (2, 2, 40, 8)
    q, k, v, do = (torch.randn(shape, generator=g) for _ in range(4))
    flat = lambda t: t.reshape(-1, *t.shape[2:])
    ro, rm, rl = _oracle_fwd(flat(q), flat(k), flat(v), True)
    rg = _oracle_bwd(flat(q), flat(k), flat(v), ro, flat(do), rm, rl, True)
    outs, grads = [], []
    for r in range(3):
        o, m, l = sharded_flash_fwd(q, k, v, True, gather=False, attn=_oracle_fwd, world=3, rank=r)
        outs.append(o)
        grads.append(sharded_flash_bwd(q, k, v, o, do, m, l, True, gather=False,
                                       attn_bwd=_oracle_bwd, world=3, rank=r))
    assert [o.shape[0] for o in outs] == [2, 1, 1]
    np.testing.assert_allclose(torch.cat(outs).numpy(), ro.numpy(), atol=1e-6)
    for i in range(3):
        np.testing.assert_allclose(torch.cat([gr[i] for gr in grads]).numpy(), rg[i].numpy(), atol=1e-5)
    with pytest.raises(ValueError, match="rows"):
        sharded_flash_bwd(q, k, v, outs[0], do, m, l, True, gather=False, attn_bwd=_oracle_bwd,
                          world=3, rank=2)


def _oracle_fwd(q, k, v, causal):
    from oracle import attention as A
    o, m, l = A.attention_fwd(q.numpy(), k.numpy(), v.numpy(), causal)
    return torch.from_numpy(o), torch.from_numpy(m), torch.from_numpy(l)


def _oracle_bwd(q, k, v, o, do, m, l, causal):
    from oracle import attention as A
    g = A.attention_bwd(*(t.numpy() for t in (q, k, v, o, do, m, l)), causal)
    return tuple(torch.from_numpy(np.ascontiguousarray(x)) for x in g)


def _worker(rank, world, port, shape, causal, errq):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "llmsys-project-flashattn_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from minitorch.shard import sharded_flash_bwd, sharded_flash_fwd
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        g = torch.Generator().manual_seed(0)
        q, k, v, do = (torch.randn(shape, generator=g) for _ in range(4))
        o, m, l = sharded_flash_fwd(q, k, v, causal, attn=_oracle_fwd)
        ro, rm, rl = _oracle_fwd(q.reshape(-1, *shape[2:]), k.reshape(-1, *shape[2:]),
                                 v.reshape(-1, *shape[2:]), causal)
        np.testing.assert_allclose(o.reshape(ro.shape).numpy(), ro.numpy(), atol=1e-6)
        np.testing.assert_allclose(m.reshape(rm.shape).numpy(), rm.numpy(), atol=1e-6)
        dq, dk, dv = sharded_flash_bwd(q, k, v, o, do, m, l, causal, attn_bwd=_oracle_bwd)
        flat = lambda t: t.reshape(-1, *t.shape[2:])
        ref = _oracle_bwd(flat(q), flat(k), flat(v), flat(o), flat(do), flat(m), flat(l), causal)
        for got, want in zip((dq, dk, dv), ref):
            np.testing.assert_allclose(flat(got).numpy(), want.numpy(), atol=1e-5)
        # without gather: this rank's rows only
        os_, _, _ = sharded_flash_fwd(q, k, v, causal, gather=False, attn=_oracle_fwd)
        lo, hi = bh_range(shape[0] * shape[1], world, rank)
        np.testing.assert_allclose(os_.numpy(), ro[lo:hi].numpy(), atol=1e-6)
        # the no-gather training path: rank-local O/m/l straight into the backward
        os_, ms_, ls_ = sharded_flash_fwd(q, k, v, causal, gather=False, attn=_oracle_fwd)
        lg = sharded_flash_bwd(q, k, v, os_, do, ms_, ls_, causal, gather=False, attn_bwd=_oracle_bwd)
        for got, want in zip(lg, ref):
            np.testing.assert_allclose(got.numpy(), want[lo:hi].numpy(), atol=1e-5)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surfaced to the parent
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("shape,causal", [((2, 2, 48, 16), False), ((1, 3, 33, 8), True)])
def test_sharded_fwd_bwd_gloo_world2(shape, causal):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, shape, causal, errq)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _chunk_worker(rank, world, port, shape, causal, chunks, errq):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "llmsys-project-flashattn_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from minitorch.shard import sharded_flash_fwd
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        g = torch.Generator().manual_seed(7)
        q, k, v = (torch.randn(shape, generator=g) for _ in range(3))
        one = sharded_flash_fwd(q, k, v, causal, attn=_oracle_fwd)
        many = sharded_flash_fwd(q, k, v, causal, attn=_oracle_fwd, chunks=chunks)
        for a, b in zip(one, many):  # the overlapped chunked gather changes nothing
            assert a.shape == b.shape and torch.equal(a, b), "chunked gather differs"
        # an explicit rank that is not this process's own, with gather: refused
        with pytest.raises(ValueError, match="not this process's group rank"):
            sharded_flash_fwd(q, k, v, causal, attn=_oracle_fwd, world=world, rank=(rank + 1) % world)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surfaced to the parent
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


@pytest.mark.parametrize("world,shape,causal,chunks", [(2, (2, 4, 40, 8), False, 2),
                                                      (4, (2, 8, 24, 8), True, 2)])
def test_chunked_overlapped_gather_bit_identical(world, shape, causal, chunks):
    """The chunked forward (all-gather of finished chunks overlapping the next chunk's
    forward, block-cyclic rows) returns exactly the unchunked gathered O, m, l."""
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_chunk_worker, args=(r, world, port, shape, causal, chunks, errq))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_chunk_rows_cover_every_head_once():
    from minitorch.shard import chunk_rows
    for bh, world, chunks in ((128, 8, 2), (1024, 8, 4), (16, 2, 4)):
        seen = sorted(r for rank in range(world) for c in range(chunks)
                      for r in range(*chunk_rows(bh, world, rank, chunks, c)))
        assert seen == list(range(bh))
        # chunk c of all ranks is one contiguous range, rank order
        for c in range(chunks):
            spans = [chunk_rows(bh, world, rank, chunks, c) for rank in range(world)]
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
