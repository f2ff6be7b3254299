"""The B*H-sharded forward and backward on the GPU:
minitorch/shard.py driving the HIP kernels through the C ABI, with the output all-gather
over RCCL (``backend="nccl"`` is RCCL on ROCm), checked against the CPU oracle.

One GPU per box here, so the RCCL group has world size 1 (the all-gather runs, over one
rank); the multi-rank logic is covered by the world-size-2 gloo tests in
tests/test_shard_cpu.py, and the ragged split is exercised here without a collective by
computing each rank's rows of a 3-way split in one process (explicit world/rank,
``gather=False``, the rank-local forward fed straight into the backward)."""
import socket

import numpy as np
import pytest

from oracle import attention as A

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rccl_group():
    import torch
    import torch.distributed as dist
    assert torch.cuda.is_available(), "needs an MI355X"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1)
    yield dist
    dist.destroy_process_group()


def _inputs(torch, shape, dtype, seed):
    rng = np.random.default_rng(seed)
    arrs = [rng.standard_normal(shape).astype(np.float32) for _ in range(4)]
    if dtype == torch.bfloat16:
        arrs = [A.bf16_round(a) for a in arrs]
    return arrs, [torch.from_numpy(a).to("cuda").to(dtype) for a in arrs]


def _tol(dtype, torch):
    # fp32: the reference MHA bound; bf16: the bounds of tests/test_flash_gpu.py
    return (1e-5, 1e-5) if dtype == torch.float32 else (2e-2, 2e-2)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_sharded_fwd_bwd_rccl_world1(rccl_group, causal, dt, parity_record):
    """gather=True through RCCL all_gather_into_tensor (world size 1) on the HIP path."""
    import torch
    from minitorch.shard import sharded_flash_bwd, sharded_flash_fwd
    dtype = torch.float32 if dt == "fp32" else torch.bfloat16
    shape = (2, 3, 192, 64)
    (q, k, v, do), (tq, tk, tv, tdo) = _inputs(torch, shape, dtype, 11)
    o, m, l = sharded_flash_fwd(tq, tk, tv, causal)
    dq, dk, dv = sharded_flash_bwd(tq, tk, tv, o, tdo, m, l, causal)
    torch.cuda.synchronize()
    ro, rm, rl = A.attention_fwd(q, k, v, causal)
    rg = A.attention_bwd(q, k, v, ro, do, rm, rl, causal)
    otol, gtol = _tol(dtype, torch)
    err_o = float(np.abs(o.float().cpu().numpy() - ro).max())
    assert err_o <= otol, err_o
    for name, got, want in zip("QKV", (dq, dk, dv), rg):
        scale = max(1.0, float(np.abs(want).max()))
        err = float(np.abs(got.float().cpu().numpy() - want).max())
        assert err <= gtol * scale, f"d{name} {err:.3e}"
    parity_record("test_sharded_fwd_bwd_rccl_world1", f"{dt} causal={causal} {shape}", max_abs_o=err_o,
                  bound_o=otol)


@pytest.mark.parametrize("causal", [False, True])
def test_sharded_ragged_local_bwd(causal):
    """Each rank's rows of a ragged 3-way split of B*H = 8 (3/3/2 heads), forward without
    gather, its rank-local O/m/l into the backward: the pieces equal the unsharded oracle
    result rows."""
    import torch
    from minitorch.shard import bh_range, sharded_flash_bwd, sharded_flash_fwd
    shape = (2, 4, 160, 64)
    (q, k, v, do), (tq, tk, tv, tdo) = _inputs(torch, shape, torch.float32, 12)
    flat = lambda a: a.reshape(-1, *a.shape[2:])
    ro, rm, rl = A.attention_fwd(flat(q), flat(k), flat(v), causal)
    rg = A.attention_bwd(flat(q), flat(k), flat(v), ro, flat(do), rm, rl, causal)
    for r in range(3):
        lo, hi = bh_range(8, 3, r)
        o, m, l = sharded_flash_fwd(tq, tk, tv, causal, gather=False, world=3, rank=r)
        assert o.shape == (hi - lo, 160, 64) and m.shape == (hi - lo, 160)
        grads = sharded_flash_bwd(tq, tk, tv, o, tdo, m, l, causal, gather=False, world=3, rank=r)
        torch.cuda.synchronize()
        np.testing.assert_allclose(o.cpu().numpy(), ro[lo:hi], atol=1e-5)
        for got, want in zip(grads, rg):
            np.testing.assert_allclose(got.cpu().numpy(), want[lo:hi], atol=1e-5)
