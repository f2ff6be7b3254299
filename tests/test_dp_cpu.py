"""World-size-2 ``gloo`` test of the data-parallel training step (minitorch/dp.py) on CPU:
two ranks on half batches + gradient all-reduce reproduce the single-process full-batch
step of a DecoderLM (NumPy test backend; on GPUs the same code all-reduces device
gradients over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _setup_path():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "llmsys-project-flashattn_amd"), os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _model_and_data():
    import minitorch
    from cpu_backend import NumpyOps
    backend = minitorch.TensorBackend(NumpyOps)
    np.random.seed(0)
    lm = minitorch.DecoderLM(n_vocab=20, n_embd=16, n_head=4, n_positions=8, p_dropout=0.0,
                             backend=backend, use_fused_kernel=True, use_flash_attention=True,
                             n_layer=1)
    rng = np.random.default_rng(1)
    idx = rng.integers(0, 20, (4, 8)).astype(np.float32)
    tgt = rng.integers(0, 20, (4, 8)).astype(np.float32)
    return minitorch, backend, lm, idx, tgt


def _loss_fn(minitorch, backend):
    def f(model, x, y):
        b, t = x.shape
        logits = model(minitorch.tensor_from_numpy(x, backend))
        loss = minitorch.softmax_loss(logits.view(b * t, 20),
                                      minitorch.tensor_from_numpy(y.reshape(-1), backend))
        return loss.sum() / (b * t)
    return f


def _worker(rank, world, port, errq):
    _setup_path()
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        from minitorch import dp
        minitorch, backend, lm, idx, tgt = _model_and_data()
        params = lm.parameters()
        dp.broadcast_parameters(params)
        opt = minitorch.SGD(params, lr=0.5)
        loss_fn = _loss_fn(minitorch, backend)
        loss = dp.train_step(lm, opt, loss_fn, dp.shard_rows(idx, world, rank),
                             dp.shard_rows(tgt, world, rank))
        got = [p.value.to_numpy() for p in lm.parameters()]
        # reference: one process, full batch
        minitorch, backend, ref, idx, tgt = _model_and_data()
        ropt = minitorch.SGD(ref.parameters(), lr=0.5)
        ropt.zero_grad()
        l_full = loss_fn(ref, idx, tgt)
        l_full.backward()
        ropt.step()
        for a, (name, p) in zip(got, ref.named_parameters()):
            np.testing.assert_allclose(a, p.value.to_numpy(), rtol=1e-5, atol=1e-6, err_msg=name)
        np.testing.assert_allclose(loss, float(l_full.item()), rtol=1e-5)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_rows():
    _setup_path()
    from minitorch.dp import shard_rows
    x = np.arange(12).reshape(6, 2)
    assert shard_rows(x, 3, 1).tolist() == [[4, 5], [6, 7]]
    with pytest.raises(ValueError):
        shard_rows(x, 4, 0)


def test_dp_step_matches_full_batch_gloo_world2():
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, errq)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
