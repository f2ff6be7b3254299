"""The graph-captured training step (minitorch/graphs.py StepGraph) against the same step run
eagerly: a DecoderLM with dropout and the fused Adam (config 5's step at reduced size), two
copies from the same initial weights and the same NumPy seed, one stepped eagerly and one by
replays. Every replay must reproduce the eager step bit for bit: the loss of each step, and
after the run every parameter and both Adam moments. That holds only if each replay draws
fresh dropout seeds in the eager order and advances Adam's bias correction."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _setup(minitorch, backend, p_dropout, seed=0):
    np.random.seed(seed)
    B, T, V, E, H = 8, 24, 300, 64, 4
    lm = minitorch.DecoderLM(n_vocab=V, n_embd=E, n_head=H, n_positions=T + 1, p_dropout=p_dropout,
                             backend=backend, use_fused_kernel=True, use_flash_attention=True)
    opt = minitorch.Adam(lm.parameters(), lr=1e-3)
    rng = np.random.default_rng(1)
    tok = rng.integers(0, V, size=(B, T + 1)).astype(np.float32)
    kv = rng.integers(T // 2, T + 1, size=B).astype(np.int64)
    w = (np.arange(T)[None, :] < kv[:, None]).astype(np.float32)
    x = minitorch.tensor_from_numpy(tok[:, :-1].copy(), backend)
    y = minitorch.tensor_from_numpy(tok[:, 1:].reshape(-1).copy(), backend)
    wt = minitorch.tensor_from_numpy(w.reshape(-1).copy(), backend)

    def step():
        opt.zero_grad()
        logits = lm(x, kv_len=kv).view(B * T, V)
        loss = (minitorch.softmax_loss(logits, y) * wt).sum() / wt.sum()
        loss.backward()
        opt.step()
        return loss

    return lm, opt, step


def _state(lm, opt):
    out = []
    for p in lm.parameters():
        out.append(p.value.to_numpy().copy())
        st = opt._states[id(p)]
        out.append(st["exp_avg"].to_numpy().copy())
        out.append(st["exp_avg_sq"].to_numpy().copy())
        out.append(np.array(st["step"]))
    return out


@pytest.mark.parametrize("p_dropout", [0.0, 0.1])
def test_step_graph_matches_eager_bitwise(p_dropout):
    import torch
    assert torch.cuda.is_available(), "needs an MI355X"
    import minitorch
    from minitorch import _hip
    from minitorch.graphs import StepGraph
    _hip.lib()
    backend = minitorch.TensorBackend(minitorch.HipKernelOps)
    warmup, replays = 2, 4

    lm_e, opt_e, step_e = _setup(minitorch, backend, p_dropout)
    lm_g, opt_g, step_g = _setup(minitorch, backend, p_dropout)

    np.random.seed(123)
    eager_losses = []
    for _ in range(warmup + replays):
        eager_losses.append(float(step_e().to_numpy()[0]))
    torch.cuda.synchronize()
    eager_state = _state(lm_e, opt_e)

    np.random.seed(123)
    g = StepGraph(step_g, warmup=warmup)
    graph_losses = []
    for _ in range(replays):
        loss = g.replay()
        torch.cuda.synchronize()
        graph_losses.append(float(loss.to_numpy()[0]))
    graph_state = _state(lm_g, opt_g)

    assert g.replays == replays
    if p_dropout > 0:
        assert len(g._seed_fns) > 0, "the captured step should own dropout seed slots"
    assert len(g._f32_fns) >= 1, "the captured Adam should read its step size from a slot"
    assert graph_losses == eager_losses[warmup:], (graph_losses, eager_losses)
    for a, b in zip(eager_state, graph_state):
        np.testing.assert_array_equal(a, b)


def test_step_graph_new_batches_match_eager():
    """Replays fed a new batch each time through copy_into (tokens, labels, loss weights and a
    device kv_len tensor in fixed buffers) match eager steps over the same batch sequence bit for
    bit: losses, parameters and Adam moments."""
    import torch
    assert torch.cuda.is_available(), "needs an MI355X"
    import minitorch
    from minitorch.graphs import StepGraph, copy_into
    backend = minitorch.TensorBackend(minitorch.HipKernelOps)
    B, T, V, E, H = 8, 24, 300, 64, 4
    rng = np.random.default_rng(3)
    batches = []
    for _ in range(5):
        tok = rng.integers(0, V, size=(B, T + 1)).astype(np.float32)
        kv = rng.integers(T // 3, T + 1, size=B).astype(np.float32)
        w = (np.arange(T)[None, :] < kv[:, None]).astype(np.float32)
        batches.append((tok[:, :-1].copy(), tok[:, 1:].reshape(-1).copy(), w.reshape(-1).copy(), kv))

    def make():
        np.random.seed(0)
        lm = minitorch.DecoderLM(n_vocab=V, n_embd=E, n_head=H, n_positions=T + 1, p_dropout=0.1,
                                 backend=backend, use_fused_kernel=True, use_flash_attention=True)
        opt = minitorch.Adam(lm.parameters(), lr=1e-3)
        bufs = [minitorch.tensor_from_numpy(a, backend) for a in batches[0]]
        x, y, wt, kvt = bufs

        def step():
            opt.zero_grad()
            loss = (minitorch.softmax_loss(lm(x, kv_len=kvt).view(B * T, V), y) * wt).sum() / wt.sum()
            loss.backward()
            opt.step()
            return loss
        return lm, opt, bufs, step

    lm_e, opt_e, bufs_e, step_e = make()
    np.random.seed(7)
    eager = []
    for i in [0, 0, 1, 2, 3, 4]:
        for t, a in zip(bufs_e, batches[i]):
            copy_into(t, a)
        eager.append(float(step_e().to_numpy()[0]))
    torch.cuda.synchronize()

    lm_g, opt_g, bufs_g, step_g = make()
    np.random.seed(7)
    g = StepGraph(step_g, warmup=2)
    graph = []
    for i in [1, 2, 3, 4]:
        for t, a in zip(bufs_g, batches[i]):
            copy_into(t, a)
        loss = g.replay()
        torch.cuda.synchronize()
        graph.append(float(loss.to_numpy()[0]))
    assert graph == eager[2:], (graph, eager)
    for a, b in zip(_state(lm_e, opt_e), _state(lm_g, opt_g)):
        np.testing.assert_array_equal(a, b)


def test_step_graph_config5_size_matches_eager():
    """The same bitwise check at config 5's size (B=128, T=39, V=10000, n_embd 256, 8 heads): the
    replayed graph then holds the kernels the small model never reaches, the column reductions
    with arrival counters (4992 x 256 bias gradients) and the split-K LM-head dX GEMM with its
    scratch partials."""
    import torch
    assert torch.cuda.is_available(), "needs an MI355X"
    import minitorch
    from minitorch.graphs import StepGraph
    backend = minitorch.TensorBackend(minitorch.HipKernelOps)
    B, T, V, E, H = 128, 39, 10000, 256, 8
    rng = np.random.default_rng(9)
    tok = rng.integers(0, V, size=(B, T + 1)).astype(np.float32)
    kv = rng.integers(T // 2, T + 1, size=B).astype(np.int64)
    w = (np.arange(T)[None, :] < kv[:, None]).astype(np.float32)

    def make():
        np.random.seed(0)
        lm = minitorch.DecoderLM(n_vocab=V, n_embd=E, n_head=H, n_positions=T + 1, p_dropout=0.1,
                                 backend=backend, use_fused_kernel=True, use_flash_attention=True)
        opt = minitorch.Adam(lm.parameters(), lr=1e-4)
        x = minitorch.tensor_from_numpy(tok[:, :-1].copy(), backend)
        y = minitorch.tensor_from_numpy(tok[:, 1:].reshape(-1).copy(), backend)
        wt = minitorch.tensor_from_numpy(w.reshape(-1).copy(), backend)

        def step():
            opt.zero_grad()
            loss = (minitorch.softmax_loss(lm(x, kv_len=kv).view(B * T, V), y) * wt).sum() / wt.sum()
            loss.backward()
            opt.step()
            return loss
        return lm, opt, step

    lm_e, opt_e, step_e = make()
    np.random.seed(5)
    eager = [float(step_e().to_numpy()[0]) for _ in range(4)]
    torch.cuda.synchronize()
    lm_g, opt_g, step_g = make()
    np.random.seed(5)
    g = StepGraph(step_g, warmup=2)
    graph = []
    for _ in range(2):
        loss = g.replay()
        torch.cuda.synchronize()
        graph.append(float(loss.to_numpy()[0]))
    assert graph == eager[2:], (graph, eager)
    for a, b in zip(_state(lm_e, opt_e), _state(lm_g, opt_g)):
        np.testing.assert_array_equal(a, b)


def test_step_graph_fails_loudly_on_host_sync():
    """A step that needs the host inside it (a device value read back) cannot be captured:
    the capture raises instead of recording a step that would replay wrong."""
    import torch
    assert torch.cuda.is_available(), "needs an MI355X"
    import minitorch
    from minitorch.graphs import StepGraph
    backend = minitorch.TensorBackend(minitorch.HipKernelOps)
    a = minitorch.tensor_from_numpy(np.ones((4, 4), dtype=np.float32), backend)

    def step():
        return float((a * 2.0).sum().item())

    with pytest.raises(Exception):
        StepGraph(step, warmup=1)
