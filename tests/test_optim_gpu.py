"""The multi-tensor Adam kernel (``mt_adam_step``, minitorch/optim.py's HIP path) against
the optimizer's tensor-op arithmetic restated in NumPy float32 (reference
minitorch/optim.py:50-79, second moment on (1 - beta2) as in this package's Adam), over
several steps, ragged sizes (the 4-element tail path), more tensors than one launch takes
(24), and one DecoderLM-sized parameter list through ``minitorch.Adam``."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mt():
    import torch
    assert torch.cuda.is_available(), "needs an MI355X"
    import minitorch
    from minitorch import _hip
    _hip.lib()
    return minitorch, minitorch.TensorBackend(minitorch.HipKernelOps)


def _np_adam(p, g, m, v, t, lr, b1, b2, eps):
    f = np.float32
    m = m * f(b1) + g * f(1 - b1)
    v = v * f(b2) + (g * g) * f(1 - b2)
    step = f(lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t))
    return p - (step * m) / (np.sqrt(v) + f(eps)), m, v


def test_adam_kernel_vs_numpy(mt):
    import torch
    from minitorch import _hip
    rng = np.random.default_rng(3)
    sizes = [1, 3, 4, 5, 1023, 1024, 1025, 4097, 256 * 256 + 7] + [17 * i + 1 for i in range(1, 25)]
    ps = [rng.standard_normal(n).astype(np.float32) for n in sizes]
    ms = [np.zeros(n, np.float32) for n in sizes]
    vs = [np.zeros(n, np.float32) for n in sizes]
    dp = [torch.from_numpy(x.copy()).cuda() for x in ps]
    dm = [torch.zeros(n, device="cuda") for n in sizes]
    dv = [torch.zeros(n, device="cuda") for n in sizes]
    lr, b1, b2, eps = 1e-3, 0.9, 0.999, 1e-8
    for t in range(1, 4):
        gs = [(rng.standard_normal(n) * 10.0 ** rng.integers(-4, 2)).astype(np.float32) for n in sizes]
        dg = [torch.from_numpy(x).cuda() for x in gs]
        step = lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
        _hip.adam_step([x.data_ptr() for x in dp], [x.data_ptr() for x in dg], [x.data_ptr() for x in dm],
                       [x.data_ptr() for x in dv], sizes, b1, b2, eps, step)
        for i in range(len(sizes)):
            ps[i], ms[i], vs[i] = _np_adam(ps[i], gs[i], ms[i], vs[i], t, lr, b1, b2, eps)
    torch.cuda.synchronize()
    for i in range(len(sizes)):
        np.testing.assert_allclose(dm[i].cpu().numpy(), ms[i], rtol=1e-6, atol=0)
        np.testing.assert_allclose(dv[i].cpu().numpy(), vs[i], rtol=1e-6, atol=0)
        # p: the update is ~lr, so compare it relative to the update size
        np.testing.assert_allclose(dp[i].cpu().numpy(), ps[i], rtol=0, atol=1e-7 * max(1.0, np.abs(ps[i]).max()))


def test_adam_fused_matches_tensor_ops(mt, monkeypatch):
    """minitorch.Adam on a DecoderLM's parameters: the fused path against the tensor-op path
    (the same optimizer with the fused kernel disabled) after two steps, bit for bit (the
    kernel rounds every product and sum as the tensor ops do, divides through the reciprocal
    and takes the square root with powf(v, 0.5), as Inv and PowerScalar do)."""
    import torch
    minitorch, backend = mt
    from minitorch import optim

    def run(fused):
        rng = np.random.default_rng(0)
        lm = minitorch.DecoderLM(n_vocab=500, n_embd=64, n_head=4, n_positions=16, p_dropout=0.0,
                                 backend=backend, use_fused_kernel=True, use_flash_attention=True)
        for i, p in enumerate(lm.parameters()):  # deterministic weights
            arr = np.random.default_rng(i).standard_normal(p.value.shape).astype(np.float32) * 0.05
            p.update(minitorch.tensor_from_numpy(arr, backend))
        opt = minitorch.Adam(lm.parameters(), lr=1e-2)
        x = minitorch.tensor_from_numpy(rng.integers(0, 500, (4, 16)).astype(np.float32), backend)
        y = minitorch.tensor_from_numpy(rng.integers(0, 500, (64,)).astype(np.float32), backend)
        if not fused:
            monkeypatch.setattr(optim, "_fusable", lambda *ts: False)
        for _ in range(2):
            opt.zero_grad()
            loss = minitorch.softmax_loss(lm(x).view(64, 500), y).sum() / 64
            loss.backward()
            opt.step()
        monkeypatch.undo()
        torch.cuda.synchronize()
        return [p.value.to_numpy() for p in lm.parameters()]

    a, b = run(True), run(False)
    assert len(a) == len(b) > 24
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
