"""The fused softmax cross-entropy (mt_softmax_xent_fw / _bw, minitorch.nn.softmax_loss on the
HIP backend) against the reference's composition on the same backend (logsumexp - one-hot
pick, minitorch/nn.py) and against a NumPy float64 restatement: per-row loss and the logits
gradient, for class counts with and without 16-B rows (C % 4), the config-5 vocabulary
(10000) and rows with extreme logits."""
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


def _np_xent(x, t, g):
    x = x.astype(np.float64)
    m = x.max(axis=1, keepdims=True)
    lse = m[:, 0] + np.log(np.exp(x - m).sum(axis=1))
    loss = lse - x[np.arange(len(t)), t]
    p = np.exp(x - lse[:, None])
    p[np.arange(len(t)), t] -= 1.0
    return loss, p * g[:, None]


@pytest.mark.parametrize("rows,C", [(7, 5), (5, 4), (64, 1000), (33, 1023), (16, 16384), (8, 16388), (4992, 10000)])
def test_softmax_xent_vs_numpy_and_composition(mt, rows, C):
    minitorch, backend = mt
    from minitorch import nn
    rng = np.random.default_rng(rows + C)
    x = (rng.standard_normal((rows, C)) * 3).astype(np.float32)
    x[0, :] += 60.0  # a row far from zero
    x[-1, 1] = 80.0  # a spike
    t = rng.integers(0, C, rows)
    g = rng.standard_normal(rows).astype(np.float32)
    loss_ref, dx_ref = _np_xent(x, t, g)

    def run(fused):
        xt = minitorch.tensor_from_numpy(x, backend)
        xt.requires_grad_(True)
        tt = minitorch.tensor_from_numpy(t.astype(np.float32), backend)
        gt = minitorch.tensor_from_numpy(g, backend)
        if fused:
            loss = nn.softmax_loss(xt, tt)
        else:  # the reference's composition on the same backend
            picked = (xt * nn.one_hot(tt, C)).sum(dim=1)
            loss = (nn.logsumexp(xt, dim=1) - picked).view(rows)
        (loss * gt).sum().backward()
        return loss.to_numpy(), xt.grad.to_numpy()

    lf, df = run(True)
    lc, dc = run(False)
    np.testing.assert_allclose(lf, loss_ref, rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(df, dx_ref, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(lf, lc, rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(df, dc, rtol=1e-4, atol=1e-6)
