"""Host-side minitorch machinery on a NumPy test backend (no GPU): tensor layout,
autodiff, module wiring and the MultiHeadAttention flash/plain/fused branches vs
torch.nn.MultiheadAttention (the reference's test recipe,
tests/test_flash_attention.py:24-186)."""
import numpy as np
import pytest
import torch

import minitorch
from cpu_backend import NumpyOps

BACKEND = minitorch.TensorBackend(NumpyOps)


def t(a, grad=False):
    return minitorch.tensor_from_numpy(np.asarray(a, np.float32), BACKEND, grad)


def test_tensor_data_layout():
    td = minitorch.TensorData(np.arange(24, dtype=np.float32), (2, 3, 4))
    assert td.strides == (12, 4, 1) and td.is_contiguous()
    p = td.permute(2, 0, 1)
    assert p.shape == (4, 2, 3) and p.strides == (1, 12, 4)
    assert not p.is_contiguous()
    np.testing.assert_array_equal(p.to_numpy(), np.arange(24).reshape(2, 3, 4).transpose(2, 0, 1))
    assert minitorch.shape_broadcast((2, 1, 4), (3, 1)) == (2, 3, 4)
    with pytest.raises(minitorch.IndexingError):
        minitorch.shape_broadcast((2, 3), (4, 3))


def test_autodiff_elementwise_and_reduce():
    x = np.random.default_rng(0).standard_normal((3, 4)).astype(np.float32)
    a = t(x, True)
    y = ((a * a).exp() / (a + 3.0)).sum(1).log().sum()
    y.backward()
    xt = torch.tensor(x, dtype=torch.float64, requires_grad=True)
    yt = torch.log(((xt * xt).exp() / (xt + 3.0)).sum(1) + 1e-6).sum()
    yt.backward()
    np.testing.assert_allclose(a.grad.to_numpy(), xt.grad.numpy(), rtol=1e-4, atol=1e-5)


def test_autodiff_matmul_permute_view():
    rng = np.random.default_rng(1)
    x, w = rng.standard_normal((2, 3, 5)), rng.standard_normal((5, 4))
    a, b = t(x, True), t(w, True)
    out = (a.view(6, 5) @ b).view(2, 3, 4).permute(2, 0, 1).contiguous().sum()
    out.backward()
    xt = torch.tensor(x, requires_grad=True)
    wt = torch.tensor(w, requires_grad=True)
    (xt.reshape(6, 5) @ wt).sum().backward()
    np.testing.assert_allclose(a.grad.to_numpy(), xt.grad.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(b.grad.to_numpy(), wt.grad.numpy(), rtol=1e-5, atol=1e-5)


def test_module_parameters():
    mha = minitorch.MultiHeadAttention(16, 4, True, 0.0, bias=False, backend=BACKEND,
                                       use_flash_attention=True)
    names = [n for n, _ in mha.named_parameters()]
    assert names == ["q_projection.weights", "k_projection.weights",
                     "v_projection.weights", "out_projection.weights"]
    layer = minitorch.TransformerLayer(16, 4, 0.0, 1e-5, True, BACKEND, use_flash_attention=True)
    assert layer.attention.use_flash_attention and layer.attention.causal


def _mha_vs_torch(causal, use_flash, use_fused, B=2, N=12, E=16, H=4, seed=10):
    np.random.seed(seed)
    torch.manual_seed(seed)
    data = np.random.rand(B, N, E)
    X = minitorch.tensor_from_numpy(data, BACKEND, True)
    X_ = torch.tensor(data, dtype=torch.float32, requires_grad=True)
    layer_ = torch.nn.MultiheadAttention(E, H, 0.0, bias=False, batch_first=True, dtype=torch.float32)
    layer = minitorch.MultiHeadAttention(E, H, causal, 0.0, bias=False, backend=BACKEND,
                                         use_fused_kernel=use_fused, use_flash_attention=use_flash)
    w_qkv = layer_.in_proj_weight.detach().numpy().T.copy()
    for name, w in zip(("q_projection", "k_projection", "v_projection"), np.split(w_qkv, 3, -1)):
        getattr(layer, name).weights.value = minitorch.tensor_from_numpy(w.copy(), BACKEND, True)
    layer.out_projection.weights.value = minitorch.tensor_from_numpy(
        layer_.out_proj.weight.detach().numpy().T.copy(), BACKEND, True)
    mask = torch.triu(-float("inf") * torch.ones(N, N), 1) if causal else None
    result = layer(X)
    result_, _ = layer_(X_, X_, X_, attn_mask=mask)
    np.testing.assert_allclose(result.to_numpy(), result_.detach().numpy(), atol=1e-5, rtol=1e-5)
    result.sum().backward()
    result_.sum().backward()
    np.testing.assert_allclose(X.grad.to_numpy(), X_.grad.detach().numpy(), atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(layer.out_projection.weights.value.grad.to_numpy(),
                               layer_.out_proj.weight.grad.detach().numpy().T, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("branch", ["flash", "plain", "fused"])
def test_mha_branches_vs_torch(causal, branch):
    _mha_vs_torch(causal, branch == "flash", branch == "fused")


def test_decoder_lm_step_cpu():
    lm = minitorch.DecoderLM(n_vocab=20, n_embd=16, n_head=4, n_positions=8, p_dropout=0.0,
                             backend=BACKEND, use_fused_kernel=True, use_flash_attention=True,
                             n_layer=1)
    idx = minitorch.tensor_from_numpy(np.random.randint(0, 20, (2, 8)).astype(np.float32), BACKEND)
    logits = lm(idx)
    assert logits.shape == (2, 8, 20)
    loss = minitorch.softmax_loss(logits.view(16, 20), minitorch.tensor_from_numpy(
        np.random.randint(0, 20, (16,)).astype(np.float32), BACKEND)).sum() / 16
    loss.backward()
    missing = [n for n, p in lm.named_parameters() if p.value.grad is None]
    assert not missing, missing
    before = lm.lm_head.weights.value.to_numpy().copy()
    opt = minitorch.Adam(lm.parameters(), lr=1e-3)
    opt.step()
    assert np.abs(lm.lm_head.weights.value.to_numpy() - before).max() > 0
