"""Config-5 parity: the transformer block and the DecoderLM
training step on the HIP backend.

* ``TransformerLayer`` against ``torch.nn.TransformerEncoderLayer(norm_first=True,
  gelu-tanh)`` with the reference's weight-injection recipe and tolerances
  (reference tests/test_modules_transformer.py:113-207: batch 2/32, seq 128, n_embd
  32/64, 4 heads, causal, no bias, ln_eps 1e-5, atol = rtol = 1e-5 on the output and on
  dX after ``result.sum().backward()``), for the plain, the flash and the fused-LN +
  flash attention branches.
* One DecoderLM step at config 5's width (n_vocab 10000, n_embd 256, 8 heads, seq 39;
  reference project/run_machine_translation.py:397-407) with the fused HIP LayerNorm and
  flash attention, against the same model, weights and tokens on the CPU test backend
  (tests/cpu_backend.py: NumPy ops, the CPU oracle for the attention): loss and every
  parameter gradient.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mt():
    import torch
    assert torch.cuda.is_available(), "needs an MI355X"
    import minitorch
    from minitorch import _hip
    _hip.lib()  # fail loudly if the HIP library is missing
    return minitorch, minitorch.TensorBackend(minitorch.HipKernelOps)


@pytest.mark.parametrize("branch", ["plain", "flash", "fused_flash"])
@pytest.mark.parametrize("batch_size,n_embd", [(2, 32), (2, 64), (32, 32), (32, 64)])
def test_transformer_layer_vs_torch(mt, batch_size, n_embd, branch, parity_record):
    import torch
    minitorch, backend = mt
    seq_len, num_heads = 128, 4
    np.random.seed(10)
    torch.manual_seed(10)
    data = np.random.randn(batch_size, seq_len, n_embd)
    X = minitorch.tensor_from_numpy(data.copy(), backend, True)
    X_ = torch.tensor(data, dtype=torch.float32, requires_grad=True)
    layer_ = torch.nn.TransformerEncoderLayer(
        d_model=n_embd, nhead=num_heads, dim_feedforward=256, dropout=0,
        activation=lambda x: torch.nn.functional.gelu(x, approximate="tanh"),
        batch_first=True, norm_first=True, bias=False, dtype=torch.float32,
        # the fused LayerNorm is the reference kernel's contract (layernorm_kernel.cu:
        # var = E[x²] − μ² + 1e-8, no eps argument): torch gets that eps for that branch
        layer_norm_eps=1e-8 if branch == "fused_flash" else 1e-5)
    layer = minitorch.TransformerLayer(
        n_embd=n_embd, n_head=num_heads, p_dropout=0, ln_eps=layer_.norm1.eps, bias=False,
        backend=backend, use_fused_kernel=branch == "fused_flash",
        use_flash_attention=branch != "plain")
    w_qkv = layer_.self_attn.in_proj_weight.detach().numpy().T.copy()
    w_q, w_k, w_v = (w.copy() for w in np.split(w_qkv, 3, -1))
    put = lambda mod, w: setattr(mod.weights, "value", minitorch.tensor_from_numpy(w, backend, True))
    put(layer.attention.q_projection, w_q)
    put(layer.attention.k_projection, w_k)
    put(layer.attention.v_projection, w_v)
    put(layer.attention.out_projection, layer_.self_attn.out_proj.weight.detach().numpy().T.copy())
    put(layer.ff.linear_in, layer_.linear1.weight.detach().numpy().T.copy())
    put(layer.ff.linear_out, layer_.linear2.weight.detach().numpy().T.copy())
    M = torch.triu(-float("inf") * torch.ones(seq_len, seq_len), 1)

    result = layer(X)
    result_ = layer_(X_, M)
    tol = 1e-5
    got, want = result.to_numpy(), result_.detach().numpy()
    np.testing.assert_allclose(got, want, atol=tol, rtol=tol)
    result.sum().backward()
    result_.sum().backward()
    gx, gx_ = X.grad.to_numpy(), X_.grad.detach().numpy()
    np.testing.assert_allclose(gx, gx_, atol=tol, rtol=tol)
    parity_record("test_transformer_layer_vs_torch", f"{branch} B={batch_size} E={n_embd}",
                  max_abs_out=float(np.abs(got - want).max()),
                  max_abs_dx=float(np.abs(gx - gx_).max()), bound=tol)


def test_decoder_lm_step_hip_vs_cpu(mt, parity_record):
    import minitorch
    from cpu_backend import NumpyOps
    _, hip = mt
    cpu = minitorch.TensorBackend(NumpyOps)
    V, E, H, B, T = 10000, 256, 8, 4, 39
    kw = dict(n_vocab=V, n_embd=E, n_head=H, n_positions=40, p_dropout=0.0,
              use_fused_kernel=True, use_flash_attention=True)
    lm_h = minitorch.DecoderLM(backend=hip, **kw)
    lm_c = minitorch.DecoderLM(backend=cpu, **kw)
    ph, pc = dict(lm_h.named_parameters()), dict(lm_c.named_parameters())
    assert ph.keys() == pc.keys()
    for name, p in ph.items():  # the HIP model's random init, copied to the CPU model
        pc[name].update(minitorch.tensor_from_numpy(p.value.to_numpy().copy(), cpu))
    rng = np.random.default_rng(7)
    # a right-padded batch with the reference's loss weights (run_machine_translation.py:
    # 119-141, 186-192): source tokens weight 0, target tokens 1, padding 0; the flash path
    # masks the padding keys (kv_len)
    from bench import synthetic_mt_batch
    batch = synthetic_mt_batch(rng, B, T, V)
    idx, tgt, w, kv = batch["input_ids"], batch["labels"], batch["label_token_weights"], batch["kv_len"]

    def step(lm, backend):
        logits = lm(minitorch.tensor_from_numpy(idx, backend), kv_len=kv)
        loss = minitorch.softmax_loss(logits.view(B * T, V),
                                      minitorch.tensor_from_numpy(tgt.reshape(-1), backend))
        wt = minitorch.tensor_from_numpy(w.reshape(-1), backend)
        loss = (loss * wt).sum() / wt.sum()
        loss.backward()
        return loss.item()

    loss_h, loss_c = step(lm_h, hip), step(lm_c, cpu)
    assert abs(loss_h - loss_c) <= 1e-5 * abs(loss_c), (loss_h, loss_c)
    # Each gradient within 1e-4 of its own max-abs, floored at 1e-3 of the largest gradient
    # of the model: the key-projection bias gradient is zero in exact arithmetic (a bias on
    # every key adds q·b to a whole score row, which the softmax cancels), so its own scale
    # is rounding noise.
    grads = {n: (ph[n].value.grad, pc[n].value.grad) for n in ph}
    assert all(a is not None and b is not None for a, b in grads.values())
    grads = {n: (a.to_numpy(), b.to_numpy()) for n, (a, b) in grads.items()}
    gmax = max(float(np.abs(b).max()) for _, b in grads.values())
    worst = 0.0
    for name, (a, b) in grads.items():
        scale = max(float(np.abs(b).max()), 1e-3 * gmax)
        err = float(np.abs(a - b).max()) / scale
        assert err <= 1e-4, f"{name}: max|Δgrad| / scale = {err:.2e}"
        worst = max(worst, err)
    parity_record("test_decoder_lm_step_hip_vs_cpu", f"V={V} E={E} H={H} B={B} T={T} padded, weighted loss",
                  loss_hip=loss_h, loss_cpu=loss_c, worst_rel_grad=worst, bound_rel_grad=1e-4)
