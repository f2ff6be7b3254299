"""Autodiff ``Function``s and tensor constructors (reference ``minitorch/tensor_functions.py``).

The fused functions are the hot path of the north star:
``FlashAttention`` / ``FlashAttentionCausal`` (reference :472-516) call
``Q.f.flash_attention[_causal]_fw`` and save ``(Q, K, V, O, m, l)``; their backward calls
``out_grad.f.flash_attention[_causal]_bw``. ``Attn_Softmax`` saves the softmax *output*
(what its backward needs; the reference saves the input and then mis-unpacks it,
:440/:447) and ``LayerNorm`` saves ``(inp, gamma, beta, var, mean)``.
"""
from __future__ import annotations

import random
from typing import Any, List, Optional, Tuple

import numpy as np

from . import operators
from .autodiff import Context
from .tensor_data import TensorData, UserShape, _prod, datatype, strides_from_shape


def wrap_tuple(x: Any) -> tuple:
    return x if isinstance(x, tuple) else (x,)


_History = _Tensor = None  # tensor.History / tensor.Tensor, bound on the first Function.apply


class Function:
    @classmethod
    def _backward(cls, ctx: Context, grad_out) -> tuple:
        return wrap_tuple(cls.backward(ctx, grad_out))

    @classmethod
    def _forward(cls, ctx: Context, *inps):
        return cls.forward(ctx, *inps)

    @classmethod
    def apply(cls, *vals):
        global _History, _Tensor
        if _Tensor is None:  # bound once (tensor.py imports this module; an import per call was host time)
            from .tensor import History as _History, Tensor as _Tensor  # noqa: F811
        History, Tensor = _History, _Tensor
        raw_vals = []
        need_grad = False
        for v in vals:
            if v.requires_grad():
                need_grad = True
            raw_vals.append(v.detach())
        ctx = Context(not need_grad)
        c = cls._forward(ctx, *raw_vals)
        back = History(cls, ctx, vals) if need_grad else None
        return Tensor(c._tensor, back, backend=c.backend)


class Neg(Function):
    @staticmethod
    def forward(ctx, t1):
        return t1.f.neg_map(t1)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output.f.neg_map(grad_output)


class Inv(Function):
    @staticmethod
    def forward(ctx, t1):
        ctx.save_for_backward(t1)
        return t1.f.inv_map(t1)

    @staticmethod
    def backward(ctx, grad_output):
        (t1,) = ctx.saved_values
        return grad_output.f.inv_back_zip(t1, grad_output)


class Add(Function):
    @staticmethod
    def forward(ctx, t1, t2):
        return t1.f.add_zip(t1, t2)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output, grad_output


class Mul(Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return a.f.mul_zip(a, b)

    @staticmethod
    def backward(ctx, grad_output):
        a, b = ctx.saved_values
        return grad_output.f.mul_zip(b, grad_output), grad_output.f.mul_zip(a, grad_output)


class PowerScalar(Function):
    @staticmethod
    def forward(ctx, a, scalar):
        ctx.save_for_backward(a, scalar)
        return a.f.pow_scalar_zip(a, scalar)

    @staticmethod
    def backward(ctx, grad_output):
        a, scalar = ctx.saved_values
        s = scalar.item()
        # d/da a^s = s * a^(s-1)
        da = grad_output.f.mul_zip(
            grad_output,
            a.f.mul_zip(a.f.pow_scalar_zip(a, a._ensure_tensor(s - 1.0)), a._ensure_tensor(s)))
        return da, 0.0


class Tanh(Function):
    @staticmethod
    def forward(ctx, a):
        out = a.f.tanh_map(a)
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        (out,) = ctx.saved_values
        one_minus = out.f.add_zip(out._ensure_tensor(1.0), out.f.neg_map(out.f.mul_zip(out, out)))
        return grad_output.f.mul_zip(grad_output, one_minus)


class Sigmoid(Function):
    @staticmethod
    def forward(ctx, t1):
        out = t1.f.sigmoid_map(t1)
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        (s,) = ctx.saved_values
        ds = s.f.mul_zip(s, s.f.add_zip(s._ensure_tensor(1.0), s.f.neg_map(s)))
        return grad_output.f.mul_zip(grad_output, ds)


class ReLU(Function):
    @staticmethod
    def forward(ctx, t1):
        ctx.save_for_backward(t1)
        return t1.f.relu_map(t1)

    @staticmethod
    def backward(ctx, grad_output):
        (t1,) = ctx.saved_values
        return grad_output.f.relu_back_zip(t1, grad_output)


class Log(Function):
    @staticmethod
    def forward(ctx, t1):
        ctx.save_for_backward(t1)
        return t1.f.log_map(t1)

    @staticmethod
    def backward(ctx, grad_output):
        (t1,) = ctx.saved_values
        return grad_output.f.log_back_zip(t1, grad_output)


class Exp(Function):
    @staticmethod
    def forward(ctx, t1):
        out = t1.f.exp_map(t1)
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        (out,) = ctx.saved_values
        return grad_output.f.mul_zip(out, grad_output)


class Sum(Function):
    @staticmethod
    def forward(ctx, a, dim):
        ctx.save_for_backward(a.shape, dim)
        return a.f.add_reduce(a, int(dim.item()))

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output, 0.0


class All(Function):
    @staticmethod
    def forward(ctx, a, dim):
        if dim is not None:
            return a.f.mul_reduce(a, int(dim.item()))
        return a.f.mul_reduce(a.contiguous().view(int(operators.prod(a.shape))), 0)


class LT(Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a.shape, b.shape)
        return a.f.lt_zip(a, b)

    @staticmethod
    def backward(ctx, grad_output):
        a_shape, b_shape = ctx.saved_values
        return grad_output.zeros(a_shape), grad_output.zeros(b_shape)


class EQ(Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a.shape, b.shape)
        return a.f.eq_zip(a, b)

    @staticmethod
    def backward(ctx, grad_output):
        a_shape, b_shape = ctx.saved_values
        return grad_output.zeros(a_shape), grad_output.zeros(b_shape)


class IsClose(Function):
    @staticmethod
    def forward(ctx, a, b):
        return a.f.is_close_zip(a, b)


class Permute(Function):
    @staticmethod
    def forward(ctx, a, order):
        order_l = [int(order[i]) for i in range(order.size)]
        ctx.save_for_backward(order_l)
        return a._new(a._tensor.permute(*order_l))

    @staticmethod
    def backward(ctx, grad_output):
        (order_l,) = ctx.saved_values
        inv = [0] * len(order_l)
        for i, o in enumerate(order_l):
            inv[o] = i
        return grad_output._new(grad_output._tensor.permute(*inv)), 0.0


class SoftmaxXent(Function):
    """Per-row softmax cross-entropy, the reference's softmax_loss (minitorch/nn.py:
    logsumexp(logits, 1) - logits[target]) as one backend kernel each way; target (class
    ids) gets no gradient."""

    @staticmethod
    def forward(ctx, logits, target):
        loss, lse = logits.f.softmax_xent_fw(logits, target)
        ctx.save_for_backward(logits, target, lse)
        return loss

    @staticmethod
    def backward(ctx, grad_output):
        logits, target, lse = ctx.saved_values
        return logits.f.softmax_xent_bw(grad_output, logits, target, lse), 0.0


class BiasGelu(Function):
    """GELU_tanh(x + bias) for a 2-D x and a [cols] bias: FeedForward's linear_in bias add and
    GELU (reference modules_transfomer.py FeedForward, nn.py GELU) as one backend kernel each
    way; the bias gradient is the column sum of dx."""

    @staticmethod
    def forward(ctx, x, bias):
        ctx.save_for_backward(x, bias)
        return x.f.bias_gelu_fw(x, bias)

    @staticmethod
    def backward(ctx, grad_output):
        x, bias = ctx.saved_values
        dx = x.f.bias_gelu_bw(grad_output, x, bias)
        db = x.f.add_reduce(dx, 0)
        from .tensor import Tensor
        return dx, Tensor.make(db._tensor._storage, bias.shape, backend=db.backend)


class EmbeddingGather(Function):
    """Embedding lookup W[ids] as one backend kernel each way (the reference forms
    one_hot(ids, V) @ W, modules_basic.py Embedding): same values (a row of W is the one-hot
    product's exact result), dW the per-id sums of the output gradient; the ids get none."""

    @staticmethod
    def forward(ctx, ids, weight):
        ctx.save_for_backward(ids, weight.shape[0])
        return ids.f.embedding_fw(ids, weight)

    @staticmethod
    def backward(ctx, grad_output):
        ids, V = ctx.saved_values
        return 0.0, grad_output.f.embedding_bw(grad_output, ids, V)


class _DeviceSeed:
    """A dropout seed held in device memory (its address), for graph-captured steps."""
    __slots__ = ("ptr",)

    def __init__(self, ptr: int):
        self.ptr = ptr


class DropoutMask(Function):
    """Dropout with the keep mask drawn on the device from a seed (keep = u > p, then scaled by
    1 / (1 - p), reference modules_basic.py Dropout) in one kernel, and redrawn from the same
    seed in the backward; p is a host constant, the seed comes from NumPy's global generator
    (np.random.seed reproduces a run, as with rand())."""

    @staticmethod
    def forward(ctx, x, p):
        rate = float(p.item())
        scale = float(np.float32(1.0) / np.float32(1.0 - rate))
        from . import graphs
        g = graphs.capturing()
        if g is not None:
            # a captured step (graphs.StepGraph): the seed lives in a device slot that each
            # replay refills with this same draw, and the kernels read it from there
            seed = _DeviceSeed(g.seed_slot(lambda: int(np.random.randint(0, 2**63 - 1, dtype=np.int64))))
        else:
            seed = int(np.random.randint(0, 2**63 - 1, dtype=np.int64))
        ctx.save_for_backward(rate, scale, seed)
        return x.f.dropout_fw(x, rate, scale, seed)

    @staticmethod
    def backward(ctx, grad_output):
        rate, scale, seed = ctx.saved_values
        return grad_output.f.dropout_fw(grad_output, rate, scale, seed), 0.0


class View(Function):
    @staticmethod
    def forward(ctx, a, shape):
        ctx.save_for_backward(a.shape)
        if not a._tensor.is_dense():
            raise AssertionError("Must be contiguous to view")
        shape2 = [int(shape[i]) for i in range(shape.size)]
        return _Tensor.make(a._tensor._storage, tuple(shape2), backend=a.backend)

    @staticmethod
    def backward(ctx, grad_output):
        (original,) = ctx.saved_values
        g = grad_output if grad_output._tensor.is_dense() else grad_output.contiguous()
        return _Tensor.make(g._tensor._storage, original, backend=g.backend), 0.0


class Copy(Function):
    @staticmethod
    def forward(ctx, a):
        return a.f.id_map(a)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output


class MatMul(Function):
    @staticmethod
    def forward(ctx, t1, t2):
        ctx.save_for_backward(t1, t2)
        return t1.f.matrix_multiply(t1, t2)

    @staticmethod
    def backward(ctx, grad_output):
        t1, t2 = ctx.saved_values

        def transpose(a):
            order = list(range(a.dims))
            order[-2], order[-1] = order[-1], order[-2]
            return a._new(a._tensor.permute(*order))

        return (grad_output.f.matrix_multiply(grad_output, transpose(t2)),
                grad_output.f.matrix_multiply(transpose(t1), grad_output))


class Attn_Softmax(Function):  # noqa: N801 - reference name
    @staticmethod
    def forward(ctx, inp, mask):
        out = inp.f.attn_softmax_fw(inp, mask)
        ctx.save_for_backward(out, mask.shape)
        return out

    @staticmethod
    def backward(ctx, out_grad):
        out, mask_shape = ctx.saved_values
        dinp, _ = out_grad.f.attn_softmax_bw(out_grad, out)
        return dinp, out_grad.zeros(mask_shape)


class Attn_Softmax_NoMask(Function):  # noqa: N801
    """Row softmax without an additive mask; ``future`` (a host constant 0/1) masks
    col > row inside the kernel (the decoder self-attention case)."""

    @staticmethod
    def forward(ctx, inp, future):
        out = inp.f.attn_softmax_fw(inp, None, mask_future=bool(future.item()))
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, out_grad):
        (out,) = ctx.saved_values
        dinp, _ = out_grad.f.attn_softmax_bw(out_grad, out)
        return dinp, 0.0


class LayerNorm(Function):
    @staticmethod
    def forward(ctx, inp, gamma, beta):
        ln_res, var, means = inp.f.layernorm_fw(inp, gamma, beta)
        ctx.save_for_backward(inp, gamma, beta, var, means)
        return ln_res

    @staticmethod
    def backward(ctx, out_grad):
        inp, gamma, beta, var, means = ctx.saved_values
        return out_grad.f.layernorm_bw(out_grad, inp, gamma, beta, var, means)


def _kv_kw(kv):
    """The optional key-padding lengths (a [B] constant tensor) as the ops' keyword."""
    return {} if kv is None else {"kv_len": kv}


class FlashAttention(Function):
    """Reference tensor_functions.py:472-497. An optional 4th input is a constant [B]
    tensor of valid key counts (key padding, mt_flash_attn_*_varlen); it gets no gradient."""

    @staticmethod
    def forward(ctx, Q, K, V, kv=None):  # noqa: N803 - reference names
        O, m, l = Q.f.flash_attention_fw(Q, K, V, **_kv_kw(kv))
        ctx.save_for_backward(Q, K, V, O, m, l, kv)
        return O

    @staticmethod
    def backward(ctx, out_grad):
        Q, K, V, O, m, l, kv = ctx.saved_values
        g = out_grad.f.flash_attention_bw(Q, K, V, O, out_grad, m, l, **_kv_kw(kv))
        return g if kv is None else tuple(g) + (0.0,)


class FlashAttentionCausal(Function):
    """Reference tensor_functions.py:501-516; kv as in FlashAttention."""

    @staticmethod
    def forward(ctx, Q, K, V, kv=None):  # noqa: N803
        O, m, l = Q.f.flash_attention_causal_fw(Q, K, V, **_kv_kw(kv))
        ctx.save_for_backward(Q, K, V, O, m, l, kv)
        return O

    @staticmethod
    def backward(ctx, out_grad):
        Q, K, V, O, m, l, kv = ctx.saved_values
        g = out_grad.f.flash_attention_causal_bw(Q, K, V, O, out_grad, m, l, **_kv_kw(kv))
        return g if kv is None else tuple(g) + (0.0,)


# ---- constructors --------------------------------------------------------------------
def _backend_or_raise(backend):
    if backend is None:
        raise ValueError("a TensorBackend is required (e.g. TensorBackend(HipKernelOps))")
    return backend


def zeros(shape: UserShape, backend=None):
    from .tensor import Tensor
    backend = _backend_or_raise(backend)
    shape = tuple(int(s) for s in shape)
    if backend.cuda:
        import torch
        size = _prod(shape) if shape else 1
        st = torch.zeros(size, dtype=torch.float32, device="cuda")
        return Tensor(TensorData(st, shape), backend=backend)
    t = Tensor.make(np.zeros(int(np.prod(shape)) if shape else 1, dtype=datatype), shape, backend=backend)
    return t


def ones(shape: UserShape, backend=None):
    from .tensor import Tensor
    backend = _backend_or_raise(backend)
    shape = tuple(int(s) for s in shape)
    t = Tensor.make(np.ones(int(np.prod(shape)) if shape else 1, dtype=datatype), shape, backend=backend)
    t._type_(backend)
    return t


def rand(shape: UserShape, backend=None, requires_grad: bool = False):
    from .tensor import Tensor
    backend = _backend_or_raise(backend)
    if getattr(backend, "rand_uniform", None) is not None:
        # device draw; the seed comes from NumPy's global generator so np.random.seed()
        # still makes a run reproducible
        import torch
        from .tensor import Tensor
        size = int(np.prod(shape)) if shape else 1  # every element is drawn: no zero fill
        t = Tensor(TensorData(torch.empty(size, dtype=torch.float32, device="cuda"), tuple(shape)),
                   backend=backend)
        backend.rand_uniform(t, int(np.random.randint(0, 2**63 - 1, dtype=np.int64)))
        t.requires_grad_(requires_grad)
        return t
    vals = np.array([random.random() for _ in range(int(np.prod(shape)))], dtype=datatype)
    t = Tensor.make(vals, tuple(shape), backend=backend)
    t._type_(backend)
    t.requires_grad_(requires_grad)
    return t


def _tensor(ls, shape: UserShape, backend=None, requires_grad: bool = False):
    from .tensor import Tensor
    backend = _backend_or_raise(backend)
    t = Tensor.make(np.array(ls, dtype=datatype), tuple(shape), backend=backend)
    t._type_(backend)
    t.requires_grad_(requires_grad)
    return t


def tensor(ls: Any, backend=None, requires_grad: bool = False):
    arr = np.array(ls, dtype=datatype)
    shape = arr.shape if arr.shape else (1,)
    return _tensor(arr.reshape(-1).tolist(), shape, backend=backend, requires_grad=requires_grad)


def tensor_from_numpy(ls: np.ndarray, backend=None, requires_grad: bool = False):
    """Copy a NumPy array into a new tensor on ``backend`` (device-resident for HIP)."""
    from .tensor import Tensor
    backend = _backend_or_raise(backend)
    arr = np.ascontiguousarray(ls, dtype=datatype)
    shape = arr.shape if arr.shape else (1,)
    t = Tensor(TensorData(arr.reshape(-1).copy(), shape, strides_from_shape(shape)), backend=backend)
    t._type_(backend)
    t.requires_grad_(requires_grad)
    return t


def zeros_tensor_from_numpy(shape, backend=None):
    return zeros(shape, backend=backend)


def ones_tensor_from_numpy(shape, backend=None):
    return ones(shape, backend=backend)


# ---- gradient checking ------------------------------------------------------------------
def grad_central_difference(f: Any, *vals, arg: int = 0, epsilon: float = 1e-6, ind=None) -> float:
    x = vals[arg]
    up = np.zeros(x.shape, dtype=np.float64)
    up[ind] = epsilon
    vals1 = [x if j != arg else x + tensor_from_numpy(up, x.backend) for j, x in enumerate(vals)]
    vals2 = [x if j != arg else x - tensor_from_numpy(up, x.backend) for j, x in enumerate(vals)]
    delta = f(*vals1).sum() - f(*vals2).sum()
    return delta[0] / (2.0 * epsilon)


def grad_check(f: Any, *vals, tol: float = 1e-6) -> None:
    for x in vals:
        x.requires_grad_(True)
        x.zero_grad_()
    random.seed(10)
    out = f(*vals)
    out.sum().backward()
    for i, x in enumerate(vals):
        ind = x._tensor.sample()
        check = grad_central_difference(f, *vals, arg=i, ind=ind)
        assert x.grad is not None
        np.testing.assert_allclose(x.grad[ind], check, 1e-2, 1e-2)
