"""A NumPy ``TensorOps`` for the CPU-only tests -- TEST INFRASTRUCTURE ONLY.

It lets ``-m "not gpu"`` tests exercise the host-side minitorch machinery (Tensor,
autodiff, views/permutes, Module wiring, MultiHeadAttention plumbing) without a GPU.
It is never importable from the shipped package; the fused attention ops delegate to
the CPU oracle (``oracle/attention.py``), which only tests may use.
"""
from __future__ import annotations

import numpy as np

from minitorch import operators
from minitorch.tensor import Tensor
from minitorch.tensor_data import TensorData, shape_broadcast
from minitorch.tensor_ops import TensorOps
from oracle import attention as A

_NP = {
    operators.add: np.add, operators.mul: np.multiply, operators.id: lambda x: x,
    operators.neg: np.negative, operators.lt: lambda x, y: (x < y).astype(np.float32),
    operators.eq: lambda x, y: (x == y).astype(np.float32),
    operators.sigmoid: lambda x: 1.0 / (1.0 + np.exp(-x)),
    operators.relu: lambda x: np.maximum(x, 0), operators.relu_back: lambda x, d: np.where(x > 0, d, 0),
    operators.log: lambda x: np.log(x + operators.EPS), operators.log_back: lambda x, d: d / (x + operators.EPS),
    operators.exp: np.exp, operators.inv: lambda x: 1.0 / x,
    operators.inv_back: lambda x, d: -(1.0 / x ** 2) * d,
    operators.is_close: lambda x, y: (np.abs(x - y) < 1e-2).astype(np.float32),
    operators.max: np.maximum, operators.pow: np.power, operators.tanh: np.tanh,
}


def _arr(t: Tensor) -> np.ndarray:
    return t._tensor.to_numpy()


def _new(a: np.ndarray, backend) -> Tensor:
    a = np.ascontiguousarray(a, dtype=np.float32)
    return Tensor(TensorData(a.reshape(-1), a.shape), backend=backend)


class NumpyOps(TensorOps):
    cuda = False

    @staticmethod
    def map(fn):
        f = _NP[fn]

        def ret(a, out=None):
            r = np.broadcast_to(f(_arr(a)), out.shape if out is not None else a.shape)
            if out is None:
                return _new(r, a.backend)
            for idx in out._tensor.indices():
                out._tensor.set(idx, float(r[idx]))
            return out
        return ret

    @staticmethod
    def cmap(fn):
        return NumpyOps.map(fn)

    @staticmethod
    def zip(fn):
        f = _NP[fn]

        def ret(a, b):
            shape = shape_broadcast(a.shape, b.shape)
            return _new(np.broadcast_to(f(_arr(a), _arr(b)), shape), a.backend)
        return ret

    @staticmethod
    def reduce(fn, start=0.0):
        f = _NP[fn]

        def ret(a, dim):
            x = _arr(a)
            r = np.full(x.shape[:dim] + (1,) + x.shape[dim + 1:], start, np.float32)
            for j in range(x.shape[dim]):
                r = f(r, np.take(x, [j], axis=dim))
            return _new(r, a.backend)
        return ret

    @staticmethod
    def matrix_multiply(a, b):
        return _new(np.matmul(_arr(a).astype(np.float64), _arr(b).astype(np.float64)), a.backend)

    @staticmethod
    def attn_softmax_fw(inp, mask, mask_future=False):
        x = _arr(inp)
        if mask is not None:
            x = x + _arr(mask)
        if mask_future:
            T = x.shape[-1]
            x = np.where(np.triu(np.ones((x.shape[-2], T)), 1) > 0, -1e8, x)
        e = np.exp(x - x.max(-1, keepdims=True))
        return _new(e / (e.sum(-1, keepdims=True) + 1e-8), inp.backend)

    @staticmethod
    def attn_softmax_bw(out_grad, soft_inp):
        g, y = _arr(out_grad), _arr(soft_inp)
        return _new(y * (g - (g * y).sum(-1, keepdims=True)), out_grad.backend), soft_inp

    @staticmethod
    def layernorm_fw(inp, gamma, beta):
        x = _arr(inp).astype(np.float64)
        mean = x.mean(-1)
        var = (x * x).mean(-1) - mean ** 2 + 1e-8
        y = _arr(gamma) * (x - mean[:, None]) / np.sqrt(var[:, None]) + _arr(beta)
        b = inp.backend
        return _new(y, b), _new(var, b), _new(mean, b)

    @staticmethod
    def layernorm_bw(out_grad, inp, gamma, beta, var, mean):
        x, dy, g = (_arr(t).astype(np.float64) for t in (inp, out_grad, gamma))
        v, m = _arr(var).astype(np.float64), _arr(mean).astype(np.float64)
        rsd = 1 / np.sqrt(v)[:, None]
        xh = (x - m[:, None]) * rsd
        dyg = dy * g
        dx = (dyg - dyg.mean(-1, keepdims=True) - xh * (dyg * xh).mean(-1, keepdims=True)) * rsd
        b = inp.backend
        return _new(dx, b), _new((dy * xh).sum(0)[None], b), _new(dy.sum(0)[None], b)

    @staticmethod
    def _kv(kv_len):
        return None if kv_len is None else _arr(kv_len).reshape(-1).astype(np.int64)

    @staticmethod
    def _fw(Q, K, V, causal, kv_len=None):
        o, m, l = A.attention_fwd(_arr(Q), _arr(K), _arr(V), causal, NumpyOps._kv(kv_len))
        b = Q.backend
        return _new(o, b), _new(m, b), _new(l, b)

    @staticmethod
    def _bw(Q, K, V, O, dO, m, l, causal, kv_len=None):
        g = A.attention_bwd(_arr(Q), _arr(K), _arr(V), _arr(O), _arr(dO), _arr(m), _arr(l), causal,
                            NumpyOps._kv(kv_len))
        return tuple(_new(x, Q.backend) for x in g)

    @staticmethod
    def flash_attention_fw(Q, K, V, kv_len=None):
        return NumpyOps._fw(Q, K, V, False, kv_len)

    @staticmethod
    def flash_attention_bw(Q, K, V, O, dO, m, l, kv_len=None):
        return NumpyOps._bw(Q, K, V, O, dO, m, l, False, kv_len)

    @staticmethod
    def flash_attention_causal_fw(Q, K, V, kv_len=None):
        return NumpyOps._fw(Q, K, V, True, kv_len)

    @staticmethod
    def flash_attention_causal_bw(Q, K, V, O, dO, m, l, kv_len=None):
        return NumpyOps._bw(Q, K, V, O, dO, m, l, True, kv_len)
