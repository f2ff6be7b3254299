"""Backend plugin API (reference ``minitorch/tensor_ops.py:22-105``).

An ops class (``TensorOps`` subclass) supplies higher-order ``map``/``zip``/``reduce``,
``matrix_multiply`` and the eight fused kernels; ``TensorBackend(ops)`` binds them to
the attribute table every ``Tensor`` dispatches through (``t.f``). The attribute names
are the reference's, so ``TensorBackend(HipKernelOps)`` is a drop-in for
``TensorBackend(CudaKernelOps)``.
"""
from __future__ import annotations

from typing import TYPE_CHECKING, Callable, Optional, Type

from typing_extensions import Protocol

from . import operators

if TYPE_CHECKING:
    from .tensor import Tensor


class MapProto(Protocol):
    def __call__(self, x: "Tensor", out: Optional["Tensor"] = ..., /) -> "Tensor": ...


class TensorOps:
    cuda = False

    @staticmethod
    def map(fn: Callable[[float], float]) -> MapProto:
        raise NotImplementedError

    @staticmethod
    def cmap(fn: Callable[[float], float]) -> Callable[["Tensor", "Tensor"], "Tensor"]:
        raise NotImplementedError

    @staticmethod
    def zip(fn: Callable[[float, float], float]) -> Callable[["Tensor", "Tensor"], "Tensor"]:
        raise NotImplementedError

    @staticmethod
    def reduce(fn: Callable[[float, float], float], start: float = 0.0) -> Callable[["Tensor", int], "Tensor"]:
        raise NotImplementedError

    @staticmethod
    def matrix_multiply(a: "Tensor", b: "Tensor") -> "Tensor":
        raise NotImplementedError

    # fused kernels (reference tensor_ops.py:96-104)
    @staticmethod
    def attn_softmax_fw(inp, mask, mask_future=False):
        raise NotImplementedError

    @staticmethod
    def attn_softmax_bw(out_grad, soft_inp):
        raise NotImplementedError

    @staticmethod
    def layernorm_fw(inp, gamma, beta):
        raise NotImplementedError

    @staticmethod
    def layernorm_bw(out_grad, inp, gamma, beta, var, mean):
        raise NotImplementedError

    @staticmethod
    def flash_attention_fw(Q, K, V):
        raise NotImplementedError

    @staticmethod
    def flash_attention_bw(Q, K, V, O, dO, m, l):
        raise NotImplementedError

    @staticmethod
    def flash_attention_causal_fw(Q, K, V):
        raise NotImplementedError

    @staticmethod
    def flash_attention_causal_bw(Q, K, V, O, dO, m, l):
        raise NotImplementedError


class TensorBackend:
    def __init__(self, ops: Type[TensorOps]):
        self.ops = ops
        # maps
        self.neg_map = ops.map(operators.neg)
        self.sigmoid_map = ops.map(operators.sigmoid)
        self.relu_map = ops.map(operators.relu)
        self.log_map = ops.map(operators.log)
        self.exp_map = ops.map(operators.exp)
        self.id_map = ops.map(operators.id)
        self.id_cmap = ops.cmap(operators.id)
        self.inv_map = ops.map(operators.inv)
        self.tanh_map = ops.map(operators.tanh)
        # zips
        self.add_zip = ops.zip(operators.add)
        self.mul_zip = ops.zip(operators.mul)
        self.lt_zip = ops.zip(operators.lt)
        self.eq_zip = ops.zip(operators.eq)
        self.is_close_zip = ops.zip(operators.is_close)
        self.relu_back_zip = ops.zip(operators.relu_back)
        self.log_back_zip = ops.zip(operators.log_back)
        self.inv_back_zip = ops.zip(operators.inv_back)
        self.pow_scalar_zip = ops.zip(operators.pow)
        # reduces
        self.add_reduce = ops.reduce(operators.add, 0.0)
        self.mul_reduce = ops.reduce(operators.mul, 1.0)
        self.max_reduce = ops.reduce(operators.max, -1e9)
        self.matrix_multiply = ops.matrix_multiply
        self.cuda = ops.cuda
        # optional device RNG (HipKernelOps.rand_uniform); None -> host draws
        self.rand_uniform = getattr(ops, "rand_uniform", None)
        # fused softmax cross-entropy (optional: a backend without it keeps the composition)
        self.softmax_xent_fw = getattr(ops, "softmax_xent_fw", None)
        self.softmax_xent_bw = getattr(ops, "softmax_xent_bw", None)
        # fused FeedForward pieces (optional: a backend without them keeps the compositions)
        self.bias_gelu_fw = getattr(ops, "bias_gelu_fw", None)
        self.bias_gelu_bw = getattr(ops, "bias_gelu_bw", None)
        self.dropout_fw = getattr(ops, "dropout_fw", None)
        self.embedding_fw = getattr(ops, "embedding_fw", None)
        self.embedding_bw = getattr(ops, "embedding_bw", None)
        # fused kernels
        self.attn_softmax_fw = ops.attn_softmax_fw
        self.attn_softmax_bw = ops.attn_softmax_bw
        self.layernorm_fw = ops.layernorm_fw
        self.layernorm_bw = ops.layernorm_bw
        self.flash_attention_fw = ops.flash_attention_fw
        self.flash_attention_bw = ops.flash_attention_bw
        self.flash_attention_causal_fw = ops.flash_attention_causal_fw
        self.flash_attention_causal_bw = ops.flash_attention_causal_bw
