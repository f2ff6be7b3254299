"""Basic modules (reference ``minitorch/modules_basic.py``): Embedding, Dropout, Linear,
LayerNorm1d and FusedLayerNorm (the HIP LayerNorm kernel). Fixes vs the reference:
LayerNorm1d applies its weights/bias (reference :194-198 drops them)."""
from __future__ import annotations

import numpy as np

from .module import Module, Parameter
from .nn import one_hot
from .tensor import Tensor
from .tensor_functions import rand, ones, tensor_from_numpy, zeros


class Embedding(Module):
    def __init__(self, num_embeddings: int, embedding_dim: int, backend):
        super().__init__()
        self.backend = backend
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.weights = Parameter(tensor_from_numpy(
            np.random.normal(0, 1, (num_embeddings, embedding_dim)), backend=backend, requires_grad=True))

    def forward(self, x: Tensor) -> Tensor:
        bs, seq_len = x.shape
        if getattr(x.backend, "embedding_fw", None) is not None:
            # the device backend gathers the rows (and sums dW per id) instead of the one-hot
            # product: the same values without the [tokens x V] one-hot matrix and its GEMMs
            from .tensor_functions import EmbeddingGather
            return EmbeddingGather.apply(x, self.weights.value)
        oh = one_hot(x, self.num_embeddings).view(bs * seq_len, self.num_embeddings)
        return (oh @ self.weights.value).view(bs, seq_len, self.embedding_dim)


class Dropout(Module):
    def __init__(self, p_dropout: float = 0.1):
        super().__init__()
        self.p_dropout = p_dropout

    def forward(self, x: Tensor) -> Tensor:
        if self.p_dropout == 0 or not self.training:
            return x
        # keep with probability 1 - p, scale by 1 / (1 - p) (reference modules_basic.py
        # Dropout, which draws the mask with np.random.binomial on the host); here the
        # uniform draw is on the device when the backend has one, and a backend with the fused
        # kernel draws, masks and scales in one pass each way (DropoutMask)
        if getattr(x.backend, "dropout_fw", None) is not None and x._tensor.on_device:
            from .tensor_functions import DropoutMask
            return DropoutMask.apply(x, x._const(self.p_dropout))
        keep = rand(x.shape, backend=x.backend) > self.p_dropout
        return (x * keep) / (1 - self.p_dropout)


class Linear(Module):
    def __init__(self, in_size: int, out_size: int, bias: bool, backend):
        super().__init__()
        bound = (1 / in_size) ** 0.5
        self.out_size = out_size
        self.weights = Parameter(tensor_from_numpy(
            np.random.uniform(-bound, bound, (in_size, out_size)), backend=backend, requires_grad=True))
        if bias:
            self.bias = Parameter(tensor_from_numpy(
                np.random.uniform(-bound, bound, (out_size,)), backend=backend, requires_grad=True))

    def forward(self, x: Tensor) -> Tensor:
        batch, in_size = x.shape
        out = x @ self.weights.value
        if self.bias is not None:
            out = out + self.bias.value
        return out


class LayerNorm1d(Module):
    def __init__(self, dim: int, eps: float, backend):
        super().__init__()
        self.dim = dim
        self.eps = eps
        self.weights = Parameter(ones((dim,), backend=backend))
        self.bias = Parameter(zeros((dim,), backend=backend))

    def forward(self, x: Tensor) -> Tensor:
        mean = x.mean(dim=1)
        var = x.var(dim=1)
        norm = (x - mean) / ((var + self.eps) ** 0.5)
        return norm * self.weights.value + self.bias.value


class FusedLayerNorm(Module):
    """LayerNorm on the fused HIP kernel (reference modules_basic.py:202-210)."""

    def __init__(self, n_embd: int, backend):
        super().__init__()
        self.n_embd = n_embd
        self.weights = Parameter(ones((n_embd,), backend=backend))
        self.bias = Parameter(zeros((n_embd,), backend=backend))

    @property
    def gamma(self) -> Tensor:
        return self.weights.value

    @property
    def beta(self) -> Tensor:
        return self.bias.value

    def forward(self, x: Tensor) -> Tensor:
        return x.layernorm(self.weights.value, self.bias.value)
