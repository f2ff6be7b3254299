"""Neural-network helpers (reference ``minitorch/nn.py``): max/softmax/logsoftmax,
dropout, GELU (tanh form), one_hot, logsumexp and the softmax cross-entropy loss.
``softmax`` is the unfused composition the reference's CPU attention uses
(``e = exp(x - max); e / sum(e)``, nn.py:104-123)."""
from __future__ import annotations

import math
from typing import Tuple

import numpy as np

from .autodiff import Context
from .tensor import Tensor
from .tensor_functions import Function, rand, tensor_from_numpy


class Max(Function):
    @staticmethod
    def forward(ctx: Context, input: Tensor, dim: Tensor) -> Tensor:  # noqa: A002
        out = input.f.max_reduce(input, int(dim.item()))
        ctx.save_for_backward(input, out)
        return out

    @staticmethod
    def backward(ctx: Context, grad_output: Tensor):
        input, out = ctx.saved_values  # noqa: A001
        return input.f.mul_zip(input.f.eq_zip(out, input), grad_output), 0.0


def max(input: Tensor, dim: int) -> Tensor:  # noqa: A001,A002
    return Max.apply(input, input._const(dim))


def argmax(input: Tensor, dim: int) -> Tensor:  # noqa: A002
    out = input.f.max_reduce(input, dim)
    return out == input


def softmax(input: Tensor, dim: int) -> Tensor:  # noqa: A002
    e = (input - Max.apply(input, input._const(dim))).exp()
    return e / e.sum(dim=dim)


def logsoftmax(input: Tensor, dim: int) -> Tensor:  # noqa: A002
    m = Max.apply(input, input._const(dim))
    return input - ((input - m).exp().sum(dim=dim).log() + m)


def dropout(input: Tensor, rate: float, ignore: bool = False) -> Tensor:  # noqa: A002
    if ignore or rate <= 0.0:
        return input
    r = rand(input.shape, backend=input.backend)
    return input * (r > rate)


def GELU(input: Tensor) -> Tensor:  # noqa: N802,A002 - reference name
    """tanh-approximated GELU (torch ``approximate='tanh'``)."""
    return 0.5 * input * (1 + (math.sqrt(2 / math.pi) * (input + 0.044715 * (input ** 3))).tanh())


_CLASS_IDS: dict = {}


def one_hot(input: Tensor, num_classes: int) -> Tensor:  # noqa: A002
    """(*) integer-valued indices -> (*, num_classes) one-hot rows.

    The reference builds ``np.eye(num_classes)[idx]`` on the host and copies it in
    (minitorch/nn.py:212-222): at config 5 (4992 rows x 10000 classes) that is 200 MB built
    and transferred per call, about half of a training step. Here it is one broadcast
    ``==`` of the indices against a cached 0..num_classes-1 row on the tensor's own
    backend (a device zip kernel on the HIP backend). Same values, same shape."""
    be = input.backend
    key = (num_classes, id(be))
    ids = _CLASS_IDS.get(key)
    if ids is None:
        ids = tensor_from_numpy(np.arange(num_classes, dtype=np.float32), backend=be)
        _CLASS_IDS[key] = ids
    shape = tuple(input.shape)
    return input.contiguous().view(*shape, 1) == ids.view(*([1] * len(shape)), num_classes)


def logsumexp(input: Tensor, dim: int) -> Tensor:  # noqa: A002
    m = max(input, dim=dim)
    return m + (input - m).exp().sum(dim=dim).log()


def softmax_loss(logits: Tensor, target: Tensor) -> Tensor:
    """Per-row cross-entropy logsumexp(logits) - logits[target] (reference minitorch/nn.py).
    A backend with a fused kernel (HipKernelOps.softmax_xent_fw / _bw) computes it in one pass
    each way; otherwise the reference's composition."""
    batch = logits.shape[0]
    be = logits.backend
    if getattr(be, "softmax_xent_fw", None) is not None and logits.dims == 2 and logits._tensor.on_device:
        from .tensor_functions import SoftmaxXent
        t = target if target._tensor.is_dense() else target.contiguous()
        return SoftmaxXent.apply(logits, t if t.dims == 1 else t.view(batch))
    picked = (logits * one_hot(target, logits.shape[1])).sum(dim=1)
    return (logsumexp(logits, dim=1) - picked).view(batch)
