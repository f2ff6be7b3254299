"""``Tensor``: the user-facing autodiff tensor (reference ``minitorch/tensor.py``).

Same surface as the reference (operators, ``view``/``permute``/``contiguous``,
``backward``, and the fused entry points ``attn_softmax``, ``layernorm``,
``flash_attention``, ``flash_attention_causal`` at reference :424-436). Every op
dispatches through ``self.f`` (the ``TensorBackend``).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Any, Iterable, List, Optional, Sequence, Tuple, Type, Union

import numpy as np

from . import operators
from .autodiff import Context, Variable, backpropagate
from .tensor_data import TensorData, UserIndex, UserShape, datatype, shape_broadcast
from .tensor_functions import (
    EQ, LT, Add, All, Attn_Softmax, Attn_Softmax_NoMask, Copy, Exp, FlashAttention,
    FlashAttentionCausal, Inv, IsClose, LayerNorm, Log, MatMul, Mul, Neg, Permute,
    PowerScalar, ReLU, Sigmoid, Sum, Tanh, View, tensor_from_numpy,
)

TensorLike = Union[float, int, "Tensor"]


@dataclass
class History:
    last_fn: Optional[Type] = None
    ctx: Optional[Context] = None
    inputs: Sequence["Tensor"] = ()


_tensor_count = 0
_DEV_SCALARS: dict = {}  # (value, backend id) -> shared device constant (Tensor._ensure_tensor)


class Tensor:
    def __init__(self, v: TensorData, back: Optional[History] = None, name: Optional[str] = None,
                 backend=None):
        global _tensor_count
        _tensor_count += 1
        self.unique_id = _tensor_count
        assert isinstance(v, TensorData)
        assert backend is not None
        self._tensor = v
        self.history = back
        self.backend = backend
        self.grad: Optional[Tensor] = None
        self._name = name  # None: the unique id, formatted on first use (name)
        self.f = backend

    @property
    def name(self) -> str:
        return self._name if self._name is not None else str(self.unique_id)

    @name.setter
    def name(self, value: str) -> None:
        self._name = value

    # ---- grad flags ------------------------------------------------------------------
    def requires_grad_(self, x: bool) -> None:
        self.history = History() if x else None

    def requires_grad(self) -> bool:
        return self.history is not None

    # ---- properties ------------------------------------------------------------------
    def to_numpy(self) -> np.ndarray:
        return self._tensor.to_numpy()

    @property
    def shape(self) -> Tuple[int, ...]:
        return self._tensor.shape

    @property
    def size(self) -> int:
        return self._tensor.size

    @property
    def dims(self) -> int:
        return self._tensor.dims

    def _ensure_tensor(self, b: TensorLike) -> "Tensor":
        if isinstance(b, (int, float, np.floating, np.integer)):
            if self.backend.cuda:
                # one device-resident constant per value, filled once and then shared (no
                # host-to-device copy and no fill launch per scalar operand; no kernel writes
                # into an operand, and gradients are always fresh tensors or copies)
                # keyed on the fp32 bit pattern: -0.0 and 0.0 stay distinct, and a NaN
                # operand finds its cached constant like any other value
                key = (struct.pack("<f", float(b)), id(self.backend))
                c = _DEV_SCALARS.get(key)
                if c is None:
                    import torch
                    st = torch.full((1,), float(b), dtype=torch.float32, device="cuda")
                    c = Tensor(TensorData(st, (1,)), backend=self.backend)
                    # one made inside a graph capture is filled only when the graph runs: not
                    # shared with eager code
                    from .graphs import capturing
                    if len(_DEV_SCALARS) < 4096 and capturing() is None:
                        _DEV_SCALARS[key] = c
                return c
            return Tensor.make([float(b)], (1,), backend=self.backend)
        b._type_(self.backend)
        return b

    # ---- operators -------------------------------------------------------------------
    def __add__(self, b: TensorLike) -> "Tensor":
        return Add.apply(self, self._ensure_tensor(b))

    def __sub__(self, b: TensorLike) -> "Tensor":
        return Add.apply(self, -self._ensure_tensor(b))

    def __mul__(self, b: TensorLike) -> "Tensor":
        return Mul.apply(self, self._ensure_tensor(b))

    def __truediv__(self, b: TensorLike) -> "Tensor":
        return Mul.apply(self, Inv.apply(self._ensure_tensor(b)))

    def __rtruediv__(self, b: TensorLike) -> "Tensor":
        return Mul.apply(self._ensure_tensor(b), Inv.apply(self))

    def __matmul__(self, b: "Tensor") -> "Tensor":
        return MatMul.apply(self, b)

    def __lt__(self, b: TensorLike) -> "Tensor":
        return LT.apply(self, self._ensure_tensor(b))

    def __eq__(self, b: TensorLike) -> "Tensor":  # type: ignore[override]
        return EQ.apply(self, self._ensure_tensor(b))

    def __gt__(self, b: TensorLike) -> "Tensor":
        return LT.apply(self._ensure_tensor(b), self)

    def __neg__(self) -> "Tensor":
        return Neg.apply(self)

    def __radd__(self, b: TensorLike) -> "Tensor":
        return self + b

    def __rmul__(self, b: TensorLike) -> "Tensor":
        return self * b

    def __pow__(self, b: TensorLike) -> "Tensor":
        if isinstance(b, (int, float)):
            return PowerScalar.apply(self, self._ensure_tensor(b))
        if len(b.shape) == 1 and b.shape[0] == 1:
            return PowerScalar.apply(self, b)
        raise NotImplementedError("power with a non-scalar exponent")

    __hash__ = object.__hash__

    def _const(self, x: float) -> "Tensor":
        """A host-resident constant (shape/dim parameters that are never differentiated)."""
        return Tensor.make([float(x)], (1,), backend=self.backend, device=False)

    def all(self, dim: Optional[int] = None) -> "Tensor":
        if dim is None:
            return All.apply(self.contiguous().view(self.size), self._const(0))
        return All.apply(self, self._const(dim))

    def is_close(self, y: "Tensor") -> "Tensor":
        return IsClose.apply(self, y)

    def sigmoid(self) -> "Tensor":
        return Sigmoid.apply(self)

    def relu(self) -> "Tensor":
        return ReLU.apply(self)

    def log(self) -> "Tensor":
        return Log.apply(self)

    def exp(self) -> "Tensor":
        return Exp.apply(self)

    def tanh(self) -> "Tensor":
        return Tanh.apply(self)

    def item(self) -> float:
        assert self.size == 1
        return self._tensor.get((0,) * self.dims)

    def sum(self, dim: Optional[int] = None) -> "Tensor":
        if dim is None:
            return Sum.apply(self.contiguous().view(self.size), self._const(0))
        return Sum.apply(self, self._const(dim))

    def mean(self, dim: Optional[int] = None) -> "Tensor":
        if dim is not None:
            return self.sum(dim) / self.shape[dim]
        return self.sum() / self.size

    def var(self, dim: Optional[int] = None) -> "Tensor":
        if dim is not None:
            diff = self - self.mean(dim)
            return (diff * diff).sum(dim) / self.shape[dim]
        flat = self.contiguous().view(self.size)
        diff = flat - flat.mean(0)
        return (diff * diff).sum(0).view(1) / self.size

    def permute(self, *order: int) -> "Tensor":
        return Permute.apply(self, Tensor.make([float(o) for o in order], (len(order),),
                                               backend=self.backend, device=False))

    def view(self, *shape: int) -> "Tensor":
        return View.apply(self, Tensor.make([float(s) for s in shape], (len(shape),),
                                            backend=self.backend, device=False))

    def contiguous(self) -> "Tensor":
        # already row-major: the tensor itself (a copy would change nothing but cost a launch
        # and a buffer on the device backend)
        if self._tensor.is_dense():
            return self
        return Copy.apply(self)

    def __repr__(self) -> str:
        return self._tensor.to_string()

    def __getitem__(self, key: Union[int, UserIndex]) -> float:
        key2 = (key,) if isinstance(key, int) else key
        return self._tensor.get(key2)

    def __setitem__(self, key: Union[int, UserIndex], val: float) -> None:
        key2 = (key,) if isinstance(key, int) else key
        self._tensor.set(key2, val)

    # ---- internal ----------------------------------------------------------------------
    def _type_(self, backend) -> None:
        self.backend = backend
        self.f = backend
        if backend.cuda:
            self._tensor.to_cuda_()

    def _new(self, tensor_data: TensorData) -> "Tensor":
        return Tensor(tensor_data, backend=self.backend)

    @staticmethod
    def make(storage, shape: UserShape, strides=None, backend=None, device: Optional[bool] = None) -> "Tensor":
        t = Tensor(TensorData(storage, shape, strides), backend=backend)
        if device and not t._tensor.on_device:
            t._tensor.to_cuda_()
        return t

    def expand(self, other: "Tensor") -> "Tensor":
        """Reduce a broadcast gradient ``other`` back to this tensor's shape."""
        if self.shape == other.shape:
            return other
        true_shape = shape_broadcast(self.shape, other.shape)
        if self.shape == true_shape or other.shape != true_shape:
            buf = self.zeros(true_shape)
            self.backend.id_map(other, buf)
            if self.shape == true_shape:
                return buf
            out = buf
        else:  # the reductions below read `other` through its strides: no staging copy
            out = other
        orig_shape = [1] * (len(out.shape) - len(self.shape)) + list(self.shape)
        for dim, s in enumerate(out.shape):
            if orig_shape[dim] == 1 and s != 1:
                out = self.backend.add_reduce(out, dim)
        if out is other:  # no reduction ran (only leading size-1 dims differ)
            td = other._tensor
            if td.on_device and td.is_dense() and int(td._storage.numel()) == td.size:
                # the same values in this tensor's shape: a view (gradients are never updated in
                # place, see accumulate_derivative)
                return Tensor.make(td._storage, self.shape, backend=self.backend)
            out = self.backend.id_map(other)
        assert out.size == self.size, f"{out.shape} {self.shape}"
        return Tensor.make(out._tensor._storage, self.shape, backend=self.backend)

    def zeros(self, shape: Optional[UserShape] = None) -> "Tensor":
        from .tensor_functions import zeros
        return zeros(self.shape if shape is None else shape, backend=self.backend)

    def tuple(self):
        return self._tensor.tuple()

    def detach(self) -> "Tensor":
        return Tensor(self._tensor, backend=self.backend)

    # ---- autodiff ----------------------------------------------------------------------
    def accumulate_derivative(self, x: Any) -> None:
        assert self.is_leaf(), "Only leaf variables can have derivatives."
        if self.grad is None:
            # the first gradient is 0 + x without the zero fill and the add. A dense device
            # gradient that spans its whole storage is taken as it is (nothing updates a
            # gradient in place: the fused Adam reads it, the data-parallel all-reduce gives
            # .grad a new tensor, the next accumulation adds into a new one); anything else
            # (a strided view, host storage) is copied into a dense tensor of its own
            td = x._tensor
            if td.on_device and td.is_dense() and int(td._storage.numel()) == td.size:
                self.grad = Tensor(td, backend=self.backend)
            else:
                self.grad = Tensor(self.backend.id_map(x)._tensor, backend=self.backend)
            return
        self.grad = Tensor(self.backend.add_zip(self.grad, x)._tensor, backend=self.backend)

    def is_leaf(self) -> bool:
        return self.history is not None and self.history.last_fn is None

    def is_constant(self) -> bool:
        return self.history is None

    @property
    def parents(self) -> Iterable[Variable]:
        assert self.history is not None
        return self.history.inputs

    def chain_rule(self, d_output: Any) -> Iterable[Tuple[Variable, Any]]:
        h = self.history
        assert h is not None and h.last_fn is not None and h.ctx is not None
        x = h.last_fn._backward(h.ctx, d_output)
        assert len(x) == len(h.inputs), f"Bug in function {h.last_fn}"
        return [(inp, None if inp.is_constant() else inp.expand(self._ensure_tensor(d_in)))
                for inp, d_in in zip(h.inputs, x)]

    def backward(self, grad_output: Optional["Tensor"] = None) -> None:
        if grad_output is None:
            assert self.shape == (1,), "Must provide grad_output if non-scalar"
            # on the HIP backend the shared device constant 1.0: no host-to-device copy (a
            # pageable copy waits for the queued forward and cannot be captured in a graph)
            grad_output = (self._ensure_tensor(1.0) if self.backend.cuda else
                           Tensor.make([1.0], (1,), backend=self.backend))
        backpropagate(self, grad_output)

    def zero_grad_(self) -> None:
        self.grad = None

    # ---- fused kernels (reference tensor.py:424-436) -------------------------------------
    def attn_softmax(self, mask: Optional["Tensor"] = None, mask_future: bool = False) -> "Tensor":
        if mask is None:
            return Attn_Softmax_NoMask.apply(self, self._const(1.0 if mask_future else 0.0))
        if mask_future:
            raise NotImplementedError("pass either an additive mask or mask_future")
        return Attn_Softmax.apply(self, mask)

    def layernorm(self, gamma: "Tensor", beta: "Tensor") -> "Tensor":
        return LayerNorm.apply(self, gamma, beta)

    def flash_attention(self, K: "Tensor", V: "Tensor", kv_len: Optional["Tensor"] = None) -> "Tensor":  # noqa: N803
        """kv_len: optional constant [B] tensor of valid key counts (key padding)."""
        if kv_len is None:
            return FlashAttention.apply(self, K, V)
        return FlashAttention.apply(self, K, V, kv_len)

    def flash_attention_causal(self, K: "Tensor", V: "Tensor", kv_len: Optional["Tensor"] = None) -> "Tensor":  # noqa: N803
        if kv_len is None:
            return FlashAttentionCausal.apply(self, K, V)
        return FlashAttentionCausal.apply(self, K, V, kv_len)
