"""Tensor storage + layout (reference ``minitorch/tensor_data.py:150-293``).

A ``TensorData`` is a flat fp32 storage plus (shape, strides) in elements. The storage
is either a host NumPy array or -- the MI355X path -- a 1-D ``torch.float32`` tensor
resident in HBM (PyTorch-ROCm is used only as the device allocator; the arithmetic on
it is done by ``libminitorch_hip.so``). ``to_cuda_`` moves a host storage to the device
once; nothing moves back implicitly (``to_numpy`` is an explicit copy).
"""
from __future__ import annotations

import functools
import random
from typing import Iterable, Optional, Sequence, Tuple, Union

import numpy as np

MAX_DIMS = 32

datatype = np.float32
Storage = Union[np.ndarray, "object"]  # np.ndarray (host) or torch.Tensor (device)
OutIndex = np.ndarray
Index = np.ndarray
Shape = np.ndarray
Strides = np.ndarray
UserIndex = Sequence[int]
UserShape = Sequence[int]
UserStrides = Sequence[int]


class IndexingError(RuntimeError):
    pass


def index_to_position(index: Index, strides: Strides) -> int:
    return int(sum(int(i) * int(s) for i, s in zip(index, strides)))


def to_index(ordinal: int, shape: Shape, out_index: OutIndex) -> None:
    cur = int(ordinal)
    for d in range(len(shape) - 1, -1, -1):
        out_index[d] = cur % int(shape[d])
        cur //= int(shape[d])


def broadcast_index(big_index: Index, big_shape: Shape, shape: Shape, out_index: OutIndex) -> None:
    off = len(big_shape) - len(shape)
    for d in range(len(shape)):
        out_index[d] = 0 if shape[d] == 1 else big_index[d + off]


@functools.lru_cache(maxsize=4096)
def _shape_broadcast(a: Tuple[int, ...], b: Tuple[int, ...]) -> Tuple[int, ...]:
    n = max(len(a), len(b))
    a = (1,) * (n - len(a)) + a
    b = (1,) * (n - len(b)) + b
    out = []
    for x, y in zip(a, b):
        if x != y and x != 1 and y != 1:
            raise IndexingError(f"Cannot broadcast {a} and {b}")
        out.append(max(x, y))
    return tuple(out)


def shape_broadcast(shape1: UserShape, shape2: UserShape) -> Tuple[int, ...]:
    # memoised on the int tuples: a model step broadcasts the same few shape pairs hundreds
    # of times (host time of the config-5 step)
    return _shape_broadcast(tuple(map(int, shape1)), tuple(map(int, shape2)))


@functools.lru_cache(maxsize=4096)
def _strides_from_shape(shape: Tuple[int, ...]) -> Tuple[int, ...]:
    out, acc = [], 1
    for s in reversed(shape):
        out.append(acc)
        acc *= s
    return tuple(reversed(out))


def strides_from_shape(shape: UserShape) -> Tuple[int, ...]:
    return _strides_from_shape(tuple(map(int, shape)))


@functools.lru_cache(maxsize=4096)
def _prod(shape: Tuple[int, ...]) -> int:
    size = 1
    for s in shape:
        size *= s
    return size


def _is_device(storage) -> bool:
    return not isinstance(storage, np.ndarray)


class TensorData:
    _storage: Storage

    def __init__(self, storage, shape: UserShape, strides: Optional[UserStrides] = None):
        if isinstance(storage, np.ndarray):
            self._storage = np.ascontiguousarray(storage, dtype=datatype).reshape(-1)
            self._on_dev = False
        elif isinstance(storage, (list, tuple)):
            self._storage = np.array(storage, dtype=datatype).reshape(-1)
            self._on_dev = False
        else:  # device storage (torch tensor)
            self._storage = storage
            self._on_dev = True
        shape = tuple(map(int, shape))
        strides = _strides_from_shape(shape) if strides is None else tuple(map(int, strides))
        if len(strides) != len(shape):
            raise IndexingError(f"Len of strides {strides} must match {shape}.")
        self.shape = shape
        self.strides = strides
        self.dims = len(shape)
        self.size = _prod(shape)

    # NumPy forms of shape / strides, built on first use and cached (shape and strides are
    # fixed at construction; the index helpers and the CPU backend take these forms); the
    # device path never needs them, and building two arrays per tensor was a measurable
    # share of minitorch's per-op host time in the config-5 step
    @functools.cached_property
    def _shape(self) -> np.ndarray:
        a = np.array(self.shape, dtype=np.int64)
        a.flags.writeable = False
        return a

    @functools.cached_property
    def _strides(self) -> np.ndarray:
        a = np.array(self.strides, dtype=np.int64)
        a.flags.writeable = False
        return a

    # ---- placement --------------------------------------------------------------
    @property
    def on_device(self) -> bool:
        # kept beside the storage (set where the storage is): this is asked thousands of
        # times per model step (host time of the config-5 step)
        return self._on_dev

    def to_cuda_(self) -> None:
        if not self._on_dev:
            import torch
            self._storage = torch.from_numpy(self._storage).to("cuda", non_blocking=False)
            self._on_dev = True

    def data_ptr(self) -> int:
        if not self.on_device:
            raise RuntimeError("host storage has no device pointer")
        return self._storage.data_ptr()

    def storage_numpy(self) -> np.ndarray:
        if self.on_device:
            return self._storage.detach().cpu().numpy()
        return self._storage

    def to_numpy(self) -> np.ndarray:
        flat = self.storage_numpy()
        if self.dims == 0:
            return flat[:1].copy()
        view = np.lib.stride_tricks.as_strided(
            flat, shape=self.shape, strides=tuple(s * flat.itemsize for s in self.strides))
        return np.array(view, dtype=datatype)

    # ---- layout -----------------------------------------------------------------
    def is_contiguous(self) -> bool:
        last = None
        for st in self.strides:
            if last is not None and st > last:
                return False
            last = st
        return True

    def is_dense(self) -> bool:
        """Row-major with no gaps (size-1 dims ignored)."""
        expect = 1
        for d in range(self.dims - 1, -1, -1):
            if self.shape[d] != 1 and self.strides[d] != expect:
                return False
            expect *= self.shape[d]
        return True

    @staticmethod
    def shape_broadcast(shape_a: UserShape, shape_b: UserShape) -> UserShape:
        return shape_broadcast(shape_a, shape_b)

    def index(self, index: Union[int, UserIndex]) -> int:
        if isinstance(index, (int, np.integer)):
            index = (int(index),)
        index = tuple(index)
        if len(index) != self.dims:
            raise IndexingError(f"Index {index} must be size of {self.shape}.")
        pos = 0
        for i, s, st in zip(index, self.shape, self.strides):
            i = int(i)
            if i >= s or i < 0:
                raise IndexingError(f"Index {index} out of range {self.shape}.")
            pos += i * st
        return pos

    def indices(self) -> Iterable[UserIndex]:
        lshape = self._shape
        out_index = np.zeros(self.dims, dtype=np.int64)
        for i in range(self.size):
            to_index(i, lshape, out_index)
            yield tuple(int(x) for x in out_index)

    def sample(self) -> UserIndex:
        return tuple(random.randint(0, s - 1) for s in self.shape)

    def get(self, key: UserIndex) -> float:
        pos = self.index(key)
        if self.on_device:
            return float(self._storage[pos].item())
        return float(self._storage[pos])

    def set(self, key: UserIndex, val: float) -> None:
        pos = self.index(key)
        self._storage[pos] = float(val)

    def tuple(self) -> Tuple[Storage, Shape, Strides]:
        return (self._storage, self._shape, self._strides)

    def permute(self, *order: int) -> "TensorData":
        if sorted(order) != list(range(self.dims)):
            raise IndexingError(f"Must give a position to each dimension. Shape: {self.shape} Order: {order}")
        return TensorData(self._storage, tuple(self.shape[o] for o in order),
                          tuple(self.strides[o] for o in order))

    def to_string(self) -> str:
        return np.array2string(self.to_numpy(), precision=5)
