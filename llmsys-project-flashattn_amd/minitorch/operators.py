"""Scalar operators of the minitorch surface (reference ``minitorch/operators.py``).

They name the elementwise functions a backend applies; ``HipKernelOps`` maps each one
to the device function id of ``libminitorch_hip.so`` (the reference's combine.cu ids),
so their identity matters more than their Python bodies. The bodies give the exact
scalar semantics the HIP kernels implement (e.g. ``log`` adds ``EPS``, ``is_close``
is a 1e-2 window) and are what the CPU test backend in ``tests/`` evaluates.
"""
from __future__ import annotations

import math
from typing import Callable, Iterable, List

EPS = 1e-6


def mul(x: float, y: float) -> float:
    return x * y


def id(x: float) -> float:  # noqa: A001 - reference name
    return x


def add(x: float, y: float) -> float:
    return x + y


def neg(x: float) -> float:
    return -x


def lt(x: float, y: float) -> float:
    return 1.0 if x < y else 0.0


def eq(x: float, y: float) -> float:
    return 1.0 if x == y else 0.0


def max(x: float, y: float) -> float:  # noqa: A001 - reference name
    return x if x > y else y


def is_close(x: float, y: float) -> float:
    return 1.0 if (x - y < 1e-2) and (y - x < 1e-2) else 0.0


def sigmoid(x: float) -> float:
    if x >= 0:
        return 1.0 / (1.0 + math.exp(-x))
    e = math.exp(x)
    return e / (1.0 + e)


def relu(x: float) -> float:
    return x if x > 0 else 0.0


def log(x: float) -> float:
    return math.log(x + EPS)


def exp(x: float) -> float:
    return math.exp(x)


def log_back(x: float, d: float) -> float:
    return d / (x + EPS)


def inv(x: float) -> float:
    return 1.0 / x


def inv_back(x: float, d: float) -> float:
    return -(1.0 / x ** 2) * d


def relu_back(x: float, d: float) -> float:
    return d if x > 0 else 0.0


def pow(x: float, y: float) -> float:  # noqa: A001 - reference name
    return x ** y


def tanh(x: float) -> float:
    return math.tanh(x)


# Higher-order helpers (list-level, kept for API completeness).
def map(fn: Callable[[float], float]) -> Callable[[Iterable[float]], List[float]]:  # noqa: A001
    return lambda ls: [fn(x) for x in ls]


def zipWith(fn: Callable[[float, float], float]):  # noqa: N802 - reference name
    return lambda a, b: [fn(x, y) for x, y in zip(a, b)]


def reduce(fn: Callable[[float, float], float], start: float):
    def _r(ls: Iterable[float]) -> float:
        acc = start
        for x in ls:
            acc = fn(acc, x)
        return acc
    return _r


def prod(ls: Iterable[float]) -> float:
    return reduce(mul, 1.0)(ls)


def sum(ls: Iterable[float]) -> float:  # noqa: A001 - reference name
    return reduce(add, 0.0)(ls)


# Device function ids of libminitorch_hip.so (reference src/combine.cu:12-29).
FN_IDS = {
    add: 1, mul: 2, id: 3, neg: 4, lt: 5, eq: 6, sigmoid: 7, relu: 8, relu_back: 9,
    log: 10, log_back: 11, exp: 12, inv: 13, inv_back: 14, is_close: 15, max: 16,
    pow: 17, tanh: 18,
}
