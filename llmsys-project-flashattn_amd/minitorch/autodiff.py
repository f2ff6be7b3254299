"""Reverse-mode autodiff driver (reference ``minitorch/autodiff.py:93-195``).

``backpropagate`` walks the graph in reverse topological order and accumulates
derivatives per variable; leaf variables receive them through
``accumulate_derivative``. The traversal is iterative (no recursion limit on deep
graphs such as a multi-layer DecoderLM step).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Iterable, List, Tuple

from typing_extensions import Protocol


def central_difference(f: Any, *vals: Any, arg: int = 0, epsilon: float = 1e-6) -> Any:
    up = list(vals)
    dn = list(vals)
    up[arg] = up[arg] + epsilon
    dn[arg] = dn[arg] - epsilon
    return (f(*up) - f(*dn)) / (2.0 * epsilon)


class Variable(Protocol):
    def accumulate_derivative(self, x: Any) -> None: ...

    @property
    def unique_id(self) -> int: ...

    def is_leaf(self) -> bool: ...

    def is_constant(self) -> bool: ...

    @property
    def parents(self) -> Iterable["Variable"]: ...

    def chain_rule(self, d_output: Any) -> Iterable[Tuple["Variable", Any]]: ...


def topological_sort(variable: Variable) -> List[Variable]:
    """Variables reachable from ``variable``, each after every variable it feeds."""
    order: List[Variable] = []
    seen = set()
    stack = [(variable, False)]
    while stack:
        var, done = stack.pop()
        if done:
            order.append(var)
            continue
        if var.unique_id in seen or var.is_constant():
            continue
        seen.add(var.unique_id)
        stack.append((var, True))
        if not var.is_leaf():
            for p in var.parents:
                if p.unique_id not in seen and not p.is_constant():
                    stack.append((p, False))
    order.reverse()
    return order


def backpropagate(variable: Variable, deriv: Any) -> None:
    derivatives = {variable.unique_id: deriv}
    for var in topological_sort(variable):
        d = derivatives.pop(var.unique_id, None)
        if d is None:
            continue
        if var.is_leaf():
            var.accumulate_derivative(d)
            continue
        for parent, pd in var.chain_rule(d):
            if parent.is_constant():
                continue
            prev = derivatives.get(parent.unique_id)
            derivatives[parent.unique_id] = pd if prev is None else prev + pd


@dataclass
class Context:
    no_grad: bool = False
    saved_values: Tuple[Any, ...] = field(default_factory=tuple)

    def save_for_backward(self, *values: Any) -> None:
        if self.no_grad:
            return
        self.saved_values = values

    @property
    def saved_tensors(self) -> Tuple[Any, ...]:
        return self.saved_values
