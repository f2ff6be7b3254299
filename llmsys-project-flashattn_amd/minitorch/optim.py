"""Optimizers (reference ``minitorch/optim.py``). The reference's Adam uses
``(1 - beta1)`` for the second moment (optim.py:70); this one uses ``(1 - beta2)``."""
from __future__ import annotations

import math
from typing import Sequence

from .module import Parameter


class Optimizer:
    def __init__(self, parameters: Sequence[Parameter]):
        self.parameters = parameters

    def zero_grad(self) -> None:
        for p in self.parameters:
            if p.value is not None and getattr(p.value, "grad", None) is not None:
                p.value.grad = None


class SGD(Optimizer):
    def __init__(self, parameters: Sequence[Parameter], lr: float = 1.0):
        super().__init__(parameters)
        self.lr = lr

    def step(self) -> None:
        for p in self.parameters:
            if p.value is not None and getattr(p.value, "grad", None) is not None:
                p.update(p.value.detach() - self.lr * p.value.grad)


class Adam(Optimizer):
    def __init__(self, parameters: Sequence[Parameter], lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8):
        super().__init__(parameters)
        self.lr, self.beta1, self.beta2, self.eps = lr, beta1, beta2, eps
        self._states = {id(p): {} for p in parameters}

    def step(self) -> None:
        for p in self.parameters:
            grad = getattr(p.value, "grad", None) if p.value is not None else None
            if grad is None:
                continue
            st = self._states[id(p)]
            if not st:
                st["step"] = 0
                st["exp_avg"] = grad.zeros()
                st["exp_avg_sq"] = grad.zeros()
            st["step"] += 1
            st["exp_avg"] = st["exp_avg"] * self.beta1 + grad * (1 - self.beta1)
            st["exp_avg_sq"] = st["exp_avg_sq"] * self.beta2 + (grad * grad) * (1 - self.beta2)
            bc1 = 1.0 - self.beta1 ** st["step"]
            bc2 = 1.0 - self.beta2 ** st["step"]
            step_size = self.lr * math.sqrt(bc2) / bc1
            denom = st["exp_avg_sq"] ** 0.5 + self.eps
            p.update(p.value.detach() - step_size * st["exp_avg"] / denom)
