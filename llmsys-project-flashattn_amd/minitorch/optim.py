"""Optimizers (reference ``minitorch/optim.py``). The reference's Adam uses
``(1 - beta1)`` for the second moment (optim.py:68); this one uses ``(1 - beta2)``.

On the HIP backend, Adam updates every parameter whose value, gradient and moments are
dense fp32 device buffers in one multi-tensor kernel (``mt_adam_step``): the same arithmetic
and order as the tensor-op form below, bit for bit (tests/test_optim_gpu.py), but in place:
the parameter's storage is updated (the tensor-op form gives ``p.value`` a new tensor) and
``p.value.grad`` is left as it is (neither path clears it; call ``zero_grad``). Anything else
takes the tensor-op form, which is also the CPU backend's path. Inside a graph capture
(``graphs.StepGraph``) the fused launch reads its step size from a device slot that every replay
refills after advancing the step counters (``mt_adam_step_dstep``)."""
from __future__ import annotations

import math
from typing import Sequence

from . import graphs as _graphs
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
        g = _graphs.capturing()
        fused = {}  # step count -> [(param, grad, state)]
        for p in self.parameters:
            grad = getattr(p.value, "grad", None) if p.value is not None else None
            if grad is None:
                continue
            st = self._states[id(p)]
            if not st:
                if g is not None:
                    raise RuntimeError("Adam: a parameter got its first gradient inside a graph capture; "
                                       "warm the step up eagerly first")
                st["step"] = 0
                st["exp_avg"] = grad.zeros()
                st["exp_avg_sq"] = grad.zeros()
            if _fusable(p.value, grad, st["exp_avg"], st["exp_avg_sq"]):
                # captured: each replay advances the counter (graphs.StepGraph slot below)
                fused.setdefault(st["step"] + 1, []).append((p, grad, st))
                if g is None:
                    st["step"] += 1
                continue
            if g is not None:
                raise RuntimeError("Adam: only the fused multi-tensor path (dense fp32 device buffers) "
                                   "can run inside a graph capture")
            st["step"] += 1
            st["exp_avg"] = st["exp_avg"] * self.beta1 + grad * (1 - self.beta1)
            st["exp_avg_sq"] = st["exp_avg_sq"] * self.beta2 + (grad * grad) * (1 - self.beta2)
            p.update(p.value.detach() - self._step_size(st["step"]) * st["exp_avg"] / (st["exp_avg_sq"] ** 0.5 + self.eps))
        for t, group in fused.items():
            from . import _hip
            step_ptr = None
            if g is not None:
                states = [st for _, _, st in group]

                def advance(states=states):
                    for st in states:
                        st["step"] += 1
                    return self._step_size(states[0]["step"])
                step_ptr = g.f32_slot(advance)
            _hip.adam_step([p.value._tensor.data_ptr() for p, _, _ in group],
                           [gr._tensor.data_ptr() for _, gr, _ in group],
                           [st["exp_avg"]._tensor.data_ptr() for _, _, st in group],
                           [st["exp_avg_sq"]._tensor.data_ptr() for _, _, st in group],
                           [p.value._tensor.size for p, _, _ in group],
                           self.beta1, self.beta2, self.eps, self._step_size(t), step_size_ptr=step_ptr)

    def _step_size(self, t: int) -> float:
        bc1 = 1.0 - self.beta1 ** t
        bc2 = 1.0 - self.beta2 ** t
        return self.lr * math.sqrt(bc2) / bc1


def _fusable(*ts) -> bool:
    """Dense fp32 device buffers of one size, each exactly its tensor (no view offset)."""
    n = ts[0]._tensor.size
    for t in ts:
        td = t._tensor
        if not td.on_device or td.size != n or not td.is_dense():
            return False
        st = td._storage
        if st.dtype.itemsize != 4 or not st.dtype.is_floating_point or st.numel() != n or st.storage_offset() != 0:
            return False
    return True
