"""One training step captured as one hipGraph and replayed (HIP backend).

minitorch's autodiff issues a training step as a few hundred small launches from Python (config
5, the reference's machine-translation step, project/run_machine_translation.py:195-237: ≈ 330
launches, ≈ 4 ms of GPU work behind ≈ 7.6 ms of host work). ``StepGraph`` runs the step a few
times eagerly (shapes, caches, the allocator and the optimizer state settle), captures one more
call of it on its own stream (``torch.cuda.graph``: every launch of the library goes to torch's
current stream, which the capture redirects), and afterwards replays the graph: one launch per
step, with the host free.

What varies between steps without being a tensor is produced on the host before each replay
and read by the kernels from device memory, so a replay computes what an eager call would:

* dropout seeds (``DropoutMask``): each call in the captured step owns a uint64 slot; a replay
  draws every slot from NumPy's global generator in the eager call order (``np.random.seed``
  reproduces a run as before) and the kernels read the seed from the slot (``mt_dropout_dseed``);
* Adam's bias-corrected step size (``Adam.step``, fused path only): a replay advances the step
  counters and writes lr·sqrt(1 − β₂ᵗ)/(1 − β₁ᵗ) as one fp32 (``mt_adam_step_dstep``).

The slots are copied host → device (pinned, asynchronous, on the replay stream) ahead of the
graph launch. Inputs are the tensors the step function closes over: to feed a new batch, copy it
into those tensors' storage (``StepGraph`` itself never reallocates them). The tensors the
captured call returned are the replay's outputs, overwritten by every replay.

Anything in the step that needs the host inside the step (a synchronising copy, ``.item()`` on
a device value, a host-side constant created for the first time) fails loudly during capture:
run it once more in the warm-up, or keep it out of the step."""
from __future__ import annotations

from typing import Any, Callable, List, Optional

import numpy as np

_CAPTURING: Optional["StepGraph"] = None


def capturing() -> Optional["StepGraph"]:
    """The StepGraph whose capture is running (None outside a capture)."""
    return _CAPTURING


def copy_into(t, array) -> None:
    """Copy host data into the device storage of a minitorch tensor in place (same element
    count), on torch's current stream: how a captured step's fixed inputs take the next batch
    before ``replay()``. (A pageable host-to-device copy: the host waits for it.)"""
    import torch
    src = torch.as_tensor(np.ascontiguousarray(array, dtype=np.float32).reshape(-1))
    dst = t._tensor._storage
    if not isinstance(dst, torch.Tensor) or dst.numel() != src.numel() or not t._tensor.is_dense():
        raise ValueError("copy_into needs a dense device tensor of the array's size")
    dst.copy_(src)


class StepGraph:
    """Capture ``step_fn`` (a no-argument callable: forward, backward, optimizer step) once
    and replay it. ``warmup`` eager calls run first, on the capture stream."""

    SEED_SLOTS = 4096
    F32_SLOTS = 1024
    RING = 4  # pinned host staging buffers in flight (the host may run RING replays ahead)

    def __init__(self, step_fn: Callable[[], Any], warmup: int = 3):
        import torch
        if warmup < 1:
            raise ValueError("StepGraph needs at least one eager warm-up call")
        self.fn = step_fn
        self.stream = torch.cuda.Stream()
        self._seed_fns: List[Callable[[], int]] = []
        self._f32_fns: List[Callable[[], float]] = []
        self._seed_dev = torch.zeros(self.SEED_SLOTS, dtype=torch.int64, device="cuda")
        self._f32_dev = torch.zeros(self.F32_SLOTS, dtype=torch.float32, device="cuda")
        self._host = [(torch.zeros(self.SEED_SLOTS, dtype=torch.int64).pin_memory(),
                       torch.zeros(self.F32_SLOTS, dtype=torch.float32).pin_memory(),
                       torch.cuda.Event()) for _ in range(self.RING)]
        self._ring = 0
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            for _ in range(warmup):
                step_fn()
        torch.cuda.current_stream().wait_stream(self.stream)
        self.graph = torch.cuda.CUDAGraph()
        global _CAPTURING
        _CAPTURING = self
        try:
            with torch.cuda.graph(self.graph, stream=self.stream):
                self.outputs = step_fn()
        finally:
            _CAPTURING = None
        self.replays = 0

    # ---- slots (called by the ops while the capture runs) ---------------------------------
    def seed_slot(self, draw: Callable[[], int]) -> int:
        """Device address of a fresh uint64 seed slot; ``draw()`` fills it before each replay."""
        i = len(self._seed_fns)
        if i >= self.SEED_SLOTS:
            raise RuntimeError(f"StepGraph: more than {self.SEED_SLOTS} seeded ops in one step")
        self._seed_fns.append(draw)
        return self._seed_dev.data_ptr() + 8 * i

    def f32_slot(self, produce: Callable[[], float]) -> int:
        """Device address of a fresh fp32 slot; ``produce()`` fills it before each replay."""
        i = len(self._f32_fns)
        if i >= self.F32_SLOTS:
            raise RuntimeError(f"StepGraph: more than {self.F32_SLOTS} per-step scalars in one step")
        self._f32_fns.append(produce)
        return self._f32_dev.data_ptr() + 4 * i

    # ---- replay ------------------------------------------------------------------------
    def replay(self) -> Any:
        """One step: the host-produced slots (in capture order), their copy to the device and
        the graph launch, all on torch's current stream. Returns the captured outputs."""
        import torch
        hs, hf, ev = self._host[self._ring]
        self._ring = (self._ring + 1) % self.RING
        ev.synchronize()  # the copy that last read this staging buffer has run
        ns, nf = len(self._seed_fns), len(self._f32_fns)
        if ns:
            # in capture order: NumPy's generator advances exactly as in the eager calls
            hs_np = hs.numpy()
            for i, f in enumerate(self._seed_fns):
                v = int(f()) & 0xFFFFFFFFFFFFFFFF
                hs_np[i] = v - (1 << 64) if v >> 63 else v  # the uint64's bits as int64
        if nf:
            hf_np = hf.numpy()
            for i, f in enumerate(self._f32_fns):
                hf_np[i] = np.float32(f())
        if ns:
            self._seed_dev[:ns].copy_(hs[:ns], non_blocking=True)
        if nf:
            self._f32_dev[:nf].copy_(hf[:nf], non_blocking=True)
        ev.record()
        self.graph.replay()
        self.replays += 1
        return self.outputs

    __call__ = replay
