"""Golden-vector generator -- TEST INFRASTRUCTURE, runs only in the survey/build container.

Produces ``tests/golden/attn_*.npz`` by running the *reference's own* minitorch CPU
attention (``FastOps`` + ``nn.softmax`` + autodiff) on seeded inputs, exactly the
composition ``MultiHeadAttention.self_attention`` uses on its non-flash branch
(reference ``minitorch/modules_transfomer.py:177-193``; causal mask
``-finfo(float32).max * triu(ones, 1)`` from ``:63-71``).

numba is not installed in this image, so a small stand-in package (``njit``/``jit``
-> identity decorator, ``prange`` -> ``range``, ``cuda.is_available()`` -> False)
is written to a temporary directory and put in front of the reference on
``sys.path``. The reference itself is only imported from ``/root/reference``; nothing
from it is copied into this repository -- only the numeric input/output arrays.

Caveats that shape the recipe (verified in this container):
* ``TensorBackend(FastOps)`` raises because FastOps lacks the 8 fused attributes
  read at reference ``tensor_ops.py:97-104`` -> copy them from ``SimpleOps``.
* ``FastOps.matrix_multiply`` is only correct for <=3-D tensors
  (``fast_ops.py:332-349``) -> flatten (B,H,N,d) to (B*H,N,d), as
  ``CudaKernelOps.matrix_multiply`` does (``cuda_kernel_ops.py:357-369``).
* The backward uses a RANDOM upstream gradient dO, never ``sum()`` (a ``sum()``
  upstream makes every dO row identical and hides dV errors).

Usage (from the repo root, in the build container only)::

    python oracle/gen_golden.py [case ...]   # writes tests/golden/attn_*.npz
"""
from __future__ import annotations

import os
import sys
import tempfile
import time

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")

_NUMBA_STANDIN = '''
import sys, types
def _deco(*a, **k):
    return a[0] if (len(a) == 1 and callable(a[0]) and not k) else (lambda f: f)
njit = jit = _deco
prange = range
float64 = float32 = float
int32 = int
class _Shared:
    @staticmethod
    def array(shape, dtype):
        import numpy as np
        return np.zeros(shape)
class _Cuda(types.ModuleType):
    def __init__(self):
        super().__init__("numba.cuda")
        self.shared = _Shared()
    def jit(self, *a, **k):
        return _deco(*a, **k)
    def is_available(self):
        return False
    def is_cuda_array(self, x):
        return False
    def to_device(self, x):
        return x
cuda = _Cuda()
sys.modules["numba.cuda"] = cuda
'''

# (name, B, H, N, d, causal, seed) -- C1 shape from BASELINE.json configs[0] plus a
# ragged N (tail handling: N not a multiple of any tile) and an odd head dim.
CASES = [
    ("c1", 1, 2, 128, 32, False, 0),
    ("c1_causal", 1, 2, 128, 32, True, 1),
    ("ragged", 1, 2, 100, 32, False, 2),
    ("ragged_causal", 1, 2, 100, 32, True, 3),
    ("odd_d_causal", 2, 1, 67, 20, True, 4),
]
# key padding: the reference's [B, to_len] additive mask (src/softmax_kernel.cu:26-33: 0 for
# tokens, -inf for padding) on the same composition; (name, B, H, N, d, causal, seed, kv_len)
VARLEN_CASES = [
    ("varlen", 2, 2, 96, 32, False, 5, (60, 96)),
    ("varlen_causal", 3, 1, 80, 32, True, 6, (33, 80, 1)),
]


def _import_reference():
    tmp = tempfile.mkdtemp(prefix="numba_standin_")
    os.makedirs(os.path.join(tmp, "numba"))
    with open(os.path.join(tmp, "numba", "__init__.py"), "w") as f:
        f.write(_NUMBA_STANDIN)
    sys.path[:0] = [tmp, REF]
    import minitorch  # noqa: E402  (the reference package)
    from minitorch.fast_ops import FastOps
    from minitorch.tensor_ops import SimpleOps

    class CPUOps(FastOps):
        pass

    for name in ("attn_softmax_fw", "attn_softmax_bw", "layernorm_fw", "layernorm_bw",
                 "flash_attention_fw", "flash_attention_bw",
                 "flash_attention_causal_fw", "flash_attention_causal_bw"):
        setattr(CPUOps, name, getattr(SimpleOps, name))
    return minitorch, minitorch.TensorBackend(CPUOps)


def run_case(mt, backend, B, H, N, d, causal, seed, kv_len=None):
    rng = np.random.default_rng(seed)
    q = rng.standard_normal((B, H, N, d)).astype(np.float32)
    k = rng.standard_normal((B, H, N, d)).astype(np.float32)
    v = rng.standard_normal((B, H, N, d)).astype(np.float32)
    do = rng.standard_normal((B, H, N, d)).astype(np.float32)
    BH = B * H
    Q = mt.tensor_from_numpy(q.reshape(BH, N, d), backend, True)
    K = mt.tensor_from_numpy(k.reshape(BH, N, d), backend, True)
    V = mt.tensor_from_numpy(v.reshape(BH, N, d), backend, True)
    kT = K.permute(0, 2, 1).contiguous()
    scores = (Q @ kT) / (d ** 0.5)
    if causal:
        mask = -np.finfo(np.float32).max * np.triu(np.ones((BH, N, N), dtype=np.float32), 1)
        scores = scores + mt.tensor_from_numpy(mask, backend, True)
    if kv_len is not None:  # [B, to_len] padding mask broadcast over heads and queries
        pad = np.where(np.arange(N)[None, :] < np.asarray(kv_len)[:, None], 0.0, -np.inf)
        pad = np.broadcast_to(pad[:, None, None, :], (B, H, N, N)).reshape(BH, N, N)
        scores = scores + mt.tensor_from_numpy(np.ascontiguousarray(pad, dtype=np.float32), backend, False)
    O = mt.softmax(scores, dim=2) @ V
    O.backward(mt.tensor_from_numpy(do.reshape(BH, N, d), backend, False))
    shp = (B, H, N, d)
    return dict(
        q=q, k=k, v=v, do=do,
        o=O.to_numpy().reshape(shp).astype(np.float32),
        dq=Q.grad.to_numpy().reshape(shp).astype(np.float32),
        dk=K.grad.to_numpy().reshape(shp).astype(np.float32),
        dv=V.grad.to_numpy().reshape(shp).astype(np.float32),
        causal=np.array(causal), B=np.array(B), H=np.array(H), N=np.array(N), d=np.array(d),
        **({} if kv_len is None else {"kv_len": np.asarray(kv_len, np.int32)}),
        source=np.array("reference minitorch FastOps+nn.softmax+autodiff (numba stand-in)"),
    )


def main():
    os.makedirs(OUT, exist_ok=True)
    mt, backend = _import_reference()
    only = set(sys.argv[1:])  # optional case names
    cases = [c + (None,) for c in CASES] + list(VARLEN_CASES)
    for name, B, H, N, d, causal, seed, kv_len in cases:
        if only and name not in only:
            continue
        t0 = time.time()
        arrays = run_case(mt, backend, B, H, N, d, causal, seed, kv_len)
        path = os.path.join(OUT, f"attn_{name}.npz")
        np.savez_compressed(path, **arrays)
        print(f"{name}: (B,H,N,d)=({B},{H},{N},{d}) causal={causal} -> {path} "
              f"[{time.time() - t0:.1f}s]")


if __name__ == "__main__":
    main()
