"""Config-5 step census (diagnostics): which C-ABI calls one DecoderLM training step makes,
grouped by entry point and operand layout, so the remaining strided copies / broadcasts can be
traced to the model code that issues them.
usage: python scripts/c5_op_census.py"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llmsys-project-flashattn_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

import minitorch
from minitorch import _hip
from bench import synthetic_mt_batch

B, T, V, E, H = 128, 39, 10000, 256, 8
backend = minitorch.TensorBackend(minitorch.HipKernelOps)
rng = np.random.default_rng(0)
lm = minitorch.DecoderLM(n_vocab=V, n_embd=E, n_head=H, n_positions=40, p_dropout=0.1, backend=backend,
                         use_fused_kernel=True, use_flash_attention=True)
opt = minitorch.Adam(lm.parameters(), lr=1e-4)
batch = synthetic_mt_batch(rng, B, T, V)
x = minitorch.tensor_from_numpy(batch["input_ids"], backend)
y = minitorch.tensor_from_numpy(batch["labels"].reshape(-1), backend)
w = minitorch.tensor_from_numpy(batch["label_token_weights"].reshape(-1), backend)
kv = batch["kv_len"]


def step():
    opt.zero_grad()
    loss = (minitorch.softmax_loss(lm(x, kv_len=kv).view(B * T, V), y) * w).sum() / w.sum()
    loss.backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()

lib = _hip.lib()
counts = collections.Counter()
where = {}


def wrap(name, describe):
    fn = getattr(lib, name)

    def w(*args):
        key = (name,) + describe(args)
        counts[key] += 1
        if key not in where:
            st = [f for f in traceback.extract_stack()[:-1] if "minitorch" in f.filename and "hip_kernel_ops" not in f.filename]
            where[key] = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-6:])
        return fn(*args)
    setattr(lib, name, w)


def arr(a, n):
    return tuple(a[i] for i in range(n))


wrap("mt_tensor_map", lambda a: (a[0], arr(a[2], a[4]), arr(a[3], a[4]), arr(a[7], a[8])))
wrap("mt_tensor_zip", lambda a: (a[0], arr(a[2], a[4]), arr(a[6], a[8]), arr(a[7], a[8]), arr(a[10], a[12]), arr(a[11], a[12])))
wrap("mt_tensor_reduce", lambda a: (a[0], arr(a[5], a[7]), arr(a[6], a[7]), a[8]))
wrap("mt_matmul_f32", lambda a: (a[3], a[4], a[5], a[6]))
# every other entry point: counted by name
for nm in sorted(n for n in dir(lib) if n.startswith("mt_")):
    if nm in ("mt_tensor_map", "mt_tensor_zip", "mt_tensor_reduce", "mt_matmul_f32") or "version" in nm \
            or "error" in nm or "workspace" in nm or "policy" in nm or "set_" in nm or not callable(getattr(lib, nm)):
        continue
    wrap(nm, lambda a: ())
# host-to-device copies of host-built tensors (each a synchronous copy on the stream)
from minitorch.tensor_data import TensorData
_to_cuda = TensorData.to_cuda_


def _counted_to_cuda(self):
    if not self.on_device:
        st = [f for f in traceback.extract_stack()[:-1] if "minitorch" in f.filename or "scripts" in f.filename]
        key = ("to_cuda_", tuple(self.shape))
        counts[key] += 1
        where.setdefault(key, " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-6:]))
    return _to_cuda(self)


TensorData.to_cuda_ = _counted_to_cuda
step()
torch.cuda.synchronize()
tot = sum(counts.values())
print(f"C-ABI calls in one step: {tot}")
for k, c in counts.most_common():
    print(f"{c:4d}  {k}  [{where[k]}]")
