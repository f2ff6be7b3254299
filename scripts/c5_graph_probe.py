"""C5 DecoderLM training step (forward, backward, Adam; bench.py's c5 leg) eager against its
hipGraph replay (minitorch/graphs.py StepGraph: fresh dropout seeds and Adam step size per
replay). Prints one JSON line: eager and replay ms per step, capture time, launches per step.
usage: python scripts/c5_graph_probe.py [steps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llmsys-project-flashattn_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

import minitorch
from bench import synthetic_mt_batch

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
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
kv = batch["kv_len"]  # cached on the device by value (modules_transfomer._kv_tensor)


def step():
    opt.zero_grad()
    loss = (minitorch.softmax_loss(lm(x, kv_len=kv).view(B * T, V), y) * w).sum() / w.sum()
    loss.backward()
    opt.step()
    return loss


from minitorch.graphs import StepGraph

for _ in range(3):
    step()
torch.cuda.synchronize()
out = {}
t0 = time.perf_counter()
for _ in range(steps):
    step()
torch.cuda.synchronize()
out["eager_ms"] = round((time.perf_counter() - t0) / steps * 1e3, 3)
t0 = time.perf_counter()
try:
    g = StepGraph(step, warmup=2)
except Exception as e:  # noqa: BLE001
    import traceback
    traceback.print_exc()
    out["capture_error"] = repr(e)[:600]
    print(json.dumps(out))
    sys.exit(1)
out["capture_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
out["seed_slots"], out["f32_slots"] = len(g._seed_fns), len(g._f32_fns)
g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    loss = g.replay()
torch.cuda.synchronize()
out["replay_ms"] = round((time.perf_counter() - t0) / steps * 1e3, 3)
out["loss_after_replays"] = float(loss.to_numpy()[0])
print(json.dumps(out))
