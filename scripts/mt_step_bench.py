"""Config 5 timing: one DecoderLM training step (forward, backward, Adam) of the reference's
machine-translation setup (n_vocab 10000, n_embd 256, n_head 8, batch 128, seq 39;
reference project/run_machine_translation.py:397-407) on synthetic tokens, on the HIP
backend with fused LayerNorm + softmax and flash attention. Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import numpy as np
import torch

import minitorch

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
B, T, V, E, H = 128, 39, 10000, 256, 8
backend = minitorch.TensorBackend(minitorch.HipKernelOps)
rng = np.random.default_rng(0)
lm = minitorch.DecoderLM(n_vocab=V, n_embd=E, n_head=H, n_positions=40, p_dropout=0.1, backend=backend,
                         use_fused_kernel=True, use_flash_attention=True)
opt = minitorch.Adam(lm.parameters(), lr=1e-4)
x = minitorch.tensor_from_numpy(rng.integers(0, V, (B, T)).astype(np.float32), backend)
y = minitorch.tensor_from_numpy(rng.integers(0, V, (B * T,)).astype(np.float32), backend)


def step():
    opt.zero_grad()
    logits = lm(x)
    loss = minitorch.softmax_loss(logits.view(B * T, V), y).sum() / (B * T)
    loss.backward()
    opt.step()
    return loss


for _ in range(2):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    loss = step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
print(json.dumps({"config": "C5 DecoderLM step (B=128, T=39, E=256, H=8, V=10000, 4 layers)",
                  "ms_per_step": round(dt * 1e3, 2), "tokens_per_s": round(B * T / dt, 1),
                  "loss": float(loss.item())}))
