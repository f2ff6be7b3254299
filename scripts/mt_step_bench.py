"""Config 5 timing: one DecoderLM training step (forward, backward, Adam) of the reference's
machine-translation setup (n_vocab 10000, n_embd 256, n_head 8, batch 128, seq 39;
reference project/run_machine_translation.py:397-407) on the synthetic right-padded batch
and weighted loss of bench.py's C5 leg, on the HIP backend with fused LayerNorm + softmax
and flash attention. Prints one JSON line: the step time and its phases (forward, backward,
optimizer; each bracketed by a device sync, so the phases sum to more than the pipelined
step), and the op / launch counts per step.
usage: python scripts/mt_step_bench.py [steps] [--prof FILE]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# MT_PKG_ROOT: another copy of the package (A/B of host-side changes)
sys.path.insert(0, os.environ.get("MT_PKG_ROOT") or os.path.join(ROOT, "llmsys-project-flashattn_amd"))
import numpy as np
import torch

import minitorch
from bench import synthetic_mt_batch

args = [a for a in sys.argv[1:] if not a.startswith("--")]
steps = int(args[0]) if args else 5
prof = sys.argv[sys.argv.index("--prof") + 1] if "--prof" in sys.argv else None
B, T, V, E, H = 128, 39, 10000, 256, 8
backend = minitorch.TensorBackend(minitorch.HipKernelOps)
if os.environ.get("MT_GEMM") == "own":  # A/B: the library's own fp32 MFMA GEMM for every matmul
    from minitorch import _hip
    _hip.lib().mt_set_gemm_backend(1)
rng = np.random.default_rng(0)
lm = minitorch.DecoderLM(n_vocab=V, n_embd=E, n_head=H, n_positions=40, p_dropout=0.1, backend=backend,
                         use_fused_kernel=True, use_flash_attention=True)
opt = minitorch.Adam(lm.parameters(), lr=1e-4)
batch = synthetic_mt_batch(rng, B, T, V)
x = minitorch.tensor_from_numpy(batch["input_ids"], backend)
y = minitorch.tensor_from_numpy(batch["labels"].reshape(-1), backend)
w = minitorch.tensor_from_numpy(batch["label_token_weights"].reshape(-1), backend)
kv = batch["kv_len"]


def fwd():
    return (minitorch.softmax_loss(lm(x, kv_len=kv).view(B * T, V), y) * w).sum() / w.sum()


def step():
    opt.zero_grad()
    loss = fwd()
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

phase = {"fwd": 0.0, "bwd": 0.0, "opt": 0.0}
for _ in range(steps):
    opt.zero_grad()
    torch.cuda.synchronize()
    a = time.perf_counter()
    loss = fwd()
    torch.cuda.synchronize()
    b = time.perf_counter()
    loss.backward()
    torch.cuda.synchronize()
    c = time.perf_counter()
    opt.step()
    torch.cuda.synchronize()
    d = time.perf_counter()
    phase["fwd"] += b - a
    phase["bwd"] += c - b
    phase["opt"] += d - c
gc_ms = {}
import gc
for mode in ("freeze", "disable"):
    gc.collect()
    if mode == "freeze":
        gc.freeze()
    else:
        gc.disable()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    gc_ms[mode] = round((time.perf_counter() - t0) / steps * 1e3, 2)
gc.enable()
gc.unfreeze()
n_params = len(list(lm.parameters()))
out = {"config": "C5 DecoderLM step (B=128, T=39, E=256, H=8, V=10000, 4 layers), padded, weighted loss",
       "ms_per_step": round(dt * 1e3, 2), "tokens_per_s": round(B * T / dt, 1),
       "phase_ms": {k: round(v / steps * 1e3, 2) for k, v in phase.items()},
       "gc_variants_ms": gc_ms, "n_params": n_params, "loss": float(loss.item())}
if prof:
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pr.dump_stats(prof)
    with open(prof + ".txt", "w") as f:
        st = pstats.Stats(pr, stream=f)
        st.sort_stats("tottime").print_stats(45)
        st.sort_stats("cumulative").print_stats(45)
print(json.dumps(out))
