"""Round 6: minitorch MultiHeadAttention (flash, the reference test's case) X.grad under the
fp32 split ring backward in X3 form (knob 0) and fp32-MFMA form (knob 65), each compared with
torch fp32 on the GPU (the test's comparison) and with torch float64 (a checker): the worst
|err| / (1e-5 + 1e-5 |ref|) and the max |err|.
usage: MT_DIAG=1 python scripts/probe_mha_x3.py"""
import copy, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llmsys-project-flashattn_amd"))
import numpy as np
import torch
import minitorch
from minitorch import _hip
_hip.use_library(os.path.join(os.path.dirname(_hip.LIB_PATH), "diag", "libminitorch_hip_diag.so"))
backend = minitorch.TensorBackend(minitorch.HipKernelOps)


def ratio(a, r):
    return float(np.max(np.abs(a - r) / (1e-5 + 1e-5 * np.abs(r)))), float(np.max(np.abs(a - r)))


CASES = [(2, 1024, 1024, 16, True), (2, 1024, 1024, 16, False), (4, 256, 512, 16, True), (2, 512, 512, 16, True)]
if os.environ.get("CASES"):  # e.g. CASES="2,4096,256,4,1;2,4096,256,4,0"
    CASES = [tuple(int(x) for x in c.split(",")) for c in os.environ["CASES"].split(";")]
for (bs, n, e, h, causal) in CASES:
    causal = bool(causal)
    np.random.seed(10)
    torch.manual_seed(10)
    data = np.random.rand(bs, n, e)
    layer_ = torch.nn.MultiheadAttention(e, h, 0.0, bias=False, batch_first=True, dtype=torch.float32, device="cuda")
    M = torch.triu(-float("inf") * torch.ones(n, n, device="cuda"), 1) if causal else None
    X_ = torch.tensor(data, dtype=torch.float32, requires_grad=True, device="cuda")
    layer_(X_, X_, X_, attn_mask=M, need_weights=False)[0].sum().backward()
    l64 = copy.deepcopy(layer_).double()
    X64 = torch.tensor(data, dtype=torch.float64, requires_grad=True, device="cuda")
    l64(X64, X64, X64, attn_mask=None if M is None else M.double(), need_weights=False)[0].sum().backward()
    lc = copy.deepcopy(layer_).cpu()
    Xc = torch.tensor(data, dtype=torch.float32, requires_grad=True)
    lc(Xc, Xc, Xc, attn_mask=None if M is None else M.cpu(), need_weights=False)[0].sum().backward()
    g32, g64 = X_.grad.cpu().numpy(), X64.grad.cpu().numpy()
    print(f"{(bs, n, e, h)} causal={causal}: torch fp32 (GPU) vs float64 {ratio(g32, g64)}, torch fp32 (CPU) "
          f"vs float64 {ratio(Xc.grad.numpy(), g64)}", flush=True)
    for kn in os.environ.get("KNOBS", "0,65").split(","):
        os.environ["MT_KNOB"] = kn
        layer = minitorch.MultiHeadAttention(e, h, causal, 0.0, bias=False, backend=backend,
                                             use_fused_kernel=False, use_flash_attention=True)
        w_qkv = layer_.in_proj_weight.detach().cpu().numpy().T.copy()
        for name, w in zip(("q_projection", "k_projection", "v_projection"), np.split(w_qkv, 3, -1)):
            getattr(layer, name).weights.value = minitorch.tensor_from_numpy(w.copy(), backend, True)
        layer.out_projection.weights.value = minitorch.tensor_from_numpy(
            layer_.out_proj.weight.detach().cpu().numpy().T.copy(), backend, True)
        X = minitorch.tensor_from_numpy(data, backend, True)
        layer(X).sum().backward()
        g = X.grad.to_numpy()
        print(f"   knob {kn}: vs torch fp32 GPU {ratio(g, g32)}  CPU {ratio(g, Xc.grad.numpy())}  vs float64 "
              f"{ratio(g, g64)}", flush=True)
    os.environ["MT_KNOB"] = "0"
