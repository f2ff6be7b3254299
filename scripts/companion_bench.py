"""Achieved bandwidth of the companion kernels (fused attention softmax fw/bw, LayerNorm fw/bw,
csrc/softmax_layernorm.hip) through the C ABI, on the GPU box.

Algorithmic bytes per launch (fp32): softmax fw read inp + write out (+ the mask rows), bw read
dout + soft, write dinp; LayerNorm fw read x, write y (+ gamma, beta, mean, var), bw read dout
and x, write dx (+ gamma, beta, mean, var, dgamma, dbeta). Mean of 50 launches after 10 warm-up
launches, HIP events on the launch stream. Shapes: the C5 DecoderLM ones and larger ones that
leave the caches (MI355X: 4 MB L2 per XCD, 256 MB MALL).
usage: python scripts/companion_bench.py [out.json]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "llmsys-project-flashattn_amd"))
import ctypes  # noqa: E402

import torch  # noqa: E402

from minitorch import _hip  # noqa: E402

PEAK = 8.0e12  # HBM3E, MI355X_MICROARCH.md


def timed(fn, reps=50, warm=10):
    for _ in range(warm):
        fn()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    L = _hip.lib()
    s = _hip.stream_ptr()
    g = torch.Generator(device="cuda").manual_seed(0)
    rows_out = []

    def rec(kind, shape, nbytes, sec):
        r = {"kernel": kind, "shape": list(shape), "us": round(sec * 1e6, 2),
             "algorithmic_bytes": int(nbytes), "gbps": round(nbytes / sec / 1e9, 1),
             "frac_of_hbm_peak": round(nbytes / sec / PEAK, 3)}
        rows_out.append(r)
        print(json.dumps(r), flush=True)

    i64 = ctypes.c_int64 * 4
    for (B, nh, F, T, masked, fut) in ((128, 8, 39, 39, True, False), (128, 8, 39, 39, False, True),
                                       (8, 16, 1024, 1024, True, False), (8, 16, 1024, 1024, False, True),
                                       (4, 16, 2048, 2048, True, False)):
        x = torch.randn((B, nh, F, T), device="cuda", generator=g)
        out = torch.empty_like(x)
        mask = torch.zeros((B, T), device="cuda") if masked else None
        ms = i64(T, 0, 0, 1) if masked else None  # [B, to]: b stride T, broadcast over h, row
        mp = mask.data_ptr() if masked else None
        f = lambda: _hip.check(L.mt_attn_softmax_fw(out.data_ptr(), x.data_ptr(), mp, B, nh, F, T, ms,
                                                    int(fut), s), "softmax_fw")
        nbytes = 2 * x.numel() * 4 + (mask.numel() * 4 if masked else 0)
        rec("attn_softmax_fw" + ("_mask" if masked else "") + ("_future" if fut else ""), x.shape,
            nbytes, timed(f))
        dout = torch.randn_like(x)
        dinp = torch.empty_like(x)
        fb = lambda: _hip.check(L.mt_attn_softmax_bw(dinp.data_ptr(), dout.data_ptr(), out.data_ptr(),
                                                     B * nh * F, T, s), "softmax_bw")
        if not fut:
            rec("attn_softmax_bw", x.shape, 3 * x.numel() * 4, timed(fb))
        del x, out, dout, dinp, mask
    for (R, H) in ((4992, 256), (65536, 1024), (16384, 4096)):
        x = torch.randn((R, H), device="cuda", generator=g)
        gm, bt = torch.randn((H,), device="cuda", generator=g), torch.randn((H,), device="cuda", generator=g)
        y, var, mean = torch.empty_like(x), torch.empty((R,), device="cuda"), torch.empty((R,), device="cuda")
        f = lambda: _hip.check(L.mt_layernorm_fw(y.data_ptr(), var.data_ptr(), mean.data_ptr(), x.data_ptr(),
                                                 gm.data_ptr(), bt.data_ptr(), R, H, s), "layernorm_fw")
        rec("layernorm_fw", x.shape, 2 * x.numel() * 4 + 2 * H * 4 + 2 * R * 4, timed(f))
        dout = torch.randn_like(x)
        dx = torch.empty_like(x)
        dg, db = torch.empty((1, H), device="cuda"), torch.empty((1, H), device="cuda")
        ws = torch.empty(max(1, L.mt_layernorm_bw_workspace_bytes(R, H) // 4), device="cuda")
        fb = lambda: _hip.check(L.mt_layernorm_bw(dg.data_ptr(), db.data_ptr(), dx.data_ptr(), dout.data_ptr(),
                                                  x.data_ptr(), gm.data_ptr(), bt.data_ptr(), var.data_ptr(),
                                                  mean.data_ptr(), R, H, ws.data_ptr(), s), "layernorm_bw")
        rec("layernorm_bw", x.shape, 3 * x.numel() * 4 + 4 * H * 4 + 2 * R * 4, timed(fb))
        del x, y, dout, dx, ws
    if len(sys.argv) > 1:
        json.dump(rows_out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
