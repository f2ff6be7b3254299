"""ctypes binding of ``libminitorch_hip.so`` (C ABI declared in ``include/minitorch_hip.h``).

This is the MI355X counterpart of the reference's ctypes loading block
(reference ``minitorch/cuda_kernel_ops.py:25-29``): one library, located next to
this file rather than relative to the CWD, with every ``argtypes`` declared once.
There is no fallback: if the library is missing the first call raises.

Device buffers are torch tensors (PyTorch-ROCm is used for memory, streams and
``torch.distributed`` only); every computation goes through the HIP kernels.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
# MT_HIP_LIB: another build of the library (diagnostics: _lib/diag/libminitorch_hip_diag.so,
# `make DIAG=1`, which adds the A/B kernel policies) for tests and scripts; the package
# default is the product library
LIB_PATH = os.environ.get("MT_HIP_LIB") or os.path.join(_HERE, "_lib", "libminitorch_hip.so")

MT_F32 = 0
MT_BF16 = 1

_lib = None

_i64 = ctypes.c_int64
_int = ctypes.c_int
_vp = ctypes.c_void_p
_fp = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_int64)
_ip = ctypes.POINTER(ctypes.c_int)
_vpp = ctypes.POINTER(ctypes.c_void_p)

# name -> (restype, argtypes); mirrors include/minitorch_hip.h
_PROTOS = {
    "mt_last_error": (ctypes.c_char_p, []),
    "mt_abi_version": (_int, []),
    "mt_flash_set_kernel_policy": (_int, [_int]),
    "mt_flash_get_kernel_policy": (_int, []),
    "mt_scratch_bytes": (_i64, []),
    "mt_scratch_release": (_int, []),
    "mt_flash_attn_fwd": (_int, [_int, _int, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64,
                                 _i64p, _i64p, _i64p, _i64p, _vp]),
    "mt_flash_attn_fwd_varlen": (_int, [_int, _int, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64,
                                        _i64, _i64p, _i64p, _i64p, _i64p, _vp, _vp]),
    "mt_flash_attn_bwd_workspace_bytes": (_i64, [_i64, _i64, _i64, _i64]),
    "mt_flash_attn_bwd": (_int, [_int, _int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                 _i64, _i64, _i64, _i64, _i64p, _vp, _vp]),
    "mt_flash_attn_bwd_varlen": (_int, [_int, _int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                        _i64, _i64, _i64, _i64, _i64p, _vp, _vp, _vp]),
    "mt_flash_attn_bwd_v3": (_int, [_int, _int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                    _i64, _i64, _i64, _i64, _i64p, _vp, _vp, _i64, _vp]),
    "mt_attn_softmax_fw": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64p, _int, _vp]),
    "mt_attn_softmax_bw": (_int, [_vp, _vp, _vp, _i64, _i64, _vp]),
    "mt_layernorm_fw": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp]),
    "mt_bias_gelu_fw": (_int, [_vp, _vp, _vp, _i64, _i64, _vp]),
    "mt_bias_gelu_bw": (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _vp]),
    "mt_dropout": (_int, [_vp, _vp, _i64, ctypes.c_float, ctypes.c_float, ctypes.c_uint64, _vp]),
    "mt_dropout_dseed": (_int, [_vp, _vp, _i64, ctypes.c_float, ctypes.c_float, _vp, _vp]),
    "mt_embedding_fw": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _vp]),
    "mt_embedding_bw": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _vp]),
    "mt_softmax_xent_fw": (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _vp]),
    "mt_softmax_xent_bw": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp]),
    "mt_layernorm_bw_workspace_bytes": (_i64, [_i64, _i64]),
    "mt_layernorm_bw": (_int, [_vp] * 9 + [_i64, _i64, _vp, _vp]),
    "mt_tensor_map": (_int, [_int, _vp, _i64p, _i64p, _int, _vp, _i64p, _i64p, _int, _vp]),
    "mt_tensor_zip": (_int, [_int, _vp, _i64p, _i64p, _int, _vp, _i64p, _i64p, _int,
                             _vp, _i64p, _i64p, _int, _vp]),
    "mt_tensor_reduce": (_int, [_int, _vp, _i64p, _i64p, _vp, _i64p, _i64p, _int, _int,
                                ctypes.c_float, _vp]),
    "mt_matmul_f32": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64p, _i64p, _i64p, _vp]),
    "mt_rand_uniform": (_int, [_vp, _i64, ctypes.c_uint64, _vp]),
    "mt_adam_step": (_int, [_int, _vpp, _vpp, _vpp, _vpp, _i64p, ctypes.c_double, ctypes.c_double,
                            ctypes.c_double, ctypes.c_double, _vp]),
    "mt_adam_step_dstep": (_int, [_int, _vpp, _vpp, _vpp, _vpp, _i64p, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_double, _vp, _vp]),
    "mt_set_gemm_backend": (None, [_int]),
    "launch_attn_softmax": (None, [_fp, _fp, _int, _int, _int, _int, ctypes.c_bool, _vp]),
    "launch_attn_softmax_bw": (None, [_fp, _fp, _int, _int, _vp]),
    "launch_layernorm": (None, [_fp] * 6 + [_int, _int, _vp]),
    "launch_layernorm_bw": (None, [_fp] * 9 + [_int, _int, _vp, _vp]),
    "tensorMap": (None, [_fp, _ip, _ip, _int, _fp, _ip, _ip, _int, _int, _int]),
    "tensorZip": (None, [_fp, _ip, _ip, _int, _int, _fp, _ip, _ip, _int, _int,
                         _fp, _ip, _ip, _int, _int, _int]),
    "tensorReduce": (None, [_fp, _ip, _ip, _int, _fp, _ip, _ip, _int, ctypes.c_float, _int, _int]),
    "MatrixMultiply": (None, [_fp, _ip, _ip, _fp, _ip, _ip, _fp, _ip, _ip, _int, _int, _int]),
    "launch_flashattention_forward": (None, [_fp] * 6 + [_int] * 4),
    "launch_flashattention_backward": (None, [_fp] * 10 + [_int] * 4),
    "launch_flashattention_forward_causal": (None, [_fp] * 6 + [_int] * 4),
    "launch_flashattention_backward_causal": (None, [_fp] * 10 + [_int] * 4),
}


def lib() -> ctypes.CDLL:
    """Load the HIP library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `make -C {os.path.dirname(_HERE)}` "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        # One HIP runtime per process: torch's. Device buffers and streams are torch's, and
        # loaded first the library would bind /opt/rocm's libamdhip64 beside torch's bundled
        # one, which on some boxes then reports "no ROCm-capable device" for every call
        # (scripts/probe_runtime.py). With torch imported first, the library's libamdhip64
        # dependency resolves (by soname) to the runtime torch already mapped.
        try:
            import torch  # noqa: F401
        except ImportError:  # plain C-ABI use without torch: the library's own runtime
            pass
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _PROTOS.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
        _bind_fast(l)
    return _lib


fast = None  # the _mtfast extension bound to the loaded library (None: the ops use ctypes)


def _bind_fast(l: ctypes.CDLL) -> None:
    """Hand the generic entry points' addresses of the loaded library to the _mtfast CPython
    extension (csrc/mtfast.c: tuples in, no ctypes marshalling), when it was built."""
    global fast
    try:
        from . import _mtfast
    except ImportError:
        fast = None
        return
    addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
    _mtfast.bind(addr(l.mt_tensor_map), addr(l.mt_tensor_zip), addr(l.mt_tensor_reduce), addr(l.mt_matmul_f32))
    fast = _mtfast


def use_library(path: str) -> ctypes.CDLL:
    """Load a different build of the library (diagnostics only: scripts/ablate*.py load
    ``_lib/diag/libminitorch_hip_diag.so``, built by ``make DIAG=1``). The package itself
    always loads LIB_PATH."""
    global _lib, LIB_PATH
    if _lib is not None:
        raise RuntimeError("use_library() must run before the first lib() call")
    LIB_PATH = path
    return lib()


def set_policy(policy: int) -> None:
    """Select a kernel policy for A/B timing (mt_flash_set_kernel_policy; raises for an
    id the library rejects)."""
    check(lib().mt_flash_set_kernel_policy(int(policy)), "mt_flash_set_kernel_policy")


class policy:
    """``with _hip.policy(p): ...`` runs the block under kernel policy p, then restores
    the previous one."""

    def __init__(self, p: int):
        self.p = int(p)

    def __enter__(self):
        self.prev = lib().mt_flash_get_kernel_policy()
        set_policy(self.p)
        return self

    def __exit__(self, *exc):
        set_policy(self.prev)
        return False


def register(name: str, restype, argtypes) -> None:
    """Declare an additional export (used by the companion-kernel modules)."""
    _PROTOS[name] = (restype, argtypes)
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.restype = restype
        fn.argtypes = argtypes


def check(status: int, what: str) -> None:
    if status != 0:
        msg = lib().mt_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed: {msg}")


# ---- torch plumbing -------------------------------------------------------------
def _torch():
    import torch
    return torch


def stream_ptr(device=None) -> int:
    """The current torch stream of `device` (default: the current device) as a raw
    hipStream_t. Uses the raw-stream accessor when present (no Stream object per call)."""
    torch = _torch()
    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if raw is not None and (device is None or isinstance(device, int)):
        return raw(torch.cuda.current_device() if device is None else device)
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(t) -> int:
    torch = _torch()
    if t.dtype == torch.float32:
        return MT_F32
    if t.dtype == torch.bfloat16:
        return MT_BF16
    raise TypeError(f"unsupported dtype {t.dtype} (float32 or bfloat16)")


def strides3(t) -> ctypes.Array:
    """(batch, head, seq) element strides of a [B, H, N, d] tensor with unit-stride d."""
    if t.dim() != 4:
        raise ValueError(f"expected a 4-D [B,H,N,d] tensor, got shape {tuple(t.shape)}")
    if t.stride(3) != 1 and t.shape[3] != 1:
        raise ValueError("the head dimension must be unit-stride")
    return (ctypes.c_int64 * 3)(t.stride(0), t.stride(1), t.stride(2))


def _check_dev(*ts) -> None:
    for t in ts:
        if not t.is_cuda:
            raise ValueError("HIP flash attention needs device (cuda) tensors")


def _kv_arg(kv_len, B, device):
    """kv_len as the C ABI takes it: a device int32 [B] (None stays None)."""
    if kv_len is None:
        return None
    torch = _torch()
    kv = torch.as_tensor(kv_len, device=device).to(torch.int32).contiguous()
    if kv.shape != (B,):
        raise ValueError(f"kv_len must have shape ({B},), got {tuple(kv.shape)}")
    return kv


def flash_fwd(q, k, v, causal: bool = False, out=None, m=None, l=None, stream: Optional[int] = None,
              kv_len=None, out_dtype=None):
    """Device-pointer forward on torch tensors [B,H,N,d] (fp32 or bf16, any strides
    with unit-stride d). Returns (O, m, l); O has q's dtype, m/l are fp32 [B,H,N].
    kv_len: optional [B] valid-key counts (key padding: keys >= kv_len[b] are masked,
    mt_flash_attn_fwd_varlen). out_dtype=torch.float32 with bf16 inputs (or an fp32 `out`):
    the bf16 kernels write O in fp32, without its final bf16 rounding (MT_BF16_F32OUT)."""
    torch = _torch()
    _check_dev(q, k, v)
    B, H, N, d = q.shape
    if k.shape != q.shape or v.shape != q.shape:
        raise ValueError(f"q/k/v shapes differ: {tuple(q.shape)} {tuple(k.shape)} {tuple(v.shape)}")
    if not (q.dtype == k.dtype == v.dtype):
        raise TypeError("q/k/v dtypes differ")
    code = dtype_code(q)
    f32o = q.dtype == torch.bfloat16 and (out_dtype == torch.float32 or
                                          (out is not None and out.dtype == torch.float32))
    if out is None:
        out = torch.empty_like(q, dtype=torch.float32 if f32o else q.dtype,
                               memory_format=torch.contiguous_format)
    if f32o:
        code = 2  # MT_BF16_F32OUT
    if m is None:
        m = torch.empty((B, H, N), dtype=torch.float32, device=q.device)
    if l is None:
        l = torch.empty((B, H, N), dtype=torch.float32, device=q.device)
    st = stream_ptr(q.device) if stream is None else stream
    kv = _kv_arg(kv_len, B, q.device)
    if kv is None:
        check(lib().mt_flash_attn_fwd(code, int(causal), q.data_ptr(), k.data_ptr(),
                                      v.data_ptr(), out.data_ptr(), m.data_ptr(), l.data_ptr(),
                                      B, H, N, d, strides3(q), strides3(k), strides3(v),
                                      strides3(out), st), "mt_flash_attn_fwd")
    else:
        check(lib().mt_flash_attn_fwd_varlen(code, int(causal), q.data_ptr(), k.data_ptr(),
                                             v.data_ptr(), out.data_ptr(), m.data_ptr(), l.data_ptr(),
                                             B, H, N, d, strides3(q), strides3(k), strides3(v),
                                             strides3(out), kv.data_ptr(), st),
              "mt_flash_attn_fwd_varlen")
    return out, m, l


def flash_bwd(q, k, v, o, do, m, l, causal: bool = False, dq=None, dk=None, dv=None,
              workspace=None, stream: Optional[int] = None, kv_len=None):
    """Device-pointer backward. Returns (dQ, dK, dV) in q's dtype. kv_len: as flash_fwd."""
    torch = _torch()
    _check_dev(q, k, v, o, do, m, l)
    B, H, N, d = q.shape
    dq = torch.empty_like(q, memory_format=torch.contiguous_format) if dq is None else dq
    dk = torch.empty_like(k, memory_format=torch.contiguous_format) if dk is None else dk
    dv = torch.empty_like(v, memory_format=torch.contiguous_format) if dv is None else dv
    if workspace is None:
        nbytes = lib().mt_flash_attn_bwd_workspace_bytes(B, H, N, d)
        workspace = torch.empty(nbytes // 4, dtype=torch.float32, device=q.device)
    m = m.contiguous().float()
    l = l.contiguous().float()
    strides = (ctypes.c_int64 * 24)()
    for i, t in enumerate((q, k, v, o, do, dq, dk, dv)):
        s = strides3(t)
        strides[3 * i:3 * i + 3] = list(s)
    st = stream_ptr(q.device) if stream is None else stream
    kv = _kv_arg(kv_len, B, q.device)
    args = (dtype_code(q), int(causal), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
            do.data_ptr(), m.data_ptr(), l.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
            B, H, N, d, strides)
    # the size-checked entry (ABI 3): a workspace the caller sized too small is an error
    check(lib().mt_flash_attn_bwd_v3(*args, None if kv is None else kv.data_ptr(),
                                     workspace.data_ptr(), workspace.numel() * workspace.element_size(),
                                     st), "mt_flash_attn_bwd_v3")
    return dq, dk, dv


def scratch_bytes() -> int:
    """Device bytes the library's stream scratch holds between calls (mt_scratch_bytes)."""
    return int(lib().mt_scratch_bytes())


def scratch_release() -> None:
    """Free the library's stream scratch that no captured graph holds (mt_scratch_release)."""
    check(lib().mt_scratch_release(), "mt_scratch_release")


def exported_symbols() -> Sequence[str]:
    return tuple(_PROTOS)


def adam_step(params, grads, exp_avg, exp_avg_sq, numels, beta1, beta2, eps, step_size,
              step_size_ptr: Optional[int] = None) -> None:
    """One multi-tensor Adam launch (mt_adam_step) over dense fp32 device buffers given as
    raw pointers, in place, on the current stream. step_size_ptr: read the step size from
    that device fp32 instead (mt_adam_step_dstep, a graph-captured step)."""
    n = len(params)
    arr = ctypes.c_void_p * max(1, n)
    ptrs = (n, arr(*params), arr(*grads), arr(*exp_avg), arr(*exp_avg_sq), (ctypes.c_int64 * max(1, n))(*numels),
            beta1, beta2, eps)
    if step_size_ptr is None:
        check(lib().mt_adam_step(*ptrs, step_size, stream_ptr()), "mt_adam_step")
    else:
        check(lib().mt_adam_step_dstep(*ptrs, step_size_ptr, stream_ptr()), "mt_adam_step_dstep")
