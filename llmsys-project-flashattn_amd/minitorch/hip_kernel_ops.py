"""``HipKernelOps``: the MI355X backend for ``TensorBackend`` (drop-in for the reference's
``CudaKernelOps``, ``minitorch/cuda_kernel_ops.py``).

Every storage is device-resident (``cuda = True``): tensors are uploaded once by
``tensor_from_numpy`` and every operator -- map/zip/reduce/matmul and the fused softmax,
LayerNorm and FlashAttention kernels -- runs as a stream-ordered HIP kernel from
``libminitorch_hip.so`` on device pointers. The reference instead round-trips every
operand host->device->host inside each launcher (flashattention_kernel.cu:284-324,
combine.cu:345-382). There is no CPU fallback: a missing library raises.

Fused-op contracts (reference cuda_kernel_ops.py:439-892):
  attn_softmax_fw(inp, mask)              -> softmax(inp + mask) (new tensor)
  attn_softmax_bw(out_grad, soft_inp)     -> (inp_grad, soft_inp)
  layernorm_fw(inp, gamma, beta)          -> (ln_res, var, means)
  layernorm_bw(dout, inp, gamma, beta, var, mean) -> (inp_grad, gamma_grad[1,H], beta_grad[1,H])
  flash_attention[_causal]_fw(Q, K, V)    -> (O, m, l)      P = exp(s - m) / l
  flash_attention[_causal]_bw(Q, K, V, O, dO, m, l) -> (dQ, dK, dV)
Q/K/V may be strided views (e.g. the permuted projections of MultiHeadAttention): the
kernels take (batch, head, seq) strides, so no ``.contiguous()`` copy is made.
"""
from __future__ import annotations

import ctypes
import os
import functools
from typing import Callable, Optional

import numpy as np

from . import _hip
from . import operators
from .tensor import Tensor
from .tensor_data import TensorData, _prod, shape_broadcast
from .tensor_ops import MapProto, TensorOps


@functools.lru_cache(maxsize=4096)
def _i64_cached(vals: tuple) -> ctypes.Array:
    return (ctypes.c_int64 * max(1, len(vals)))(*vals)


def _i64(vals) -> ctypes.Array:
    """int64 array argument; shapes/strides repeat every step, so the ctypes arrays are
    cached by value (the callee only reads them). TensorData already holds them as tuples
    of Python ints, which go to the cache as they are."""
    if type(vals) is not tuple:
        vals = tuple(int(v) for v in vals)
    return _i64_cached(vals)


_RIGHT_T = os.environ.get("MT_RIGHT_T", "1") != "0"  # A/B switch (scripts/gpu_colab.sh)


_torch_mod = None


def _out(like: Tensor, shape) -> Tensor:
    """Uninitialised dense fp32 device output (every kernel below writes all of it)."""
    global _torch_mod
    if _torch_mod is None:
        import torch
        _torch_mod = torch
    shape = tuple(map(int, shape))
    st = _torch_mod.empty(_prod(shape), dtype=_torch_mod.float32, device="cuda")
    return Tensor(TensorData(st, shape), backend=like.backend)


def _dev(t: Tensor) -> Tensor:
    if not t._tensor.on_device:
        t._tensor.to_cuda_()
    return t


def _ptr(t: Tensor) -> int:
    return _dev(t)._tensor.data_ptr()


def _dense(t: Tensor) -> Tensor:
    return t if t._tensor.is_dense() else t.contiguous()


def _stream() -> int:
    return _hip.stream_ptr()


def _fn_id(fn: Callable) -> int:
    try:
        return operators.FN_IDS[fn]
    except KeyError:
        raise NotImplementedError(f"no device kernel for {getattr(fn, '__name__', fn)}") from None


def _torch_view(t: Tensor):
    """A torch view of a minitorch tensor's storage with its shape and strides (plumbing
    for the flash entry points, which read strides from torch tensors)."""
    import torch
    st = _dev(t)._tensor._storage
    return torch.as_strided(st, t.shape, t._tensor.strides)


def _layout_like(t: Tensor) -> tuple:
    """Strides of a dense buffer of t's shape whose dims are laid out in t's stride order
    (outermost = largest stride; ties keep the dim order): t's own layout when t is a
    permutation of a dense tensor, row-major when t is dense."""
    shape, st = t.shape, t._tensor.strides
    order = sorted(range(len(shape)), key=lambda i: (-st[i], i))
    out = [0] * len(shape)
    acc = 1
    for i in reversed(order):
        out[i] = acc
        acc *= shape[i]
    return tuple(out)


def _wrap(storage, shape, backend, strides=None) -> Tensor:
    return Tensor(TensorData(storage, tuple(shape), strides), backend=backend)


class HipKernelOps(TensorOps):
    cuda = True

    @staticmethod
    def map(fn: Callable[[float], float]) -> MapProto:
        fid = _fn_id(fn)

        def ret(a: Tensor, out: Optional[Tensor] = None) -> Tensor:
            if out is None:
                out = _out(a, a.shape)
            L = _hip.lib()
            if _hip.fast is not None:
                _hip.check(_hip.fast.map(fid, _ptr(out), out.shape, out._tensor.strides, _ptr(a), a.shape,
                                         a._tensor.strides, _stream()), "map")
                return out
            _hip.check(L.mt_tensor_map(
                fid, _ptr(out), _i64(out.shape), _i64(out._tensor.strides), out.dims,
                _ptr(a), _i64(a.shape), _i64(a._tensor.strides), a.dims, _stream()), "map")
            return out

        return ret

    @staticmethod
    def cmap(fn: Callable[[float], float]) -> Callable[[Tensor, Tensor], Tensor]:
        fid = _fn_id(fn)

        def ret(a: Tensor, out: Tensor) -> Tensor:
            L = _hip.lib()
            if _hip.fast is not None:
                _hip.check(_hip.fast.map(fid, _ptr(out), out.shape, out._tensor.strides, _ptr(a), a.shape,
                                         a._tensor.strides, _stream()), "cmap")
                return out
            _hip.check(L.mt_tensor_map(
                fid, _ptr(out), _i64(out.shape), _i64(out._tensor.strides), out.dims,
                _ptr(a), _i64(a.shape), _i64(a._tensor.strides), a.dims, _stream()), "cmap")
            return out

        return ret

    @staticmethod
    def zip(fn: Callable[[float, float], float]) -> Callable[[Tensor, Tensor], Tensor]:
        fid = _fn_id(fn)

        def ret(a: Tensor, b: Tensor) -> Tensor:
            shape = shape_broadcast(a.shape, b.shape)
            out = _out(a, shape)
            L = _hip.lib()
            if _hip.fast is not None:
                _hip.check(_hip.fast.zip(fid, _ptr(out), out.shape, out._tensor.strides, _ptr(a), a.shape,
                                         a._tensor.strides, _ptr(b), b.shape, b._tensor.strides, _stream()), "zip")
                return out
            _hip.check(L.mt_tensor_zip(
                fid, _ptr(out), _i64(out.shape), _i64(out._tensor.strides), out.dims,
                _ptr(a), _i64(a.shape), _i64(a._tensor.strides), a.dims,
                _ptr(b), _i64(b.shape), _i64(b._tensor.strides), b.dims, _stream()), "zip")
            return out

        return ret

    @staticmethod
    def reduce(fn: Callable[[float, float], float], start: float = 0.0) -> Callable[[Tensor, int], Tensor]:
        fid = _fn_id(fn)

        def ret(a: Tensor, dim: int) -> Tensor:
            shape = list(a.shape)
            shape[dim] = 1
            out = _out(a, shape)
            L = _hip.lib()
            if _hip.fast is not None:
                _hip.check(_hip.fast.reduce(fid, _ptr(out), out.shape, out._tensor.strides, _ptr(a), a.shape,
                                            a._tensor.strides, int(dim), float(start), _stream()), "reduce")
                return out
            _hip.check(L.mt_tensor_reduce(
                fid, _ptr(out), _i64(out.shape), _i64(out._tensor.strides),
                _ptr(a), _i64(a.shape), _i64(a._tensor.strides), a.dims, int(dim),
                ctypes.c_float(start), _stream()), "reduce")
            return out

        return ret

    @staticmethod
    def matrix_multiply(a: Tensor, b: Tensor) -> Tensor:
        """Batched a @ b over broadcast leading dims (reference cuda_kernel_ops.py:340-437
        flattens to 3-D the same way)."""
        both_2d = a.dims == 2 and b.dims == 2

        Mo, No = a.shape[-2], b.shape[-1]

        def gemm_ready(t: Tensor, left: bool) -> bool:
            # a layout the GEMM takes as it is: row-major (with a row pitch), or, for the left
            # operand of a product with a small output, the transpose of a row-major matrix
            # (MatMul.backward's dW = xᵀ·dy: rocBLAS op T with split-K, 12 µs against 28 µs +
            # the transposing copy at config 5). Otherwise the copy: rocBLAS's op-T kernels
            # measured slower on the other shapes (LM-head dW 2.3 ms against 0.25 ms, dX = dy·Wᵀ
            # 16.6 against 11.4 µs + copy; profiles/r4_c5_gemm_layouts.txt)
            r, c = t.shape[-2], t.shape[-1]
            sr, sc = t._tensor.strides[-2], t._tensor.strides[-1]
            if t._tensor.is_dense() or (sc == 1 and sr >= c):
                return True
            if sr != 1 or sc < r:
                return False
            if left:
                return Mo <= 1024 and No <= 1024
            # a small transposed right operand (the linears' Wᵀ in dX = dy·Wᵀ): op T, no copy
            return _RIGHT_T and r <= 1024 and c <= 1024

        def lift(t: Tensor, left: bool) -> Tensor:
            # a 2-D operand as a batch of one over the same storage (a backend op: no autodiff
            # View, whose shape tensor and Function record cost host time on every matmul)
            if not gemm_ready(t, left):
                t = t.contiguous()
            st = t._tensor.strides
            return _wrap(t._tensor._storage, (1,) + tuple(t.shape), t.backend, (t.size,) + tuple(st))

        if both_2d:
            # the common case (every Linear): no batch, no lifted views, one output tensor
            if not gemm_ready(a, True):
                a = a.contiguous()
            if not gemm_ready(b, False):
                b = b.contiguous()
            M, K = a.shape
            K2, N = b.shape
            assert K == K2, f"matmul shape mismatch {a.shape} @ {b.shape}"
            out = _out(a, (M, N))
            sa, sb = a._tensor.strides, b._tensor.strides
            L = _hip.lib()
            if _hip.fast is not None:
                _hip.check(_hip.fast.matmul(_ptr(out), _ptr(a), _ptr(b), 1, M, N, K, (M * K, sa[0], sa[1]),
                                            (K * N, sb[0], sb[1]), (M * N, N, 1), _stream()), "matmul")
                return out
            _hip.check(L.mt_matmul_f32(_ptr(out), _ptr(a), _ptr(b), 1, M, N, K,
                                                _i64((M * K, sa[0], sa[1])), _i64((K * N, sb[0], sb[1])),
                                                _i64((M * N, N, 1)), _stream()), "matmul")
            return out
        if a.dims == 2:
            a = lift(a, True)
        if b.dims == 2:
            b = lift(b, False)
        lead = tuple(shape_broadcast(a.shape[:-2], b.shape[:-2]))
        M, K = a.shape[-2], a.shape[-1]
        K2, N = b.shape[-2], b.shape[-1]
        assert K == K2, f"matmul shape mismatch {a.shape} @ {b.shape}"
        batch = _prod(lead) if lead else 1

        def batch_view(t: Tensor):
            # (batch stride, row stride, col stride); a broadcast operand gets stride 0.
            if t.dims == 3 and len(lead) == 1:
                bs = 0 if t.shape[0] == 1 and batch > 1 else t._tensor.strides[0]
                return t, (bs, t._tensor.strides[1], t._tensor.strides[2])
            tl = t.shape[:-2]
            if _prod(tuple(tl)) == 1 and batch > 1:
                return t, (0, t._tensor.strides[-2], t._tensor.strides[-1])
            if tuple(tl) != lead:
                raise NotImplementedError(f"partial batch broadcast {t.shape} vs {lead}")
            if not t._tensor.is_dense() and not (t.dims == 3 and gemm_ready(t, t is a)):
                t = t.contiguous()
            s = t._tensor.strides
            return t, (s[-3], s[-2], s[-1])

        a, sa = batch_view(a)
        b, sb = batch_view(b)
        out = _out(a, lead + (M, N))
        so = (M * N, N, 1)
        if _hip.lib() is not None and _hip.fast is not None:
            _hip.check(_hip.fast.matmul(_ptr(out), _ptr(a), _ptr(b), batch, M, N, K, tuple(map(int, sa)),
                                        tuple(map(int, sb)), so, _stream()), "matmul")
        else:
            _hip.check(_hip.lib().mt_matmul_f32(_ptr(out), _ptr(a), _ptr(b), batch, M, N, K,
                                                _i64(sa), _i64(sb), _i64(so), _stream()), "matmul")
        if both_2d:
            return _wrap(out._tensor._storage, (M, N), out.backend)
        return out

    @staticmethod
    def rand_uniform(out: Tensor, seed: int) -> Tensor:
        """Fill the dense fp32 ``out`` with U[0,1) on the device (counter-based hash of
        (seed, index)); the reference draws dropout randomness on the host
        (tensor_functions.rand, modules_basic.py Dropout)."""
        assert out._tensor.is_dense()
        _hip.check(_hip.lib().mt_rand_uniform(_ptr(out), out.size, seed & 0xFFFFFFFFFFFFFFFF,
                                              _stream()), "rand_uniform")
        return out

    # ---- fused kernels -------------------------------------------------------------------
    @staticmethod
    def bias_gelu_fw(x: Tensor, bias: Tensor) -> Tensor:
        """GELU_tanh(x + bias) over the rows of a 2-D x (FeedForward's linear_in bias + GELU,
        reference modules_transfomer.py FeedForward) in one pass."""
        x, b = _dense(x), _dense(bias)
        rows, cols = x.shape
        out = _out(x, (rows, cols))
        _hip.check(_hip.lib().mt_bias_gelu_fw(_ptr(out), _ptr(x), _ptr(b), rows, cols, _stream()),
                   "bias_gelu_fw")
        return out

    @staticmethod
    def bias_gelu_bw(grad: Tensor, x: Tensor, bias: Tensor) -> Tensor:
        g, x, b = _dense(grad), _dense(x), _dense(bias)
        rows, cols = x.shape
        dx = _out(x, (rows, cols))
        _hip.check(_hip.lib().mt_bias_gelu_bw(_ptr(dx), _ptr(g), _ptr(x), _ptr(b), rows, cols, _stream()),
                   "bias_gelu_bw")
        return dx

    @staticmethod
    def dropout_fw(x: Tensor, p: float, scale: float, seed: int) -> Tensor:
        """x * (u > p) * scale with u the device uniform draw of (seed, index) (the mask of
        rand(shape) > p, never stored: the backward redraws it from the seed)."""
        x = _dense(x)
        out = _out(x, x.shape)
        if isinstance(seed, int):
            _hip.check(_hip.lib().mt_dropout(_ptr(out), _ptr(x), x.size, ctypes.c_float(p), ctypes.c_float(scale),
                                             seed & 0xFFFFFFFFFFFFFFFF, _stream()), "dropout")
        else:  # a device-resident seed (tensor_functions._DeviceSeed, a graph-captured step)
            _hip.check(_hip.lib().mt_dropout_dseed(_ptr(out), _ptr(x), x.size, ctypes.c_float(p),
                                                   ctypes.c_float(scale), seed.ptr, _stream()), "dropout")
        return out

    @staticmethod
    def embedding_fw(ids: Tensor, weight: Tensor) -> Tensor:
        """W[ids] for float token ids of any shape: rows of the [V, E] weight (reference
        modules_basic.py Embedding: one_hot(ids) @ W, a 25.6 GFLOP product at config 5)."""
        ids, w = _dense(ids), _dense(weight)
        V, E = w.shape
        out = _out(w, tuple(ids.shape) + (E,))
        _hip.check(_hip.lib().mt_embedding_fw(_ptr(out), _ptr(ids), _ptr(w), ids.size, V, E, _stream()),
                   "embedding_fw")
        return out

    @staticmethod
    def embedding_bw(grad: Tensor, ids: Tensor, num_embeddings: int) -> Tensor:
        """dW [V, E]: the rows of grad summed per token id (fixed order: deterministic)."""
        g, ids = _dense(grad), _dense(ids)
        E = g.shape[-1]
        dw = _out(g, (num_embeddings, E))
        _hip.check(_hip.lib().mt_embedding_bw(_ptr(dw), _ptr(g), _ptr(ids), ids.size, num_embeddings, E,
                                              _stream()), "embedding_bw")
        return dw

    @staticmethod
    def softmax_xent_fw(logits: Tensor, target: Tensor):
        """(loss[rows], lse[rows]) of the reference's softmax_loss (nn.py) in one pass."""
        x = _dense(logits)
        t = _dense(target)
        rows, C = x.shape
        loss = _out(x, (rows,))
        lse = _out(x, (rows,))
        _hip.check(_hip.lib().mt_softmax_xent_fw(_ptr(loss), _ptr(lse), _ptr(x), _ptr(t), rows, C,
                                                 _stream()), "softmax_xent_fw")
        return loss, lse

    @staticmethod
    def softmax_xent_bw(grad: Tensor, logits: Tensor, target: Tensor, lse: Tensor) -> Tensor:
        g, x, t = _dense(grad), _dense(logits), _dense(target)
        rows, C = x.shape
        dx = _out(x, (rows, C))
        _hip.check(_hip.lib().mt_softmax_xent_bw(_ptr(dx), _ptr(g), _ptr(x), _ptr(t), _ptr(lse), rows, C,
                                                 _stream()), "softmax_xent_bw")
        return dx

    @staticmethod
    def attn_softmax_fw(inp: Tensor, mask: Optional[Tensor], mask_future: bool = False) -> Tensor:
        B, nh, T_from, T_to = inp.shape
        x = inp if inp._tensor.is_dense() else inp.contiguous()
        out = _out(x, x.shape)  # the kernel writes every element
        mptr, ms = None, None
        if mask is not None:
            mshape = (1,) * (4 - mask.dims) + tuple(mask.shape)
            mstr = (0,) * (4 - mask.dims) + tuple(mask._tensor.strides)
            ms = _i64([0 if mshape[i] == 1 else mstr[i] for i in range(4)])
            mptr = _ptr(mask)
        _hip.check(_hip.lib().mt_attn_softmax_fw(_ptr(out), _ptr(x), mptr, B, nh, T_from, T_to, ms,
                                                 int(mask_future), _stream()), "attn_softmax_fw")
        return out

    @staticmethod
    def attn_softmax_bw(out_grad: Tensor, soft_inp: Tensor):
        g = out_grad if out_grad._tensor.is_dense() else out_grad.contiguous()
        y = soft_inp if soft_inp._tensor.is_dense() else soft_inp.contiguous()
        rows = int(np.prod(y.shape[:-1]))
        dinp = _out(g, g.shape)
        _hip.check(_hip.lib().mt_attn_softmax_bw(_ptr(dinp), _ptr(g), _ptr(y), rows, y.shape[-1],
                                                 _stream()), "attn_softmax_bw")
        return dinp, soft_inp

    @staticmethod
    def layernorm_fw(inp: Tensor, gamma: Tensor, beta: Tensor):
        x = inp if inp._tensor.is_dense() else inp.contiguous()
        rows, H = x.shape
        gm, bt = _dense(gamma), _dense(beta)  # held: their device buffers must outlive the launch
        ln = _out(x, x.shape)
        var = _out(x, (rows,))
        mean = _out(x, (rows,))
        _hip.check(_hip.lib().mt_layernorm_fw(_ptr(ln), _ptr(var), _ptr(mean), _ptr(x),
                                              _ptr(gm), _ptr(bt),
                                              rows, H, _stream()), "layernorm_fw")
        return ln, var, mean

    @staticmethod
    def layernorm_bw(out_grad: Tensor, inp: Tensor, gamma: Tensor, beta: Tensor, var: Tensor,
                     mean: Tensor):
        import torch
        g = out_grad if out_grad._tensor.is_dense() else out_grad.contiguous()
        x = inp if inp._tensor.is_dense() else inp.contiguous()
        rows, H = x.shape
        gm, bt = _dense(gamma), _dense(beta)
        dx = _out(x, x.shape)
        dgamma = _out(x, (1, H))
        dbeta = _out(x, (1, H))
        ws = torch.empty(max(1, _hip.lib().mt_layernorm_bw_workspace_bytes(rows, H) // 4),
                         dtype=torch.float32, device="cuda")
        _hip.check(_hip.lib().mt_layernorm_bw(_ptr(dgamma), _ptr(dbeta), _ptr(dx), _ptr(g), _ptr(x),
                                              _ptr(gm), _ptr(bt),
                                              _ptr(var), _ptr(mean), rows, H, ws.data_ptr(),
                                              _stream()), "layernorm_bw")
        return dx, dgamma, dbeta

    @staticmethod
    def _kv(kv_len):
        """A [B] key-padding length tensor (minitorch Tensor, device storage) as the int32
        device vector the C ABI takes, or None."""
        if kv_len is None:
            return None
        import torch
        return _torch_view(kv_len).reshape(-1).to(torch.int32)

    @staticmethod
    def _flash_fw(Q: Tensor, K: Tensor, V: Tensor, causal: bool, kv_len=None):
        """O is laid out like Q's storage: for MultiHeadAttention's permuted projection views
        ([B,N,H,d] storage seen as [B,H,N,d]) O's storage is [B,N,H,d] too, so the block's
        ``O.permute(0, 2, 1, 3).contiguous()`` is a view, not a copy (the kernels take strides)."""
        import torch
        B, H, N, d = Q.shape
        backend = Q.backend
        so = _layout_like(Q)
        o = torch.empty(B * H * N * d, dtype=torch.float32, device="cuda")
        m = torch.empty(B * H * N, dtype=torch.float32, device="cuda")
        l = torch.empty(B * H * N, dtype=torch.float32, device="cuda")
        _hip.flash_fwd(_torch_view(Q), _torch_view(K), _torch_view(V), causal,
                       out=torch.as_strided(o, (B, H, N, d), so), m=m.view(B, H, N), l=l.view(B, H, N),
                       kv_len=HipKernelOps._kv(kv_len))
        return (_wrap(o, (B, H, N, d), backend, so), _wrap(m, (B, H, N), backend),
                _wrap(l, (B, H, N), backend))

    @staticmethod
    def _flash_bw(Q, K, V, O, dO, m, l, causal: bool, kv_len=None):
        """dQ, dK, dV laid out like Q, K, V: the permuted projection views' gradients flow back
        through Permute and View with no contiguous copy."""
        import torch
        B, H, N, d = Q.shape
        backend = Q.backend
        lay = [_layout_like(t) for t in (Q, K, V)]
        bufs = [torch.empty(B * H * N * d, dtype=torch.float32, device="cuda") for _ in range(3)]
        g = [torch.as_strided(b, (B, H, N, d), s) for b, s in zip(bufs, lay)]
        _hip.flash_bwd(_torch_view(Q), _torch_view(K), _torch_view(V), _torch_view(O),
                       _torch_view(dO), _torch_view(m), _torch_view(l), causal,
                       dq=g[0], dk=g[1], dv=g[2], kv_len=HipKernelOps._kv(kv_len))
        return tuple(_wrap(b, (B, H, N, d), backend, s) for b, s in zip(bufs, lay))

    # reference cuda_kernel_ops.py:605-892; kv_len (optional keyword, [B] valid key counts):
    # key padding through mt_flash_attn_*_varlen
    @staticmethod
    def flash_attention_fw(Q: Tensor, K: Tensor, V: Tensor, kv_len=None):
        return HipKernelOps._flash_fw(Q, K, V, False, kv_len)

    @staticmethod
    def flash_attention_bw(Q, K, V, O, dO, m, l, kv_len=None):
        return HipKernelOps._flash_bw(Q, K, V, O, dO, m, l, False, kv_len)

    @staticmethod
    def flash_attention_causal_fw(Q: Tensor, K: Tensor, V: Tensor, kv_len=None):
        return HipKernelOps._flash_fw(Q, K, V, True, kv_len)

    @staticmethod
    def flash_attention_causal_bw(Q, K, V, O, dO, m, l, kv_len=None):
        return HipKernelOps._flash_bw(Q, K, V, O, dO, m, l, True, kv_len)
