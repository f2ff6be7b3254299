"""ctypes binding of the C oracle (``oracle/attn_ref.c``) -- TEST INFRASTRUCTURE ONLY.

Used by ``tests/`` for large-size parity checks and by ``bench.py``'s
``cpu_baseline`` leg. Never imported by the shipped operator path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_attn.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        f = ctypes.POINTER(ctypes.c_float)
        i64 = ctypes.c_int64
        _lib.oracle_attn_fwd.argtypes = [f, f, f, f, f, f, i64, i64, i64, ctypes.c_int, ctypes.c_int]
        _lib.oracle_attn_fwd.restype = None
        _lib.oracle_attn_bwd.argtypes = [f, f, f, f, f, f, f, f, f, i64, i64, i64,
                                         ctypes.c_int, ctypes.c_int]
        _lib.oracle_attn_bwd.restype = None
        ip = ctypes.POINTER(ctypes.c_int)
        _lib.oracle_attn_fwd_kv.argtypes = [f, f, f, f, f, f, i64, i64, i64, ctypes.c_int, ip, ctypes.c_int]
        _lib.oracle_attn_fwd_kv.restype = None
        _lib.oracle_attn_bwd_kv.argtypes = [f, f, f, f, f, f, f, f, f, i64, i64, i64,
                                            ctypes.c_int, ip, ctypes.c_int]
        _lib.oracle_attn_bwd_kv.restype = None
        _lib.oracle_num_threads.restype = ctypes.c_int
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def num_threads() -> int:
    return lib().oracle_num_threads()


def _kv_rows(kv_len, lead):
    """[B] key-padding lengths of a (B, H, ...) batch -> one int32 per (b, h) row (or None)."""
    if kv_len is None:
        return None
    kv = np.asarray(kv_len, np.int32).reshape(-1)
    reps = int(np.prod(lead[1:])) if len(lead) > 1 else 1
    return np.ascontiguousarray(np.repeat(kv, reps), np.int32)


def _ip(a):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def attn_fwd(q, k, v, causal=False, nthreads=0, kv_len=None):
    """q,k,v: (..., N, d) fp32 -> (o, m, l) through the C restatement. kv_len: optional [B]
    key-padding lengths of a (B, H, N, d) batch."""
    q, k, v = (np.ascontiguousarray(a, dtype=np.float32) for a in (q, k, v))
    *lead, N, d = q.shape
    BH = int(np.prod(lead)) if lead else 1
    o = np.empty_like(q)
    m = np.empty(tuple(lead) + (N,), np.float32)
    l = np.empty_like(m)
    kv = _kv_rows(kv_len, lead)
    lib().oracle_attn_fwd_kv(_p(q), _p(k), _p(v), _p(o), _p(m), _p(l), BH, N, d, int(causal),
                             _ip(kv), nthreads)
    return o, m, l


def attn_bwd(q, k, v, do, m, l, causal=False, nthreads=0, kv_len=None):
    q, k, v, do, m, l = (np.ascontiguousarray(a, dtype=np.float32) for a in (q, k, v, do, m, l))
    *lead, N, d = q.shape
    BH = int(np.prod(lead)) if lead else 1
    dq, dk, dv = np.empty_like(q), np.empty_like(q), np.empty_like(q)
    kv = _kv_rows(kv_len, lead)
    lib().oracle_attn_bwd_kv(_p(q), _p(k), _p(v), _p(do), _p(m), _p(l), _p(dq), _p(dk), _p(dv),
                             BH, N, d, int(causal), _ip(kv), nthreads)
    return dq, dk, dv
