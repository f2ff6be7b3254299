"""CPU-side checks of the C ABI: the library loads and exports every symbol the
header declares (no kernel is launched here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", f) for f in sorted(os.listdir(os.path.join(ROOT, "include")))
           if f.endswith(".h")]


def _declared(path):
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", text, flags=re.M)
    return sorted(set(n for n in names if n not in ("if", "extern")))


def test_headers_present():
    assert HEADERS


def test_library_exports_every_declared_symbol():
    from minitorch import _hip
    if not os.path.exists(_hip.LIB_PATH):
        pytest.skip("library not built")
    lib = _hip.lib()  # torch first: one HIP runtime per process
    missing = []
    for h in HEADERS:
        for name in _declared(h):
            if not hasattr(lib, name):
                missing.append((os.path.basename(h), name))
    assert not missing, missing


def test_python_binding_covers_header():
    from minitorch import _hip
    declared = set()
    for h in HEADERS:
        declared.update(_declared(h))
    lib = _hip.lib()  # also applies every argtypes declaration
    assert declared <= set(_hip.exported_symbols()), declared - set(_hip.exported_symbols())
    assert lib.mt_abi_version() == 3
    # fp32 delta + log2-LSE per row, 256-B aligned; at d = 64 also the fused bf16 backward's
    # arrival counters (u32 [B*H][ceil(N/64)], 256-B aligned) and the dQ partial slab of one
    # group of heads: min(B*H, 2^30 // head) heads of ceil(N/64) * ceil(N/256) * 8 KiB each
    def fused(B, H, N):
        head = -(-N // 64) * -(-N // 256) * 8192
        cnt = -(-(B * H * -(-N // 64) * 4) // 256) * 256
        return cnt + min(B * H, 2 ** 30 // head) * head
    assert lib.mt_flash_attn_bwd_workspace_bytes(2, 3, 5, 7) == 256
    # ... or, when larger, the fp32 fused ring backward's partials (fa_bwd_fused_ring): one group
    # of at most 1 GiB of ceil(N/256) * N * 64 fp32 per head (C2: 128 MiB, above the bf16 64 MiB)
    def ring(B, H, N):
        head = -(-N // 256) * N * 256
        return min(B * H, 2 ** 30 // head) * head
    assert lib.mt_flash_attn_bwd_workspace_bytes(8, 16, 1024, 64) == 2 * 128 * 1024 * 4 + ring(8, 16, 1024)
    assert ring(8, 16, 1024) == 2 ** 27 > fused(8, 16, 1024)
    assert lib.mt_flash_attn_bwd_workspace_bytes(2, 3, 300, 48) == 2 * 6 * 300 * 4 + 256 - (2 * 6 * 300 * 4) % 256 + ring(2, 3, 300)
    assert lib.mt_flash_attn_bwd_workspace_bytes(8, 16, 4096, 64) == 2 * 128 * 4096 * 4 + fused(8, 16, 4096)
    assert fused(8, 16, 4096) == 128 * 64 * 4 + 2 ** 30  # C3: one launch, 1 GiB of partials
    # longer sequences: head groups that reuse a slab of at most 1 GiB (N = 16384: 8 heads)
    assert lib.mt_flash_attn_bwd_workspace_bytes(1, 16, 16384, 64) == 2 * 16 * 16384 * 4 + fused(1, 16, 16384)
    # large batches no longer scale the slab (round 3: 32 GiB at (64,16,8192,64))
    big = lib.mt_flash_attn_bwd_workspace_bytes(64, 16, 8192, 64)
    assert big == 2 * 1024 * 8192 * 4 + fused(64, 16, 8192) and big < 2 ** 31
    # past one head's slab within 1 GiB (N > 46336) the split backward needs the rows only
    assert lib.mt_flash_attn_bwd_workspace_bytes(1, 1, 46336, 64) > 2 * 46336 * 4 + 255
    assert lib.mt_flash_attn_bwd_workspace_bytes(1, 1, 46400, 64) == 2 * 46400 * 4
    # the fused form needs its lse2 | delta rows under 2^31 bytes (one LDS-DMA buffer)
    bh = 2 ** 31 // (2 * 8192 * 4)
    assert lib.mt_flash_attn_bwd_workspace_bytes(1, bh - 1, 8192, 64) > 2 * (bh - 1) * 8192 * 4 + 255
    assert lib.mt_flash_attn_bwd_workspace_bytes(1, bh, 8192, 64) == 2 * bh * 8192 * 4


def test_bwd_v3_rejects_small_workspace():
    """mt_flash_attn_bwd_v3 checks the caller's workspace size before touching any pointer
    (host-only: the size check precedes every launch)."""
    from minitorch import _hip
    lib = _hip.lib()
    need = lib.mt_flash_attn_bwd_workspace_bytes(8, 16, 4096, 64)
    dummy = ctypes.c_void_p(16)
    rc = lib.mt_flash_attn_bwd_v3(1, 0, *([dummy] * 10), 8, 16, 4096, 64, None, None, dummy,
                                  need - 1, None)
    assert rc != 0 and b"workspace" in lib.mt_last_error()


def test_errors_are_reported_not_fatal():
    from minitorch import _hip
    lib = _hip.lib()
    rc = lib.mt_flash_attn_fwd(7, 0, None, None, None, None, None, None, 1, 1, 1, 1,
                               None, None, None, None, None)
    assert rc != 0
    assert b"dtype" in lib.mt_last_error()


@pytest.mark.parametrize("sizes,msg", [
    ((0, 1, 64, 64), b"bad sizes"),        # empty batch
    ((1, 0, 64, 64), b"bad sizes"),        # no heads
    ((1, 1, 0, 64), b"bad sizes"),         # empty sequence
    ((1, 1, 64, 0), b"bad sizes"),         # zero head dim
    ((1, 1, 64, 4097), b"out of range"),   # d > 4096
    ((1, 1, 2 ** 30 + 1, 64), b"out of range"),
])
def test_size_validation_before_any_device_call(sizes, msg):
    """Empty and oversized shapes are refused with a status and a message before the library
    touches the device (so this runs without a GPU), forward and backward alike."""
    from minitorch import _hip
    lib = _hip.lib()
    for dtype in (0, 1):  # MT_F32, MT_BF16
        assert lib.mt_flash_attn_fwd(dtype, 0, None, None, None, None, None, None, *sizes,
                                     None, None, None, None, None) != 0
        assert msg in lib.mt_last_error()
        assert lib.mt_flash_attn_bwd(dtype, 1, None, None, None, None, None, None, None, None,
                                     None, None, *sizes, None, None, None) != 0
        assert msg in lib.mt_last_error()


def test_kernel_policy_switch_rejects_unknown_ids():
    """Only policies that compute the default's attention are selectable: the timing-only
    ablations (wrong results by construction) are not in the product library, and unknown
    ids leave the policy unchanged with a status."""
    from minitorch import _hip
    lib = _hip.lib()
    assert lib.mt_flash_get_kernel_policy() == 0
    for bad in (-1, 7, 16, 80, 86, 91, 96, 97, 10, 15, 1000):
        assert lib.mt_flash_set_kernel_policy(bad) != 0, bad
        assert b"unknown policy" in lib.mt_last_error()
        assert lib.mt_flash_get_kernel_policy() == 0
    with _hip.policy(120):
        assert lib.mt_flash_get_kernel_policy() == 120
    assert lib.mt_flash_get_kernel_policy() == 0
    with pytest.raises(RuntimeError):
        _hip.set_policy(97)


def test_product_library_policy_list():
    """The product library ships the kernels some default selects, and its policy switch takes
    exactly 0 (defaults), 1 (generic kernels), 120 / 121 (fused / split bf16 backward); the
    A/B schedules are in the diagnostics build (make DIAG=1)."""
    from minitorch import _hip
    if os.environ.get("MT_HIP_LIB"):
        pytest.skip("a non-product library is loaded")
    lib = _hip.lib()
    accepted = [p for p in range(0, 200) if lib.mt_flash_set_kernel_policy(p) == 0]
    lib.mt_flash_set_kernel_policy(0)
    assert accepted == [0, 1, 120, 121]
    import subprocess
    syms = subprocess.run(["nm", "-C", "--defined-only", _hip.LIB_PATH], capture_output=True,
                          text=True).stdout
    for absent in ("fa_bwd_dkv_bf16_w64", "fa_bwd_dq_pipe", "fa_bwd_dkv_bf16_st", "fa_fwd_bf16_sp2",
                   "fa_fwd_bf16_pp", "launch_fwd_v4_deep"):
        assert absent not in syms, absent


def test_product_library_has_no_ablation_kernels():
    """The product .so carries no instantiation of the wrong-result ablation templates."""
    from minitorch import _hip
    import subprocess
    if not os.path.exists(_hip.LIB_PATH):
        pytest.skip("library not built")
    syms = subprocess.run(["nm", "-C", "-D", "--defined-only", _hip.LIB_PATH], capture_output=True,
                          text=True).stdout
    assert "launch_fwd_v4_ablation" not in syms


def test_mtfast_extension_bound_and_checks_arguments():
    """The _mtfast CPython extension (csrc/mtfast.c) is built beside the package, bound to the
    loaded library's entry points at load, and rejects malformed arguments before any call
    (no GPU needed: nothing below reaches the library)."""
    from minitorch import _hip
    _hip.lib()
    assert _hip.fast is not None, "minitorch/_mtfast*.so missing: make -C llmsys-project-flashattn_amd"
    f = _hip.fast
    with pytest.raises(TypeError):
        f.map(1, 0, [4], (1,), 0, (4,), (1,), 0)          # a list where a tuple belongs
    with pytest.raises(TypeError):
        f.zip(1, 0, (4,), (1,))                            # wrong arity
    with pytest.raises(ValueError):
        f.map(1, 0, tuple(range(17)), (1,), 0, (4,), (1,), 0)  # more than 16 dims
    with pytest.raises(ValueError):
        f.matmul(0, 0, 0, 1, 2, 2, 2, (4, 2), (4, 2, 1), (4, 2, 1), 0)  # strides not triples
    # a strides tuple shorter (or longer) than its shape
    with pytest.raises(ValueError):
        f.map(1, 0, (2, 4), (4,), 0, (2, 4), (4, 1), 0)
    with pytest.raises(ValueError):
        f.zip(1, 0, (4,), (1,), 0, (4,), (1,), 0, (2, 4), (4,), 0)
    with pytest.raises(ValueError):
        f.reduce(1, 0, (1,), (1,), 0, (4, 1), (1,), 0, 0.0, 0)
