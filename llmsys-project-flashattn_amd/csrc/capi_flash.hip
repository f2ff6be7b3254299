// C ABI for the FlashAttention kernels (include/minitorch_hip.h).
//
// Device-pointer entry points (mt_flash_attn_*) plus host-pointer wrappers with the
// exact names and argument order of the reference launchers
// (src/flashattention_kernel.cu:259, :352, :694, :761), so the reference's ctypes
// binding (minitorch/cuda_kernel_ops.py:605-892) can load this library unchanged.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "../../include/minitorch_hip.h"
#include "fa_common.h"
#include <algorithm>

namespace mt {
hipError_t launch_fwd_generic(const AttnArgs& a, bool bf16_io, bool vec, bool causal,
                              hipStream_t st);
hipError_t launch_fwd_fast(const AttnArgs& a, bool causal, int variant, hipStream_t st,
                           bool* handled);
hipError_t launch_fwd_v2(const AttnArgs& a, bool causal, int nw, int resc, hipStream_t st,
                         bool* handled);
hipError_t launch_fwd_v3(const AttnArgs& a, bool causal, int variant, hipStream_t st, bool* handled);
hipError_t launch_fwd_v4(const AttnArgs& a, bool causal, int nw, bool pk, hipStream_t st,
                         bool* handled, int pair = 0);
hipError_t launch_fwd_v4_ablation(const AttnArgs& a, int abl, hipStream_t st);
hipError_t launch_fwd_v4_deep(const AttnArgs& a, bool causal, bool pk, hipStream_t st);
hipError_t launch_fwd_v5(const AttnArgs& a, bool causal, int ahead, int var, hipStream_t st,
                         bool* handled);
hipError_t launch_fwd_d128(const AttnArgs& a, bool causal, int nw, bool dma, hipStream_t st,
                           bool* handled, int pair = 0);
hipError_t launch_bwd_bf16(const AttnArgs& a, bool causal, int variant, hipStream_t st, bool* handled);
hipError_t launch_bwd_generic(const AttnArgs& a, bool bf16_io, bool vec, bool causal,
                              hipStream_t st);

static thread_local char g_err[512] = "";
static int g_kernel_policy = 0;  // 0: default bf16 MFMA kernels, 1: generic kernels only,
                                 // other values: A/B variants (fa_fwd_fast/v2/v3/v4.hip,
                                 // listed in tests/test_flash_gpu.py FAST_POLICIES)

int set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return 1;
}
int check_hip(hipError_t e, const char* where) {
  if (e == hipSuccess) return 0;
  return set_error("%s: %s", where, hipGetErrorString(e));
}

static void fill_strides(int64_t dst[3], const int64_t* src, int64_t H, int64_t N, int64_t d) {
  if (src) {
    dst[0] = src[0]; dst[1] = src[1]; dst[2] = src[2];
  } else {
    dst[0] = H * N * d; dst[1] = N * d; dst[2] = d;
  }
}

// 16-B vector path allowed: d and every row/batch/head stride a multiple of the
// 16-B element count, and every base pointer 16-B aligned.
static bool vec_ok(int64_t d, int esize, std::initializer_list<const int64_t*> strides,
                   std::initializer_list<const void*> ptrs) {
  const int64_t epc = 16 / esize;
  if (d % epc) return false;
  for (const int64_t* s : strides)
    for (int i = 0; i < 3; ++i)
      if (s[i] % epc) return false;
  for (const void* p : ptrs)
    if (p && ((uintptr_t)p & 15)) return false;
  return true;
}

static int check_sizes(int dtype, int64_t B, int64_t H, int64_t N, int64_t d) {
  if (dtype != MT_F32 && dtype != MT_BF16) return set_error("unsupported dtype %d", dtype);
  if (B <= 0 || H <= 0 || N <= 0 || d <= 0)
    return set_error("bad sizes B=%lld H=%lld N=%lld d=%lld", (long long)B, (long long)H,
                     (long long)N, (long long)d);
  if (N > (1 << 30) || B * H > (1ll << 31) - 1 || d > 4096)
    return set_error("sizes out of range (N=%lld, B*H=%lld, d=%lld; d <= 4096)", (long long)N,
                     (long long)(B * H), (long long)d);
  return 0;
}

}  // namespace mt

using namespace mt;

extern "C" {

const char* mt_last_error(void) { return g_err; }
void mt_flash_set_kernel_policy(int policy) { g_kernel_policy = policy; }
int mt_abi_version(void) { return 1; }

int mt_flash_attn_fwd(int dtype, int causal, const void* q, const void* k, const void* v,
                      void* o, float* m, float* l, int64_t B, int64_t H, int64_t N, int64_t d,
                      const int64_t* q_strides, const int64_t* k_strides,
                      const int64_t* v_strides, const int64_t* o_strides, void* stream) {
  if (check_sizes(dtype, B, H, N, d)) return 1;
  if (!q || !k || !v || !o) return set_error("mt_flash_attn_fwd: null tensor pointer");
  AttnArgs a;
  memset(&a, 0, sizeof(a));
  a.q = q; a.k = k; a.v = v; a.out = o; a.m = m; a.l = l;
  fill_strides(a.sq, q_strides, H, N, d);
  fill_strides(a.sk, k_strides, H, N, d);
  fill_strides(a.sv, v_strides, H, N, d);
  fill_strides(a.so, o_strides, H, N, d);
  a.B = (int)B; a.H = (int)H; a.N = (int)N; a.d = (int)d;
  a.scale = (float)(1.0 / sqrt((double)d));
  a.scale_log2 = (float)(1.4426950408889634 / sqrt((double)d));
  const int es = dtype == MT_BF16 ? 2 : 4;
  const bool vec = vec_ok(d, es, {a.sq, a.sk, a.sv, a.so}, {q, k, v, o});
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MT_BF16 && vec && g_kernel_policy != 1) {
    bool handled = false;
    hipError_t e = hipSuccess;
    if (g_kernel_policy >= 7 && g_kernel_policy <= 9)
      e = launch_fwd_v2(a, causal != 0, g_kernel_policy == 8 ? 8 : 4, g_kernel_policy == 9, st,
                        &handled);
    if (g_kernel_policy >= 16 && g_kernel_policy <= 20)
      e = launch_fwd_v3(a, causal != 0, g_kernel_policy - 16, st, &handled);
    if (g_kernel_policy >= 21 && g_kernel_policy <= 24)
      e = launch_fwd_v4(a, causal != 0, (g_kernel_policy & 1) ? 4 : 8, g_kernel_policy >= 23, st,
                        &handled);
    // default at d = 64: v5 (two query blocks per wave) for non-causal N % 64 == 0, else
    // 4-wave v4 (packed-f32 softmax arithmetic when non-causal, scalar when causal: the
    // faster of each in the A/B, profiles/r1_ab_*)
    if ((g_kernel_policy == 25 || g_kernel_policy == 26) && d == 64 &&
        ((int64_t)N + 128) * std::max(a.sk[2], a.sv[2]) * 2 < ((int64_t)1 << 31)) {
      e = launch_fwd_v4_deep(a, causal != 0, g_kernel_policy == 25, st);  // 4-wave, deep staging
      handled = true;
    }
    if (g_kernel_policy >= 27 && g_kernel_policy <= 29)
      e = launch_fwd_v5(a, causal != 0, 2 * (g_kernel_policy - 26), g_kernel_policy == 27 ? 4 : 0, st,
                        &handled);
    if (g_kernel_policy == 39 && !causal)  // 37 + static priority for the younger 4 waves
      e = launch_fwd_v5(a, false, 2, 2048 + 1028 + 4096, st, &handled);
    if (g_kernel_policy == 38 && !causal)  // 4 waves, register staging (the previous default)
      e = launch_fwd_v5(a, false, 2, 4, st, &handled);
    if (g_kernel_policy == 31)  // tile loop not unrolled (the pre-unroll default)
      e = launch_fwd_v5(a, causal != 0, 2, 0, st, &handled);
    if (g_kernel_policy == 35 && !causal)  // LDS-DMA staging
      e = launch_fwd_v5(a, false, 2, 1028, st, &handled);
    if ((g_kernel_policy == 36 || g_kernel_policy == 37) && !causal)  // 8 waves (37: + LDS-DMA)
      e = launch_fwd_v5(a, false, 2, g_kernel_policy == 36 ? 2048 + 4 : 2048 + 1028, st, &handled);
    if (g_kernel_policy == 50 || g_kernel_policy == 51)  // causal v4, heavy + light block pairs
      e = launch_fwd_v4(a, causal != 0, g_kernel_policy == 50 ? 4 : 8, !causal, st, &handled, true);
    if (g_kernel_policy == 63 || g_kernel_policy == 64)  // 50 / 51 with the light block first
      e = launch_fwd_v4(a, causal != 0, g_kernel_policy == 63 ? 4 : 8, !causal, st, &handled, 2);
    if (g_kernel_policy == 61 && !causal)  // 56 with the LDS-DMA issued from inline asm
      e = launch_fwd_v5(a, false, 2, 2048 + 623620, st, &handled);
    if (g_kernel_policy >= 56 && g_kernel_policy <= 58 && !causal)  // 54 + exp-to-use distance
      // of one MFMA slot (57 / 58: LDS operand reads 3 / 4 MFMAs ahead instead of 2)
      e = launch_fwd_v5(a, false, g_kernel_policy - 54, 2048 + 99332, st, &handled);
    if ((g_kernel_policy == 54 || g_kernel_policy == 55) && !causal)  // 37 (55: + priority) with
      // the Vᵀ fragments of P2 kept in registers for P4 (half the V LDS reads)
      e = launch_fwd_v5(a, false, 2, 2048 + (g_kernel_policy == 54 ? 33796 : 37892), st, &handled);
    if (g_kernel_policy >= 46 && g_kernel_policy <= 49 && !causal) {
      // 37 (+ static priority at 49) with: 46 single-issue f32 softmax VALU (no v_pk_*),
      // 47 waves 4-7 staggered half a tile behind waves 0-3, 48 both
      static const int kVar[4] = {9220, 17412, 25604, 21508};
      e = launch_fwd_v5(a, false, 2, 2048 + kVar[g_kernel_policy - 46], st, &handled);
    }
    if (g_kernel_policy == 97)  // diagnostics only (wrong results): no scale-and-shift
      e = launch_fwd_v5(a, causal != 0, 2, 2, st, &handled);
    if (g_kernel_policy >= 80 && g_kernel_policy <= 86 && !causal) {
      // diagnostics only (wrong results): unrolled v5 minus one component (fa_fwd_v5.hip)
      static const int kAbl[7] = {12, 28, 4, 68, 132, 260, 6};  // 82 = the default (see v5)
      e = launch_fwd_v5(a, false, 2, kAbl[g_kernel_policy - 80], st, &handled);
    }
    if (g_kernel_policy >= 91 && g_kernel_policy <= 96 && d == 64 && !causal) {
      e = launch_fwd_v4_ablation(a, g_kernel_policy - 90, st);  // diagnostics only
      handled = true;
    }
    if (g_kernel_policy == 0) {
      // v5 for non-causal N % 64 == 0. Causal v5 (policies 27-31) is correct but slower
      // than the 4-wave v4 (790 vs 811 TF/s at C3, 813 vs 836 at (1,16,16384,64)):
      // 256-query workgroups balance the triangle worse and its diagonal tiles run serially.
      // Non-causal default: 8 waves per workgroup with LDS-DMA K/V staging (policy 37:
      // 993 vs 967 TF/s for the 4-wave register-staged form, profiles/r1_ab_v5_nw8.txt).
      // Then (policy 56): the Vᵀ fragments of P2 kept in registers for P4 (+1.8 %,
      // profiles/r1_ab_v5_vkeep.txt) and each pair's row-sum add / bf16 pack one MFMA slot
      // after its exponentials (no trans-use s_nop; +2.2 % more, profiles/r1_ab_v5_defer.txt).
      if (!causal) e = launch_fwd_v5(a, false, 2, 2048 + 99332, st, &handled);
      // Causal: v4 with heavy + light query blocks paired per workgroup
      // (profiles/r1_ab_causal_pair.txt): 4 waves (policy 50) below N = 8192 (860 vs 806
      // TF/s unpaired at C3, 824 for 8 waves), 8 waves (policy 51) from there (934 vs 898
      // for 4 waves at (1,16,16384,64)). The light block of each pair runs first
      // (policies 63 / 64, profiles/r1_ab_causal_lightfirst.txt): same time (±1 %), and
      // the heavy block finds the light block's K/V tiles still in L2, so HBM traffic at C3
      // drops from 321 to 273 MB per launch (algorithmic 270 MB).
      if (!handled)
        e = launch_fwd_v4(a, causal != 0, causal && N >= 8192 ? 8 : 4, !causal, st, &handled,
                          causal ? 2 : 0);
    }
    // d = 128: the pipelined frozen-reference kernel (fa_fwd_d128.hip). Default: 8 waves
    // non-causal, 4 causal (warm-clock A/B, profiles/r1_ab_d128_warm.txt: non-causal 1085 vs
    // 1001 TF/s at (8,16,4096,128), 1143 vs 1046 at (1,16,16384,128); causal 846 vs 819).
    // 32 / 33 force 8 / 4 waves; 44 / 45 the same with LDS-DMA staging (neutral to -3 %).
    if (!handled && (g_kernel_policy == 0 || (g_kernel_policy >= 32 && g_kernel_policy <= 33) ||
                     (g_kernel_policy >= 44 && g_kernel_policy <= 45) || g_kernel_policy == 52 ||
                     g_kernel_policy == 53 || (g_kernel_policy >= 63 && g_kernel_policy <= 65))) {
      // 44 / 45: 8 / 4 waves with LDS-DMA staging; 52 / 53: causal heavy + light block
      // pairs per workgroup, 4 / 8 waves
      const int nw = (g_kernel_policy == 32 || g_kernel_policy == 44 || g_kernel_policy == 53) ? 8
                     : (g_kernel_policy == 33 || g_kernel_policy == 45 || g_kernel_policy == 52 ||
                        g_kernel_policy == 63) ? 4
                     : 8;
      // causal default: 8 waves with paired query blocks (policy 53: 944 vs 866 TF/s for
      // unpaired 4 waves at (8,16,4096,128), 1101 vs 1020 at (1,16,16384,128))
      e = launch_fwd_d128(a, causal != 0, nw, g_kernel_policy == 44 || g_kernel_policy == 45, st,
                          &handled,
                          g_kernel_policy >= 63 || (g_kernel_policy == 0 && causal) ? 2  // light first
                          : g_kernel_policy >= 52                                    ? 1
                                                                                     : 0);
    }
    // any shape the kernels above decline: the single-phase kernel, 8 waves by default
    // (faster than 4 at d = 128: 959 vs 802 TF/s at (1,16,16384,128))
    if (!handled)
      e = launch_fwd_fast(a, causal != 0, g_kernel_policy == 0 ? 2 : g_kernel_policy, st, &handled);
    if (handled) return check_hip(e, "mt_flash_attn_fwd(fast)");
  }
  return check_hip(launch_fwd_generic(a, dtype == MT_BF16, vec, causal != 0, st),
                   "mt_flash_attn_fwd");
}

int64_t mt_flash_attn_bwd_workspace_bytes(int64_t B, int64_t H, int64_t N, int64_t d) {
  (void)d;
  return 2 * B * H * N * (int64_t)sizeof(float);
}

int mt_flash_attn_bwd(int dtype, int causal, const void* q, const void* k, const void* v,
                      const void* o, const void* dout, const float* m, const float* l,
                      void* dq, void* dk, void* dv, int64_t B, int64_t H, int64_t N,
                      int64_t d, const int64_t* strides, void* workspace, void* stream) {
  if (check_sizes(dtype, B, H, N, d)) return 1;
  if (!q || !k || !v || !o || !dout || !m || !l || !dq || !dk || !dv || !workspace)
    return set_error("mt_flash_attn_bwd: null pointer argument");
  AttnArgs a;
  memset(&a, 0, sizeof(a));
  a.q = q; a.k = k; a.v = v; a.o = o; a.dout = dout;
  a.dq = dq; a.dk = dk; a.dv = dv;
  a.m = (float*)m; a.l = (float*)l;
  a.lse2 = (float*)workspace;
  a.delta = a.lse2 + B * H * N;
  int64_t* dst[8] = {a.sq, a.sk, a.sv, a.so, a.sdo, a.sdq, a.sdk, a.sdv};
  for (int i = 0; i < 8; ++i) fill_strides(dst[i], strides ? strides + 3 * i : nullptr, H, N, d);
  a.B = (int)B; a.H = (int)H; a.N = (int)N; a.d = (int)d;
  a.scale = (float)(1.0 / sqrt((double)d));
  a.scale_log2 = (float)(1.4426950408889634 / sqrt((double)d));
  const int es = dtype == MT_BF16 ? 2 : 4;
  const bool vec = vec_ok(d, es, {a.sq, a.sk, a.sv, a.so, a.sdo, a.sdq, a.sdk, a.sdv},
                          {q, k, v, o, dout, dq, dk, dv});
  if (dtype == MT_BF16 && vec && g_kernel_policy != 1) {
    bool handled = false;
    // 40: software-pipelined dK/dV (A/B variant). An in-wave interleaved dQ tile was
    // measured 1.7 % slower than the plain tile and removed (profiles/r1_ab_bwd_dq.txt).
    // dK/dV variants: 0 32-query steps, 1 software-pipelined (policy 40), 2 64-query steps
    // (policy 42). Default: 2 non-causal (1.912 vs 1.952 ms at C3), 0 causal (1.12 vs
    // 1.31 ms: the masked diagonal steps spill in the 64-query form); policy 43 forces 0.
    const int variant = g_kernel_policy == 40   ? 1
                        : g_kernel_policy == 42 ? 2
                        : g_kernel_policy == 62 ? 3  // 64-query steps, one wave per SIMD
                        : g_kernel_policy == 66 ? 4  // 64-query steps, Q / dO by LDS-DMA
                        : g_kernel_policy == 43 ? 0
                                                : (causal ? 0 : 2);
    const hipError_t e = launch_bwd_bf16(a, causal != 0, variant, (hipStream_t)stream, &handled);
    if (handled) return check_hip(e, "mt_flash_attn_bwd(bf16)");
  }
  return check_hip(launch_bwd_generic(a, dtype == MT_BF16, vec, causal != 0, (hipStream_t)stream),
                   "mt_flash_attn_bwd");
}

// ---- reference-compatible host-pointer wrappers ---------------------------------
struct DevBuf {
  void* p = nullptr;
  ~DevBuf() { if (p) (void)hipFree(p); }
};

static int host_fwd(float* Q, float* K, float* V, float* O, float* l, float* m, int B, int nh,
                    int N, int d, int causal, const char* name) {
  const size_t n = (size_t)B * nh * N * d, r = (size_t)B * nh * N;
  DevBuf dq, dk, dv, dof, dm, dl;
  if (check_hip(hipMalloc(&dq.p, n * 4), name) || check_hip(hipMalloc(&dk.p, n * 4), name) ||
      check_hip(hipMalloc(&dv.p, n * 4), name) || check_hip(hipMalloc(&dof.p, n * 4), name) ||
      check_hip(hipMalloc(&dm.p, r * 4), name) || check_hip(hipMalloc(&dl.p, r * 4), name))
    goto fail;
  if (check_hip(hipMemcpy(dq.p, Q, n * 4, hipMemcpyHostToDevice), name) ||
      check_hip(hipMemcpy(dk.p, K, n * 4, hipMemcpyHostToDevice), name) ||
      check_hip(hipMemcpy(dv.p, V, n * 4, hipMemcpyHostToDevice), name))
    goto fail;
  if (mt_flash_attn_fwd(MT_F32, causal, dq.p, dk.p, dv.p, dof.p, (float*)dm.p, (float*)dl.p, B, nh,
                        N, d, nullptr, nullptr, nullptr, nullptr, nullptr))
    goto fail;
  if (check_hip(hipDeviceSynchronize(), name) ||
      check_hip(hipMemcpy(O, dof.p, n * 4, hipMemcpyDeviceToHost), name) ||
      check_hip(hipMemcpy(m, dm.p, r * 4, hipMemcpyDeviceToHost), name) ||
      check_hip(hipMemcpy(l, dl.p, r * 4, hipMemcpyDeviceToHost), name))
    goto fail;
  return 0;
fail:
  fprintf(stderr, "%s failed: %s\n", name, g_err);
  return 1;
}

static int host_bwd(float* Q, float* K, float* V, float* O, float* dQ, float* dK, float* dV,
                    float* dO, float* l, float* m, int B, int nh, int N, int d, int causal,
                    const char* name) {
  const size_t n = (size_t)B * nh * N * d, r = (size_t)B * nh * N;
  DevBuf bufs[11];
  float* hin[5] = {Q, K, V, O, dO};
  for (int i = 0; i < 8; ++i)
    if (check_hip(hipMalloc(&bufs[i].p, n * 4), name)) goto fail;
  if (check_hip(hipMalloc(&bufs[8].p, r * 4), name) || check_hip(hipMalloc(&bufs[9].p, r * 4), name) ||
      check_hip(hipMalloc(&bufs[10].p, (size_t)mt_flash_attn_bwd_workspace_bytes(B, nh, N, d)), name))
    goto fail;
  for (int i = 0; i < 5; ++i)
    if (check_hip(hipMemcpy(bufs[i].p, hin[i], n * 4, hipMemcpyHostToDevice), name)) goto fail;
  if (check_hip(hipMemcpy(bufs[8].p, m, r * 4, hipMemcpyHostToDevice), name) ||
      check_hip(hipMemcpy(bufs[9].p, l, r * 4, hipMemcpyHostToDevice), name))
    goto fail;
  if (mt_flash_attn_bwd(MT_F32, causal, bufs[0].p, bufs[1].p, bufs[2].p, bufs[3].p, bufs[4].p,
                        (const float*)bufs[8].p, (const float*)bufs[9].p, bufs[5].p, bufs[6].p,
                        bufs[7].p, B, nh, N, d, nullptr, bufs[10].p, nullptr))
    goto fail;
  if (check_hip(hipDeviceSynchronize(), name) ||
      check_hip(hipMemcpy(dQ, bufs[5].p, n * 4, hipMemcpyDeviceToHost), name) ||
      check_hip(hipMemcpy(dK, bufs[6].p, n * 4, hipMemcpyDeviceToHost), name) ||
      check_hip(hipMemcpy(dV, bufs[7].p, n * 4, hipMemcpyDeviceToHost), name))
    goto fail;
  return 0;
fail:
  fprintf(stderr, "%s failed: %s\n", name, g_err);
  return 1;
}

void launch_flashattention_forward(float* Q, float* K, float* V, float* O, float* l, float* m,
                                   int B, int nh, int N, int d) {
  host_fwd(Q, K, V, O, l, m, B, nh, N, d, 0, "launch_flashattention_forward");
}
void launch_flashattention_forward_causal(float* Q, float* K, float* V, float* O, float* l,
                                          float* m, int B, int nh, int N, int d) {
  host_fwd(Q, K, V, O, l, m, B, nh, N, d, 1, "launch_flashattention_forward_causal");
}
void launch_flashattention_backward(float* Q, float* K, float* V, float* O, float* dQ,
                                    float* dK, float* dV, float* dO, float* l, float* m, int B,
                                    int nh, int N, int d) {
  host_bwd(Q, K, V, O, dQ, dK, dV, dO, l, m, B, nh, N, d, 0, "launch_flashattention_backward");
}
void launch_flashattention_backward_causal(float* Q, float* K, float* V, float* O, float* dQ,
                                           float* dK, float* dV, float* dO, float* l,
                                           float* m, int B, int nh, int N, int d) {
  host_bwd(Q, K, V, O, dQ, dK, dV, dO, l, m, B, nh, N, d, 1,
           "launch_flashattention_backward_causal");
}

}  // extern "C"
