// Generic strided tensor kernels for the minitorch backend: map, zip, reduce and
// batched matmul on device-resident fp32 storage.
//
// Counterpart of the reference's combine.cu (map/zip/reduce :213-310, MatrixMultiply
// :148-210, C ABI :315-580). Function ids are the reference's (combine.cu:12-29) so its
// fn_map (cuda_kernel_ops.py:33-53) indexes this library unchanged; the scalar
// functions follow minitorch/operators.py (log and log_back add EPS = 1e-6, sigmoid is
// the two-sided stable form, is_close |x - y| < 1e-2).
//
// MI355X design: device pointers and stream-ordered launches (the reference copies
// every operand host<->device per call), int64 indexing, grid-stride loops sized for
// 256 CUs, a contiguous fast path, wave-per-row reductions for long reduce axes. The
// batched matmul is a plain library GEMM: rocBLAS sgemm_strided_batched whenever each
// operand has a unit stride in one of its two dims (every Linear / attention / one-hot
// product of the model), else our own exact-fp32 MFMA kernel (v_mfma_f32_32x32x2_f32)
// for arbitrary strides.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <vector>

#include <rocblas/rocblas.h>

#include "../../include/minitorch_hip.h"
#include "fa_common.h"

namespace mt {

int set_error(const char* fmt, ...);
int check_hip(hipError_t e, const char* where);

constexpr int kMaxDims = 8;

struct Layout {
  int64_t shape[kMaxDims];
  int64_t strides[kMaxDims];
  int dims;
  int contiguous;
};

enum FnId {
  FN_ADD = 1, FN_MUL = 2, FN_ID = 3, FN_NEG = 4, FN_LT = 5, FN_EQ = 6, FN_SIGMOID = 7,
  FN_RELU = 8, FN_RELU_BACK = 9, FN_LOG = 10, FN_LOG_BACK = 11, FN_EXP = 12, FN_INV = 13,
  FN_INV_BACK = 14, FN_IS_CLOSE = 15, FN_MAX = 16, FN_POW = 17, FN_TANH = 18
};

__device__ __forceinline__ float apply_fn(int fn, float x, float y) {
  switch (fn) {
    case FN_ADD: return x + y;
    case FN_MUL: return x * y;
    case FN_ID: return x;
    case FN_NEG: return -x;
    case FN_LT: return x < y ? 1.f : 0.f;
    case FN_EQ: return x == y ? 1.f : 0.f;
    case FN_SIGMOID: return x >= 0.f ? 1.f / (1.f + expf(-x)) : expf(x) / (1.f + expf(x));
    case FN_RELU: return x > 0.f ? x : 0.f;
    case FN_RELU_BACK: return x > 0.f ? y : 0.f;
    case FN_LOG: return logf(x + 1e-6f);
    case FN_LOG_BACK: return y / (x + 1e-6f);
    case FN_EXP: return expf(x);
    case FN_INV: return 1.f / x;
    case FN_INV_BACK: return -(1.f / (x * x)) * y;
    case FN_IS_CLOSE: return (x - y < 1e-2f) && (y - x < 1e-2f) ? 1.f : 0.f;
    case FN_MAX: return x > y ? x : y;
    case FN_POW: return powf(x, y);
    case FN_TANH: return tanhf(x);
    default: return __builtin_nanf("");
  }
}

// Position in `in` of the element broadcast to out-ordinal i (shapes right-aligned). I: the
// index type, int32 whenever every ordinal and offset fits (host-checked): the 64-bit
// division per dimension is a long software sequence on the GPU, and it made the strided
// copies and broadcasts of the minitorch step several times slower than their bytes.
template <typename I>
__device__ __forceinline__ I bcast_pos(I i, const Layout& out, const Layout& in) {
  I pos = 0;
  const int off = out.dims - in.dims;
  for (int d = out.dims - 1; d >= 0; --d) {
    const I sh = (I)out.shape[d];
    const I q = i / sh;
    const I idx = i - q * sh;
    i = q;
    const int e = d - off;
    if (e >= 0 && in.shape[e] != 1) pos += idx * (I)in.strides[e];
  }
  return pos;
}
template <typename I>
__device__ __forceinline__ I out_pos(I i, const Layout& out) {
  if (out.contiguous) return i;
  I pos = 0;
  for (int d = out.dims - 1; d >= 0; --d) {
    const I sh = (I)out.shape[d];
    const I q = i / sh;
    pos += (i - q * sh) * (I)out.strides[d];
    i = q;
  }
  return pos;
}

template <typename I>
__global__ __launch_bounds__(256) void map_kernel(int fn, float* out, Layout ol, int64_t n,
                                                  const float* in, Layout il, int same) {
  const I step = (I)gridDim.x * blockDim.x;
  for (I i = (I)blockIdx.x * blockDim.x + threadIdx.x; i < (I)n; i += step) {
    const float x = same ? in[i] : in[bcast_pos<I>(i, ol, il)];
    out[same ? i : out_pos<I>(i, ol)] = apply_fn(fn, x, 0.f);
  }
}

template <typename I>
__global__ __launch_bounds__(256) void zip_kernel(int fn, float* out, Layout ol, int64_t n,
                                                  const float* a, Layout al, const float* b,
                                                  Layout bl, int same) {
  const I step = (I)gridDim.x * blockDim.x;
  for (I i = (I)blockIdx.x * blockDim.x + threadIdx.x; i < (I)n; i += step) {
    const float x = same ? a[i] : a[bcast_pos<I>(i, ol, al)];
    const float y = same ? b[i] : b[bcast_pos<I>(i, ol, bl)];
    out[same ? i : out_pos<I>(i, ol)] = apply_fn(fn, x, y);
  }
}

// Dense fast paths (16 B per lane where the sizes allow): every operand contiguous in the
// output's order, the second operand either the same shape (BMODE 0), one element (1), or a
// contiguous block repeated along the leading dims (2: out[i] op b[i % nb], a bias row);
// SWAP puts the repeated operand on the left.
template <int BMODE, bool SWAP>
__global__ __launch_bounds__(256) void zip_dense_kernel(int fn, float* __restrict__ out, int64_t n,
                                                        const float* __restrict__ a,
                                                        const float* __restrict__ b, int64_t nb) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const float b0 = BMODE == 1 ? b[0] : 0.f;
  if (n % 4 == 0 && (BMODE != 2 || nb % 4 == 0)) {
    const float4* a4 = (const float4*)a;
    float4* o4 = (float4*)out;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += step) {
      const float4 x = a4[i];
      float4 y;
      if (BMODE == 0) y = ((const float4*)b)[i];
      else if (BMODE == 1) y = make_float4(b0, b0, b0, b0);
      else y = ((const float4*)b)[i % (nb / 4)];
      float4 r;
      r.x = SWAP ? apply_fn(fn, y.x, x.x) : apply_fn(fn, x.x, y.x);
      r.y = SWAP ? apply_fn(fn, y.y, x.y) : apply_fn(fn, x.y, y.y);
      r.z = SWAP ? apply_fn(fn, y.z, x.z) : apply_fn(fn, x.z, y.z);
      r.w = SWAP ? apply_fn(fn, y.w, x.w) : apply_fn(fn, x.w, y.w);
      o4[i] = r;
    }
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
    const float x = a[i];
    const float y = BMODE == 0 ? b[i] : BMODE == 1 ? b0 : b[i % nb];
    out[i] = SWAP ? apply_fn(fn, y, x) : apply_fn(fn, x, y);
  }
}
__global__ __launch_bounds__(256) void map_dense_kernel(int fn, float* __restrict__ out, int64_t n,
                                                        const float* __restrict__ a) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  if (n % 4 == 0) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += step) {
      const float4 x = ((const float4*)a)[i];
      ((float4*)out)[i] = make_float4(apply_fn(fn, x.x, 0.f), apply_fn(fn, x.y, 0.f),
                                      apply_fn(fn, x.z, 0.f), apply_fn(fn, x.w, 0.f));
    }
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step)
    out[i] = apply_fn(fn, a[i], 0.f);
}

// out has a's shape with shape[dim] = 1. One wave per output element (lanes stride the
// reduce axis, then a butterfly); short axes use one lane per output instead.
__global__ __launch_bounds__(256) void reduce_wave_kernel(int fn, float* out, Layout ol,
                                                          int64_t n_out, const float* a,
                                                          Layout al, int dim, float start) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t len = al.shape[dim], st = al.strides[dim];
  for (int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); o < n_out; o += nw) {
    const int64_t base = bcast_pos<int64_t>(o, ol, al);  // out and a share shapes except dim (=1)
    float acc = 0.f;
    bool have = false;
    for (int64_t j = lane; j < len; j += 64) {
      const float x = a[base + j * st];
      acc = have ? apply_fn(fn, acc, x) : x;
      have = true;
    }
    // Butterfly over the lanes that saw elements; `start` is applied once at the end.
    for (int off = 32; off > 0; off >>= 1) {
      const float y = __shfl_xor(acc, off);
      const bool hy = __shfl_xor((int)have, off) != 0;
      if (hy) acc = have ? apply_fn(fn, acc, y) : y;
      have = have || hy;
    }
    if (lane == 0) out[out_pos<int64_t>(o, ol)] = have ? apply_fn(fn, start, acc) : start;
  }
}
// Few outputs over a long axis (the loss sums of config 5: 4992 -> 1, where one wave per output
// ran 23 µs): one 1024-thread workgroup per output, 8 loads in flight per lane, the lanes'
// partials folded by a butterfly per wave and then in wave order through LDS (deterministic).
template <int FN>
__global__ __launch_bounds__(1024) void reduce_block_kernel(int fn_rt, float* out, Layout ol, const float* a,
                                                            Layout al, int dim, float start) {
  const int fn = FN >= 0 ? FN : fn_rt;
  __shared__ float wsum[16];
  __shared__ int whave[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t o = blockIdx.x;
  const int64_t len = al.shape[dim], st = al.strides[dim];
  const int64_t base = bcast_pos<int64_t>(o, ol, al);
  float acc = 0.f;
  bool have = false;
  for (int64_t j0 = threadIdx.x; j0 < len; j0 += 8 * 1024) {
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = a[base + min(j0 + (int64_t)u * 1024, len - 1) * st];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (j0 + (int64_t)u * 1024 >= len) break;
      acc = have ? apply_fn(fn, acc, x[u]) : x[u];
      have = true;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const float y = __shfl_xor(acc, off);
    const bool hy = __shfl_xor((int)have, off) != 0;
    if (hy) acc = have ? apply_fn(fn, acc, y) : y;
    have = have || hy;
  }
  if (lane == 0) { wsum[w] = acc; whave[w] = have; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = 0.f;
    bool hv = false;
    for (int k = 0; k < 16; ++k) {
      if (!whave[k]) continue;
      v = hv ? apply_fn(fn, v, wsum[k]) : wsum[k];
      hv = true;
    }
    out[out_pos<int64_t>(o, ol)] = hv ? apply_fn(fn, start, v) : start;
  }
}
__global__ __launch_bounds__(256) void reduce_thread_kernel(int fn, float* out, Layout ol,
                                                            int64_t n_out, const float* a,
                                                            Layout al, int dim, float start) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int64_t len = al.shape[dim], st = al.strides[dim];
  for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < n_out; o += step) {
    const int64_t base = bcast_pos<int64_t>(o, ol, al);
    float acc = start;
    for (int64_t j = 0; j < len; ++j) acc = apply_fn(fn, acc, a[base + j * st]);
    out[out_pos<int64_t>(o, ol)] = acc;
  }
}

// Column reductions (a contiguous [outer][len][inner] tensor reduced over len with inner >= 16:
// the bias gradients, column sums of [rows, cols] activations such as the LM head's 4992 x
// 10000). The columns are split into 64-wide blocks and the rows into R chunks, so the grid
// fills the chip even for 256 columns (one workgroup per column block ran 4 workgroups
// there: 100 µs per 4992 x 256 sum). Workgroup (column block, chunk): 16 waves over the
// chunk's rows (a wave reads 64 consecutive floats of a row: coalesced), folded in wave order
// through LDS into the chunk's partial; reduce_cols_fold then folds the R <= 16 partials of
// each column in chunk order (fixed order: deterministic). R = 1 writes the result directly.
// Both kernels are latency-bound at these sizes (5 MB for a 4992 x 256 sum; 14 + 12 µs at
// C5): the fold issues all its loads unconditionally (clamped indices) before it folds, and
// each extra round of 16 partial loads cost it ≈ 5 µs (R = 39 chunks of 128 rows: 22 µs).
constexpr int kColRMax = 16;
__global__ __launch_bounds__(1024) void reduce_cols_kernel(int fn, float* __restrict__ out,
                                                           float* __restrict__ part_out,
                                                           int* __restrict__ have_out,
                                                           const float* __restrict__ a, int64_t len,
                                                           int64_t inner, int64_t chunk, float start) {
  __shared__ float part[16][64];
  __shared__ int have_s[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + tx;
  const int r = blockIdx.y, R = gridDim.y, o = blockIdx.z;
  const float* src = a + (int64_t)o * len * inner + i;
  const int64_t j0 = (int64_t)r * chunk, j1 = min(len, j0 + chunk);
  float acc = 0.f;
  bool have = false;
  if (i < inner) {
#pragma unroll 8
    for (int64_t j = j0 + ty; j < j1; j += 16) {
      const float x = src[j * inner];
      acc = have ? apply_fn(fn, acc, x) : x;
      have = true;
    }
  }
  part[ty][tx] = acc;
  have_s[ty][tx] = have;
  __syncthreads();
  if (ty == 0 && i < inner) {
    float v = 0.f;
    bool hv = false;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (!have_s[k][tx]) continue;
      v = hv ? apply_fn(fn, v, part[k][tx]) : part[k][tx];
      hv = true;
    }
    if (R == 1) {
      out[(int64_t)o * inner + i] = hv ? apply_fn(fn, start, v) : start;
    } else {
      const int64_t w = ((int64_t)o * R + r) * inner + i;
      part_out[w] = v;
      have_out[w] = hv;
    }
  }
}
__global__ __launch_bounds__(256) void reduce_cols_fold(int fn, float* __restrict__ out,
                                                        const float* __restrict__ part,
                                                        const int* __restrict__ have, int64_t inner,
                                                        int R, int64_t n, float start) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  const int64_t o = t / inner, i = t % inner;
  const float* p = part + o * R * inner + i;
  const int* h = have + o * R * inner + i;
  float v = 0.f;
  bool hv = false;
#pragma unroll
  for (int r0 = 0; r0 < kColRMax; r0 += 16) {
    if (r0 >= R) break;
    float x[16];
    int hx[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {  // 16 loads in flight, then the ordered fold
      const int64_t rr = min(r0 + r, R - 1);
      x[r] = p[rr * inner];
      hx[r] = h[rr * inner];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (r0 + r >= R || !hx[r]) continue;
      v = hv ? apply_fn(fn, v, x[r]) : x[r];
      hv = true;
    }
  }
  out[t] = hv ? apply_fn(fn, start, v) : start;
}

// Column-group reduction (round 5) for [outer][len][inner], inner % 4 = 0, 16-byte aligned rows,
// len up to 8192: one workgroup owns 4 adjacent columns (a float4 per row) over ALL rows, so no
// partial ever leaves the workgroup: no scratch, no fence, no arrival counter. Lane t takes rows
// t, t + T, ... (8 loads in flight) and folds them in row order; the T lane values fold by a
// fixed pairwise tree through LDS: deterministic. Each load instruction of a
// wave touches 64 rows, one 16-B piece of each 128-B line; the 8 column groups sharing a line are
// placed on one XCD (blockIdx % 8 picks the XCD), so each line still comes from HBM once.
// Config 5's 4992 x 256 bias gradient: 4.8 µs against 9.1 µs for the one-pass chunked form,
// whose cross-XCD hand-off (release fence, agent atomic, acquire, fold) alone costs 6.4 µs
// (scripts/colsum_bench.hip).
__device__ __forceinline__ void fold4(int fn, float4& v, bool& hv, const float4& y, bool hy) {
  if (!hy) return;
  if (!hv) { v = y; hv = true; return; }
  v.x = apply_fn(fn, v.x, y.x); v.y = apply_fn(fn, v.y, y.y);
  v.z = apply_fn(fn, v.z, y.z); v.w = apply_fn(fn, v.w, y.w);
}
template <int FN>
__global__ __launch_bounds__(1024) void reduce_colgroup_kernel(int fn_rt, float* __restrict__ out,
                                                               const float* __restrict__ a, int64_t len,
                                                               int64_t inner, int ncg, int xcd_map,
                                                               float start) {
  const int fn = FN >= 0 ? FN : fn_rt;
  __shared__ float4 red[1024];
  const int b = blockIdx.x, o = blockIdx.y;
  // xcd_map: the 8 groups of line L sit at blockIdx b with b % 8 == L % 8
  const int cg = xcd_map ? (((b & 7) + 8 * ((b >> 3) >> 3)) * 8 + ((b >> 3) & 7)) : b;
  if (cg >= ncg) return;  // padding workgroups of the XCD map: uniform, before any barrier
  const int t = threadIdx.x, T = blockDim.x;  // T = min(1024, len)
  const float* src = a + (int64_t)o * len * inner + (int64_t)cg * 4;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  bool hv = false;
  for (int64_t j = t; j < len; j += 8 * (int64_t)T) {
    float4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)  // masked, not clamped: a load instruction costs per row it touches
      x[u] = j + (int64_t)u * T < len ? *(const float4*)(src + (j + (int64_t)u * T) * inner)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 8; ++u) fold4(fn, v, hv, x[u], j + (int64_t)u * T < len);
  }
  // every lane holds at least one row (T <= len): a fixed pairwise tree through LDS
  // (measured 1 µs faster than a shuffle butterfly plus a wave-order fold at 4992 x 256)
  red[t] = v;
  __syncthreads();
  int p2 = 1;
  while (p2 < T) p2 <<= 1;
  for (int s = p2 >> 1; s > 0; s >>= 1) {
    if (t < s && t + s < T) {
      float4 x = red[t];
      const float4 y = red[t + s];
      x.x = apply_fn(fn, x.x, y.x); x.y = apply_fn(fn, x.y, y.y);
      x.z = apply_fn(fn, x.z, y.z); x.w = apply_fn(fn, x.w, y.w);
      red[t] = x;
    }
    __syncthreads();
  }
  if (t == 0) {
    float4 r = red[0];
    r.x = apply_fn(fn, start, r.x); r.y = apply_fn(fn, start, r.y);
    r.z = apply_fn(fn, start, r.z); r.w = apply_fn(fn, start, r.w);
    *(float4*)(out + (int64_t)o * inner + (int64_t)cg * 4) = r;
  }
}

// One-pass column reduction (round 5) for [outer][len][inner] with inner % 4 = 0 and 16-byte
// aligned rows: workgroup (column block of 256, row chunk r, outer o) has 8 waves; a lane owns 4
// adjacent columns (float4 loads: a wave reads one 1 KiB row segment per load) and a wave takes
// every 8th row of the chunk, 8 loads in flight; the 8 wave partials fold through LDS in wave
// order. With R > 1 chunks the chunk's partial goes to the scratch, the workgroup counts its
// arrival on the column block's counter (agent scope, after a release fence), and the last of
// the R arrivals folds the R partials in chunk order (8 waves over consecutive chunk ranges, then
// in wave order through LDS), writes the result and resets the counter for the next launch.
// Fixed association for a given shape: deterministic. Replaces the reduce + fold pair at config
// 5's bias gradients (4992 x 256: 16.6 + 8.6 µs per call in the C5 step, scripts/reduce_probe.py).
constexpr int kCol1Waves = 8;
template <int FN>  // FN >= 0: the op folded in at compile time (add, mul, max); -1: fn at run time
__global__ __launch_bounds__(512) void reduce_cols1_kernel(int fn_rt, float* __restrict__ out,
                                                           float* __restrict__ part,
                                                           unsigned* __restrict__ counters,
                                                           const float* __restrict__ a, int64_t len,
                                                           int64_t inner, int64_t chunk, float start) {
  const int fn = FN >= 0 ? FN : fn_rt;
  __shared__ float4 red[kCol1Waves][64];
  __shared__ int have_s[kCol1Waves];
  __shared__ int last_s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cbn = gridDim.x, R = gridDim.y, r = blockIdx.y, o = blockIdx.z;
  const int64_t col = (int64_t)blockIdx.x * 256 + lane * 4;
  const bool live = col < inner;
  const int64_t j0 = (int64_t)r * chunk, j1 = min(len, j0 + chunk);
  const float* src = a + (int64_t)o * len * inner + col;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  bool have = false;
  if (live) {
    for (int64_t j = j0 + w; j < j1; j += 8 * kCol1Waves) {
      float4 x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {  // 8 loads in flight (clamped rows, folded only when in range)
        const int64_t jj = min(j + (int64_t)u * kCol1Waves, j1 - 1);
        x[u] = *(const float4*)(src + jj * inner);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (j + (int64_t)u * kCol1Waves >= j1) break;
        if (!have) { acc = x[u]; have = true; continue; }
        acc.x = apply_fn(fn, acc.x, x[u].x); acc.y = apply_fn(fn, acc.y, x[u].y);
        acc.z = apply_fn(fn, acc.z, x[u].z); acc.w = apply_fn(fn, acc.w, x[u].w);
      }
    }
  }
  red[w][lane] = acc;
  if (lane == 0) have_s[w] = have;
  __syncthreads();
  if (w == 0) {
    float4 v = red[0][lane];  // wave 0 always has a row: every chunk holds at least one
    for (int k = 1; k < kCol1Waves; ++k) {
      if (!have_s[k]) break;  // waves past the chunk's last row
      const float4 y = red[k][lane];
      v.x = apply_fn(fn, v.x, y.x); v.y = apply_fn(fn, v.y, y.y);
      v.z = apply_fn(fn, v.z, y.z); v.w = apply_fn(fn, v.w, y.w);
    }
    if (R == 1) {
      if (live) {
        v.x = apply_fn(fn, start, v.x); v.y = apply_fn(fn, start, v.y);
        v.z = apply_fn(fn, start, v.z); v.w = apply_fn(fn, start, v.w);
        *(float4*)(out + (int64_t)o * inner + col) = v;
      }
    } else {
      if (live) *(float4*)(part + ((int64_t)o * R + r) * inner + col) = v;
      __threadfence();  // release the partial at agent scope before the arrival
      if (lane == 0) {
        const unsigned prev = __hip_atomic_fetch_add(counters + (int64_t)o * cbn + blockIdx.x, 1u,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_s = prev == (unsigned)(R - 1);
      }
    }
  }
  if (R == 1) return;  // uniform: every wave leaves before the second barrier
  __syncthreads();
  if (!last_s) return;
  __threadfence();  // acquire: the other chunks' partials
  const int per = (R + kCol1Waves - 1) / kCol1Waves;
  const int r0 = w * per, r1 = min(R, r0 + per);
  const float* p = part + (int64_t)o * R * inner + col;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live && r0 < r1) {
    // the partials come from other XCDs' workgroups (misses in this XCD's L2): 16 loads in
    // flight per batch, folded in chunk order, instead of one dependent miss per partial
    v = *(const float4*)(p + (int64_t)r0 * inner);
    for (int q = r0 + 1; q < r1; q += 16) {
      float4 y[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) y[u] = *(const float4*)(p + (int64_t)min(q + u, r1 - 1) * inner);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        if (q + u < r1) {
          v.x = apply_fn(fn, v.x, y[u].x); v.y = apply_fn(fn, v.y, y[u].y);
          v.z = apply_fn(fn, v.z, y[u].z); v.w = apply_fn(fn, v.w, y[u].w);
        }
      }
    }
  }
  red[w][lane] = v;
  if (lane == 0) have_s[w] = r0 < r1;
  __syncthreads();
  if (w == 0) {
    float4 t = red[0][lane];
    for (int k = 1; k < kCol1Waves; ++k) {
      if (!have_s[k]) break;
      const float4 y = red[k][lane];
      t.x = apply_fn(fn, t.x, y.x); t.y = apply_fn(fn, t.y, y.y);
      t.z = apply_fn(fn, t.z, y.z); t.w = apply_fn(fn, t.w, y.w);
    }
    if (live) {
      t.x = apply_fn(fn, start, t.x); t.y = apply_fn(fn, start, t.y);
      t.z = apply_fn(fn, start, t.z); t.w = apply_fn(fn, start, t.w);
      *(float4*)(out + (int64_t)o * inner + col) = t;
    }
    if (lane == 0) counters[(int64_t)o * cbn + blockIdx.x] = 0u;  // ready for the next launch
  }
}

namespace {
struct ScratchSlot { int pool; int dev; hipStream_t st; void* buf; size_t cap; bool captured; };
std::mutex g_scratch_mu;
ScratchSlot g_scratch[128] = {};
int g_nscratch = 0;
// buffers a stream capture was handed and then outgrown: a captured hipGraph replays with the
// address it was captured with, so they stay allocated for the life of the process
std::vector<std::pair<void*, size_t>> g_scratch_kept;
}  // namespace

void* stream_scratch(int pool, size_t bytes, hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return nullptr;
  const bool capturing = cs != hipStreamCaptureStatusNone;
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  ScratchSlot* s = nullptr;
  for (int i = 0; i < g_nscratch && !s; ++i)
    if (g_scratch[i].pool == pool && g_scratch[i].dev == dev && g_scratch[i].st == st) s = &g_scratch[i];
  if (!s) {
    if (g_nscratch == 128) return nullptr;  // the caller then takes its path without scratch
    s = &g_scratch[g_nscratch++];
    *s = ScratchSlot{pool, dev, st, nullptr, 0, false};
  }
  if (s->cap < bytes) {
    if (capturing) return nullptr;  // no allocation inside a capture
    // the reduction pool doubles (many small, growing asks); the padded-copy pool takes the
    // exact size (its callers chunk to at most kPadScratchCap bytes)
    if (pool != kScratchPad) bytes = std::max(bytes, 2 * s->cap);
    if (s->buf) {
      if (s->captured) {
        g_scratch_kept.emplace_back(s->buf, s->cap);
      } else {
        // nothing but this stream's pending work can use it: free it once that has run
        if (hipStreamSynchronize(st) != hipSuccess) return nullptr;
        (void)hipFree(s->buf);
      }
      s->buf = nullptr;
      s->cap = 0;
      s->captured = false;
    }
    void* nb = nullptr;
    if (hipMalloc(&nb, bytes) != hipSuccess) return nullptr;
    s->buf = nb;
    s->cap = bytes;
  }
  if (capturing) s->captured = true;
  return s->buf;
}

static void* reduce_scratch(size_t bytes, hipStream_t st) { return stream_scratch(kScratchReduce, bytes, st); }

// Arrival counters of the one-pass column reduction, one zeroed block per (device, stream),
// allocated once outside any capture; each launch's last arrivals reset the counters they used.
constexpr int64_t kColCounters = 1 << 16;
static unsigned* reduce_counters(hipStream_t st) {
  struct Slot { int dev; hipStream_t st; unsigned* buf; };
  static std::mutex mu;
  static Slot slots[64] = {};
  static int nslots = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  for (int i = 0; i < nslots; ++i)
    if (slots[i].dev == dev && slots[i].st == st) return slots[i].buf;
  if (nslots == 64) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  unsigned* b = nullptr;
  if (hipMalloc(&b, kColCounters * sizeof(unsigned)) != hipSuccess) return nullptr;
  // zeroed in the stream's own order: a legacy hipMemset need not precede work on a non-blocking
  // stream (torch's side streams), and a counter left at garbage never elects a last arrival
  if (hipMemsetAsync(b, 0, kColCounters * sizeof(unsigned), st) != hipSuccess) { (void)hipFree(b); return nullptr; }
  slots[nslots++] = Slot{dev, st, b};
  return b;
}

// Batched GEMM C[b] = A[b] @ B[b], fp32, exact fp32 MFMA. A: [M,K], B: [K,N], C: [M,N],
// arbitrary element strides; batch stride 0 broadcasts. 64x64 output tile per 256-thread
// workgroup (4 waves, 32x32 each), K staged 16 at a time through LDS.
struct GemmArgs {
  const float* a; const float* b; float* c;
  int64_t M, N, K;
  int64_t sab, sam, sak, sbb, sbk, sbn, scb, scm, scn;
};

__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs g) {
  constexpr int BM = 64, BN = 64, BK = 16, LDT = BK + 4;
  __shared__ __attribute__((aligned(16))) float sA[BM * LDT];
  __shared__ __attribute__((aligned(16))) float sB[BN * LDT];  // Bᵀ tile: [n][k]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t bz = blockIdx.z;
  const int64_t m0 = (int64_t)blockIdx.y * BM, n0 = (int64_t)blockIdx.x * BN;
  const float* A = g.a + bz * g.sab;
  const float* B = g.b + bz * g.sbb;
  f32x16 acc = f32x16{};
  for (int64_t k0 = 0; k0 < g.K; k0 += BK) {
    __syncthreads();
    for (int e = tid; e < BM * BK; e += 256) {
      const int r = e / BK, kk = e % BK;
      const int64_t gm = m0 + r, gk = k0 + kk;
      sA[r * LDT + kk] = (gm < g.M && gk < g.K) ? A[gm * g.sam + gk * g.sak] : 0.f;
      const int64_t gn = n0 + r;
      sB[r * LDT + kk] = (gn < g.N && gk < g.K) ? B[gk * g.sbk + gn * g.sbn] : 0.f;
    }
    __syncthreads();
    const f32x8 af = row_frag<float>(sA + (wm * 32 + c32) * LDT + 8 * hf);
    const f32x8 bf = row_frag<float>(sB + (wn * 32 + c32) * LDT + 8 * hf);
    mma(acc, af, bf);
  }
  // acc: column (n) on the lane, rows (m) acc_row(r, hf).
  float* C = g.c + bz * g.scb;
  const int64_t gn = n0 + wn * 32 + c32;
  if (gn < g.N) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t gm = m0 + wm * 32 + acc_row(r, hf);
      if (gm < g.M) C[gm * g.scm + gn * g.scn] = acc[r];
    }
  }
}

// Batched fp32 GEMM C[b] = A[b]·B[b] on the bf16 MFMA with every operand in three bf16 pieces
// (fa_common.h mma_x3: six v_mfma_f32_32x32x16_bf16 per 16-deep k step, fp32 accuracy, 2.67x
// the v_mfma_f32_32x32x2_f32 rate; the flash kernels' fp32 path uses the same split). A 64x64
// tile per 256-thread workgroup (2 x 2 waves of 32x32), K staged 32 at a time: every thread
// loads two 16-B chunks of A and of B along each operand's unit-stride dimension into
// registers one stage ahead, splits them and writes 8 B per chunk to each of the three bf16
// planes of a two-stage LDS ring. An operand contiguous along k (AK / BK) keeps planes
// [row][k] and its MFMA fragment is two 8-B row reads; one contiguous along m (A) or n (B) keeps
// planes [k][row] read by ds_read_b64_tr_b16 (the flash kernels' transposed V reads). Both take
// the k order of that transposed read (element j of lane half h: k = 8 (j >> 2) + 4 h + (j & 3)),
// so A and B agree. The MFMA accumulator is flushed into an fp32 register sum every 256 k (a
// VALU add), so no single MFMA accumulation chain grows with K. Split-K: slice z % S covers k in
// [slice·ks, (slice+1)·ks) and writes C (S = 1) or its own [S][M][N] partial (gemm_slice_sum).
struct GemmX3Args {
  const float* a; const float* b; float* c;
  int64_t M, N, K, ks;  // ks: k per slice
  int64_t sab, sam, sak, sbb, sbk, sbn, scb, scm, scn;
  int S;
};
constexpr int kGxLDK = 40;                 // [row][k] plane row: 32 k + 8
constexpr int kGxLDR = 72;                 // [k][row] plane row: 64 rows + 8
constexpr int kGxPlane = 64 * kGxLDK;      // one plane (bf16 elements; 32 x 72 = 2304 fits too)
constexpr int kGxStage = 6 * kGxPlane;     // A h, m, l then B h, m, l
static_assert(32 * kGxLDR <= kGxPlane, "plane size");
template <bool AK, bool BK, bool VEC>
__global__ __launch_bounds__(256, 2) void gemm_x3_kernel(GemmX3Args g) {
  __shared__ __attribute__((aligned(16))) bf16 sm[2 * kGxStage];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t bz = blockIdx.z / g.S, slice = blockIdx.z % g.S;
  const int64_t m0 = (int64_t)blockIdx.y * 64, n0 = (int64_t)blockIdx.x * 64;
  const float* A = g.a + bz * g.sab;
  const float* B = g.b + bz * g.sbb;
  const int64_t kbeg = slice * g.ks, kend = min(g.K, kbeg + g.ks);
  // 16-B chunk c of an operand tile: along k (KC): row c / 8, k 4 (c % 8); along the rows:
  // k c / 16, rows 4 (c % 16)
  auto chunk = [&](const float* base, int64_t rs, int64_t rlim, int64_t r, int64_t k, bool kc) -> float4 {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t lim = kc ? kend : rlim;  // the contiguous dimension's end
    const int64_t i0 = kc ? k : r;         // its index
    if ((kc ? r >= rlim : k >= kend)) return v;
    const float* p = base + (kc ? r * rs + k : k * rs + r);
    if (VEC && i0 + 3 < lim) return *(const float4*)p;
    if (i0 < lim) v.x = p[0];
    if (i0 + 1 < lim) v.y = p[1];
    if (i0 + 2 < lim) v.z = p[2];
    if (i0 + 3 < lim) v.w = p[3];
    return v;
  };
  float4 ra[2], rb[2];
  auto load = [&](int64_t k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      ra[i] = AK ? chunk(A, g.sam, g.M, m0 + c / 8, k0 + 4 * (c % 8), true)
                 : chunk(A, g.sak, g.M, m0 + 4 * (c % 16), k0 + c / 16, false);
      rb[i] = BK ? chunk(B, g.sbn, g.N, n0 + c / 8, k0 + 4 * (c % 8), true)
                 : chunk(B, g.sbk, g.N, n0 + 4 * (c % 16), k0 + c / 16, false);
    }
  };
  auto store = [&](int st) __attribute__((always_inline)) {
    bf16* base = sm + st * kGxStage;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
#pragma unroll
      for (int op = 0; op < 2; ++op) {
        const float4 v = op ? rb[i] : ra[i];
        const bool kc = op ? BK : AK;
        unsigned h0, m0_, l0, h1, m1, l1;
        x3_split2(v.x, v.y, h0, m0_, l0);
        x3_split2(v.z, v.w, h1, m1, l1);
        bf16* pl = base + 3 * op * kGxPlane + (kc ? (c / 8) * kGxLDK + 4 * (c % 8) : (c / 16) * kGxLDR + 4 * (c % 16));
        *(uint2*)(pl) = make_uint2(h0, h1);
        *(uint2*)(pl + kGxPlane) = make_uint2(m0_, m1);
        *(uint2*)(pl + 2 * kGxPlane) = make_uint2(l0, l1);
      }
    }
  };
  // the fragment of k step ks for row `row` (m or n) of a plane: row reads or transposed reads
  typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
  auto frag = [&](const bf16* pl, int row, int ks, bool kc) -> bf16x8 {
    if (kc) {
      const bf16* q = pl + row * kGxLDK + 16 * ks + 4 * hf;
      const u32x2 lo = *(const u32x2*)q, hi = *(const u32x2*)(q + 8);
      const unsigned u[4] = {lo[0], lo[1], hi[0], hi[1]};
      return __builtin_bit_cast(bf16x8, u);
    }
    return col_frag<bf16>(pl, kGxLDR, 16 * ks + 4 * hf, row - c32, lane);
  };
  f32x16 tot = f32x16{}, acc = f32x16{};
  const int nst = (int)((kend - kbeg + 31) / 32);
  if (nst > 0) {
    load(kbeg);
    store(0);
    if (nst > 1) load(kbeg + 32);
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const bf16* base = sm + (st & 1) * kGxStage;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ra_ = wm * 32 + c32, rb_ = wn * 32 + c32;
      X3Frag fa, fb;
      fa.h = frag(base, ra_, ks, AK);
      fa.m = frag(base + kGxPlane, ra_, ks, AK);
      fa.l = frag(base + 2 * kGxPlane, ra_, ks, AK);
      fb.h = frag(base + 3 * kGxPlane, rb_, ks, BK);
      fb.m = frag(base + 4 * kGxPlane, rb_, ks, BK);
      fb.l = frag(base + 5 * kGxPlane, rb_, ks, BK);
      // C[m][n] += A[m][k]·B[k][n]: A's row m as the A operand, B's column n as the B operand
      mma_x3(acc, fa, fb);
    }
    if ((st & 7) == 7 || st + 1 == nst) {  // flush every 256 k
#pragma unroll
      for (int r = 0; r < 16; ++r) tot[r] += acc[r];
      acc = f32x16{};
    }
    if (st + 1 < nst) {
      store((st + 1) & 1);
      if (st + 2 < nst) load(kbeg + 32 * (st + 2));
    }
    __syncthreads();
  }
  // tot: column n0 + 32 wn + c32 on the lane, rows m0 + 32 wm + acc_row(r, hf)
  const int64_t gn = n0 + wn * 32 + c32;
  if (gn >= g.N) return;
  float* C = g.c + (g.S > 1 ? slice * g.M * g.N : bz * g.scb);
  const int64_t scm = g.S > 1 ? g.N : g.scm, scn = g.S > 1 ? 1 : g.scn;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t gm = m0 + wm * 32 + acc_row(r, hf);
    if (gm < g.M) C[gm * scm + gn * scn] = tot[r];
  }
}

// The same GEMM on a 128x128 tile (gemm_x3 takes it where those tiles alone fill the chip):
// 2 x 2 waves of 64x64 (2 x 2 MFMA tiles of 32x32 each), K staged 16 at a time through a
// two-stage ring of six planes (72 KiB: two workgroups per CU, two waves per SIMD). Each loaded
// element is split once and feeds 128 outputs (64 in gemm_x3_kernel), and every barrier covers
// 24 MFMAs per wave (12 there). Each k-step's six products go to a fresh sum added to the
// running fp32 sum with a VALU add (fa_common.h x3_tile_sum). Split-K as gemm_x3_kernel.
constexpr int kGbLDK = 24;                 // [row][k] plane row: 16 k + 8
constexpr int kGbLDR = 136;                // [k][row] plane row: 128 rows + 8
constexpr int kGbPlane = 128 * kGbLDK;     // 3072 elements (16 x 136 = 2176 fits too)
constexpr int kGbStage = 6 * kGbPlane;
static_assert(16 * kGbLDR <= kGbPlane, "plane size");
template <bool AK, bool BK, bool VEC>
__global__ __launch_bounds__(256, 2) void gemm_x3_big(GemmX3Args g) {
  extern __shared__ __attribute__((aligned(16))) bf16 smb[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t bz = blockIdx.z / g.S, slice = blockIdx.z % g.S;
  const int64_t m0 = (int64_t)blockIdx.y * 128, n0 = (int64_t)blockIdx.x * 128;
  const float* A = g.a + bz * g.sab;
  const float* B = g.b + bz * g.sbb;
  const int64_t kbeg = slice * g.ks, kend = min(g.K, kbeg + g.ks);
  auto chunk = [&](const float* base, int64_t rs, int64_t rlim, int64_t r, int64_t k, bool kc) -> float4 {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t lim = kc ? kend : rlim;
    const int64_t i0 = kc ? k : r;
    if ((kc ? r >= rlim : k >= kend)) return v;
    const float* p = base + (kc ? r * rs + k : k * rs + r);
    if (VEC && i0 + 3 < lim) return *(const float4*)p;
    if (i0 < lim) v.x = p[0];
    if (i0 + 1 < lim) v.y = p[1];
    if (i0 + 2 < lim) v.z = p[2];
    if (i0 + 3 < lim) v.w = p[3];
    return v;
  };
  // 16-B chunk c (0..511) of a 128 x 16 operand tile: along k: row c / 4, k 4 (c % 4); along
  // the rows: k c / 32, rows 4 (c % 32)
  float4 ra[2], rb[2];
  auto load = [&](int64_t k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      ra[i] = AK ? chunk(A, g.sam, g.M, m0 + c / 4, k0 + 4 * (c % 4), true)
                 : chunk(A, g.sak, g.M, m0 + 4 * (c % 32), k0 + c / 32, false);
      rb[i] = BK ? chunk(B, g.sbn, g.N, n0 + c / 4, k0 + 4 * (c % 4), true)
                 : chunk(B, g.sbk, g.N, n0 + 4 * (c % 32), k0 + c / 32, false);
    }
  };
  auto store = [&](int st) __attribute__((always_inline)) {
    bf16* base = smb + st * kGbStage;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      x3_store4(base + (AK ? (c / 4) * kGbLDK + 4 * (c % 4) : (c / 32) * kGbLDR + 4 * (c % 32)), kGbPlane,
                __builtin_bit_cast(uint4, ra[i]));
      x3_store4(base + 3 * kGbPlane + (BK ? (c / 4) * kGbLDK + 4 * (c % 4) : (c / 32) * kGbLDR + 4 * (c % 32)),
                kGbPlane, __builtin_bit_cast(uint4, rb[i]));
    }
  };
  typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
  auto frag = [&](const bf16* pl, int row, int ks, bool kc) -> bf16x8 {
    if (kc) {
      const bf16* q = pl + row * kGbLDK + 16 * ks + 4 * hf;
      const u32x2 lo = *(const u32x2*)q, hi = *(const u32x2*)(q + 8);
      const unsigned u[4] = {lo[0], lo[1], hi[0], hi[1]};
      return __builtin_bit_cast(bf16x8, u);
    }
    return col_frag<bf16>(pl, kGbLDR, 16 * ks + 4 * hf, row - c32, lane);
  };
  f32x16 tot[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) tot[i][j] = f32x16{};
  const int nst = (int)((kend - kbeg + 15) / 16);
  if (nst > 0) {
    load(kbeg);
    store(0);
    if (nst > 1) load(kbeg + 16);
  }
  __syncthreads();
#pragma nounroll
  for (int st = 0; st < nst; ++st) {
    const bf16* base = smb + (st & 1) * kGbStage;
    {
      constexpr int ks = 0;
      X3Frag fb[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int rb_ = wn * 64 + 32 * j + c32;
        fb[j].h = frag(base + 3 * kGbPlane, rb_, ks, BK);
        fb[j].m = frag(base + 4 * kGbPlane, rb_, ks, BK);
        fb[j].l = frag(base + 5 * kGbPlane, rb_, ks, BK);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ra_ = wm * 64 + 32 * i + c32;
        X3Frag fa;
        fa.h = frag(base, ra_, ks, AK);
        fa.m = frag(base + kGbPlane, ra_, ks, AK);
        fa.l = frag(base + 2 * kGbPlane, ra_, ks, AK);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x16 t = f32x16{};
          mma_x3(t, fa, fb[j]);
          tot[i][j] += t;
        }
      }
    }
    if (st + 1 < nst) {
      store((st + 1) & 1);
      if (st + 2 < nst) load(kbeg + 16 * (st + 2));
    }
    __syncthreads();
  }
  float* C = g.c + (g.S > 1 ? slice * g.M * g.N : bz * g.scb);
  const int64_t scm = g.S > 1 ? g.N : g.scm, scn = g.S > 1 ? 1 : g.scn;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t gn = n0 + wn * 64 + 32 * j + c32;
    if (gn >= g.N) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gm = m0 + wm * 64 + 32 * i + acc_row(r, hf);
        if (gm < g.M) C[gm * scm + gn * scn] = tot[i][j][r];
      }
  }
}

// C = Σ_s part[s] (slice order: deterministic), C at row stride scm, column stride scn
__global__ __launch_bounds__(256) void gemm_slice_sum(float* __restrict__ c, const float* __restrict__ part,
                                                      int64_t M, int64_t N, int S, int64_t scm, int64_t scn) {
  const int64_t n = M * N, step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += step) {
    float a = part[t];
    for (int s = 1; s < S; ++s) a += part[s * n + t];
    const int64_t m = t / N, j = t - m * N;
    c[m * scm + j * scn] = a;
  }
}

static Layout make_layout(const int64_t* shape, const int64_t* strides, int dims) {
  Layout l;
  memset(&l, 0, sizeof(l));
  l.dims = dims;
  int64_t expect = 1;
  l.contiguous = 1;
  for (int d = dims - 1; d >= 0; --d) {
    l.shape[d] = shape[d];
    l.strides[d] = strides[d];
    if (shape[d] != 1 && strides[d] != expect) l.contiguous = 0;
    expect *= shape[d];
  }
  return l;
}
static bool same_shape(const Layout& a, const Layout& b) {
  if (a.dims != b.dims) return false;
  for (int d = 0; d < a.dims; ++d)
    if (a.shape[d] != b.shape[d]) return false;
  return true;
}
// every ordinal the grid-stride loops form (below n plus one grid stride, at most
// grid_for's 4096 x 256) and every element offset of the layouts below 2^31 (int32 indexing)
static bool fits_i32(int64_t n, std::initializer_list<const Layout*> ls) {
  if (n + ((int64_t)4096 * 256) >= ((int64_t)1 << 31)) return false;
  for (const Layout* l : ls) {
    int64_t e = 0;
    for (int d = 0; d < l->dims; ++d)
      if (l->shape[d] > 1) e += (l->shape[d] - 1) * (l->strides[d] < 0 ? -l->strides[d] : l->strides[d]);
    if (e >= ((int64_t)1 << 31)) return false;
  }
  return true;
}
static int64_t numel(const Layout& l) {
  int64_t n = 1;
  for (int d = 0; d < l.dims; ++d) n *= l.shape[d];
  return n;
}
// b repeats along out's leading dims: contiguous, and its shape (leading 1s dropped) equals
// out's trailing dims
static bool trailing_block(const Layout& out, const Layout& b) {
  if (!b.contiguous) return false;
  int lead = 0;
  while (lead < b.dims - 1 && b.shape[lead] == 1) ++lead;
  const int k = b.dims - lead;
  if (k > out.dims) return false;
  for (int j = 0; j < k; ++j)
    if (b.shape[lead + j] != out.shape[out.dims - k + j]) return false;
  return true;
}
static unsigned grid_for(int64_t n, int per_block = 256) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g > 256 * 16) g = 256 * 16;
  return (unsigned)(g < 1 ? 1 : g);
}
static int check_dims(int d) {
  if (d < 1 || d > kMaxDims) return set_error("tensor rank %d outside 1..%d", d, kMaxDims);
  return 0;
}

}  // namespace mt

using namespace mt;

// ---- counter-based uniform RNG ---------------------------------------------------------
// u[i] = top 24 bits of splitmix64(seed + golden·(i+1)) / 2^24, in [0, 1). Stateless: a
// launch is reproducible from (seed, n) and any element is independent of the grid.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ void rand_uniform_kernel(float* out, int64_t n, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = mix64(seed + 0x9e3779b97f4a7c15ull * (uint64_t)(i + 1));
    out[i] = (float)(h >> 40) * (1.0f / 16777216.0f);
  }
}

// Fused feed-forward pieces of the minitorch step (reference minitorch/modules_transfomer.py
// FeedForward, :233-277: dropout(linear_out(GELU(linear_in(x))))): the bias add of linear_in
// with the tanh-form GELU (minitorch/nn.py GELU, torch approximate='tanh'), forward and
// backward in one pass each, and dropout with its keep mask drawn from the counter-based
// uniform above (u > p keeps, as rand(shape) > p does) and redrawn in the backward from the
// same seed, so no mask is stored. Rows of `cols` contiguous floats; 16 B per lane where the
// row length allows.
__device__ __forceinline__ float gelu_tanh(float u, float& t, float& dt) {
  constexpr float k = 0.7978845608028654f;  // sqrt(2 / pi)
  const float u2 = u * u;
  t = tanhf(k * (u + 0.044715f * (u2 * u)));
  dt = k * (1.f + 3.f * 0.044715f * u2);   // d(inner)/du
  return 0.5f * u * (1.f + t);
}
template <bool BW>
__global__ __launch_bounds__(256) void bias_gelu_kernel(float* __restrict__ out, const float* __restrict__ x,
                                                        const float* __restrict__ bias,
                                                        const float* __restrict__ dy, int64_t n, int64_t cols,
                                                        int vec) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  auto one = [&](float xv, float bv, float g) -> float {
    float t, dt;
    const float u = xv + bv;
    const float y = gelu_tanh(u, t, dt);
    if (!BW) return y;
    // d/du 0.5 u (1 + t) = 0.5 (1 + t) + 0.5 u (1 - t^2) dt
    return g * (0.5f * (1.f + t) + 0.5f * u * (1.f - t * t) * dt);
  };
  if (vec) {  // cols % 4 == 0, 16-B aligned rows
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += step) {
      const float4 xv = ((const float4*)x)[i];
      const float4 bv = ((const float4*)bias)[i % (cols / 4)];
      const float4 g = BW ? ((const float4*)dy)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      ((float4*)out)[i] = make_float4(one(xv.x, bv.x, g.x), one(xv.y, bv.y, g.y), one(xv.z, bv.z, g.z),
                                      one(xv.w, bv.w, g.w));
    }
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step)
    out[i] = one(x[i], bias[i % cols], BW ? dy[i] : 0.f);
}

__global__ __launch_bounds__(256) void dropout_kernel(float* __restrict__ out, const float* __restrict__ x,
                                                      int64_t n, float p, float scale, uint64_t seed,
                                                      const uint64_t* __restrict__ seedp) {
  // seedp: the seed in device memory (a graph-captured step draws a fresh one per replay)
  if (seedp) seed = *seedp;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
    const uint64_t h = mix64(seed + 0x9e3779b97f4a7c15ull * (uint64_t)(i + 1));
    const float u = (float)(h >> 40) * (1.0f / 16777216.0f);
    out[i] = u > p ? x[i] * scale : 0.f;
  }
}

// Embedding rows (reference modules_basic.py Embedding: one_hot(ids) @ W, a [tokens x V] x
// [V x E] product): the forward gathers W[id] (zero for an id outside [0, V), the one-hot
// row of such an id being zero); the backward sums dY rows into dW rows. ids are the float
// token ids of the minitorch tensor.
__global__ __launch_bounds__(256) void embed_fw_kernel(float* __restrict__ out, const float* __restrict__ ids,
                                                       const float* __restrict__ w, int64_t ntok, int64_t V,
                                                       int64_t E) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ntok * E; i += step) {
    const int64_t t = i / E, c = i - t * E;
    const float f = ids[t];
    const int64_t id = (int64_t)f;
    out[i] = (f >= 0.f && id < V) ? w[id * E + c] : 0.f;
  }
}
// dW[v] = sum of dY[t] over the tokens t with id v (deterministic: fixed order; every row of
// dW written). One 1024-thread workgroup per kEmbVB vocabulary rows. Per pass over kEmbChunk
// tokens each of the 16 waves compacts its 128 tokens' matches (ballot, token order) into an
// LDS list of (token, row) entries; thread (group q, column c) then adds, in list order, the
// dY rows of the matches of waves 4q .. 4q + 3 (a quarter of the chunk), eight loads in
// flight; the four groups' sums are folded in group order at the end. (An id that repeats
// thousands of times, the padding id of a padded batch, is spread over the four groups.)
constexpr int kEmbVB = 8, kEmbChunk = 2048;
__global__ __launch_bounds__(1024) void embed_bw_kernel(float* __restrict__ dw, const float* __restrict__ dy,
                                                        const float* __restrict__ ids, int64_t ntok, int64_t V,
                                                        int64_t E) {
  __shared__ int list[kEmbChunk];
  __shared__ int wcount[16];
  __shared__ float fold[3][kEmbVB][256];
  constexpr int kW = kEmbChunk / 16;  // tokens per wave per pass
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, q = tid >> 8, cl = tid & 255;
  const int64_t v0 = (int64_t)blockIdx.x * kEmbVB;
  for (int64_t c0 = 0; c0 < E; c0 += 256) {
    const int64_t col = c0 + cl;
    float acc[kEmbVB];
#pragma unroll
    for (int k = 0; k < kEmbVB; ++k) acc[k] = 0.f;
    for (int64_t t0 = 0; t0 < ntok; t0 += kEmbChunk) {
      int* my = list + w * kW;
      int n = 0;
#pragma unroll
      for (int k = 0; k < kW; k += 64) {
        const int64_t t = t0 + w * kW + k + lane;
        int rel = -1;
        if (t < ntok) {
          const float f = ids[t];
          const int64_t id = (int64_t)f;
          if (f >= 0.f && id >= v0 && id < v0 + kEmbVB) rel = (int)(id - v0);
        }
        const unsigned long long m = __ballot(rel >= 0);
        if (rel >= 0) my[n + __popcll(m & ((1ull << lane) - 1))] = (w * kW + k + lane) | (rel << 12);
        n += __popcll(m);
      }
      if (lane == 0) wcount[w] = n;
      __syncthreads();
      if (col < E) {
        const float* g = dy + t0 * E + col;
        for (int ww = 4 * q; ww < 4 * q + 4; ++ww) {
          const int* l = list + ww * kW;
          const int nw = wcount[ww];
          int j = 0;
          // 32 rows in flight, then 8, then singles; the adds stay in list order. (A padding id
          // repeated ~1250 times in config 5's batch puts ~300 rows on each thread of one
          // workgroup; 32 in flight instead of 8 took the kernel only from 72 to ≈ 70 µs, so the
          // id scan of the 1250 workgroups, not that chain, is what bounds it.)
          for (; j + 32 <= nw; j += 32) {
            int e[32];
            float x[32];
#pragma unroll
            for (int u = 0; u < 32; ++u) e[u] = l[j + u];
#pragma unroll
            for (int u = 0; u < 32; ++u) x[u] = g[(int64_t)(e[u] & 4095) * E];
#pragma unroll
            for (int u = 0; u < 32; ++u)
#pragma unroll
              for (int k = 0; k < kEmbVB; ++k)
                if (k == (e[u] >> 12)) acc[k] += x[u];
          }
          for (; j + 8 <= nw; j += 8) {
            int e[8];
            float x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) e[u] = l[j + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = g[(int64_t)(e[u] & 4095) * E];
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
              for (int k = 0; k < kEmbVB; ++k)
                if (k == (e[u] >> 12)) acc[k] += x[u];
          }
          for (; j < nw; ++j) {
            const int e = l[j];
            const float x = g[(int64_t)(e & 4095) * E];
#pragma unroll
            for (int k = 0; k < kEmbVB; ++k)
              if (k == (e >> 12)) acc[k] += x;
          }
        }
      }
      __syncthreads();
    }
    if (q > 0) {
#pragma unroll
      for (int k = 0; k < kEmbVB; ++k) fold[q - 1][k][cl] = acc[k];
    }
    __syncthreads();
    if (q == 0 && col < E) {
#pragma unroll
      for (int k = 0; k < kEmbVB; ++k)
        if (v0 + k < V) dw[(v0 + k) * E + col] = ((acc[k] + fold[0][k][cl]) + fold[1][k][cl]) + fold[2][k][cl];
    }
    __syncthreads();
  }
}

// Multi-tensor Adam (minitorch/optim.py Adam.step, reference minitorch/optim.py:52-75 with
// the second moment on (1 - beta2)): for every element of every listed tensor
//   m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g g;  p = p - step_size m / (sqrt(v) + eps)
// with step_size = lr sqrt(1 - b2^t) / (1 - b1^t) from the host, in the op-by-op path's
// order and roundings (no contraction). One launch per kAdamMax tensors: workgroup blocks
// [blk0[t], blk0[t + 1]) take tensor t, 4 elements a lane when the tensor allows it.
constexpr int kAdamMax = 24;
struct AdamArgs {
  float* p[kAdamMax];
  const float* g[kAdamMax];
  float* m[kAdamMax];
  float* v[kAdamMax];
  int64_t n[kAdamMax];
  int blk0[kAdamMax + 1];
  int nt;
  float b1, b2, c1, c2, step, eps;  // c1 = 1 - b1, c2 = 1 - b2
  const float* stepp;  // non-null: the step size in device memory (read instead of step)
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamArgs& a, float step) {
  // separately rounded products and sums, like the tensor ops (plain operators under the
  // pragma: the __f*_rn helpers are inlined from a header compiled with contraction on)
#pragma clang fp contract(off)
  m = m * a.b1 + g * a.c1;
  v = v * a.b2 + (g * g) * a.c2;
  // the tensor-op form divides as a product with the reciprocal (Tensor.__truediv__ =
  // Mul(a, Inv(b))) and takes the square root as PowerScalar's powf(v, 0.5)
  p = p - (step * m) * (1.f / (powf(v, 0.5f) + a.eps));
}

__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  int t = 0;
  while (t + 1 < a.nt && (int)blockIdx.x >= a.blk0[t + 1]) ++t;
  const int64_t n = a.n[t];
  const int64_t base = (int64_t)(blockIdx.x - a.blk0[t]) * 1024;
  float* P = a.p[t];
  const float* G = a.g[t];
  float* M = a.m[t];
  float* V = a.v[t];
  const bool vec = ((((uintptr_t)P | (uintptr_t)G | (uintptr_t)M | (uintptr_t)V) & 15) == 0);
  const float step = a.stepp ? *a.stepp : a.step;
  const int64_t i = base + 4 * threadIdx.x;
  if (vec && i + 4 <= n) {
    float4 p = *(float4*)(P + i), m = *(float4*)(M + i), v = *(float4*)(V + i);
    const float4 g = *(const float4*)(G + i);
    adam_elem(p.x, g.x, m.x, v.x, a, step);
    adam_elem(p.y, g.y, m.y, v.y, a, step);
    adam_elem(p.z, g.z, m.z, v.z, a, step);
    adam_elem(p.w, g.w, m.w, v.w, a, step);
    *(float4*)(P + i) = p;
    *(float4*)(M + i) = m;
    *(float4*)(V + i) = v;
  } else {
    for (int64_t j = i; j < min(i + 4, n); ++j) adam_elem(P[j], G[j], M[j], V[j], a, step);
  }
}

extern "C" {

int64_t mt_scratch_bytes(void) {
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  int64_t n = 0;
  for (int i = 0; i < g_nscratch; ++i) n += (int64_t)g_scratch[i].cap;
  for (const auto& k : g_scratch_kept) n += (int64_t)k.second;
  return n;
}

int mt_scratch_release(void) {
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  for (int i = 0; i < g_nscratch; ++i) {
    ScratchSlot& s = g_scratch[i];
    if (!s.buf || s.captured) continue;  // a captured graph may still replay with it
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s.st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) continue;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return set_error("mt_scratch_release: hipGetDevice failed");
    if (hipSetDevice(s.dev) != hipSuccess || hipStreamSynchronize(s.st) != hipSuccess) {
      (void)hipSetDevice(cur);
      return set_error("mt_scratch_release: stream synchronize failed");
    }
    (void)hipFree(s.buf);
    (void)hipSetDevice(cur);
    s.buf = nullptr;
    s.cap = 0;
  }
  return 0;
}

int mt_tensor_map(int fn, float* out, const int64_t* out_shape, const int64_t* out_strides,
                  int out_dims, const float* in, const int64_t* in_shape,
                  const int64_t* in_strides, int in_dims, void* stream) {
  if (check_dims(out_dims) || check_dims(in_dims)) return 1;
  Layout ol = make_layout(out_shape, out_strides, out_dims);
  Layout il = make_layout(in_shape, in_strides, in_dims);
  int64_t n = 1;
  for (int d = 0; d < out_dims; ++d) n *= out_shape[d];
  if (n == 0) return 0;
  const int same = ol.contiguous && il.contiguous && same_shape(ol, il);
  hipStream_t st = (hipStream_t)stream;
  if (same && (((uintptr_t)out | (uintptr_t)in) & 15) == 0)
    hipLaunchKernelGGL(map_dense_kernel, dim3(grid_for(n % 4 ? n : n / 4)), dim3(256), 0, st, fn, out, n, in);
  else if (fits_i32(n, {&ol, &il}))
    hipLaunchKernelGGL(map_kernel<int>, dim3(grid_for(n)), dim3(256), 0, st, fn, out, ol, n, in, il, same);
  else
    hipLaunchKernelGGL(map_kernel<int64_t>, dim3(grid_for(n)), dim3(256), 0, st, fn, out, ol, n, in, il, same);
  return check_hip(hipGetLastError(), "mt_tensor_map");
}

int mt_tensor_zip(int fn, float* out, const int64_t* out_shape, const int64_t* out_strides,
                  int out_dims, const float* a, const int64_t* a_shape, const int64_t* a_strides,
                  int a_dims, const float* b, const int64_t* b_shape, const int64_t* b_strides,
                  int b_dims, void* stream) {
  if (check_dims(out_dims) || check_dims(a_dims) || check_dims(b_dims)) return 1;
  Layout ol = make_layout(out_shape, out_strides, out_dims);
  Layout al = make_layout(a_shape, a_strides, a_dims);
  Layout bl = make_layout(b_shape, b_strides, b_dims);
  int64_t n = 1;
  for (int d = 0; d < out_dims; ++d) n *= out_shape[d];
  if (n == 0) return 0;
  const int same = ol.contiguous && al.contiguous && bl.contiguous && same_shape(ol, al) &&
                   same_shape(ol, bl);
  hipStream_t st = (hipStream_t)stream;
  // dense fast paths: one operand the output's shape and contiguous, the other the same, a
  // single element, or a contiguous block repeated along the leading dims (16-B aligned)
  const bool aligned = (((uintptr_t)out | (uintptr_t)a | (uintptr_t)b) & 15) == 0;
  const bool a_full = al.contiguous && same_shape(ol, al), b_full = bl.contiguous && same_shape(ol, bl);
  const unsigned g4 = grid_for(n % 4 ? n : n / 4);
  if (ol.contiguous && aligned && (a_full || b_full)) {
    const float* x = a_full ? a : b;  // the full operand
    const float* y = a_full ? b : a;
    const Layout& yl = a_full ? bl : al;
    const bool swap = !a_full;
    const int64_t ny = numel(yl);
    if (same) {
      hipLaunchKernelGGL((zip_dense_kernel<0, false>), dim3(g4), dim3(256), 0, st, fn, out, n, a, b, n);
      return check_hip(hipGetLastError(), "mt_tensor_zip");
    }
    if (ny == 1) {
      if (swap) hipLaunchKernelGGL((zip_dense_kernel<1, true>), dim3(g4), dim3(256), 0, st, fn, out, n, x, y, ny);
      else hipLaunchKernelGGL((zip_dense_kernel<1, false>), dim3(g4), dim3(256), 0, st, fn, out, n, x, y, ny);
      return check_hip(hipGetLastError(), "mt_tensor_zip");
    }
    if (trailing_block(ol, yl)) {
      if (swap) hipLaunchKernelGGL((zip_dense_kernel<2, true>), dim3(g4), dim3(256), 0, st, fn, out, n, x, y, ny);
      else hipLaunchKernelGGL((zip_dense_kernel<2, false>), dim3(g4), dim3(256), 0, st, fn, out, n, x, y, ny);
      return check_hip(hipGetLastError(), "mt_tensor_zip");
    }
  }
  if (fits_i32(n, {&ol, &al, &bl}))
    hipLaunchKernelGGL(zip_kernel<int>, dim3(grid_for(n)), dim3(256), 0, st, fn, out, ol, n, a, al, b, bl, same);
  else
    hipLaunchKernelGGL(zip_kernel<int64_t>, dim3(grid_for(n)), dim3(256), 0, st, fn, out, ol, n, a, al, b, bl, same);
  return check_hip(hipGetLastError(), "mt_tensor_zip");
}

int mt_tensor_reduce(int fn, float* out, const int64_t* out_shape, const int64_t* out_strides,
                     const float* a, const int64_t* a_shape, const int64_t* a_strides, int dims,
                     int reduce_dim, float start, void* stream) {
  if (check_dims(dims)) return 1;
  if (reduce_dim < 0 || reduce_dim >= dims) return set_error("reduce dim %d out of range", reduce_dim);
  Layout ol = make_layout(out_shape, out_strides, dims);
  Layout al = make_layout(a_shape, a_strides, dims);
  int64_t n = 1;
  for (int d = 0; d < dims; ++d) n *= out_shape[d];
  if (n == 0) return 0;
  int64_t inner = 1, outer = 1;
  for (int d = reduce_dim + 1; d < dims; ++d) inner *= a_shape[d];
  for (int d = 0; d < reduce_dim; ++d) outer *= a_shape[d];
  const int64_t len = a_shape[reduce_dim];
  // the one-pass form up to 64 MiB of input; above that the two-kernel form streams faster
  // (4992 x 10000, 200 MB: 57 µs against 84-90 µs at 240-2048 workgroups of the one-pass form)
  const bool al16 = ((((uintptr_t)a | (uintptr_t)out) & 15) == 0);
  static const int64_t colgroup_max = [] {  // A/B knob: MT_COLGROUP_MAX (floats)
    const char* e = getenv("MT_COLGROUP_MAX");
    return e ? (int64_t)atoll(e) : ((int64_t)8 << 20);
  }();
  if (al.contiguous && ol.contiguous && inner % 4 == 0 && al16 && len >= 2 && len <= 8192 &&
      outer <= 65535 && outer * (inner / 4) >= 32 && outer * len * inner <= colgroup_max) {
    // column groups: every workgroup owns whole columns (see reduce_colgroup_kernel)
    const int ncg = (int)(inner / 4);
    const int xcd_map = ncg >= 64;
    const unsigned gx = (unsigned)(xcd_map ? (ncg + 63) / 64 * 64 : ncg);
    const int T = (int)std::min<int64_t>(1024, len);  // every lane has a row
    const dim3 grid(gx, (unsigned)outer);
    const hipStream_t st = (hipStream_t)stream;
    if (fn == FN_ADD)
      hipLaunchKernelGGL(reduce_colgroup_kernel<FN_ADD>, grid, dim3(T), 0, st, fn, out, a, len, inner, ncg, xcd_map, start);
    else if (fn == FN_MUL)
      hipLaunchKernelGGL(reduce_colgroup_kernel<FN_MUL>, grid, dim3(T), 0, st, fn, out, a, len, inner, ncg, xcd_map, start);
    else if (fn == FN_MAX)
      hipLaunchKernelGGL(reduce_colgroup_kernel<FN_MAX>, grid, dim3(T), 0, st, fn, out, a, len, inner, ncg, xcd_map, start);
    else
      hipLaunchKernelGGL(reduce_colgroup_kernel<-1>, grid, dim3(T), 0, st, fn, out, a, len, inner, ncg, xcd_map, start);
  } else if (al.contiguous && ol.contiguous && inner % 4 == 0 && inner >= 64 && len >= 16 && outer <= 65535 &&
      outer * len * inner <= ((int64_t)16 << 20) && al16) {
    // one pass: row chunks of at least 8 rows per wave, about 256 workgroups in all
    const int64_t cb = (inner + 255) / 256;
    // about 256 workgroups, 8 rows per wave (8 beat 4, 16, 32 and 64 rows and 128 workgroups at
    // 4992 x 256: 11.4 µs, scripts/gpu_colab.sh); fewer than 4 chunks: no fold at all
    int64_t R = std::max<int64_t>(1, std::min<int64_t>(256 / (cb * outer), len / (8 * kCol1Waves)));
    if (R < 4) R = 1;
    int64_t chunk = (len + R - 1) / R;
    R = (len + chunk - 1) / chunk;  // every chunk holds a row
    float* part = nullptr;
    unsigned* ctr = nullptr;
    if (R > 1) {
      part = (float*)reduce_scratch((size_t)(outer * R * inner) * 4, (hipStream_t)stream);
      ctr = outer * cb <= kColCounters ? reduce_counters((hipStream_t)stream) : nullptr;
      if (!part || !ctr) { R = 1; chunk = len; }
    }
    const dim3 grid((unsigned)cb, (unsigned)R, (unsigned)outer);
    const hipStream_t st = (hipStream_t)stream;
    if (fn == FN_ADD)
      hipLaunchKernelGGL(reduce_cols1_kernel<FN_ADD>, grid, dim3(512), 0, st, fn, out, part, ctr, a, len, inner, chunk, start);
    else if (fn == FN_MUL)
      hipLaunchKernelGGL(reduce_cols1_kernel<FN_MUL>, grid, dim3(512), 0, st, fn, out, part, ctr, a, len, inner, chunk, start);
    else if (fn == FN_MAX)
      hipLaunchKernelGGL(reduce_cols1_kernel<FN_MAX>, grid, dim3(512), 0, st, fn, out, part, ctr, a, len, inner, chunk, start);
    else
      hipLaunchKernelGGL(reduce_cols1_kernel<-1>, grid, dim3(512), 0, st, fn, out, part, ctr, a, len, inner, chunk, start);
  } else if (al.contiguous && ol.contiguous && inner >= 16 && len >= 16 && outer <= 65535) {
    // R row chunks: as many as give the grid about 512 workgroups, at most kColRMax, chunks of
    // at least 64 rows (128 where the rows allow)
    const int64_t cb = (inner + 63) / 64;
    int64_t R = std::min<int64_t>(std::min<int64_t>(kColRMax, (len + 127) / 128),
                                  std::max<int64_t>((512 + cb * outer - 1) / (cb * outer), len / 1024));
    R = std::min<int64_t>(R, len / 64);
    if (R < 1) R = 1;
    float* part = nullptr;
    if (R > 1) {
      part = (float*)reduce_scratch((size_t)(outer * R * inner) * 8, (hipStream_t)stream);
      if (!part) R = 1;
    }
    const int64_t chunk = (len + R - 1) / R;
    hipLaunchKernelGGL(reduce_cols_kernel, dim3((unsigned)cb, (unsigned)R, (unsigned)outer), dim3(1024), 0,
                       (hipStream_t)stream, fn, out, part, (int*)(part + outer * R * inner), a, len, inner,
                       chunk, start);
    if (R > 1) {
      const int64_t no = outer * inner;
      hipLaunchKernelGGL(reduce_cols_fold, dim3((unsigned)((no + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                         fn, out, part, (const int*)(part + outer * R * inner), inner, (int)R, no, start);
    }
  } else if (n <= 512 && a_shape[reduce_dim] >= 2048) {
    const hipStream_t st = (hipStream_t)stream;
    if (fn == FN_ADD)
      hipLaunchKernelGGL(reduce_block_kernel<FN_ADD>, dim3((unsigned)n), dim3(1024), 0, st, fn, out, ol, a, al, reduce_dim, start);
    else if (fn == FN_MAX)
      hipLaunchKernelGGL(reduce_block_kernel<FN_MAX>, dim3((unsigned)n), dim3(1024), 0, st, fn, out, ol, a, al, reduce_dim, start);
    else
      hipLaunchKernelGGL(reduce_block_kernel<-1>, dim3((unsigned)n), dim3(1024), 0, st, fn, out, ol, a, al, reduce_dim, start);
  } else if (a_shape[reduce_dim] >= 64) {
    hipLaunchKernelGGL(reduce_wave_kernel, dim3(grid_for(n, 4)), dim3(256), 0,
                       (hipStream_t)stream, fn, out, ol, n, a, al, reduce_dim, start);
  } else {
    hipLaunchKernelGGL(reduce_thread_kernel, dim3(grid_for(n)), dim3(256), 0,
                       (hipStream_t)stream, fn, out, ol, n, a, al, reduce_dim, start);
  }
  return check_hip(hipGetLastError(), "mt_tensor_reduce");
}

// 0: rocBLAS where the layout allows; 1: own fp32-MFMA kernel only; 2: own X3 kernels (128x128
// tiles where they fill the chip, else 64x64); 3: X3 on 64x64 tiles only (A/B). MT_GEMM_BACKEND
// sets the process default.
static int initial_gemm_backend() {
  const char* e = getenv("MT_GEMM_BACKEND");
  const int v = e ? atoi(e) : 0;
  return v >= 0 && v <= 3 ? v : 0;
}
static int g_gemm_backend = initial_gemm_backend();

void mt_set_gemm_backend(int backend) { g_gemm_backend = backend; }

// One rocBLAS handle per device, created on first use.
static rocblas_handle blas_handle() {
  static std::mutex mu;
  static rocblas_handle handles[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (!handles[dev] && rocblas_create_handle(&handles[dev]) != rocblas_status_success) {
    handles[dev] = nullptr;
  }
  return handles[dev];
}

// Split-K: C = the S partial products [S][M][N] summed in slice order (fixed: deterministic).
// S is a template argument so the S loads of a lane are all in flight together (a run-time loop
// waited on each: 4.6 µs per call for config 5's 256 x 256 dW at S = 4).
extern "C++" {  // (inside the file's extern "C" block: templates need C++ linkage)
template <int S>
__global__ __launch_bounds__(256) void splitk_sum_kernel(float* __restrict__ c, const float* __restrict__ part,
                                                         int64_t M, int64_t N, int64_t ldc) {
  const int64_t n4 = N / 4, total = M * n4, slice = M * N;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += step) {
    const int64_t m = t / n4, j = (t - m * n4) * 4;
    const float* p = part + m * N + j;
    float4 v[S];
#pragma unroll
    for (int k = 0; k < S; ++k) v[k] = *(const float4*)(p + k * slice);
    float4 acc = v[0];
#pragma unroll
    for (int k = 1; k < S; ++k) { acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w; }
    *(float4*)(c + m * ldc + j) = acc;
  }
}
}  // extern "C++"

// Row-major C[M,N] = A[M,K]·B[K,N] as column-major Cᵀ = Bᵀ·Aᵀ. Returns false (caller
// falls back) when a layout has no unit stride or a leading dimension rocBLAS rejects.
static bool gemm_rocblas(float* c, const float* a, const float* b, int64_t batch, int64_t M,
                         int64_t N, int64_t K, const int64_t* sa, const int64_t* sb,
                         const int64_t* sc, hipStream_t st, rocblas_status* status) {
  const int64_t lim = 0x7fffffff;
  if (M > lim || N > lim || K > lim || batch > lim) return false;
  // Normalise the strides of size-1 dims (free) towards a usable layout.
  int64_t sam = sa[1], sak = sa[2], sbk = sb[1], sbn = sb[2], scm = sc[1], scn = sc[2];
  if (N == 1) scn = 1;
  if (M == 1) { scm = std::max<int64_t>(N, 1); if (sak == 1) sam = std::max<int64_t>(sam, K); }
  if (K == 1) { sak = 1; sbk = std::max<int64_t>(N, sbk); }
  if (sc[0] < 0 || scn != 1 || scm < N) return false;
  // first operand: our B as an N x K column-major matrix (op N) or its K x N transpose
  rocblas_operation opb;
  int64_t ldb;
  if (sbn == 1 && sbk >= N) { opb = rocblas_operation_none; ldb = sbk; }
  else if (sbk == 1 && sbn >= K) { opb = rocblas_operation_transpose; ldb = sbn; }
  else return false;
  // second operand: our A as a K x M column-major matrix (op N) or its M x K transpose
  rocblas_operation opa;
  int64_t lda;
  if (sak == 1 && sam >= K) { opa = rocblas_operation_none; lda = sam; }
  else if (sam == 1 && sak >= M) { opa = rocblas_operation_transpose; lda = sak; }
  else return false;
  if (lda > lim || ldb > lim || scm > lim || sa[0] < 0 || sb[0] < 0) return false;
  rocblas_handle h = blas_handle();
  if (!h) return false;
  rocblas_set_stream(h, st);
  const float alpha = 1.f, beta = 0.f;
  // A long reduction into a small output (config 5's LM-head dX: 4992 x 256 over K = 10000,
  // 78 output tiles for 256 CUs) runs as S batched K slices into partials plus an ordered sum:
  // 547 -> 197 µs at S = 8; the linears' 256 x 256 dW over K = 4992 (rocBLAS's own split,
  // 17.7 µs) 15.1 µs at S = 4 (scripts/gemm_probe.py). Only for one matrix, K >= 8192 with
  // < 128 tiles of 128 x 128 or K >= 4096 with <= 16, S | K, N % 4 = 0, 16-byte aligned rows.
  const int64_t tiles = ((M + 127) / 128) * ((N + 127) / 128);
  if (batch == 1 && ((K >= 8192 && tiles < 128) || (K >= 4096 && tiles <= 16)) && N % 4 == 0 && scm % 4 == 0 &&
      ((uintptr_t)c & 15) == 0) {
    int S = 0;
    for (int cand : {8, 4, 2})
      if (K % cand == 0 && K / cand >= 1024 && (K >= 8192 || cand <= 4)) { S = cand; break; }
    float* part = S ? (float*)reduce_scratch((size_t)S * M * N * 4, st) : nullptr;
    if (part) {
      const int64_t ks = K / S;
      // slice s: B rows [s ks, (s+1) ks) (the first operand's K offset), A columns likewise
      const int64_t strb = opb == rocblas_operation_none ? ks * ldb : ks;
      const int64_t stra = opa == rocblas_operation_none ? ks : ks * lda;
      *status = rocblas_sgemm_strided_batched(h, opb, opa, (rocblas_int)N, (rocblas_int)M, (rocblas_int)ks,
                                              &alpha, b, (rocblas_int)ldb, strb, a, (rocblas_int)lda, stra,
                                              &beta, part, (rocblas_int)N, M * N, (rocblas_int)S);
      if (*status == rocblas_status_success) {
        const dim3 g(grid_for(M * N / 4));
        if (S == 8) hipLaunchKernelGGL(splitk_sum_kernel<8>, g, dim3(256), 0, st, c, part, M, N, scm);
        else if (S == 4) hipLaunchKernelGGL(splitk_sum_kernel<4>, g, dim3(256), 0, st, c, part, M, N, scm);
        else hipLaunchKernelGGL(splitk_sum_kernel<2>, g, dim3(256), 0, st, c, part, M, N, scm);
      }
      return true;
    }
  }
  *status = rocblas_sgemm_strided_batched(h, opb, opa, (rocblas_int)N, (rocblas_int)M, (rocblas_int)K,
                                          &alpha, b, (rocblas_int)ldb, sb[0], a, (rocblas_int)lda, sa[0],
                                          &beta, c, (rocblas_int)scm, sc[0], (rocblas_int)batch);
  return true;
}

// The X3 GEMM (gemm_x3_kernel): false when a layout has no unit stride (the caller falls back).
// Split-K when one matrix has fewer than 256 output tiles and K >= 512 (config 5's 256 x 256
// weight gradients over K = 4992: 16 tiles -> 16 slices).
// big: 128x128 tiles where they fill the chip (alone or as k-slices), else 64x64.
static bool gemm_x3(float* c, const float* a, const float* b, int64_t batch, int64_t M, int64_t N,
                    int64_t K, const int64_t* sa, const int64_t* sb, const int64_t* sc, hipStream_t st,
                    bool big) {
  int64_t sam = sa[1], sak = sa[2], sbk = sb[1], sbn = sb[2];
  if (K == 1) { sak = 1; sbk = 1; }
  if (M == 1) sam = 1;
  if (N == 1) sbn = 1;
  const bool ak = sak == 1, bk = sbk == 1;
  if ((!ak && sam != 1) || (!bk && sbn != 1)) return false;
  if (batch > 65535) return false;
  // 16-B chunks: the bases and every stride but the unit one multiples of 4 floats
  const int64_t oa = ak ? sam : sak, ob = bk ? sbn : sbk;
  const bool vec = (((uintptr_t)a | (uintptr_t)b) & 15) == 0 && oa % 4 == 0 && ob % 4 == 0 &&
                   (batch == 1 || (sa[0] % 4 == 0 && sb[0] % 4 == 0));
  const int64_t tm2 = (M + 127) / 128, tn2 = (N + 127) / 128;
  // 128x128 tiles where they fill the chip, alone or as up to 8 k-slices of >= 1024
  int S2 = 1;
  if (batch == 1 && tm2 * tn2 < 256) S2 = (int)std::min<int64_t>((256 + tm2 * tn2 - 1) / (tm2 * tn2), K / 1024);
  int64_t ks2 = K;
  if (S2 > 8) S2 = 1;
  if (S2 > 1) {
    ks2 = ((K + S2 - 1) / S2 + 15) / 16 * 16;
    S2 = (int)((K + ks2 - 1) / ks2);
  }
  float* part2 = nullptr;
  if (big && batch * tm2 * tn2 * S2 >= 256 && tm2 <= 65535 &&
      (S2 == 1 || (part2 = (float*)reduce_scratch((size_t)S2 * M * N * 4, st)) != nullptr)) {
    GemmX3Args g;
    g.a = a; g.b = b; g.c = S2 > 1 ? part2 : c;
    g.M = M; g.N = N; g.K = K; g.ks = ks2; g.S = S2;
    g.sab = sa[0]; g.sam = sam; g.sak = sak;
    g.sbb = sb[0]; g.sbk = sbk; g.sbn = sbn;
    g.scb = sc[0]; g.scm = sc[1]; g.scn = sc[2];
    const dim3 grid((unsigned)tn2, (unsigned)tm2, (unsigned)(batch * S2));
    constexpr int smem = 2 * kGbStage * 2;
#define MT_GB(AKV, BKV, VV)                                                                          \
  {                                                                                                \
    static const hipError_t attr = hipFuncSetAttribute(                                            \
        (const void*)gemm_x3_big<AKV, BKV, VV>, hipFuncAttributeMaxDynamicSharedMemorySize, smem); \
    if (attr != hipSuccess) return false;                                                          \
    hipLaunchKernelGGL((gemm_x3_big<AKV, BKV, VV>), grid, dim3(256), smem, st, g);                 \
  }
    if (vec) {
      if (ak && bk) MT_GB(true, true, true)
      else if (ak) MT_GB(true, false, true)
      else if (bk) MT_GB(false, true, true)
      else MT_GB(false, false, true)
    } else {
      if (ak && bk) MT_GB(true, true, false)
      else if (ak) MT_GB(true, false, false)
      else if (bk) MT_GB(false, true, false)
      else MT_GB(false, false, false)
    }
#undef MT_GB
    if (S2 > 1)
      hipLaunchKernelGGL(gemm_slice_sum, dim3(grid_for(M * N)), dim3(256), 0, st, c, (const float*)part2, M, N, S2,
                         sc[1], sc[2]);
    return true;
  }
  const int64_t tm = (M + 63) / 64, tn = (N + 63) / 64;
  if (tm > 65535) return false;
  int S = 1;
  if (batch == 1 && tm * tn < 256 && K >= 512) {
    S = (int)std::min<int64_t>(16, std::max<int64_t>(1, 256 / (tm * tn)));
    S = (int)std::min<int64_t>(S, K / 256);
  }
  int64_t ks = K;
  float* part = nullptr;
  if (S > 1) {
    ks = ((K + S - 1) / S + 31) / 32 * 32;
    S = (int)((K + ks - 1) / ks);
    if (S > 1) part = (float*)reduce_scratch((size_t)S * M * N * 4, st);
    if (!part) { S = 1; ks = K; }
  }
  GemmX3Args g;
  g.a = a; g.b = b; g.c = S > 1 ? part : c;
  g.M = M; g.N = N; g.K = K; g.ks = ks; g.S = S;
  g.sab = sa[0]; g.sam = sam; g.sak = sak;
  g.sbb = sb[0]; g.sbk = sbk; g.sbn = sbn;
  g.scb = sc[0]; g.scm = sc[1]; g.scn = sc[2];
  const dim3 grid((unsigned)tn, (unsigned)tm, (unsigned)(batch * S));
#define MT_GX(AKV, BKV)                                                                            \
  {                                                                                                \
    if (vec) hipLaunchKernelGGL((gemm_x3_kernel<AKV, BKV, true>), grid, dim3(256), 0, st, g);      \
    else hipLaunchKernelGGL((gemm_x3_kernel<AKV, BKV, false>), grid, dim3(256), 0, st, g);         \
  }
  if (ak && bk) MT_GX(true, true)
  else if (ak) MT_GX(true, false)
  else if (bk) MT_GX(false, true)
  else MT_GX(false, false)
#undef MT_GX
  if (S > 1)
    hipLaunchKernelGGL(gemm_slice_sum, dim3(grid_for(M * N)), dim3(256), 0, st, c, (const float*)part, M, N, S,
                       sc[1], sc[2]);
  return true;
}

int mt_matmul_f32(float* c, const float* a, const float* b, int64_t batch, int64_t M, int64_t N,
                  int64_t K, const int64_t* a_strides, const int64_t* b_strides,
                  const int64_t* c_strides, void* stream) {
  if (batch <= 0 || M <= 0 || N <= 0 || K <= 0)
    return set_error("mt_matmul_f32: bad sizes %lld %lld %lld %lld", (long long)batch,
                     (long long)M, (long long)N, (long long)K);
  if ((g_gemm_backend == 2 || g_gemm_backend == 3) &&
      gemm_x3(c, a, b, batch, M, N, K, a_strides, b_strides, c_strides, (hipStream_t)stream,
              g_gemm_backend == 2))
    return check_hip(hipGetLastError(), "mt_matmul_f32(x3)");
  if (g_gemm_backend == 0) {
    rocblas_status rs = rocblas_status_success;
    if (gemm_rocblas(c, a, b, batch, M, N, K, a_strides, b_strides, c_strides, (hipStream_t)stream, &rs)) {
      if (rs != rocblas_status_success)
        return set_error("mt_matmul_f32: rocblas_sgemm_strided_batched: %s", rocblas_status_to_string(rs));
      return check_hip(hipGetLastError(), "mt_matmul_f32(rocblas)");
    }
  }
  if (batch > 65535) return set_error("mt_matmul_f32: batch %lld > 65535", (long long)batch);
  GemmArgs g;
  g.a = a; g.b = b; g.c = c; g.M = M; g.N = N; g.K = K;
  g.sab = a_strides[0]; g.sam = a_strides[1]; g.sak = a_strides[2];
  g.sbb = b_strides[0]; g.sbk = b_strides[1]; g.sbn = b_strides[2];
  g.scb = c_strides[0]; g.scm = c_strides[1]; g.scn = c_strides[2];
  dim3 grid((unsigned)((N + 63) / 64), (unsigned)((M + 63) / 64), (unsigned)batch);
  hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(256), 0, (hipStream_t)stream, g);
  return check_hip(hipGetLastError(), "mt_matmul_f32");
}

int mt_rand_uniform(float* out, int64_t n, uint64_t seed, void* stream) {
  if (n < 0) return set_error("mt_rand_uniform: n = %lld", (long long)n);
  if (n == 0) return 0;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(rand_uniform_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     out, n, seed);
  return check_hip(hipGetLastError(), "mt_rand_uniform");
}

int mt_bias_gelu_fw(float* out, const float* x, const float* bias, int64_t rows, int64_t cols, void* stream) {
  if (rows < 0 || cols <= 0) return set_error("mt_bias_gelu_fw: bad sizes %lld x %lld", (long long)rows, (long long)cols);
  const int64_t n = rows * cols;
  if (n == 0) return 0;
  const bool v4 = cols % 4 == 0 && ((((uintptr_t)out | (uintptr_t)x | (uintptr_t)bias) & 15) == 0);
  hipLaunchKernelGGL(bias_gelu_kernel<false>, dim3(grid_for(v4 ? n / 4 : n)), dim3(256), 0, (hipStream_t)stream,
                     out, x, bias, nullptr, n, cols, (int)v4);
  return check_hip(hipGetLastError(), "mt_bias_gelu_fw");
}

int mt_bias_gelu_bw(float* dx, const float* dy, const float* x, const float* bias, int64_t rows, int64_t cols,
                    void* stream) {
  if (rows < 0 || cols <= 0) return set_error("mt_bias_gelu_bw: bad sizes %lld x %lld", (long long)rows, (long long)cols);
  const int64_t n = rows * cols;
  if (n == 0) return 0;
  const bool v4 = cols % 4 == 0 && ((((uintptr_t)dx | (uintptr_t)dy | (uintptr_t)x | (uintptr_t)bias) & 15) == 0);
  hipLaunchKernelGGL(bias_gelu_kernel<true>, dim3(grid_for(v4 ? n / 4 : n)), dim3(256), 0, (hipStream_t)stream,
                     dx, x, bias, dy, n, cols, (int)v4);
  return check_hip(hipGetLastError(), "mt_bias_gelu_bw");
}

int mt_dropout(float* out, const float* x, int64_t n, float p, float scale, uint64_t seed, void* stream) {
  if (n < 0) return set_error("mt_dropout: n = %lld", (long long)n);
  if (n == 0) return 0;
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, out, x, n, p, scale, seed,
                     nullptr);
  return check_hip(hipGetLastError(), "mt_dropout");
}

int mt_dropout_dseed(float* out, const float* x, int64_t n, float p, float scale, const uint64_t* seed,
                     void* stream) {
  if (n < 0) return set_error("mt_dropout_dseed: n = %lld", (long long)n);
  if (!seed) return set_error("mt_dropout_dseed: null seed pointer");
  if (n == 0) return 0;
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, out, x, n, p, scale,
                     (uint64_t)0, seed);
  return check_hip(hipGetLastError(), "mt_dropout_dseed");
}

int mt_embedding_fw(float* out, const float* ids, const float* weight, int64_t ntok, int64_t V, int64_t E,
                    void* stream) {
  if (ntok < 0 || V <= 0 || E <= 0)
    return set_error("mt_embedding_fw: bad sizes %lld %lld %lld", (long long)ntok, (long long)V, (long long)E);
  if (ntok == 0) return 0;
  hipLaunchKernelGGL(embed_fw_kernel, dim3(grid_for(ntok * E)), dim3(256), 0, (hipStream_t)stream, out, ids, weight,
                     ntok, V, E);
  return check_hip(hipGetLastError(), "mt_embedding_fw");
}

int mt_embedding_bw(float* dweight, const float* dout, const float* ids, int64_t ntok, int64_t V, int64_t E,
                    void* stream) {
  if (ntok < 0 || V <= 0 || E <= 0)
    return set_error("mt_embedding_bw: bad sizes %lld %lld %lld", (long long)ntok, (long long)V, (long long)E);
  const int64_t nb = (V + kEmbVB - 1) / kEmbVB;
  if (nb > 0x7fffffff) return set_error("mt_embedding_bw: V = %lld", (long long)V);
  hipLaunchKernelGGL(embed_bw_kernel, dim3((unsigned)nb), dim3(1024), 0, (hipStream_t)stream, dweight, dout, ids, ntok,
                     V, E);
  return check_hip(hipGetLastError(), "mt_embedding_bw");
}

static int adam_step(int n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                     float* const* exp_avg_sq, const int64_t* numels, double beta1, double beta2, double eps,
                     double step_size, const float* step_dev, void* stream) {
  if (n_tensors < 0) return set_error("mt_adam_step: n_tensors = %d", n_tensors);
  for (int t0 = 0; t0 < n_tensors; t0 += kAdamMax) {
    AdamArgs a;
    memset(&a, 0, sizeof(a));
    // each constant rounded to fp32 once, as the tensor-op form's scalar operands are
    a.b1 = (float)beta1; a.b2 = (float)beta2; a.c1 = (float)(1.0 - beta1); a.c2 = (float)(1.0 - beta2);
    a.step = (float)step_size; a.eps = (float)eps; a.stepp = step_dev;
    int64_t blocks = 0;
    for (int t = t0; t < std::min(n_tensors, t0 + kAdamMax); ++t) {
      if (numels[t] < 0) return set_error("mt_adam_step: numel %lld", (long long)numels[t]);
      if (numels[t] == 0) continue;
      if (!params[t] || !grads[t] || !exp_avg[t] || !exp_avg_sq[t]) return set_error("mt_adam_step: null pointer");
      a.p[a.nt] = params[t]; a.g[a.nt] = grads[t]; a.m[a.nt] = exp_avg[t]; a.v[a.nt] = exp_avg_sq[t];
      a.n[a.nt] = numels[t];
      a.blk0[a.nt] = (int)blocks;
      blocks += (numels[t] + 1023) / 1024;
      if (blocks > 0x7fffffff) return set_error("mt_adam_step: too many elements");
      ++a.nt;
    }
    if (a.nt == 0) continue;
    a.blk0[a.nt] = (int)blocks;
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
    if (check_hip(hipGetLastError(), "mt_adam_step")) return 1;
  }
  return 0;
}

int mt_adam_step(int n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                 float* const* exp_avg_sq, const int64_t* numels, double beta1, double beta2, double eps,
                 double step_size, void* stream) {
  return adam_step(n_tensors, params, grads, exp_avg, exp_avg_sq, numels, beta1, beta2, eps, step_size, nullptr,
                   stream);
}

int mt_adam_step_dstep(int n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                       float* const* exp_avg_sq, const int64_t* numels, double beta1, double beta2, double eps,
                       const float* step_size, void* stream) {
  if (!step_size) return set_error("mt_adam_step_dstep: null step-size pointer");
  return adam_step(n_tensors, params, grads, exp_avg, exp_avg_sq, numels, beta1, beta2, eps, 0.0, step_size,
                   stream);
}

}  // extern "C"

// ---- reference-compatible host-pointer wrappers (combine.cu:315-580) -----------------
// Same names and argument order as the reference; host NumPy storages and int32
// shapes/strides in, results copied back into `out`. Errors are reported on stderr and in
// mt_last_error(); the process is never terminated.
namespace {
int64_t extent(const int* shape, const int* strides, int dims) {  // max offset + 1
  int64_t e = 0;
  for (int d = 0; d < dims; ++d)
    if (shape[d] > 0) e += (int64_t)(shape[d] - 1) * strides[d];
  return e + 1;
}
struct HostTensor {
  void* dev = nullptr;
  int64_t shape[mt::kMaxDims], strides[mt::kMaxDims];
  ~HostTensor() { if (dev) (void)hipFree(dev); }
  int up(const float* h, const int* shp, const int* str, int dims, const char* w) {
    if (dims < 1 || dims > mt::kMaxDims)
      return mt::set_error("%s: tensor rank %d outside 1..%d", w, dims, mt::kMaxDims);
    if (!shp || !str) return mt::set_error("%s: null shape/stride pointer", w);
    for (int d = 0; d < dims; ++d) { shape[d] = shp[d]; strides[d] = str[d]; }
    const size_t n = (size_t)extent(shp, str, dims) * sizeof(float);
    if (mt::check_hip(hipMalloc(&dev, n), w)) return 1;
    return h ? mt::check_hip(hipMemcpy(dev, h, n, hipMemcpyHostToDevice), w) : 0;
  }
  int down(float* h, const int* shp, const int* str, int dims, const char* w) {
    const size_t n = (size_t)extent(shp, str, dims) * sizeof(float);
    if (mt::check_hip(hipDeviceSynchronize(), w)) return 1;
    return mt::check_hip(hipMemcpy(h, dev, n, hipMemcpyDeviceToHost), w);
  }
};
}  // namespace

extern "C" {

void tensorMap(float* out, int* out_shape, int* out_strides, int out_size, float* in_storage,
               int* in_shape, int* in_strides, int in_size, int shape_size, int fn_id) {
  (void)out_size; (void)in_size;
  HostTensor o, i;
  const char* w = "tensorMap";
  int rc = o.up(out, out_shape, out_strides, shape_size, w) ||
           i.up(in_storage, in_shape, in_strides, shape_size, w) ||
           mt_tensor_map(fn_id, (float*)o.dev, o.shape, o.strides, shape_size,
                         (const float*)i.dev, i.shape, i.strides, shape_size, nullptr) ||
           o.down(out, out_shape, out_strides, shape_size, w);
  if (rc) fprintf(stderr, "tensorMap failed: %s\n", mt_last_error());
}

void tensorZip(float* out, int* out_shape, int* out_strides, int out_size, int out_shape_size,
               float* a_storage, int* a_shape, int* a_strides, int a_size, int a_shape_size,
               float* b_storage, int* b_shape, int* b_strides, int b_size, int b_shape_size,
               int fn_id) {
  (void)out_size; (void)a_size; (void)b_size;
  HostTensor o, a, b;
  const char* w = "tensorZip";
  int rc = o.up(out, out_shape, out_strides, out_shape_size, w) ||
           a.up(a_storage, a_shape, a_strides, a_shape_size, w) ||
           b.up(b_storage, b_shape, b_strides, b_shape_size, w) ||
           mt_tensor_zip(fn_id, (float*)o.dev, o.shape, o.strides, out_shape_size,
                         (const float*)a.dev, a.shape, a.strides, a_shape_size,
                         (const float*)b.dev, b.shape, b.strides, b_shape_size, nullptr) ||
           o.down(out, out_shape, out_strides, out_shape_size, w);
  if (rc) fprintf(stderr, "tensorZip failed: %s\n", mt_last_error());
}

void tensorReduce(float* out, int* out_shape, int* out_strides, int out_size, float* a_storage,
                  int* a_shape, int* a_strides, int reduce_dim, float reduce_value,
                  int shape_size, int fn_id) {
  (void)out_size;
  HostTensor o, a;
  const char* w = "tensorReduce";
  int rc = o.up(out, out_shape, out_strides, shape_size, w) ||
           a.up(a_storage, a_shape, a_strides, shape_size, w) ||
           mt_tensor_reduce(fn_id, (float*)o.dev, o.shape, o.strides, (const float*)a.dev,
                            a.shape, a.strides, shape_size, reduce_dim, reduce_value, nullptr) ||
           o.down(out, out_shape, out_strides, shape_size, w);
  if (rc) fprintf(stderr, "tensorReduce failed: %s\n", mt_last_error());
}

void MatrixMultiply(float* out, int* out_shape, int* out_strides, float* a_storage, int* a_shape,
                    int* a_strides, float* b_storage, int* b_shape, int* b_strides, int batch,
                    int m, int p) {
  HostTensor o, a, b;
  const char* w = "MatrixMultiply";
  int rc = o.up(nullptr, out_shape, out_strides, 3, w) ||
           a.up(a_storage, a_shape, a_strides, 3, w) || b.up(b_storage, b_shape, b_strides, 3, w);
  if (!rc) {
    int64_t as[3] = {a_shape[0] == 1 ? 0 : a.strides[0], a.strides[1], a.strides[2]};
    int64_t bs[3] = {b_shape[0] == 1 ? 0 : b.strides[0], b.strides[1], b.strides[2]};
    rc = mt_matmul_f32((float*)o.dev, (const float*)a.dev, (const float*)b.dev, batch, m, p,
                       a_shape[2], as, bs, o.strides, nullptr) ||
         o.down(out, out_shape, out_strides, 3, w);
  }
  if (rc) fprintf(stderr, "MatrixMultiply failed: %s\n", mt_last_error());
}

}  // extern "C"
