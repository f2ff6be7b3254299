// Companion kernels named in the north star: attention softmax (fwd/bwd) and LayerNorm
// (fwd/bwd), fp32, device pointers.
//
// Contracts (reference file:line):
//  * softmax fwd, src/softmax_kernel.cu:35-224: y = exp(x + mask − max) / (Σ + 1e-8) per
//    row of [B, nh, from, to]; masked entries (mask_future: col > row) take −1e8
//    (REDUCE_FLOAT_INF_NEG, includes/block_reduce.h:13) so a fully masked row stays finite.
//    The reference kernel reads an additive [B, to] mask (:26-33, :53); here the mask is
//    any tensor broadcastable to [B, nh, from, to] given by element strides, which covers
//    [B, to] and also the [B, nh, T, T] / [1, 1, T, T] masks the reference MHA passes
//    (modules_transfomer.py:140-150, defect A.9 in SURVEY.md).
//  * softmax bwd, :308-341: dx = y ∘ (dy − Σ dy∘y).
//  * LayerNorm fwd, src/layernorm_kernel.cu:36-98: μ = E[x], var = E[x²] − μ² + 1e-8
//    (stored with eps), y = γ (x − μ)/√var + β.
//  * LayerNorm bwd, :192-368: dβ = Σ dy, dγ = Σ dy·x̂,
//    dx = (dy·γ − mean(dy·γ) − x̂·mean(dy·γ·x̂)) / √var. (The reference adds eps a
//    second time inside the backward, :229/:310; this is the exact gradient of the forward.)
//
// MI355X design: one wave64 per row with butterfly reductions (no cub/cooperative-group
// dependency), grid-stride over rows, and a deterministic two-stage column reduction for
// dγ/dβ (per-block partials in a caller-given workspace, then one pass) instead of atomics.
// These kernels are HBM-bound, so each row is read from HBM exactly once: when the row
// length is a multiple of 4 and at most 4096, a lane keeps its 16-B pieces of the row in
// registers (NV float4 per lane, templated) between the reduction and the output pass
// (softmax fw/bw, LayerNorm fw, LayerNorm bw), and the LayerNorm backward computes dx and
// its rows' dγ/dβ partials in one pass (a wave per row up to hidden 1024, a workgroup per
// row above). Other shapes take the scalar kernels, which re-read the row (from L2 in
// practice).
#include <stdio.h>
#include <string.h>

#include "../../include/minitorch_hip.h"
#include "fa_common.h"

namespace mt {

int set_error(const char* fmt, ...);
int check_hip(hipError_t e, const char* where);

constexpr float kSoftmaxEps = 1e-8f;
constexpr float kMaskedLogit = -100000000.f;
constexpr float kLnEps = 1e-8f;

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}
__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
  return x;
}

static unsigned row_grid(int64_t rows) {
  int64_t g = (rows + 3) / 4;
  if (g > 256 * 32) g = 256 * 32;
  return (unsigned)(g < 1 ? 1 : g);
}

// ---------------------------------------------------------------------------- softmax
struct SoftmaxArgs {
  float* out; const float* inp; const float* mask;
  int64_t B, nh, from, to;
  int64_t ms[4];  // mask strides (b, h, row, col)
  int mask_future;
};

__global__ __launch_bounds__(256) void softmax_fw_kernel(SoftmaxArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t rows = a.B * a.nh * a.from;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    const int64_t i = r % a.from, bh = r / a.from, h = bh % a.nh, b = bh / a.nh;
    const float* x = a.inp + r * a.to;
    float* y = a.out + r * a.to;
    const float* mrow = a.mask ? a.mask + b * a.ms[0] + h * a.ms[1] + i * a.ms[2] : nullptr;
    auto logit = [&](int64_t j) {
      if (a.mask_future && j > i) return kMaskedLogit;
      float v = x[j];
      if (mrow) v += mrow[j * a.ms[3]];
      return v;
    };
    float mx = kMaskedLogit;
    for (int64_t j = lane; j < a.to; j += 64) mx = fmaxf(mx, logit(j));
    mx = wave_max(mx);
    float s = 0.f;
    for (int64_t j = lane; j < a.to; j += 64) s += __expf(logit(j) - mx);
    s = wave_sum(s);
    const float inv = 1.f / (s + kSoftmaxEps);
    for (int64_t j = lane; j < a.to; j += 64) y[j] = __expf(logit(j) - mx) * inv;
  }
}

__global__ __launch_bounds__(256) void softmax_bw_kernel(float* dinp, const float* dout,
                                                         const float* soft, int64_t rows,
                                                         int64_t len) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    const float* dy = dout + r * len;
    const float* y = soft + r * len;
    float s = 0.f;
    for (int64_t j = lane; j < len; j += 64) s += dy[j] * y[j];
    s = wave_sum(s);
    float* dx = dinp + r * len;
    for (int64_t j = lane; j < len; j += 64) dx[j] = y[j] * (dy[j] - s);
  }
}

// -------------------------------------------------------------------------- layernorm
__global__ __launch_bounds__(256) void ln_fw_kernel(float* ln, float* var_out, float* mean_out,
                                                    const float* inp, const float* gamma,
                                                    const float* beta, int64_t rows, int64_t H) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const bool vec = (H % 4) == 0;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    const float* x = inp + r * H;
    float s = 0.f, ss = 0.f;
    if (vec) {
      for (int64_t j = lane * 4; j < H; j += 256) {
        const float4 v = *(const float4*)(x + j);
        s += v.x + v.y + v.z + v.w;
        ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      }
    } else {
      for (int64_t j = lane; j < H; j += 64) { s += x[j]; ss += x[j] * x[j]; }
    }
    s = wave_sum(s);
    ss = wave_sum(ss);
    const float mean = s / (float)H;
    const float var = ss / (float)H - mean * mean + kLnEps;
    const float rsd = 1.f / sqrtf(var);
    if (lane == 0) { mean_out[r] = mean; var_out[r] = var; }
    float* y = ln + r * H;
    if (vec) {
      for (int64_t j = lane * 4; j < H; j += 256) {
        const float4 v = *(const float4*)(x + j);
        const float4 g = *(const float4*)(gamma + j), bb = *(const float4*)(beta + j);
        *(float4*)(y + j) = make_float4(g.x * ((v.x - mean) * rsd) + bb.x,
                                        g.y * ((v.y - mean) * rsd) + bb.y,
                                        g.z * ((v.z - mean) * rsd) + bb.z,
                                        g.w * ((v.w - mean) * rsd) + bb.w);
      }
    } else {
      for (int64_t j = lane; j < H; j += 64) y[j] = gamma[j] * ((x[j] - mean) * rsd) + beta[j];
    }
  }
}

__global__ __launch_bounds__(256) void ln_bw_dinp_kernel(float* dinp, const float* dout,
                                                         const float* inp, const float* gamma,
                                                         const float* var, const float* mean,
                                                         int64_t rows, int64_t H) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    const float* x = inp + r * H;
    const float* dy = dout + r * H;
    const float mu = mean[r], rsd = 1.f / sqrtf(var[r]);
    float s1 = 0.f, s2 = 0.f;
    for (int64_t j = lane; j < H; j += 64) {
      const float g = dy[j] * gamma[j];
      s1 += g;
      s2 += g * (x[j] - mu) * rsd;
    }
    s1 = wave_sum(s1) / (float)H;
    s2 = wave_sum(s2) / (float)H;
    float* dx = dinp + r * H;
    for (int64_t j = lane; j < H; j += 64) {
      const float xh = (x[j] - mu) * rsd;
      dx[j] = (dy[j] * gamma[j] - s1 - xh * s2) * rsd;
    }
  }
}

// Stage 1: block (x = 64-column group, y = row chunk) writes per-chunk partial sums
// of dβ and dγ into ws[2][chunks][H]. Stage 2 sums the chunks.
constexpr int kLnRowsPerChunk = 256;

__global__ __launch_bounds__(256) void ln_bw_dgb_partial(float* ws, const float* dout,
                                                         const float* inp, const float* var,
                                                         const float* mean, int64_t rows,
                                                         int64_t H, int64_t chunks) {
  __shared__ float sb[4][64], sg[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.y * kLnRowsPerChunk;
  const int64_t r1 = min(rows, r0 + kLnRowsPerChunk);
  float db = 0.f, dg = 0.f;
  if (col < H) {
    for (int64_t r = r0 + wave; r < r1; r += 4) {
      const float dy = dout[r * H + col];
      db += dy;
      dg += dy * (inp[r * H + col] - mean[r]) / sqrtf(var[r]);
    }
  }
  sb[wave][lane] = db;
  sg[wave][lane] = dg;
  __syncthreads();
  if (wave == 0 && col < H) {
    ws[blockIdx.y * H + col] = sb[0][lane] + sb[1][lane] + sb[2][lane] + sb[3][lane];
    ws[(chunks + blockIdx.y) * H + col] = sg[0][lane] + sg[1][lane] + sg[2][lane] + sg[3][lane];
  }
}

__global__ __launch_bounds__(256) void ln_bw_dgb_final(float* dgamma, float* dbeta,
                                                       const float* ws, int64_t H,
                                                       int64_t chunks) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col >= H) return;
  float db = 0.f, dg = 0.f;
  for (int64_t c = 0; c < chunks; ++c) {
    db += ws[c * H + col];
    dg += ws[(chunks + c) * H + col];
  }
  dbeta[col] = db;
  dgamma[col] = dg;
}

static int64_t ln_chunks(int64_t rows) { return (rows + kLnRowsPerChunk - 1) / kLnRowsPerChunk; }

// ---------------------------------------------------- register-resident row kernels (NV)
// Lane l owns the float4 pieces at columns 4 (l + 64 k), k < NV, of its wave's row; pieces
// past the row length are never read or written (len % 4 == 0, so a piece is all in or out).
template <int NV>
__global__ __launch_bounds__(256) void softmax_fw_vec(SoftmaxArgs a, int mvec) {
  const int lane = threadIdx.x & 63;
  const int64_t rows = a.B * a.nh * a.from;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    const int64_t i = r % a.from, bh = r / a.from, h = bh % a.nh, b = bh / a.nh;
    const float* x = a.inp + r * a.to;
    const float* mrow = a.mask ? a.mask + b * a.ms[0] + h * a.ms[1] + i * a.ms[2] : nullptr;
    float4 v[NV];
    float mx = kMaskedLogit;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = 4 * (lane + 64 * k);
      if (c < a.to) {
        v[k] = *(const float4*)(x + c);
        if (mrow) {
          if (mvec) {
            const float4 m = *(const float4*)(mrow + c);
            v[k].x += m.x; v[k].y += m.y; v[k].z += m.z; v[k].w += m.w;
          } else {
            v[k].x += mrow[c * a.ms[3]];
            v[k].y += mrow[(c + 1) * a.ms[3]];
            v[k].z += mrow[(c + 2) * a.ms[3]];
            v[k].w += mrow[(c + 3) * a.ms[3]];
          }
        }
        if (a.mask_future) {
          if (c > i) v[k].x = kMaskedLogit;
          if (c + 1 > i) v[k].y = kMaskedLogit;
          if (c + 2 > i) v[k].z = kMaskedLogit;
          if (c + 3 > i) v[k].w = kMaskedLogit;
        }
        mx = fmaxf(mx, fmaxf(fmaxf(v[k].x, v[k].y), fmaxf(v[k].z, v[k].w)));
      }
    }
    mx = wave_max(mx);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if (4 * (lane + 64 * k) < a.to) {
        v[k].x = __expf(v[k].x - mx); v[k].y = __expf(v[k].y - mx);
        v[k].z = __expf(v[k].z - mx); v[k].w = __expf(v[k].w - mx);
        s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
      }
    }
    const float inv = 1.f / (wave_sum(s) + kSoftmaxEps);
    float* y = a.out + r * a.to;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = 4 * (lane + 64 * k);
      if (c < a.to) *(float4*)(y + c) = make_float4(v[k].x * inv, v[k].y * inv, v[k].z * inv, v[k].w * inv);
    }
  }
}

template <int NV>
__global__ __launch_bounds__(256) void softmax_bw_vec(float* dinp, const float* dout, const float* soft,
                                                      int64_t rows, int64_t len) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    float4 dy[NV], y[NV];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = 4 * (lane + 64 * k);
      if (c < len) {
        dy[k] = *(const float4*)(dout + r * len + c);
        y[k] = *(const float4*)(soft + r * len + c);
        s += (dy[k].x * y[k].x + dy[k].y * y[k].y) + (dy[k].z * y[k].z + dy[k].w * y[k].w);
      }
    }
    s = wave_sum(s);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = 4 * (lane + 64 * k);
      if (c < len)
        *(float4*)(dinp + r * len + c) = make_float4(y[k].x * (dy[k].x - s), y[k].y * (dy[k].y - s),
                                                     y[k].z * (dy[k].z - s), y[k].w * (dy[k].w - s));
    }
  }
}

template <int NV>
__global__ __launch_bounds__(256) void ln_fw_vec(float* ln, float* var_out, float* mean_out,
                                                 const float* inp, const float* gamma,
                                                 const float* beta, int64_t rows, int64_t H) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    float4 v[NV];
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = 4 * (lane + 64 * k);
      if (c < H) {
        v[k] = *(const float4*)(inp + r * H + c);
        s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
        ss += (v[k].x * v[k].x + v[k].y * v[k].y) + (v[k].z * v[k].z + v[k].w * v[k].w);
      }
    }
    s = wave_sum(s);
    ss = wave_sum(ss);
    const float mean = s / (float)H;
    const float var = ss / (float)H - mean * mean + kLnEps;
    const float rsd = 1.f / sqrtf(var);
    if (lane == 0) { mean_out[r] = mean; var_out[r] = var; }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = 4 * (lane + 64 * k);
      if (c < H) {
        const float4 g = *(const float4*)(gamma + c), bb = *(const float4*)(beta + c);
        *(float4*)(ln + r * H + c) = make_float4(g.x * ((v[k].x - mean) * rsd) + bb.x,
                                                 g.y * ((v[k].y - mean) * rsd) + bb.y,
                                                 g.z * ((v[k].z - mean) * rsd) + bb.z,
                                                 g.w * ((v[k].w - mean) * rsd) + bb.w);
      }
    }
  }
}

// LayerNorm backward (hidden <= 1024), dx for every row and (PARTIAL) this block's dγ/dβ partial sums over its
// rows: ws[block][0][H] = Σ dy, ws[block][1][H] = Σ dy·x̂ (the four waves' register partials
// added in LDS in wave order: deterministic).
template <int NV, bool PARTIAL>
__global__ __launch_bounds__(256) void ln_bw_vec(float* dinp, float* ws, const float* dout,
                                                 const float* inp, const float* gamma,
                                                 const float* var, const float* mean, int64_t rows,
                                                 int64_t H) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t nw = (int64_t)gridDim.x * 4;
  float4 db[PARTIAL ? NV : 1], dg[PARTIAL ? NV : 1];
  if (PARTIAL) {
#pragma unroll
    for (int k = 0; k < NV; ++k) { db[k] = make_float4(0.f, 0.f, 0.f, 0.f); dg[k] = db[k]; }
  }
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < rows; r += nw) {
    const float mu = mean[r], rsd = 1.f / sqrtf(var[r]);
    float4 dy[NV], xh[NV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = 4 * (lane + 64 * k);
      if (c < H) {
        dy[k] = *(const float4*)(dout + r * H + c);
        const float4 x = *(const float4*)(inp + r * H + c), g = *(const float4*)(gamma + c);
        xh[k] = make_float4((x.x - mu) * rsd, (x.y - mu) * rsd, (x.z - mu) * rsd, (x.w - mu) * rsd);
        const float4 dyg = make_float4(dy[k].x * g.x, dy[k].y * g.y, dy[k].z * g.z, dy[k].w * g.w);
        s1 += (dyg.x + dyg.y) + (dyg.z + dyg.w);
        s2 += (dyg.x * xh[k].x + dyg.y * xh[k].y) + (dyg.z * xh[k].z + dyg.w * xh[k].w);
        if (PARTIAL) {
          db[k].x += dy[k].x; db[k].y += dy[k].y; db[k].z += dy[k].z; db[k].w += dy[k].w;
          dg[k].x += dy[k].x * xh[k].x; dg[k].y += dy[k].y * xh[k].y;
          dg[k].z += dy[k].z * xh[k].z; dg[k].w += dy[k].w * xh[k].w;
        }
      }
    }
    s1 = wave_sum(s1) / (float)H;
    s2 = wave_sum(s2) / (float)H;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = 4 * (lane + 64 * k);
      if (c < H) {
        const float4 g = *(const float4*)(gamma + c);
        *(float4*)(dinp + r * H + c) = make_float4((dy[k].x * g.x - s1 - xh[k].x * s2) * rsd,
                                                   (dy[k].y * g.y - s1 - xh[k].y * s2) * rsd,
                                                   (dy[k].z * g.z - s1 - xh[k].z * s2) * rsd,
                                                   (dy[k].w * g.w - s1 - xh[k].w * s2) * rsd);
      }
    }
  }
  if (PARTIAL) {
    __shared__ float4 sp[4][2][64 * NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      sp[wave][0][lane + 64 * k] = db[k];
      sp[wave][1][lane + 64 * k] = dg[k];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < 2 * (H / 4); j += 256) {
      const int w = j / (H / 4), c4 = j % (H / 4);
      float4 t = sp[0][w][c4];
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        const float4 u = sp[q][w][c4];
        t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
      }
      *(float4*)(ws + ((int64_t)blockIdx.x * 2 + w) * H + 4 * c4) = t;
    }
  }
}

// LayerNorm forward for 1024 < hidden <= 4096 (hidden % 4 == 0): a workgroup per row, thread t
// owning the float4 pieces t + 256 k (k < NV), γ and β in registers; the row sums go through
// LDS (one barrier per row, exchange slots alternating by row parity).
template <int NV>
__global__ __launch_bounds__(256) void ln_fw_row(float* ln, float* var_out, float* mean_out,
                                                 const float* inp, const float* gamma,
                                                 const float* beta, int64_t rows, int64_t H) {
  __shared__ float red[2][4][2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float4 gm[NV], bt[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t c = 4 * (tid + 256 * k);
    gm[k] = c < H ? *(const float4*)(gamma + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    bt[k] = c < H ? *(const float4*)(beta + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  int par = 0;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x, par ^= 1) {
    float4 v[NV];
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = 4 * (tid + 256 * k);
      if (c < H) {
        v[k] = *(const float4*)(inp + r * H + c);
        s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
        ss += (v[k].x * v[k].x + v[k].y * v[k].y) + (v[k].z * v[k].z + v[k].w * v[k].w);
      }
    }
    s = wave_sum(s);
    ss = wave_sum(ss);
    if (lane == 0) { red[par][wave][0] = s; red[par][wave][1] = ss; }
    __syncthreads();
    s = ((red[par][0][0] + red[par][1][0]) + red[par][2][0]) + red[par][3][0];
    ss = ((red[par][0][1] + red[par][1][1]) + red[par][2][1]) + red[par][3][1];
    const float mean = s / (float)H;
    const float var = ss / (float)H - mean * mean + kLnEps;
    const float rsd = 1.f / sqrtf(var);
    if (tid == 0) { mean_out[r] = mean; var_out[r] = var; }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = 4 * (tid + 256 * k);
      if (c < H)
        *(float4*)(ln + r * H + c) = make_float4(gm[k].x * ((v[k].x - mean) * rsd) + bt[k].x,
                                                 gm[k].y * ((v[k].y - mean) * rsd) + bt[k].y,
                                                 gm[k].z * ((v[k].z - mean) * rsd) + bt[k].z,
                                                 gm[k].w * ((v[k].w - mean) * rsd) + bt[k].w);
    }
  }
}

// LayerNorm backward for 1024 < hidden <= 4096 (hidden % 4 == 0): a workgroup per row, thread
// t owning the float4 pieces t + 256 k (k < NV) of every row it visits, so its dγ/dβ
// partials stay in registers; the row sums go through LDS (one barrier per row, the
// exchange slots alternating by row parity). Writes dx and the block's [2][H] slab.
template <int NV>
__global__ __launch_bounds__(256) void ln_bw_row(float* dinp, float* ws, const float* dout,
                                                 const float* inp, const float* gamma,
                                                 const float* var, const float* mean, int64_t rows,
                                                 int64_t H) {
  __shared__ float red[2][4][2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float4 db[NV], dg[NV], gm[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    db[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    dg[k] = db[k];
    const int64_t c = 4 * (tid + 256 * k);
    gm[k] = c < H ? *(const float4*)(gamma + c) : db[k];
  }
  int par = 0;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x, par ^= 1) {
    const float mu = mean[r], rsd = 1.f / sqrtf(var[r]);
    float4 dy[NV], xh[NV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = 4 * (tid + 256 * k);
      if (c < H) {
        dy[k] = *(const float4*)(dout + r * H + c);
        const float4 x = *(const float4*)(inp + r * H + c);
        xh[k] = make_float4((x.x - mu) * rsd, (x.y - mu) * rsd, (x.z - mu) * rsd, (x.w - mu) * rsd);
        const float4 g = make_float4(dy[k].x * gm[k].x, dy[k].y * gm[k].y, dy[k].z * gm[k].z, dy[k].w * gm[k].w);
        s1 += (g.x + g.y) + (g.z + g.w);
        s2 += (g.x * xh[k].x + g.y * xh[k].y) + (g.z * xh[k].z + g.w * xh[k].w);
        db[k].x += dy[k].x; db[k].y += dy[k].y; db[k].z += dy[k].z; db[k].w += dy[k].w;
        dg[k].x += dy[k].x * xh[k].x; dg[k].y += dy[k].y * xh[k].y;
        dg[k].z += dy[k].z * xh[k].z; dg[k].w += dy[k].w * xh[k].w;
      }
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) { red[par][wave][0] = s1; red[par][wave][1] = s2; }
    __syncthreads();  // (the other parity's slots were last read before this barrier)
    s1 = (((red[par][0][0] + red[par][1][0]) + red[par][2][0]) + red[par][3][0]) / (float)H;
    s2 = (((red[par][0][1] + red[par][1][1]) + red[par][2][1]) + red[par][3][1]) / (float)H;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = 4 * (tid + 256 * k);
      if (c < H)
        *(float4*)(dinp + r * H + c) = make_float4((dy[k].x * gm[k].x - s1 - xh[k].x * s2) * rsd,
                                                   (dy[k].y * gm[k].y - s1 - xh[k].y * s2) * rsd,
                                                   (dy[k].z * gm[k].z - s1 - xh[k].z * s2) * rsd,
                                                   (dy[k].w * gm[k].w - s1 - xh[k].w * s2) * rsd);
    }
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t c = 4 * (tid + 256 * k);
    if (c < H) {
      *(float4*)(ws + ((int64_t)blockIdx.x * 2) * H + c) = db[k];
      *(float4*)(ws + ((int64_t)blockIdx.x * 2 + 1) * H + c) = dg[k];
    }
  }
}

// The blocks' [2][H] slabs summed in segments of 64 slabs: block (column group x, segment y),
// wave w adds slabs 64 y + w + 4 k in order, the four waves are added in wave order
// (deterministic); out[y][2][H].
constexpr int kSlabSeg = 64;
__global__ __launch_bounds__(256) void ln_bw_vec_seg(float* out, const float* ws, int64_t H, int64_t nb) {
  __shared__ float red[4][2][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + lane;
  const int64_t s0 = (int64_t)blockIdx.y * kSlabSeg, s1 = min(nb, s0 + kSlabSeg);
  float db = 0.f, dg = 0.f;
  if (col < H) {
#pragma unroll 4
    for (int64_t c = s0 + wave; c < s1; c += 4) {
      db += ws[(2 * c) * H + col];
      dg += ws[(2 * c + 1) * H + col];
    }
  }
  red[wave][0][lane] = db;
  red[wave][1][lane] = dg;
  __syncthreads();
  if (wave == 0 && col < H) {
    out[(2 * blockIdx.y) * H + col] = ((red[0][0][lane] + red[1][0][lane]) + red[2][0][lane]) + red[3][0][lane];
    out[(2 * blockIdx.y + 1) * H + col] = ((red[0][1][lane] + red[1][1][lane]) + red[2][1][lane]) + red[3][1][lane];
  }
}

// The blocks' dγ/dβ partials in one launch (round 5): the slab [nb][2][H] read as [nb][2H], a
// workgroup per 4 adjacent columns over all nb partial rows (lane t: rows t, t + T, ...; a fixed
// pairwise tree through LDS), so nothing crosses a workgroup: deterministic, and one launch where
// the segment + final pair took two (config 5, H = 256, nb = 1024: 5.1 + 4.8 µs per LayerNorm).
// The 8 column groups sharing a 128-B line run on one XCD (blockIdx % 8).
__global__ __launch_bounds__(1024) void ln_bw_vec_colsum(float* dgamma, float* dbeta, const float* ws,
                                                         int64_t H, int64_t nb, int ncg) {
  __shared__ float4 red[1024];
  const int b = blockIdx.x;
  const int cg = ncg >= 64 ? (((b & 7) + 8 * ((b >> 3) >> 3)) * 8 + ((b >> 3) & 7)) : b;
  if (cg >= ncg) return;  // padding workgroups of the XCD placement: uniform, before the barrier
  const int t = threadIdx.x, T = blockDim.x;  // T = min(1024, nb): every lane has a row
  const int64_t W = 2 * H;
  const float* src = ws + (int64_t)cg * 4;
  float4 v = *(const float4*)(src + (int64_t)t * W);
  for (int64_t j = t + T; j < nb; j += 8 * (int64_t)T) {
    float4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      x[u] = j + (int64_t)u * T < nb ? *(const float4*)(src + (j + (int64_t)u * T) * W)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 8; ++u) { v.x += x[u].x; v.y += x[u].y; v.z += x[u].z; v.w += x[u].w; }
  }
  red[t] = v;
  __syncthreads();
  int p2 = 1;
  while (p2 < T) p2 <<= 1;
  for (int st = p2 >> 1; st > 0; st >>= 1) {
    if (t < st && t + st < T) {
      const float4 y = red[t + st];
      float4 x = red[t];
      x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
      red[t] = x;
    }
    __syncthreads();
  }
  if (t == 0) {
    const float r[4] = {red[0].x, red[0].y, red[0].z, red[0].w};
    for (int k = 0; k < 4; ++k) {
      const int64_t c = (int64_t)cg * 4 + k;
      if (c < H) dbeta[c] = r[k];
      else dgamma[c - H] = r[k];
    }
  }
}
__global__ __launch_bounds__(256) void ln_bw_vec_final(float* dgamma, float* dbeta, const float* ws,
                                                       int64_t H, int64_t nb) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col >= H) return;
  float db = 0.f, dg = 0.f;
  for (int64_t c = 0; c < nb; ++c) {
    db += ws[(2 * c) * H + col];
    dg += ws[(2 * c + 1) * H + col];
  }
  dbeta[col] = db;
  dgamma[col] = dg;
}

// float4 pieces per lane for a row of `len` (a multiple of 4): 1, 2, 4, 8 or 16; 0 when the
// row needs the scalar kernels (len % 4 != 0 or len > 4096)
static int row_nv(int64_t len) {
  if (len % 4 != 0 || len > 4096) return 0;
  const int64_t p = (len / 4 + 63) / 64;
  return p <= 1 ? 1 : p <= 2 ? 2 : p <= 4 ? 4 : p <= 8 ? 8 : 16;
}
static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
// blocks of the fused LayerNorm backward (its dγ/dβ partials are one [2][H] slab per block):
// a wave per row up to hidden 1024, a workgroup per row above
static int64_t ln_vec_blocks(int64_t rows, int64_t H) {
  const int64_t g = H <= 1024 ? (rows + 3) / 4 : rows, cap = H <= 1024 ? 1024 : 512;
  return g > cap ? cap : (g < 1 ? 1 : g);
}

// ---- softmax cross-entropy (reference minitorch/nn.py softmax_loss) -------------------------
// loss[r] = logsumexp(x[r, :]) - x[r, t_r], the reference's composition (max, shift, exp, sum,
// log, one-hot pick: ten elementwise passes over the [rows, C] logits plus as many in the
// backward) as one read of the row: an online (max, sum) per lane, combined across the
// workgroup, lse[r] kept for the backward. Backward: dx = g[r] (exp(x - lse[r]) - [j == t_r]),
// one read and one write. One 256-thread workgroup per row (grid-stride), 16-B vectors when
// the rows are 16-B aligned.
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float n = fmaxf(m, m2);
  s = (m == -INFINITY ? 0.f : s * expf(m - n)) + (m2 == -INFINITY ? 0.f : s2 * expf(m2 - n));
  m = n;
}
__device__ __forceinline__ void lse_add(float& m, float& s, float x) {
  if (x > m) {
    s = (m == -INFINITY ? 0.f : s * expf(m - x)) + 1.f;
    m = x;
  } else {
    s += expf(x - m);
  }
}

__global__ __launch_bounds__(256) void xent_fw_kernel(float* loss, float* lse, const float* x,
                                                      const float* tgt, int64_t rows, int64_t C,
                                                      int vec) {
  __shared__ float red_m[4], red_s[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const float* xr = x + r * C;
    float m = -INFINITY, s = 0.f;
    int64_t j0 = 0;
    if (vec) {
      for (int64_t j = 4 * (int64_t)tid; j + 3 < C; j += 1024) {
        const float4 v = *(const float4*)(xr + j);
        lse_add(m, s, v.x); lse_add(m, s, v.y); lse_add(m, s, v.z); lse_add(m, s, v.w);
      }
      j0 = C / 4 * 4;
    }
    for (int64_t j = j0 + tid; j < C; j += 256) lse_add(m, s, xr[j]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lse_merge(m, s, __shfl_xor(m, o), __shfl_xor(s, o));
    if (lane == 0) { red_m[w] = m; red_s[w] = s; }
    __syncthreads();
    if (tid == 0) {
      float M = red_m[0], S = red_s[0];
      for (int i = 1; i < 4; ++i) lse_merge(M, S, red_m[i], red_s[i]);
      const float l = M + logf(S);
      const int64_t t = (int64_t)tgt[r];
      lse[r] = l;
      loss[r] = l - ((t >= 0 && t < C) ? xr[t] : 0.f);
    }
    __syncthreads();
  }
}

// Rows of up to 16384 classes (16-B aligned, C % 4 == 0): the row is loaded into registers in one
// burst (up to 16 float4 per lane, all loads in flight together, where the online form above
// waits on each load before its exp), then max and sum are two workgroup reductions over the
// resident values: one exp per element and no branch. Config 5's 10000-class rows take 10 loads.
constexpr int kXentRegVec = 16;
__global__ __launch_bounds__(256) void xent_fw_reg_kernel(float* loss, float* lse, const float* x,
                                                          const float* tgt, int64_t rows, int C) {
  __shared__ float red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nk = (C + 1023) / 1024;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const float* xr = x + r * C;
    float4 v[kXentRegVec];
#pragma unroll
    for (int k = 0; k < kXentRegVec; ++k) {
      const int j = 4 * tid + 1024 * k;
      if (k < nk && j < C) v[k] = *(const float4*)(xr + j);
      else v[k] = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    }
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < kXentRegVec; ++k)
      if (k < nk) m = fmaxf(m, fmaxf(fmaxf(v[k].x, v[k].y), fmaxf(v[k].z, v[k].w)));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) red[0][w] = m;
    __syncthreads();
    const float M = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kXentRegVec; ++k)
      if (k < nk) s += (expf(v[k].x - M) + expf(v[k].y - M)) + (expf(v[k].z - M) + expf(v[k].w - M));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) red[1][w] = s;
    __syncthreads();
    if (tid == 0) {
      const float l = M + logf((red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
      const int64_t t = (int64_t)tgt[r];
      lse[r] = l;
      loss[r] = l - ((t >= 0 && t < C) ? xr[t] : 0.f);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void xent_bw_kernel(float* dx, const float* g, const float* x,
                                                      const float* tgt, const float* lse,
                                                      int64_t rows, int64_t C, int vec) {
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const float* xr = x + r * C;
    float* dr = dx + r * C;
    const float gr = g[r], l = lse[r];
    const int64_t t = (int64_t)tgt[r];
    int64_t j0 = 0;
    if (vec) {
      for (int64_t j = 4 * (int64_t)threadIdx.x; j + 3 < C; j += 1024) {
        const float4 v = *(const float4*)(xr + j);
        float4 o = make_float4(gr * (expf(v.x - l) - (j == t ? 1.f : 0.f)),
                               gr * (expf(v.y - l) - (j + 1 == t ? 1.f : 0.f)),
                               gr * (expf(v.z - l) - (j + 2 == t ? 1.f : 0.f)),
                               gr * (expf(v.w - l) - (j + 3 == t ? 1.f : 0.f)));
        *(float4*)(dr + j) = o;
      }
      j0 = C / 4 * 4;
    }
    for (int64_t j = j0 + threadIdx.x; j < C; j += 256) dr[j] = gr * (expf(xr[j] - l) - (j == t ? 1.f : 0.f));
  }
}

}  // namespace mt

using namespace mt;

extern "C" {

int mt_softmax_xent_fw(float* loss, float* lse, const float* logits, const float* target, int64_t rows,
                       int64_t classes, void* stream) {
  if (rows <= 0 || classes <= 0) return set_error("mt_softmax_xent_fw: bad sizes");
  const int vec = (classes % 4 == 0) && al16(logits);
  const unsigned grid = (unsigned)(rows < 65536 ? rows : 65536);
  if (vec && classes <= 1024 * kXentRegVec)
    hipLaunchKernelGGL(xent_fw_reg_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, loss, lse, logits,
                       target, rows, (int)classes);
  else
    hipLaunchKernelGGL(xent_fw_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, loss, lse, logits, target,
                       rows, classes, vec);
  return check_hip(hipGetLastError(), "mt_softmax_xent_fw");
}

int mt_softmax_xent_bw(float* dlogits, const float* dloss, const float* logits, const float* target,
                       const float* lse, int64_t rows, int64_t classes, void* stream) {
  if (rows <= 0 || classes <= 0) return set_error("mt_softmax_xent_bw: bad sizes");
  const int vec = (classes % 4 == 0) && al16(logits) && al16(dlogits);
  const unsigned grid = (unsigned)(rows < 65536 ? rows : 65536);
  hipLaunchKernelGGL(xent_bw_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, dlogits, dloss, logits,
                     target, lse, rows, classes, vec);
  return check_hip(hipGetLastError(), "mt_softmax_xent_bw");
}

int mt_attn_softmax_fw(float* out, const float* inp, const float* mask, int64_t B, int64_t nh,
                       int64_t from_len, int64_t to_len, const int64_t* mask_strides,
                       int mask_future, void* stream) {
  if (B <= 0 || nh <= 0 || from_len <= 0 || to_len <= 0)
    return set_error("mt_attn_softmax_fw: bad sizes");
  if (mask && !mask_strides) return set_error("mt_attn_softmax_fw: mask without strides");
  SoftmaxArgs a;
  memset(&a, 0, sizeof(a));
  a.out = out; a.inp = inp; a.mask = mask;
  a.B = B; a.nh = nh; a.from = from_len; a.to = to_len;
  if (mask)
    for (int i = 0; i < 4; ++i) a.ms[i] = mask_strides[i];
  a.mask_future = mask_future;
  const dim3 grid(row_grid(B * nh * from_len));
  hipStream_t st = (hipStream_t)stream;
  const int nv = (al16(out) && al16(inp)) ? row_nv(to_len) : 0;
  const int mvec = mask && a.ms[3] == 1 && a.ms[0] % 4 == 0 && a.ms[1] % 4 == 0 && a.ms[2] % 4 == 0 &&
                   al16(mask);
  switch (nv) {
    case 1: hipLaunchKernelGGL(softmax_fw_vec<1>, grid, dim3(256), 0, st, a, mvec); break;
    case 2: hipLaunchKernelGGL(softmax_fw_vec<2>, grid, dim3(256), 0, st, a, mvec); break;
    case 4: hipLaunchKernelGGL(softmax_fw_vec<4>, grid, dim3(256), 0, st, a, mvec); break;
    case 8: hipLaunchKernelGGL(softmax_fw_vec<8>, grid, dim3(256), 0, st, a, mvec); break;
    case 16: hipLaunchKernelGGL(softmax_fw_vec<16>, grid, dim3(256), 0, st, a, mvec); break;
    default: hipLaunchKernelGGL(softmax_fw_kernel, grid, dim3(256), 0, st, a); break;
  }
  return check_hip(hipGetLastError(), "mt_attn_softmax_fw");
}

int mt_attn_softmax_bw(float* dinp, const float* dout, const float* soft, int64_t rows,
                       int64_t softmax_len, void* stream) {
  if (rows <= 0 || softmax_len <= 0) return set_error("mt_attn_softmax_bw: bad sizes");
  const dim3 grid(row_grid(rows));
  hipStream_t st = (hipStream_t)stream;
  const int nv = (al16(dinp) && al16(dout) && al16(soft)) ? row_nv(softmax_len) : 0;
  switch (nv) {
    case 1: hipLaunchKernelGGL(softmax_bw_vec<1>, grid, dim3(256), 0, st, dinp, dout, soft, rows, softmax_len); break;
    case 2: hipLaunchKernelGGL(softmax_bw_vec<2>, grid, dim3(256), 0, st, dinp, dout, soft, rows, softmax_len); break;
    case 4: hipLaunchKernelGGL(softmax_bw_vec<4>, grid, dim3(256), 0, st, dinp, dout, soft, rows, softmax_len); break;
    case 8: hipLaunchKernelGGL(softmax_bw_vec<8>, grid, dim3(256), 0, st, dinp, dout, soft, rows, softmax_len); break;
    case 16: hipLaunchKernelGGL(softmax_bw_vec<16>, grid, dim3(256), 0, st, dinp, dout, soft, rows, softmax_len); break;
    default: hipLaunchKernelGGL(softmax_bw_kernel, grid, dim3(256), 0, st, dinp, dout, soft, rows, softmax_len); break;
  }
  return check_hip(hipGetLastError(), "mt_attn_softmax_bw");
}

int mt_layernorm_fw(float* ln_res, float* var, float* mean, const float* inp, const float* gamma,
                    const float* beta, int64_t rows, int64_t hidden, void* stream) {
  if (rows <= 0 || hidden <= 0) return set_error("mt_layernorm_fw: bad sizes");
  const dim3 grid(row_grid(rows));
  hipStream_t st = (hipStream_t)stream;
  const int nv = (al16(ln_res) && al16(inp) && al16(gamma) && al16(beta)) ? row_nv(hidden) : 0;
#define MT_LN_FW(NV) hipLaunchKernelGGL(ln_fw_vec<NV>, grid, dim3(256), 0, st, ln_res, var, mean, inp, gamma, beta, rows, hidden)
  switch (nv) {
    case 1: MT_LN_FW(1); break;
    case 2: MT_LN_FW(2); break;
    case 4: MT_LN_FW(4); break;
    case 8:  // 1024 < hidden <= 2048: a workgroup per row
      hipLaunchKernelGGL(ln_fw_row<2>, dim3((unsigned)(rows < 2048 ? rows : 2048)), dim3(256), 0, st, ln_res, var,
                         mean, inp, gamma, beta, rows, hidden);
      break;
    case 16:
      hipLaunchKernelGGL(ln_fw_row<4>, dim3((unsigned)(rows < 2048 ? rows : 2048)), dim3(256), 0, st, ln_res, var,
                         mean, inp, gamma, beta, rows, hidden);
      break;
    default:
      hipLaunchKernelGGL(ln_fw_kernel, grid, dim3(256), 0, st, ln_res, var, mean, inp, gamma, beta, rows, hidden);
      break;
  }
#undef MT_LN_FW
  return check_hip(hipGetLastError(), "mt_layernorm_fw");
}

int64_t mt_layernorm_bw_workspace_bytes(int64_t rows, int64_t hidden) {
  // fused path: one [2][H] slab per block plus one per 64-slab segment
  const int64_t nb = ln_vec_blocks(rows, hidden), vec = nb + (nb + kSlabSeg - 1) / kSlabSeg;
  const int64_t slabs = ln_chunks(rows) > vec ? ln_chunks(rows) : vec;
  return 2 * slabs * hidden * (int64_t)sizeof(float);
}

int mt_layernorm_bw(float* gamma_grad, float* beta_grad, float* inp_grad, const float* out_grad,
                    const float* inp, const float* gamma, const float* beta, const float* var,
                    const float* mean, int64_t rows, int64_t hidden, void* workspace,
                    void* stream) {
  (void)beta;
  if (rows <= 0 || hidden <= 0) return set_error("mt_layernorm_bw: bad sizes");
  if (!workspace) return set_error("mt_layernorm_bw: null workspace");
  hipStream_t st = (hipStream_t)stream;
  const int nv = (al16(inp_grad) && al16(out_grad) && al16(inp) && al16(gamma) && al16(workspace))
                     ? row_nv(hidden) : 0;
  if (nv >= 1) {  // one pass: dx and the per-block dγ/dβ partials, then the blocks' sum
    const int64_t nb = ln_vec_blocks(rows, hidden);
    float* ws = (float*)workspace;
#define MT_LN_BW(NV) hipLaunchKernelGGL((ln_bw_vec<NV, true>), dim3((unsigned)nb), dim3(256), 0, st, inp_grad, ws, out_grad, inp, gamma, var, mean, rows, hidden)
#define MT_LN_BW_ROW(NV) hipLaunchKernelGGL(ln_bw_row<NV>, dim3((unsigned)nb), dim3(256), 0, st, inp_grad, ws, out_grad, inp, gamma, var, mean, rows, hidden)
    switch (nv) {
      case 1: MT_LN_BW(1); break;
      case 2: MT_LN_BW(2); break;
      case 4: MT_LN_BW(4); break;
      case 8: MT_LN_BW_ROW(2); break;   // hidden <= 2048: 2 float4 per thread
      default: MT_LN_BW_ROW(4); break;  // hidden <= 4096
    }
#undef MT_LN_BW
#undef MT_LN_BW_ROW
    if (check_hip(hipGetLastError(), "mt_layernorm_bw(fused)")) return 1;
    if (hidden % 4 == 0 && nb >= 1) {
      const int ncg = (int)(hidden / 2);  // 2H / 4 column groups
      const unsigned gx = (unsigned)(ncg >= 64 ? (ncg + 63) / 64 * 64 : ncg);
      const int T = (int)(nb < 1024 ? nb : 1024);
      hipLaunchKernelGGL(ln_bw_vec_colsum, dim3(gx), dim3(T), 0, st, gamma_grad, beta_grad, (const float*)ws,
                         hidden, nb, ncg);
      return check_hip(hipGetLastError(), "mt_layernorm_bw(colsum)");
    }
    const int64_t nseg = (nb + kSlabSeg - 1) / kSlabSeg;
    float* ws2 = ws + 2 * nb * hidden;
    hipLaunchKernelGGL(ln_bw_vec_seg, dim3((unsigned)((hidden + 63) / 64), (unsigned)nseg), dim3(256), 0, st,
                       ws2, (const float*)ws, hidden, nb);
    if (check_hip(hipGetLastError(), "mt_layernorm_bw(segments)")) return 1;
    hipLaunchKernelGGL(ln_bw_vec_final, dim3((unsigned)((hidden + 255) / 256)), dim3(256), 0, st,
                       gamma_grad, beta_grad, (const float*)ws2, hidden, nseg);
    return check_hip(hipGetLastError(), "mt_layernorm_bw(final)");
  }
  const int64_t chunks = ln_chunks(rows);
  if (chunks > 65535) return set_error("mt_layernorm_bw: too many rows");
  hipLaunchKernelGGL(ln_bw_dgb_partial, dim3((unsigned)((hidden + 63) / 64), (unsigned)chunks),
                     dim3(256), 0, st, (float*)workspace, out_grad, inp, var, mean, rows, hidden,
                     chunks);
  if (check_hip(hipGetLastError(), "mt_layernorm_bw(partial)")) return 1;
  hipLaunchKernelGGL(ln_bw_dgb_final, dim3((unsigned)((hidden + 255) / 256)), dim3(256), 0, st,
                     gamma_grad, beta_grad, (const float*)workspace, hidden, chunks);
  if (check_hip(hipGetLastError(), "mt_layernorm_bw(final)")) return 1;
  hipLaunchKernelGGL(ln_bw_dinp_kernel, dim3(row_grid(rows)), dim3(256), 0, st, inp_grad,
                     out_grad, inp, gamma, var, mean, rows, hidden);
  return check_hip(hipGetLastError(), "mt_layernorm_bw(dinp)");
}

// ---- reference-compatible host-pointer wrappers (copy in, run, copy out) -------------
static int h2d(void** d, const void* h, size_t n, const char* w) {
  if (check_hip(hipMalloc(d, n ? n : 4), w)) return 1;
  return h ? check_hip(hipMemcpy(*d, h, n, hipMemcpyHostToDevice), w) : 0;
}

/* reference src/softmax_kernel.cu:233 — attn_mask is [batch, to_len] (or NULL). */
void launch_attn_softmax(float* inp, const float* attn_mask, int batch_size, int nhead,
                         int from_len, int to_len, bool mask_future, void* stream) {
  const size_t n = (size_t)batch_size * nhead * from_len * to_len * 4;
  const size_t mn = (size_t)batch_size * to_len * 4;
  void *d_inp = nullptr, *d_mask = nullptr;
  int64_t ms[4] = {to_len, 0, 0, 1};
  int rc = h2d(&d_inp, inp, n, "launch_attn_softmax") ||
           (attn_mask && h2d(&d_mask, attn_mask, mn, "launch_attn_softmax")) ||
           mt_attn_softmax_fw((float*)d_inp, (const float*)d_inp, (const float*)d_mask,
                              batch_size, nhead, from_len, to_len, attn_mask ? ms : nullptr,
                              mask_future ? 1 : 0, stream) ||
           check_hip(hipStreamSynchronize((hipStream_t)stream), "launch_attn_softmax") ||
           check_hip(hipMemcpy(inp, d_inp, n, hipMemcpyDeviceToHost), "launch_attn_softmax");
  if (rc) fprintf(stderr, "launch_attn_softmax failed: %s\n", mt_last_error());
  if (d_inp) (void)hipFree(d_inp);
  if (d_mask) (void)hipFree(d_mask);
}

/* reference src/softmax_kernel.cu:345 — in place on out_grad. */
void launch_attn_softmax_bw(float* out_grad, const float* soft_inp, int rows, int softmax_len,
                            void* stream) {
  const size_t n = (size_t)rows * softmax_len * 4;
  void *d_g = nullptr, *d_s = nullptr;
  int rc = h2d(&d_g, out_grad, n, "launch_attn_softmax_bw") ||
           h2d(&d_s, soft_inp, n, "launch_attn_softmax_bw") ||
           mt_attn_softmax_bw((float*)d_g, (const float*)d_g, (const float*)d_s, rows, softmax_len,
                              stream) ||
           check_hip(hipStreamSynchronize((hipStream_t)stream), "launch_attn_softmax_bw") ||
           check_hip(hipMemcpy(out_grad, d_g, n, hipMemcpyDeviceToHost), "launch_attn_softmax_bw");
  if (rc) fprintf(stderr, "launch_attn_softmax_bw failed: %s\n", mt_last_error());
  if (d_g) (void)hipFree(d_g);
  if (d_s) (void)hipFree(d_s);
}

/* reference src/layernorm_kernel.cu:101 */
void launch_layernorm(float* ln_res, float* vars, float* means, const float* inp,
                      const float* scale, const float* bias, int batch_size, int hidden_dim,
                      void* stream) {
  const size_t n = (size_t)batch_size * hidden_dim * 4, h = (size_t)hidden_dim * 4,
               r = (size_t)batch_size * 4;
  void *d_ln = nullptr, *d_var = nullptr, *d_mean = nullptr, *d_inp = nullptr, *d_g = nullptr,
       *d_b = nullptr;
  const char* w = "launch_layernorm";
  int rc = h2d(&d_ln, nullptr, n, w) || h2d(&d_var, nullptr, r, w) || h2d(&d_mean, nullptr, r, w) ||
           h2d(&d_inp, inp, n, w) || h2d(&d_g, scale, h, w) || h2d(&d_b, bias, h, w) ||
           mt_layernorm_fw((float*)d_ln, (float*)d_var, (float*)d_mean, (const float*)d_inp,
                           (const float*)d_g, (const float*)d_b, batch_size, hidden_dim, stream) ||
           check_hip(hipStreamSynchronize((hipStream_t)stream), w) ||
           check_hip(hipMemcpy(ln_res, d_ln, n, hipMemcpyDeviceToHost), w) ||
           check_hip(hipMemcpy(vars, d_var, r, hipMemcpyDeviceToHost), w) ||
           check_hip(hipMemcpy(means, d_mean, r, hipMemcpyDeviceToHost), w);
  if (rc) fprintf(stderr, "launch_layernorm failed: %s\n", mt_last_error());
  void* bufs[6] = {d_ln, d_var, d_mean, d_inp, d_g, d_b};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
}

/* reference src/layernorm_kernel.cu:370 (two streams there; one here). */
void launch_layernorm_bw(float* gamma_grad, float* betta_grad, float* inp_grad,
                         const float* out_grad, const float* inp, const float* gamma,
                         const float* betta, const float* vars, const float* means,
                         int batch_size, int hidden_dim, void* stream_1, void* stream_2) {
  (void)stream_2;
  const size_t n = (size_t)batch_size * hidden_dim * 4, h = (size_t)hidden_dim * 4,
               r = (size_t)batch_size * 4;
  const char* w = "launch_layernorm_bw";
  void *d_dg = nullptr, *d_db = nullptr, *d_dx = nullptr, *d_dy = nullptr, *d_x = nullptr,
       *d_g = nullptr, *d_b = nullptr, *d_v = nullptr, *d_m = nullptr, *d_ws = nullptr;
  int rc = h2d(&d_dg, nullptr, h, w) || h2d(&d_db, nullptr, h, w) || h2d(&d_dx, nullptr, n, w) ||
           h2d(&d_dy, out_grad, n, w) || h2d(&d_x, inp, n, w) || h2d(&d_g, gamma, h, w) ||
           h2d(&d_b, betta, h, w) || h2d(&d_v, vars, r, w) || h2d(&d_m, means, r, w) ||
           h2d(&d_ws, nullptr, (size_t)mt_layernorm_bw_workspace_bytes(batch_size, hidden_dim), w) ||
           mt_layernorm_bw((float*)d_dg, (float*)d_db, (float*)d_dx, (const float*)d_dy,
                           (const float*)d_x, (const float*)d_g, (const float*)d_b,
                           (const float*)d_v, (const float*)d_m, batch_size, hidden_dim, d_ws,
                           stream_1) ||
           check_hip(hipStreamSynchronize((hipStream_t)stream_1), w) ||
           check_hip(hipMemcpy(gamma_grad, d_dg, h, hipMemcpyDeviceToHost), w) ||
           check_hip(hipMemcpy(betta_grad, d_db, h, hipMemcpyDeviceToHost), w) ||
           check_hip(hipMemcpy(inp_grad, d_dx, n, hipMemcpyDeviceToHost), w);
  if (rc) fprintf(stderr, "launch_layernorm_bw failed: %s\n", mt_last_error());
  void* bufs[10] = {d_dg, d_db, d_dx, d_dy, d_x, d_g, d_b, d_v, d_m, d_ws};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
}

}  // extern "C"
