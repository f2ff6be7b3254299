// Column-sum microbenchmark at config 5's bias-gradient shape (4992 x 256 fp32): where the
// one-pass reduction's time goes. Variants, each timed with HIP events over 400 back-to-back
// launches:
//   load   78 workgroups load their 64-row chunk and store a partial (phase 1 alone)
//   arrive load + agent release fence + arrival atomic (no fold)
//   full   arrive + the last arriver's acquire and ordered fold (the product's form)
//   lines8 8 workgroups of 32 columns (one 128-B line per row), no hand-off
//   cols64 64 workgroups of 4 columns, 1024 threads, no hand-off
// build: hipcc -O3 --offload-arch=gfx950 scripts/colsum_bench.hip -o scripts/colsum_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

constexpr int LEN = 4992, INNER = 256, CHUNK = 64, R = LEN / CHUNK;  // 78

template <int MODE>  // 0 load, 1 arrive, 2 full
__global__ __launch_bounds__(512) void chunked(float* out, float* part, unsigned* ctr, const float* a) {
  __shared__ float4 red[8][64];
  __shared__ int last_s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = blockIdx.x;
  const float* src = a + (int64_t)r * CHUNK * INNER + lane * 4;
  float4 x[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) x[u] = *(const float4*)(src + (int64_t)(w + 8 * u) * INNER);
  float4 acc = x[0];
#pragma unroll
  for (int u = 1; u < 8; ++u) { acc.x += x[u].x; acc.y += x[u].y; acc.z += x[u].z; acc.w += x[u].w; }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0) {
    float4 v = red[0][lane];
    for (int k = 1; k < 8; ++k) { v.x += red[k][lane].x; v.y += red[k][lane].y; v.z += red[k][lane].z; v.w += red[k][lane].w; }
    *(float4*)(part + (int64_t)r * INNER + lane * 4) = v;
    if (MODE >= 1) {
      __threadfence();
      if (lane == 0) last_s = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == R - 1;
    }
  }
  if (MODE < 2) return;
  __syncthreads();
  if (!last_s) return;
  __threadfence();
  const int per = (R + 7) / 8, r0 = w * per, r1 = min(R, r0 + per);
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 y[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) y[u] = *(const float4*)(part + (int64_t)min(r0 + u, R - 1) * INNER + lane * 4);
#pragma unroll
  for (int u = 0; u < 16; ++u)
    if (r0 + u < r1) { v.x += y[u].x; v.y += y[u].y; v.z += y[u].z; v.w += y[u].w; }
  red[w][lane] = v;
  __syncthreads();
  if (w == 0) {
    float4 t = red[0][lane];
    for (int k = 1; k < 8; ++k) { t.x += red[k][lane].x; t.y += red[k][lane].y; t.z += red[k][lane].z; t.w += red[k][lane].w; }
    *(float4*)(out + lane * 4) = t;
    if (lane == 0) *ctr = 0u;
  }
}

// 8 workgroups x 32 columns: 8 lanes per row, 128 rows per pass of 1024 threads
__global__ __launch_bounds__(1024) void lines8(float* out, const float* a) {
  __shared__ float4 red[128][8];
  const int t = threadIdx.x, c = t & 7, row = t >> 3;
  const float* src = a + blockIdx.x * 32 + c * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int j = row; j < LEN; j += 128 * 8) {
    float4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = *(const float4*)(src + (int64_t)min(j + 128 * u, LEN - 1) * INNER);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (j + 128 * u < LEN) { acc.x += x[u].x; acc.y += x[u].y; acc.z += x[u].z; acc.w += x[u].w; }
  }
  red[row][c] = acc;
  __syncthreads();
  for (int s = 64; s > 0; s >>= 1) {
    if (row < s) { float4 b = red[row + s][c]; red[row][c].x += b.x; red[row][c].y += b.y; red[row][c].z += b.z; red[row][c].w += b.w; }
    __syncthreads();
  }
  if (row == 0) *(float4*)(out + blockIdx.x * 32 + c * 4) = red[0][c];
}

// 64 workgroups x 4 columns: one lane per row, 1024 rows per pass; blockIdx -> columns so that
// the 8 workgroups of one XCD (blockIdx % 8) share 128-B lines
__global__ __launch_bounds__(1024) void cols64(float* out, const float* a) {
  __shared__ float4 red[1024];
  const int t = threadIdx.x;
  const int line = blockIdx.x & 7, sub = blockIdx.x >> 3, cg = line * 8 + sub;
  const float* src = a + cg * 4;
  float4 x[5];
#pragma unroll
  for (int u = 0; u < 5; ++u) x[u] = *(const float4*)(src + (int64_t)min(t + 1024 * u, LEN - 1) * INNER);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int u = 0; u < 5; ++u)
    if (t + 1024 * u < LEN) { acc.x += x[u].x; acc.y += x[u].y; acc.z += x[u].z; acc.w += x[u].w; }
  red[t] = acc;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if (t < s) { float4 b = red[t + s]; red[t].x += b.x; red[t].y += b.y; red[t].z += b.z; red[t].w += b.w; }
    __syncthreads();
  }
  if (t == 0) *(float4*)(out + cg * 4) = red[0];
}

// the product's reduce_colgroup_kernel (csrc/combine.hip) for fn = add, T threads
__device__ __forceinline__ void fold4(float4& v, bool& hv, const float4& y, bool hy) {
  if (!hy) return;
  if (!hv) { v = y; hv = true; return; }
  v.x += y.x; v.y += y.y; v.z += y.z; v.w += y.w;
}
template <int TREE>
__global__ __launch_bounds__(1024) void prod(float* out, const float* a, int64_t len, int64_t inner, int ncg) {
  __shared__ float4 red[16];
  __shared__ float4 big[1024];
  __shared__ int have_s[16];
  const int b = blockIdx.x;
  const int cg = (((b & 7) + 8 * ((b >> 3) >> 3)) * 8 + ((b >> 3) & 7));
  if (cg >= ncg) return;
  const int t = threadIdx.x, T = blockDim.x, lane = t & 63, w = t >> 6;
  const float* src = a + (int64_t)cg * 4;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  bool hv = false;
  for (int64_t j = t; j < len; j += 8 * (int64_t)T) {
    float4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      x[u] = j + (int64_t)u * T < len ? *(const float4*)(src + (j + (int64_t)u * T) * inner)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 8; ++u) fold4(v, hv, x[u], j + (int64_t)u * T < len);
  }
  if (TREE) {
    big[t] = v;
    __syncthreads();
    for (int s = 512; s > 0; s >>= 1) {
      if (t < s) { float4 q = big[t + s]; big[t].x += q.x; big[t].y += q.y; big[t].z += q.z; big[t].w += q.w; }
      __syncthreads();
    }
    if (t == 0) *(float4*)(out + (int64_t)cg * 4) = big[0];
    return;
  }
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    float4 y;
    y.x = __shfl_xor(v.x, s); y.y = __shfl_xor(v.y, s); y.z = __shfl_xor(v.z, s); y.w = __shfl_xor(v.w, s);
    const bool hy = __shfl_xor((int)hv, s) != 0;
    if (lane & s) { float4 z = v; bool hz = hv; v = y; hv = hy; fold4(v, hv, z, hz); }
    else fold4(v, hv, y, hy);
  }
  if (lane == 0) { red[w] = v; have_s[w] = hv; }
  __syncthreads();
  if (t == 0) {
    float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
    bool hr = false;
    for (int k = 0; k < T / 64; ++k) fold4(r, hr, red[k], have_s[k] != 0);
    *(float4*)(out + (int64_t)cg * 4) = r;
  }
}

int main() {
  std::vector<float> h((size_t)LEN * INNER);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  std::vector<double> ref(INNER, 0.0);
  for (int j = 0; j < LEN; ++j) for (int c = 0; c < INNER; ++c) ref[c] += h[(size_t)j * INNER + c];
  float *a, *out, *part; unsigned* ctr;
  CK(hipMalloc(&a, h.size() * 4)); CK(hipMalloc(&out, INNER * 4)); CK(hipMalloc(&part, R * INNER * 4));
  CK(hipMalloc(&ctr, 4)); CK(hipMemset(ctr, 0, 4));
  CK(hipMemcpy(a, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch, bool check) {
    for (int i = 0; i < 20; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 400; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double err = 0;
    if (check) {
      std::vector<float> o(INNER);
      CK(hipMemcpy(o.data(), out, INNER * 4, hipMemcpyDeviceToHost));
      for (int c = 0; c < INNER; ++c) err = std::max(err, std::abs(o[c] - ref[c]));
    }
    printf("%-8s %7.2f us/launch  max_err %.3g\n", name, ms / 400 * 1e3, err);
  };
  run("load", [&] { chunked<0><<<R, 512>>>(out, part, ctr, a); }, false);
  run("arrive", [&] { chunked<1><<<R, 512>>>(out, part, ctr, a); CK(hipMemsetAsync(ctr, 0, 4)); }, false);
  run("memset", [&] { CK(hipMemsetAsync(ctr, 0, 4)); }, false);
  CK(hipMemset(ctr, 0, 4));
  run("full", [&] { chunked<2><<<R, 512>>>(out, part, ctr, a); }, true);
  run("lines8", [&] { lines8<<<8, 1024>>>(out, a); }, true);
  run("cols64", [&] { cols64<<<64, 1024>>>(out, a); }, true);
  run("prod", [&] { prod<0><<<64, 1024>>>(out, a, LEN, INNER, 64); }, true);
  run("prodtree", [&] { prod<1><<<64, 1024>>>(out, a, LEN, INNER, 64); }, true);
  run("prod", [&] { prod<0><<<64, 1024>>>(out, a, LEN, INNER, 64); }, true);
  run("cols64", [&] { cols64<<<64, 1024>>>(out, a); }, true);
  CK(hipMemset(ctr, 0, 4));
  run("full", [&] { chunked<2><<<R, 512>>>(out, part, ctr, a); }, true);
  return 0;
}
