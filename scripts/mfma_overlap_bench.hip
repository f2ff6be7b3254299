// Microbenchmark (diagnostics): does VALU work issued between v_mfma_f32_32x32x16_bf16
// instructions overlap the matrix pipe at 1 and 2 waves per SIMD, with the accumulators in
// arch VGPRs? Prints ns per MFMA per SIMD for: MFMA only; MFMA + k v_exp_f32 + 2k v_fma
// per MFMA (independent data). Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/mob this.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

template <int NEXP, int NFMA>
__global__ __launch_bounds__(256, 2) void k(float* out, int iters, float seed) {
  f32x16 acc[4] = {};
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(seed * (threadIdx.x + j));
    b[j] = (__bf16)(seed * (j + 1));
  }
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = seed * (threadIdx.x + j) * 1e-3f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      acc[m & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[m & 3], 0, 0, 0);
#pragma unroll
      for (int e = 0; e < NEXP; ++e) x[e & 7] = __builtin_amdgcn_exp2f(x[e & 7] * -0.5f);
#pragma unroll
      for (int f = 0; f < NFMA; ++f) x[(f + 3) & 7] = __builtin_fmaf(x[(f + 3) & 7], 0.999f, 1e-4f);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[i][r];
#pragma unroll
  for (int j = 0; j < 8; ++j) s += x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NEXP, int NFMA>
static void run(const char* name, int blocks_per_cu) {
  int ncu = 256;
  const int blocks = ncu * blocks_per_cu, iters = 2000;
  float* out;
  hipMalloc(&out, sizeof(float) * blocks * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k<NEXP, NFMA>), dim3(blocks), dim3(256), 0, 0, out, 10, 1.0f);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k<NEXP, NFMA>), dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // MFMAs per SIMD: blocks_per_cu waves per SIMD x iters x 16
  const double mfma_per_simd = (double)blocks_per_cu * iters * 16;
  const double tf = 2.0 * 32 * 32 * 16 * mfma_per_simd * 1024 / (ms * 1e-3) / 1e12;
  printf("%-28s waves/SIMD %d : %.2f ns per MFMA per SIMD, %.0f TF/s\n", name, blocks_per_cu,
         ms * 1e6 / mfma_per_simd, tf);
  hipFree(out);
}

int main() {
  for (int w = 1; w <= 2; ++w) {
    run<0, 0>("mfma only", w);
    run<1, 2>("mfma + 1 exp + 2 fma", w);
    run<2, 3>("mfma + 2 exp + 3 fma", w);
    run<2, 6>("mfma + 2 exp + 6 fma", w);
    run<4, 4>("mfma + 4 exp + 4 fma", w);
  }
  return 0;
}
