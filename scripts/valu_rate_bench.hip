// Microbenchmark (diagnostics): issue cost of the VALU instructions the forward softmax
// uses, alone and in the shadow of v_mfma_f32_32x32x16_bf16, at 1 and 2 waves per SIMD.
// Every op works on 8 independent registers (no dependency chains longer than 8).
// Prints cycles per op per SIMD (at the measured shader clock from s_memtime-free timing:
// the host converts ns with the clock given on the command line, default 2.0 GHz).
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/valu_rate_bench scripts/valu_rate_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(2))) float f32x2;

enum Op { EXP = 0, FMA, PKFMA, PKADD, CVT, EXPH, EXPHS, CVTH, NOP_ };

template <int OP>
__device__ __forceinline__ void op8(float (&x)[16]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (OP == EXP) asm volatile("v_exp_f32 %0, %0" : "+v"(x[j]));
    if (OP == FMA) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[j]) : "v"(x[8]), "v"(x[9]));
    if (OP == PKFMA) {
      f32x2 v = {x[2 * (j & 3)], x[2 * (j & 3) + 1]};
      const f32x2 a = {x[10], x[11]}, b = {x[12], x[13]};
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(v) : "v"(a), "v"(b));
      x[2 * (j & 3)] = v[0];
      x[2 * (j & 3) + 1] = v[1];
    }
    if (OP == PKADD) {
      f32x2 v = {x[2 * (j & 3)], x[2 * (j & 3) + 1]};
      const f32x2 a = {x[10], x[11]};
      asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(v) : "v"(a));
      x[2 * (j & 3)] = v[0];
      x[2 * (j & 3) + 1] = v[1];
    }
    if (OP == EXPH) asm volatile("v_exp_f16 %0, %0" : "+v"(x[j]));
    if (OP == EXPHS)  // the high half in place (SDWA): a packed f16 pair's second exponential
      asm volatile("v_exp_f16_sdwa %0, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1" : "+v"(x[j]));
    if (OP == CVTH) {
      unsigned r;
      asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(x[j]), "v"(x[(j + 1) & 7]));
      x[j] = __uint_as_float(r);
    }
    if (OP == CVT) {
      unsigned r;
      asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(x[j]), "v"(x[(j + 1) & 7]));
      x[j] = __uint_as_float(r);
    }
  }
}

// MFMAS: 0 = VALU only, 1 = one MFMA per group of 8*NGRP ops on 4 rotating accumulators,
// 2 = chains of 4 dependent MFMAs (accumulator m>>2), 3 = one fully dependent chain.
template <int OP, int MFMAS, int NGRP>
__global__ __launch_bounds__(256, 2) void k(float* out, int iters, float seed) {
  f32x16 acc[4] = {};
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(seed * (threadIdx.x + j));
    b[j] = (__bf16)(seed * (j + 1));
  }
  float x[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) x[j] = seed * (threadIdx.x + j) * 1e-3f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int ai = MFMAS == 1 ? (m & 3) : MFMAS == 2 ? ((m >> 2) & 1) : 0;
      if (MFMAS > 0) acc[ai] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[ai], 0, 0, 0);
#pragma unroll
      for (int g = 0; g < NGRP; ++g) op8<OP>(x);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[i][r];
#pragma unroll
  for (int j = 0; j < 16; ++j) s += x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static double g_ghz = 2.0;

template <int OP, int MFMAS, int NGRP>
static void run(const char* name, int waves_per_simd) {
  const int blocks = 256 * waves_per_simd, iters = 4000;
  float* out;
  hipMalloc(&out, sizeof(float) * blocks * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k<OP, MFMAS, NGRP>), dim3(blocks), dim3(256), 0, 0, out, 10, 1.0f);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k<OP, MFMAS, NGRP>), dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // per SIMD: waves_per_simd waves x iters x 8 groups
  const double groups = (double)waves_per_simd * iters * 8;
  const double cyc_group = ms * 1e-3 * g_ghz * 1e9 / groups;
  printf("%-34s waves/SIMD %d : %6.2f cycles per (MFMA%s + %d ops) ; %5.2f cycles/op\n", name,
         waves_per_simd, cyc_group, MFMAS ? "" : " none", 8 * NGRP, cyc_group / (8 * NGRP));
  hipFree(out);
}

int main(int argc, char** argv) {
  if (argc > 1) g_ghz = atof(argv[1]);
  for (int w = 1; w <= 2; ++w) {
    run<EXP, 0, 2>("exp only", w);
    run<FMA, 0, 2>("fma only", w);
    run<PKFMA, 0, 2>("pk_fma only", w);
    run<PKADD, 0, 2>("pk_add only", w);
    run<CVT, 0, 2>("cvt_pk_bf16 only", w);
    run<EXPH, 0, 2>("exp_f16 only", w);
    run<EXPHS, 0, 2>("exp_f16 sdwa hi only", w);
    run<CVTH, 0, 2>("cvt_pk_f16 only", w);
    run<EXP, 1, 0>("mfma only", w);
    run<EXP, 1, 1>("mfma + 8 exp", w);
    run<FMA, 1, 1>("mfma + 8 fma", w);
    run<PKFMA, 1, 1>("mfma + 8 pk_fma", w);
    run<PKADD, 1, 1>("mfma + 8 pk_add", w);
    run<CVT, 1, 1>("mfma + 8 cvt_pk", w);
    run<EXPH, 1, 1>("mfma + 8 exp_f16", w);
    run<EXPHS, 1, 1>("mfma + 8 exp_f16 sdwa hi", w);
    run<CVTH, 1, 1>("mfma + 8 cvt_pk_f16", w);
    run<EXP, 2, 0>("mfma chains of 4", w);
    run<EXP, 3, 0>("mfma one dependent chain", w);
    run<FMA, 2, 1>("mfma chains of 4 + 8 fma", w);
  }
  return 0;
}
