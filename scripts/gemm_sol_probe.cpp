// rocBLAS solution sweep for config 5's 256-wide linears (4992 x 256 x 256 fp32), in the three
// forms combine.hip's gemm_rocblas issues them (column-major view of row-major operands):
//   fwd  Y = X W       : NN, m=256 n=4992 k=256
//   dX   dX = dY Wᵀ    : TN, m=256 n=4992 k=256
//   dW   dW = Xᵀ dY    : NT, m=256 n=256  k=1248, 4 strided K slices (the product's split-K)
// For each form: the default solution's time, then every fp32 solution rocBLAS accepts for the
// problem, timed with HIP events over 200 calls; prints the five fastest.
// build: hipcc -O2 -DROCBLAS_BETA_FEATURES_API --offload-arch=gfx950 scripts/gemm_sol_probe.cpp
//        -lrocblas -o scripts/gemm_sol_probe
#define ROCBLAS_BETA_FEATURES_API
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <algorithm>
#include <cstdio>
#include <vector>

struct Form { const char* name; rocblas_operation ta, tb; int m, n, k, lda, ldb, ldc; long sa, sb, sc; int batch; };

int main() {
  rocblas_handle h;
  rocblas_create_handle(&h);
  float *A, *B, *C;
  hipMalloc(&A, 4992L * 256 * 4 * 2);
  hipMalloc(&B, 4992L * 256 * 4 * 2);
  hipMalloc(&C, 4992L * 256 * 4 * 2);
  hipMemset(A, 0, 4992L * 256 * 8);
  hipMemset(B, 0, 4992L * 256 * 8);
  const float alpha = 1.f, beta = 0.f;
  // rocBLAS A = our B (W / Wᵀ / dY), rocBLAS B = our A (X / dY / Xᵀ)
  Form forms[] = {
      {"fwd", rocblas_operation_none, rocblas_operation_none, 256, 4992, 256, 256, 256, 256, 0, 0, 0, 1},
      {"dX", rocblas_operation_transpose, rocblas_operation_none, 256, 4992, 256, 256, 256, 256, 0, 0, 0, 1},
      {"dW", rocblas_operation_none, rocblas_operation_transpose, 256, 256, 1248, 256, 256, 256,
       1248L * 256, 1248L * 256, 256L * 256, 4},
  };
  int nsol = 0;
  rocblas_gemm_ex_get_solutions_by_type(h, rocblas_datatype_f32_r, rocblas_datatype_f32_r, rocblas_datatype_f32_r,
                                        0, nullptr, &nsol);
  std::vector<rocblas_int> sols(nsol);
  rocblas_gemm_ex_get_solutions_by_type(h, rocblas_datatype_f32_r, rocblas_datatype_f32_r, rocblas_datatype_f32_r,
                                        0, sols.data(), &nsol);
  printf("%d fp32 solutions\n", nsol);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (const Form& f : forms) {
    auto call = [&](rocblas_gemm_algo algo, int idx) {
      return rocblas_gemm_strided_batched_ex(h, f.ta, f.tb, f.m, f.n, f.k, &alpha, A, rocblas_datatype_f32_r, f.lda,
                                             f.sa, B, rocblas_datatype_f32_r, f.ldb, f.sb, &beta, C,
                                             rocblas_datatype_f32_r, f.ldc, f.sc, C, rocblas_datatype_f32_r, f.ldc,
                                             f.sc, f.batch, rocblas_datatype_f32_r, algo, idx, 0);
    };
    auto timeit = [&](rocblas_gemm_algo algo, int idx) -> float {
      for (int i = 0; i < 5; ++i)
        if (call(algo, idx) != rocblas_status_success) return -1.f;
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int i = 0; i < 200; ++i) call(algo, idx);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      return ms / 200 * 1e3f;
    };
    const float def = timeit(rocblas_gemm_algo_standard, 0);
    std::vector<std::pair<float, int>> r;
    for (size_t i = 0; i < sols.size(); ++i) {
      const int s = sols[i];
      if (i % 100 == 0) { printf("  %s: %zu/%zu\n", f.name, i, sols.size()); fflush(stdout); }
      const float us = timeit(rocblas_gemm_algo_solution_index, s);
      if (us > 0) r.push_back({us, s});
    }
    std::sort(r.begin(), r.end());
    printf("%s: default %.2f us, %zu valid solutions; fastest:", f.name, def, r.size());
    for (size_t i = 0; i < r.size() && i < 5; ++i) printf(" [%d] %.2f", r[i].second, r[i].first);
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
