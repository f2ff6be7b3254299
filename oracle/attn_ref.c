/*
 * CPU ORACLE (C restatement) -- TEST INFRASTRUCTURE ONLY.
 *
 * Used by tests/ (large-size parity checks) and by bench.py's cpu_baseline leg.
 * The shipped HIP path never links or calls this file.
 *
 * Restates the reference's CPU ("fast_ops") attention, unfused and in the
 * reference's op order:
 *   S   = fp32( sum_k fp64(q_ik * k_jk) )            fast_ops.py:291-350 (fp64 acc, :339-345)
 *   S   = fp32( S * inv(sqrt(d)) )                     tensor.py:169-170  (Mul(Inv))
 *   S  += causal ? -FLT_MAX (j > i) : 0                modules_transfomer.py:63-71
 *   mx  = max_j S;  e_j = fp32(exp(S_j - mx))          nn.py:120 (Max, Exp)
 *   sum = fp32 sum_j e_j;  P_j = e_j * fp32(1/sum)     nn.py:121-122 (Sum, Inv, Mul)
 *   O   = fp32( sum_j fp64(P_j * v_jk) )
 * m = mx and l = sum are returned with the reference flash contract's meaning
 * (P = exp(S - m) / l, src/flashattention_kernel.cu:194).
 *
 * Key padding (the *_kv entry points): keys j >= kv[bh] get the reference's additive -inf
 * padding mask (src/softmax_kernel.cu:26-33, attn_mask[B, to_len]); a row with no valid key
 * returns O = 0, m = -inf, l = 0 (the reference's softmax is NaN there).
 *
 * One N-float score row per (bh, i), OpenMP over (bh, i) like numba's prange.
 * The backward is the exact gradient, fp64 accumulation, one N x N fp32 P slice
 * per (bh) and thread; OpenMP over bh.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static void score_row(const float* q, const float* k, int64_t N, int64_t d, int64_t i,
                      int causal, float inv_sqrt_d, int64_t nk, float* s) {
  for (int64_t j = 0; j < N; ++j) {
    double acc = 0.0;
    const float* kj = k + j * d;
    for (int64_t t = 0; t < d; ++t) acc += (double)(q[t] * kj[t]);
    float v = (float)acc;
    v = v * inv_sqrt_d;
    if (causal && j > i) v = v + (-FLT_MAX);
    if (j >= nk) v = v + (-INFINITY);
    s[j] = v;
  }
}

static int64_t keys_of(const int* kv, int64_t bh, int64_t N) {
  if (!kv) return N;
  const int64_t n = kv[bh];
  return n < 0 ? 0 : n > N ? N : n;
}

int oracle_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* q,k,v,o: [BH, N, d] contiguous fp32; m,l: [BH, N] (may be NULL); kv: [BH] valid keys or NULL. */
void oracle_attn_fwd_kv(const float* q, const float* k, const float* v, float* o, float* m,
                        float* l, int64_t BH, int64_t N, int64_t d, int causal, const int* kv,
                        int nthreads) {
  const float inv_sqrt_d = (float)(1.0 / (double)(float)sqrt((double)d));
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
  {
    float* s = (float*)malloc(sizeof(float) * (size_t)N);
    double* acc = (double*)malloc(sizeof(double) * (size_t)d);
#pragma omp for schedule(static) collapse(2)
    for (int64_t bh = 0; bh < BH; ++bh) {
      for (int64_t i = 0; i < N; ++i) {
        const int64_t base = bh * N * d;
        score_row(q + base + i * d, k + base, N, d, i, causal, inv_sqrt_d, keys_of(kv, bh, N), s);
        float mx = -INFINITY;
        for (int64_t j = 0; j < N; ++j) mx = s[j] > mx ? s[j] : mx;
        float sum = 0.0f;
        for (int64_t j = 0; j < N; ++j) {
          s[j] = mx == -INFINITY ? 0.0f : (float)exp((double)(s[j] - mx));
          sum += s[j];
        }
        const float inv = sum > 0.0f ? (float)(1.0 / (double)sum) : 0.0f;
        for (int64_t t = 0; t < d; ++t) acc[t] = 0.0;
        for (int64_t j = 0; j < N; ++j) {
          const float p = s[j] * inv;
          const float* vj = v + base + j * d;
          for (int64_t t = 0; t < d; ++t) acc[t] += (double)(p * vj[t]);
        }
        float* oi = o + base + i * d;
        for (int64_t t = 0; t < d; ++t) oi[t] = (float)acc[t];
        if (m) m[bh * N + i] = mx;
        if (l) l[bh * N + i] = sum;
      }
    }
    free(s);
    free(acc);
  }
}

void oracle_attn_fwd(const float* q, const float* k, const float* v, float* o, float* m,
                     float* l, int64_t BH, int64_t N, int64_t d, int causal, int nthreads) {
  oracle_attn_fwd_kv(q, k, v, o, m, l, BH, N, d, causal, NULL, nthreads);
}

/* Exact gradients. dq, dk, dv: [BH, N, d] outputs (overwritten). */
void oracle_attn_bwd_kv(const float* q, const float* k, const float* v, const float* dout,
                        const float* m, const float* l, float* dq, float* dk, float* dv,
                        int64_t BH, int64_t N, int64_t d, int causal, const int* kv,
                        int nthreads) {
  const float inv_sqrt_d = (float)(1.0 / (double)(float)sqrt((double)d));
  const double scale = 1.0 / sqrt((double)d);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
  {
    double* p = (double*)malloc(sizeof(double) * (size_t)(N * N));
    double* ds = (double*)malloc(sizeof(double) * (size_t)(N * N));
    float* s = (float*)malloc(sizeof(float) * (size_t)N);
    double* acc = (double*)malloc(sizeof(double) * (size_t)d);
    double* accK = (double*)malloc(sizeof(double) * (size_t)(N * d));
    double* accV = (double*)malloc(sizeof(double) * (size_t)(N * d));
#pragma omp for schedule(dynamic, 1)
    for (int64_t bh = 0; bh < BH; ++bh) {
      const int64_t base = bh * N * d;
      const float *Q = q + base, *K = k + base, *V = v + base, *dO = dout + base;
      for (int64_t i = 0; i < N; ++i) {
        score_row(Q + i * d, K, N, d, i, causal, inv_sqrt_d, keys_of(kv, bh, N), s);
        const double mi = m[bh * N + i], li = l[bh * N + i];
        double delta = 0.0;
        for (int64_t j = 0; j < N; ++j) {
          const double pij = li > 0.0 ? exp((double)s[j] - mi) / li : 0.0;
          double dp = 0.0;
          for (int64_t t = 0; t < d; ++t) dp += (double)dO[i * d + t] * (double)V[j * d + t];
          p[i * N + j] = pij;
          ds[i * N + j] = dp;
          delta += dp * pij;
        }
        for (int64_t j = 0; j < N; ++j) ds[i * N + j] = p[i * N + j] * (ds[i * N + j] - delta);
      }
      // The three sums run in row-major sweeps (j, then i ascending for every element, the
      // same order as the element-at-a-time loops of attention.py) so the N x N buffers are
      // read once each instead of once per output column.
      for (int64_t i = 0; i < N; ++i) {
        for (int64_t t = 0; t < d; ++t) acc[t] = 0.0;
        for (int64_t j = 0; j < N; ++j) {
          const double w = ds[i * N + j];
          for (int64_t t = 0; t < d; ++t) acc[t] += w * (double)K[j * d + t];
        }
        for (int64_t t = 0; t < d; ++t) dq[base + i * d + t] = (float)(acc[t] * scale);
      }
      for (int64_t x = 0; x < N * d; ++x) accK[x] = accV[x] = 0.0;
      for (int64_t i = 0; i < N; ++i)
        for (int64_t j = 0; j < N; ++j) {
          const double a = ds[i * N + j], b = p[i * N + j];
          for (int64_t t = 0; t < d; ++t) {
            accK[j * d + t] += a * (double)Q[i * d + t];
            accV[j * d + t] += b * (double)dO[i * d + t];
          }
        }
      for (int64_t x = 0; x < N * d; ++x) {
        dk[base + x] = (float)(accK[x] * scale);
        dv[base + x] = (float)accV[x];
      }
    }
    free(p);
    free(ds);
    free(s);
    free(acc);
    free(accK);
    free(accV);
  }
}

void oracle_attn_bwd(const float* q, const float* k, const float* v, const float* dout,
                     const float* m, const float* l, float* dq, float* dk, float* dv,
                     int64_t BH, int64_t N, int64_t d, int causal, int nthreads) {
  oracle_attn_bwd_kv(q, k, v, dout, m, l, dq, dk, dv, BH, N, d, causal, NULL, nthreads);
}
