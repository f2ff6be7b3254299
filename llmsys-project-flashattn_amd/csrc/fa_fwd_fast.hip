// FlashAttention forward, bf16 MFMA kernel specialised for head dims 64 and 128.
//
// The hot path of BASELINE.json's north star ((B,H,N,d) = (8,16,4096,64) bf16).
// Same contract as the reference forward_kernel (src/flashattention_kernel.cu:9-112):
// O = softmax(QKᵀ/√d) V with row statistics (m, l), P = exp(s − m)/l.
//
// Structure (CDNA4-first):
//  * 512-thread workgroup = 8 waves (2 per SIMD), 32 queries per wave, BQ = 256.
//    The wave's Q block lives in registers as MFMA B fragments for the whole loop.
//  * K/V tiles of 64 keys are register-staged (issue-early / write-late): the
//    global loads of tile t+1 are issued before the MFMAs of tile t and written to
//    the other LDS buffer after them; ONE barrier per tile.
//  * Sᵀ = K·Qᵀ (v_mfma_f32_32x32x16_bf16, A = K rows via ds_read_b128 from an
//    XOR-swizzled image) puts the query on the lane: the online softmax is
//    lane-local plus one v_permlane32_swap; Pᵀ feeds Oᵀ = Vᵀ·Pᵀ directly as the B
//    operand; Vᵀ comes from ds_read_b64_tr_b16 on a swizzled V image.
//  * exp2 with log2(e)/√d folded into one fma; the running max is only raised when
//    a tile's max exceeds it by more than 2^8 (deferred rescale), so the O-wide
//    rescale runs on a handful of tiles per row (P ≤ 256 stays exact enough in bf16).
//  * XCD-aware block order: all query blocks of one (b, h) run on one XCD so its
//    K/V stay in that XCD's L2; causal grids launch the heaviest blocks first.
#include "fa_common.h"

namespace mt {

namespace {

constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kBQ = 32 * kWaves;  // queries per workgroup
constexpr int kBK = 64;           // keys per tile
constexpr float kRescaleThr = 8.0f;  // log2 units

// K image, read by ds_read_b128 (16 lanes = 16 different rows, same chunk):
//   D=64  (128-B rows, 2 per 256-B bank row): chunk c of row r at c ^ ((r >> 1) & 7)
//   D=128 (256-B rows):                        chunk c of row r at c ^ (r & 15)
// so the 16 rows of a lane group hit 16 distinct 16-B bank slots.
template <int D>
__device__ __forceinline__ int k_off(int r, int c) {  // element offset of chunk c of row r
  if (D == 64) return r * D + (c ^ ((r >> 1) & 7)) * 8;
  return r * D + (c ^ (r & 15)) * 8;
}
// V image, read by ds_read_b64_tr_b16 (a half-wave reads 4 consecutive rows x 64 B):
//   D=64 : chunk c of row r at c ^ (((r >> 1) & 1) << 2)
//   D=128: chunk c of row r at c ^ ((r & 3) << 2)
// so the 4 rows land in 4 distinct 64-B quarters of the bank row.
template <int D>
__device__ __forceinline__ int v_off(int r, int c) {
  if (D == 64) return r * D + (c ^ (((r >> 1) & 1) << 2)) * 8;
  return r * D + (c ^ ((r & 3) << 2)) * 8;
}

}  // namespace

template <int D, bool CAUSAL>
__global__ __launch_bounds__(kThreads, 2) void fa_fwd_bf16_fast(AttnArgs p, int nqb) {
  constexpr int CPR = D / 8;                       // 16-B chunks per row
  constexpr int TILE_CH = kBK * CPR;               // chunks per K (or V) tile
  constexpr int LPT = TILE_CH / kThreads;          // chunks per thread per tile (1 or 2)
  constexpr int KSTEPS = D / 16;
  constexpr int DB = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* sK = (bf16*)smem;                  // [2][kBK*D]
  bf16* sV = sK + 2 * kBK * D;             // [2][kBK*D]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;

  // XCD-aware, bijective block remap: blocks sharing an XCD (hw id mod 8) take
  // consecutive logical ids, i.e. the query blocks of the same heads.
  const int nblk = gridDim.x;
  const int hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3;
  const int qd = nblk >> 3, rm = nblk & 7;
  const int logical = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + slot;
  const int bh = logical / nqb;
  int qb = logical % nqb;
  if (CAUSAL) qb = nqb - 1 - qb;  // heaviest first
  const int b = bh / p.H, hh = bh % p.H;
  const int q0 = qb * kBQ;

  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Kg = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1];
  const bf16* Vg = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1];
  const int64_t skn = p.sk[2], svn = p.sv[2];

  const int my_q = q0 + wave * 32 + c32;
  const int wq_lo = q0 + wave * 32, wq_hi = wq_lo + 31;

  // Q fragments (B operand of Sᵀ = K·Qᵀ), kept in registers.
  bf16x8 qf[KSTEPS];
  {
    const int qr = min(my_q, N - 1);
    const bf16* qrow = Qg + (int64_t)qr * p.sq[2];
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) qf[ks] = *(const bf16x8*)(qrow + ks * 16 + 8 * hf);
  }

  const int kend = CAUSAL ? min(N, q0 + kBQ) : N;
  const int ntiles = (kend + kBK - 1) / kBK;

  // Register staging of one K and one V tile.
  uint4 rk[LPT], rv[LPT];
  auto load_tile = [&](int t) {
    const int k0 = t * kBK;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int ch = tid + i * kThreads;
      const int r = ch / CPR, c = ch % CPR;
      const int key = min(k0 + r, N - 1);  // clamp: tail rows are masked later
      rk[i] = *(const uint4*)(Kg + (int64_t)key * skn + c * 8);
      rv[i] = *(const uint4*)(Vg + (int64_t)key * svn + c * 8);
    }
  };
  auto store_tile = [&](int buf) {
    bf16* k = sK + buf * kBK * D;
    bf16* v = sV + buf * kBK * D;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int ch = tid + i * kThreads;
      const int r = ch / CPR, c = ch % CPR;
      *(uint4*)(k + k_off<D>(r, c)) = rk[i];
      *(uint4*)(v + v_off<D>(r, c)) = rv[i];
    }
  };

  f32x16 O[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) O[i] = f32x16{};
  float m_run = -INFINITY;  // raw-score units (unscaled)
  float l_run = 0.f;
  const float c2 = p.scale_log2;

  load_tile(0);
  store_tile(0);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const int k0 = t * kBK;
    if (t + 1 < ntiles) load_tile(t + 1);
    const bool active = !CAUSAL || k0 <= wq_hi;
    if (active) {
      const bf16* k = sK + buf * kBK * D;
      const bf16* v = sV + buf * kBK * D;
      f32x16 S[2] = {f32x16{}, f32x16{}};
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const bf16x8 a = *(const bf16x8*)(k + k_off<D>(kb * 32 + c32, 2 * ks + hf));
          S[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], S[kb], 0, 0, 0);
        }
      // Mask only where needed: the ragged last tile and causal diagonal tiles.
      const bool need_mask = (k0 + kBK > N) || (CAUSAL && k0 + kBK - 1 > wq_lo);
      if (need_mask) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + kb * 32 + acc_row(r, hf);
            if (key >= N || (CAUSAL && key > my_q)) S[kb][r] = -INFINITY;
          }
      }
      float tmax = S[0][0];
#pragma unroll
      for (int r = 1; r < 16; ++r) tmax = fmaxf(tmax, S[0][r]);
#pragma unroll
      for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, S[1][r]);
      {
        auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(tmax), __float_as_uint(tmax),
                                                   false, false);
        tmax = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      }
      // Deferred rescale: raise the running max only when some row of the wave would
      // otherwise see exp2 arguments above kRescaleThr.
      const bool grow = (tmax - m_run) * c2 > kRescaleThr;
      if (__builtin_amdgcn_ballot_w64(grow)) {
        const float m_new = fmaxf(m_run, tmax);
        const float alpha = (m_run == -INFINITY) ? 0.f : exp2f((m_run - m_new) * c2);
        m_run = m_new;
        l_run *= alpha;
#pragma unroll
        for (int i = 0; i < DB; ++i) O[i] *= alpha;
      }
      const float mc = (m_run == -INFINITY) ? 0.f : m_run * c2;
      float rs = 0.f;
      bf16x8 pf[4];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float e = exp2f(fmaf(S[kb][8 * s + j], c2, -mc));
            rs += e;
            pf[2 * kb + s][j] = (bf16)e;
          }
      l_run += rs;
      // PV with the swizzled V image (custom transpose-read addressing).
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int kr0 = kb * 32 + 16 * s + 4 * hf;
          const int i16 = lane & 15, g = (lane >> 4) & 1;
#pragma unroll
          for (int db = 0; db < DB; ++db) {
            const int col = db * 32 + 16 * g + 4 * (i16 & 3);
            const int r1 = kr0 + (i16 >> 2), r2 = r1 + 8;
            typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
            const bf16* a1 = v + v_off<D>(r1, col >> 3) + (col & 7);
            const bf16* a2 = v + v_off<D>(r2, col >> 3) + (col & 7);
            s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
            s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a2);
            typedef __attribute__((ext_vector_type(8))) short s16x8;
            s16x8 av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            O[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av),
                                                            pf[2 * kb + s], O[db], 0, 0, 0);
          }
        }
    }
    if (t + 1 < ntiles) store_tile(buf ^ 1);
    __syncthreads();
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32);
  const float inv_l = 1.f / l_tot;
  if (my_q < N) {
    bf16* Og = (bf16*)p.out + b * p.so[0] + hh * p.so[1] + (int64_t)my_q * p.so[2];
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(Og + db * 32 + 8 * g + 4 * hf, O[db][4 * g] * inv_l, O[db][4 * g + 1] * inv_l,
               O[db][4 * g + 2] * inv_l, O[db][4 * g + 3] * inv_l, true);
    if (hf == 0) {
      const int64_t row = (int64_t)bh * N + my_q;
      if (p.m) p.m[row] = m_run * p.scale;  // natural-log units: max of s = qk/√d
      if (p.l) p.l[row] = l_tot;
    }
  }
}

template <int D, bool CAUSAL>
static hipError_t launch_fast_t(const AttnArgs& a, hipStream_t st) {
  const size_t smem = 4 * (size_t)kBK * D * sizeof(bf16);
  auto kfn = fa_fwd_bf16_fast<D, CAUSAL>;
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)smem);
  if (e != hipSuccess) return e;
  const int nqb = (a.N + kBQ - 1) / kBQ;
  const int64_t nblk = (int64_t)nqb * a.B * a.H;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kfn, dim3((unsigned)nblk), dim3(kThreads), smem, st, a, nqb);
  return hipGetLastError();
}

hipError_t launch_fwd_fast(const AttnArgs& a, bool causal, hipStream_t st, bool* handled) {
  *handled = true;
  if (a.d == 64) return causal ? launch_fast_t<64, true>(a, st) : launch_fast_t<64, false>(a, st);
  if (a.d == 128) return causal ? launch_fast_t<128, true>(a, st) : launch_fast_t<128, false>(a, st);
  *handled = false;
  return hipSuccess;
}

}  // namespace mt
