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

typedef __attribute__((ext_vector_type(2))) float f32x2;

// Row max of a lane's 32 scores (keys of both 32-key blocks), then across the two lane
// halves (same query). Built on v_max3_f32 (the TU is compiled with -fno-honor-nans so
// fmaxf lowers without canonicalising v_max on every MFMA output).
__device__ __forceinline__ float tile_max(const f32x16& a, const f32x16& b) {
  float m = fmaxf(fmaxf(a[0], a[1]), b[0]);
#pragma unroll
  for (int r = 1; r < 16; ++r) m = fmaxf(fmaxf(m, a[r]), b[r]);
  // a[1] was folded in twice above; harmless for a max.
  auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
}

// p = exp2(s*c2 - mc) for accumulator registers 8h..8h+7 of s, as a bf16 B fragment.
// The scale-and-shift runs as 4 packed v_pk_fma_f32, the exponentials as v_exp_f32.
__device__ __forceinline__ bf16x8 softmax_frag(const f32x16& s, int h, float c2, float negmc) {
  const f32x2 c = {c2, c2}, n = {negmc, negmc};
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    f32x2 x = {s[8 * h + j], s[8 * h + j + 1]};
    x = x * c + n;
    r[j] = (bf16)__builtin_amdgcn_exp2f(x[0]);
    r[j + 1] = (bf16)__builtin_amdgcn_exp2f(x[1]);
  }
  return r;
}

}  // namespace

// ABL (diagnostic builds only, never selected by default): 1 no softmax VALU, 2 no QKᵀ MFMA,
// 3 no PV MFMA, 4 no K/V staging, 5 no LDS operand reads.
template <int D, bool CAUSAL, int NW, int ABL = 0>
__global__ __launch_bounds__(64 * NW, 2) void fa_fwd_bf16_fast(AttnArgs p, int nqb) {
#ifndef MT_DIAGNOSTICS
  static_assert(ABL == 0, "ablation variants exist only in the MT_DIAGNOSTICS build");
#endif
  constexpr int kThreads = 64 * NW;
  constexpr int kBQ = 32 * NW;
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

  // Register staging of one K and one V tile (named registers: an array captured by a
  // lambda is demoted to scratch by hipcc).
  static_assert(LPT == 1 || LPT == 2 || LPT == 4, "staging layout");
  uint4 rk0, rk1, rk2, rk3, rv0, rv1, rv2, rv3;
  const int st_r = tid / CPR, st_c = tid % CPR;
  constexpr int RSTEP = kThreads / CPR;
#define SP_LD1(I_, K0_)                                                                   \
  {                                                                                       \
    const int key = min((K0_) + st_r + (I_) * RSTEP, N - 1);                              \
    rk##I_ = *(const uint4*)(Kg + (int64_t)key * skn + st_c * 8);                         \
    rv##I_ = *(const uint4*)(Vg + (int64_t)key * svn + st_c * 8);                         \
  }
#define SP_ST1(I_, BUF_)                                                                  \
  {                                                                                       \
    *(uint4*)(sK + (BUF_) * kBK * D + k_off<D>(st_r + (I_) * RSTEP, st_c)) = rk##I_;      \
    *(uint4*)(sV + (BUF_) * kBK * D + v_off<D>(st_r + (I_) * RSTEP, st_c)) = rv##I_;      \
  }
#define SP_LOAD(T_)                                                                       \
  {                                                                                       \
    SP_LD1(0, (T_) * kBK)                                                                 \
    if constexpr (LPT > 1) SP_LD1(1, (T_) * kBK)                                          \
    if constexpr (LPT > 2) { SP_LD1(2, (T_) * kBK) SP_LD1(3, (T_) * kBK) }                \
  }
#define SP_STORE(BUF_)                                                                    \
  {                                                                                       \
    SP_ST1(0, BUF_)                                                                       \
    if constexpr (LPT > 1) SP_ST1(1, BUF_)                                                \
    if constexpr (LPT > 2) { SP_ST1(2, BUF_) SP_ST1(3, BUF_) }                            \
  }

  f32x16 O[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) O[i] = f32x16{};
  f32x16 L = f32x16{};      // ones·Pᵀ: the row sum, computed on the matrix pipe
  float m_run = -INFINITY;  // raw-score units (unscaled)
  const float c2 = p.scale_log2;
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;

  SP_LOAD(0)
  SP_STORE(0)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): retire the Q loads before the loop
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const int k0 = t * kBK;
    if (ABL != 4 && t + 1 < ntiles) SP_LOAD(t + 1)
    const bool active = !CAUSAL || k0 <= wq_hi;
    if (active) {
      const bf16* k = sK + buf * kBK * D;
      const bf16* v = sV + buf * kBK * D;
      f32x16 S[2];
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          bf16x8 a = ABL == 5 ? qf[(ks + 1) % KSTEPS]
                              : *(const bf16x8*)(k + k_off<D>(kb * 32 + c32, 2 * ks + hf));
          if (ABL == 2) {
            asm volatile("" :: "v"(a));
            if (ks == 0) { S[kb] = f32x16{}; S[kb][0] = (float)t; }
          } else {
            S[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], ks ? S[kb] : f32x16{}, 0, 0, 0);
          }
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
      bf16x8 pf[4];
      if (ABL == 1) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int s = 0; s < 2; ++s) pf[2 * kb + s] = acc_frag<bf16>(S[kb], s);
      } else {
      const float tmax = tile_max(S[0], S[1]);
      // Deferred rescale: raise the running max only when some row of the wave would
      // see exp2 arguments above kRescaleThr. The O/L multiply is unconditional (alpha is
      // exactly 1 otherwise): a branch around it makes hipcc shuttle the MFMA
      // accumulators through copies on every tile, which costs more than the multiply.
      const bool grow = (tmax - m_run) * c2 > kRescaleThr;
      float alpha = 1.f;
      if (__builtin_amdgcn_ballot_w64(grow)) {
        const float m_new = fmaxf(m_run, tmax);
        alpha = (m_run == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f((m_run - m_new) * c2);
        m_run = m_new;
      }
      L *= alpha;
#pragma unroll
      for (int i = 0; i < DB; ++i) O[i] *= alpha;
      const float mc = (m_run == -INFINITY) ? 0.f : m_run * c2;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) pf[2 * kb + s] = softmax_frag(S[kb], s, c2, -mc);
      }
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
            if (ABL == 5) av = __builtin_bit_cast(s16x8, pf[(2 * kb + s + 1) & 3]);
            if (ABL == 3) {
              asm volatile("" :: "v"(av), "v"(pf[2 * kb + s]));
            } else {
              O[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av),
                                                              pf[2 * kb + s], O[db], 0, 0, 0);
            }
          }
          if (ABL != 3) L = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[2 * kb + s], L, 0, 0, 0);
        }
    }
    if (ABL != 4 && t + 1 < ntiles) SP_STORE(buf ^ 1)
    __syncthreads();
  }

  const float l_tot = L[0];
  const float inv_l = 1.f / l_tot;
  if (my_q < N) {
    const ORow Og = o_row(p, b, hh, my_q);
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(Og, db * 32 + 8 * g + 4 * hf, O[db][4 * g] * inv_l, O[db][4 * g + 1] * inv_l,
               O[db][4 * g + 2] * inv_l, O[db][4 * g + 3] * inv_l);
    if (hf == 0) {
      const int64_t row = (int64_t)bh * N + my_q;
      if (p.m) p.m[row] = m_run * p.scale;  // natural-log units: max of s = qk/√d
      if (p.l) p.l[row] = l_tot;
    }
  }
}


// ---------------------------------------------------------------------------------
// Software-pipelined variant (T15-style): each wave keeps two score tiles live. In loop
// iteration t it issues QKᵀ(t) on the matrix pipe while its VALU runs the softmax of
// tile t-1 (independent data), then PV(t-1). K tiles double-buffer; V tiles need a
// 3-slot ring because V(t-1) is still read while tile t+1 is being staged.
//   iteration t: [load tile t+1 -> regs] QKᵀ(t) ‖ softmax(t-1) ; PV(t-1) ;
//                [store tile t+1 -> LDS] ; barrier
template <int D, bool CAUSAL, int NW>
__global__ __launch_bounds__(64 * NW, 2) void fa_fwd_bf16_sp2(AttnArgs p, int nqb) {
  constexpr int kThreads = 64 * NW;
  constexpr int kBQ = 32 * NW;
  constexpr int CPR = D / 8;
  constexpr int TILE_CH = kBK * CPR;
  constexpr int LPT = TILE_CH / kThreads;
  constexpr int KSTEPS = D / 16;
  constexpr int DB = D / 32;
  constexpr int TILE = kBK * D;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* sK = (bf16*)smem;            // [2][TILE]
  bf16* sV = sK + 2 * TILE;          // [3][TILE]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;

  const int nblk = gridDim.x;
  const int hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3;
  const int qd = nblk >> 3, rm = nblk & 7;
  const int logical = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + slot;
  const int bh = logical / nqb;
  int qb = logical % nqb;
  if (CAUSAL) qb = nqb - 1 - qb;
  const int b = bh / p.H, hh = bh % p.H;
  const int q0 = qb * kBQ;

  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Kg = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1];
  const bf16* Vg = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1];
  const int64_t skn = p.sk[2], svn = p.sv[2];

  const int my_q = q0 + wave * 32 + c32;
  const int wq_lo = q0 + wave * 32, wq_hi = wq_lo + 31;

  bf16x8 qf[KSTEPS];
  {
    const int qr = min(my_q, N - 1);
    const bf16* qrow = Qg + (int64_t)qr * p.sq[2];
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) qf[ks] = *(const bf16x8*)(qrow + ks * 16 + 8 * hf);
  }
  const int kend = CAUSAL ? min(N, q0 + kBQ) : N;
  const int ntiles = (kend + kBK - 1) / kBK;

  static_assert(LPT == 1 || LPT == 2 || LPT == 4, "staging layout");
  uint4 rk0, rk1, rk2, rk3, rv0, rv1, rv2, rv3;
  const int st_r = tid / CPR, st_c = tid % CPR;
  constexpr int RSTEP = kThreads / CPR;
#define S2_LD1(I_, K0_)                                                                   \
  {                                                                                       \
    const int key = min((K0_) + st_r + (I_) * RSTEP, N - 1);                              \
    rk##I_ = *(const uint4*)(Kg + (int64_t)key * skn + st_c * 8);                         \
    rv##I_ = *(const uint4*)(Vg + (int64_t)key * svn + st_c * 8);                         \
  }
#define S2_ST1(I_, KB_, VB_)                                                              \
  {                                                                                       \
    *(uint4*)(sK + (KB_) * TILE + k_off<D>(st_r + (I_) * RSTEP, st_c)) = rk##I_;          \
    *(uint4*)(sV + (VB_) * TILE + v_off<D>(st_r + (I_) * RSTEP, st_c)) = rv##I_;          \
  }
#define S2_LOAD(T_)                                                                       \
  {                                                                                       \
    S2_LD1(0, (T_) * kBK)                                                                 \
    if constexpr (LPT > 1) S2_LD1(1, (T_) * kBK)                                          \
    if constexpr (LPT > 2) { S2_LD1(2, (T_) * kBK) S2_LD1(3, (T_) * kBK) }                \
  }
#define S2_STORE(KB_, VB_)                                                                \
  {                                                                                       \
    S2_ST1(0, KB_, VB_)                                                                   \
    if constexpr (LPT > 1) S2_ST1(1, KB_, VB_)                                            \
    if constexpr (LPT > 2) { S2_ST1(2, KB_, VB_) S2_ST1(3, KB_, VB_) }                    \
  }

  f32x16 O[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) O[i] = f32x16{};
  f32x16 L = f32x16{};
  float m_run = -INFINITY;
  const float c2 = p.scale_log2;
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;
  const int i16 = lane & 15, g16 = (lane >> 4) & 1, qr4 = i16 >> 2;
  const int vsw = (D == 64) ? (((qr4 >> 1) & 1) << 2) : ((qr4 & 3) << 2);

  f32x16 S[2];  // scores of the tile awaiting its softmax
  // Prologue: tile 0 into slot 0, QKᵀ(0), then tile 1 into K slot 1 / V slot 1.
  S2_LOAD(0)
  S2_STORE(0, 0)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): Q and tile-0 loads retired
  __syncthreads();
  if (ntiles > 1) S2_LOAD(1)
  if (!CAUSAL || 0 <= wq_hi) {
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const bf16x8 a = *(const bf16x8*)(sK + k_off<D>(kb * 32 + c32, 2 * ks + hf));
        S[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], ks ? S[kb] : f32x16{}, 0, 0, 0);
      }
  }
  if (ntiles > 1) S2_STORE(1, 1)
  __syncthreads();

  int vslot_prev = 0;  // V slot of tile t-1
  for (int t = 1; t <= ntiles; ++t) {
    if (t + 1 < ntiles) S2_LOAD(t + 1)
    // ---- QKᵀ(t) on the matrix pipe ----
    f32x16 Sn[2];
    const bool act_n = t < ntiles && (!CAUSAL || t * kBK <= wq_hi);
    if (act_n) {
      const bf16* k = sK + (t & 1) * TILE;
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const bf16x8 a = *(const bf16x8*)(k + k_off<D>(kb * 32 + c32, 2 * ks + hf));
          Sn[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], ks ? Sn[kb] : f32x16{}, 0, 0, 0);
        }
    }
    // ---- softmax(t-1) on the VALU, then PV(t-1) ----
    const int tp = t - 1;
    if (!CAUSAL || tp * kBK <= wq_hi) {
      const int k0 = tp * kBK;
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
      const float tmax = tile_max(S[0], S[1]);
      const bool grow = (tmax - m_run) * c2 > kRescaleThr;
      float alpha = 1.f;
      if (__builtin_amdgcn_ballot_w64(grow)) {
        const float m_new = fmaxf(m_run, tmax);
        alpha = (m_run == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f((m_run - m_new) * c2);
        m_run = m_new;
      }
      L *= alpha;
#pragma unroll
      for (int i = 0; i < DB; ++i) O[i] *= alpha;
      const float mc = (m_run == -INFINITY) ? 0.f : m_run * c2;
      bf16x8 pf[4];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) pf[2 * kb + s] = softmax_frag(S[kb], s, c2, -mc);
      const bf16* v = sV + vslot_prev * TILE;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int r1 = kb * 32 + 16 * s + 4 * hf + qr4;
#pragma unroll
          for (int db = 0; db < DB; ++db) {
            const int chunk = ((db * 4 + 2 * g16 + ((i16 & 3) >> 1)) ^ vsw);
            const bf16* a1 = v + r1 * D + chunk * 8 + 4 * (i16 & 1);
            typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
            s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
            s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1 + 8 * D));
            typedef __attribute__((ext_vector_type(8))) short s16x8;
            s16x8 av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            O[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av),
                                                            pf[2 * kb + s], O[db], 0, 0, 0);
          }
          L = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[2 * kb + s], L, 0, 0, 0);
        }
    }
    const int vslot_t = vslot_prev == 2 ? 0 : vslot_prev + 1;     // slot of tile t
    const int vslot_n = vslot_t == 2 ? 0 : vslot_t + 1;           // slot of tile t+1
    if (t + 1 < ntiles) S2_STORE((t + 1) & 1, vslot_n)
    __syncthreads();
    S[0] = Sn[0];
    S[1] = Sn[1];
    vslot_prev = vslot_t;
  }
#undef S2_LD1
#undef S2_ST1
#undef S2_LOAD
#undef S2_STORE

  const float l_tot = L[0];
  const float inv_l = 1.f / l_tot;
  if (my_q < N) {
    const ORow Og = o_row(p, b, hh, my_q);
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(Og, db * 32 + 8 * g + 4 * hf, O[db][4 * g] * inv_l, O[db][4 * g + 1] * inv_l,
               O[db][4 * g + 2] * inv_l, O[db][4 * g + 3] * inv_l);
    if (hf == 0) {
      const int64_t row = (int64_t)bh * N + my_q;
      if (p.m) p.m[row] = m_run * p.scale;
      if (p.l) p.l[row] = l_tot;
    }
  }
}

template <int D, bool CAUSAL, int NW>
static hipError_t launch_sp2_t(const AttnArgs& a, hipStream_t st) {
  const size_t smem = 5 * (size_t)kBK * D * sizeof(bf16);
  auto kfn = fa_fwd_bf16_sp2<D, CAUSAL, NW>;
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)smem);
  if (e != hipSuccess) return e;
  const int nqb = (a.N + 32 * NW - 1) / (32 * NW);
  const int64_t nblk = (int64_t)nqb * a.B * a.H;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kfn, dim3((unsigned)nblk), dim3(64 * NW), smem, st, a, nqb);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// Ping-pong variant (default). The 8 waves form two groups, G0 = waves 0-3 and
// G1 = waves 4-7; waves w and w+4 share a SIMD. Phases alternate, separated by one
// s_barrier: while one group runs its MFMA phase M(t) = PV(t-1) + QKᵀ(t) (plus the
// LDS staging of the next K or V tile), the other group runs the VALU-only softmax
// phase V(t') on its own scores, so every SIMD keeps one wave on the matrix pipe and
// one on the vector pipe. The row sum l is computed on the matrix pipe as ones·Pᵀ
// (bf16 P, the same values that enter PV), which moves 32 adds per tile off the VALU.
//   G0: M(0) V(0) M(1) V(1) ...        phases 0,1,2,3,...
//   G1:      M(0) V(0) M(1) ...        phases 1,2,3,4,...
// LDS: K(t) in Kbuf[t&1], written by G1 at phase 2t-1, read at phases 2t, 2t+1;
//      V(t) in Vbuf[t&1], written by G0 at phase 2t,   read at phases 2t+2, 2t+3.
template <int D, bool CAUSAL>
__global__ __launch_bounds__(kThreads, 2) void fa_fwd_bf16_pp(AttnArgs p, int nqb) {
  constexpr int ABL = 0;  // shares the diagnostic-ablation hooks of the single-phase kernel
  constexpr int CPR = D / 8;                   // 16-B chunks per row
  constexpr int TILE_CH = kBK * CPR;           // chunks per K (or V) tile
  constexpr int LPG = TILE_CH / 256;           // chunks per thread when one group stages
  constexpr int LPA = TILE_CH / kThreads;      // chunks per thread when all stage
  constexpr int KSTEPS = D / 16;
  constexpr int DB = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* sK = (bf16*)smem;                      // [2][kBK*D]
  bf16* sV = sK + 2 * kBK * D;                 // [2][kBK*D]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;
  const int gtid = tid & 255;                  // thread index within the group
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;

  const int nblk = gridDim.x;
  const int hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3;
  const int qd = nblk >> 3, rm = nblk & 7;
  const int logical = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + slot;
  const int bh = logical / nqb;
  int qb = logical % nqb;
  if (CAUSAL) qb = nqb - 1 - qb;
  const int b = bh / p.H, hh = bh % p.H;
  const int q0 = qb * kBQ;

  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Kg = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1];
  const bf16* Vg = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1];
  const int64_t skn = p.sk[2], svn = p.sv[2];

  const int my_q = q0 + wave * 32 + c32;
  const int wq_lo = q0 + wave * 32, wq_hi = wq_lo + 31;

  bf16x8 qf[KSTEPS];
  {
    const int qr = min(my_q, N - 1);
    const bf16* qrow = Qg + (int64_t)qr * p.sq[2];
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) qf[ks] = *(const bf16x8*)(qrow + ks * 16 + 8 * hf);
  }

  const int kend = CAUSAL ? min(N, q0 + kBQ) : N;
  const int ntiles = (kend + kBK - 1) / kBK;

  // Group-private staging registers: G0 streams V tiles, G1 streams K tiles.
  static_assert(LPG == 2 || LPG == 4, "staging layout");
  uint4 rs0, rs1, rs2, rs3;
  const bf16* src = grp ? Kg : Vg;
  const int64_t sstride = grp ? skn : svn;
  // chunk ch = gtid + i*256 -> row ch / CPR, column chunk ch % CPR
  const int st_r = gtid / CPR, st_c = gtid % CPR;   // i = 0; rows advance by 256/CPR per i
  constexpr int RSTEP = 256 / CPR;
#define PP_LD1(REG_, I_, T_)                                                     \
  REG_ = *(const uint4*)(src + (int64_t)min((T_) * kBK + st_r + (I_) * RSTEP, N - 1) * sstride + st_c * 8);
#define PP_STAGE_LOAD(T_)                                                       \
  { PP_LD1(rs0, 0, T_) PP_LD1(rs1, 1, T_)                                      \
    if constexpr (LPG == 4) { PP_LD1(rs2, 2, T_) PP_LD1(rs3, 3, T_) } }
#define PP_STAGE_STORE(BASE_, OFF_)                                             \
  { *(uint4*)((BASE_) + OFF_<D>(st_r, st_c)) = rs0;                            \
    *(uint4*)((BASE_) + OFF_<D>(st_r + RSTEP, st_c)) = rs1;                    \
    if constexpr (LPG == 4) {                                                  \
      *(uint4*)((BASE_) + OFF_<D>(st_r + 2 * RSTEP, st_c)) = rs2;              \
      *(uint4*)((BASE_) + OFF_<D>(st_r + 3 * RSTEP, st_c)) = rs3; } }

  // Prologue: everyone stages K(0); G0 prefetches V(0), G1 prefetches K(1).
  {
#pragma unroll
    for (int i = 0; i < LPA; ++i) {
      const int ch = tid + i * kThreads;
      const int r = ch / CPR, c = ch % CPR;
      const int key = min(r, N - 1);
      *(uint4*)(sK + k_off<D>(r, c)) = *(const uint4*)(Kg + (int64_t)key * skn + c * 8);
    }
  }
  // Retire the Q / K(0) loads here: otherwise hipcc's wait insertion carries them
  // into the loop and emits vmcnt(0) before the QKᵀ MFMAs, which also drains the
  // prefetch loads issued in the same phase (a silent serialisation).
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  if (grp == 0) {
    PP_STAGE_LOAD(0)
  } else if (ntiles > 1) {
    PP_STAGE_LOAD(1)
  }

  f32x16 O[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) O[i] = f32x16{};
  f32x16 L = f32x16{};           // ones·Pᵀ: every register holds this lane's row sum
  f32x16 S[2];
  bf16x8 pf[4];
  float m_run = -INFINITY;       // raw-score units
  const float c2 = p.scale_log2;
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;

  // V-image transpose-read bases: the swizzle term depends on the lane only.
  const int i16 = lane & 15, g16 = (lane >> 4) & 1;
  const int qr4 = i16 >> 2;              // row within the 4-row block
  const int vsw = (D == 64) ? (((qr4 >> 1) & 1) << 2) : ((qr4 & 3) << 2);

  __syncthreads();

  // Each group runs the same straight-line loop M(t) | barrier | V(t) | barrier; G1
  // starts one phase late (an idle leading barrier) and skips the final trailing one,
  // so both groups pass exactly 2*ntiles + 2 barriers.
  if (grp == 1) __syncthreads();
  for (int t = 0; t <= ntiles; ++t) {
    // ---------------- M phase: PV(t-1) + QKᵀ(t) + staging ----------------
    if (grp == 0) {
      if (t < ntiles) { PP_STAGE_STORE(sV + (t & 1) * kBK * D, v_off) }            // V(t)
      if (t + 1 < ntiles) { PP_STAGE_LOAD(t + 1) }
    } else {
      if (t + 1 < ntiles) { PP_STAGE_STORE(sK + ((t + 1) & 1) * kBK * D, k_off) }  // K(t+1)
      if (t + 2 < ntiles) { PP_STAGE_LOAD(t + 2) }
    }
    if (t > 0 && (!CAUSAL || (t - 1) * kBK <= wq_hi)) {
      const bf16* v = sV + ((t - 1) & 1) * kBK * D;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int r1 = kb * 32 + 16 * s + 4 * hf + qr4;
#pragma unroll
          for (int db = 0; db < DB; ++db) {
            const int chunk = ((db * 4 + 2 * g16 + ((i16 & 3) >> 1)) ^ vsw);
            const bf16* a1 = v + r1 * D + chunk * 8 + 4 * (i16 & 1);
            typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
            s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
            s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1 + 8 * D));
            typedef __attribute__((ext_vector_type(8))) short s16x8;
            s16x8 av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            if (ABL == 5) av = __builtin_bit_cast(s16x8, pf[(2 * kb + s + 1) & 3]);
            if (ABL == 3) {
              asm volatile("" :: "v"(av), "v"(pf[2 * kb + s]));
            } else {
              O[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av),
                                                              pf[2 * kb + s], O[db], 0, 0, 0);
            }
          }
          if (ABL != 3) L = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[2 * kb + s], L, 0, 0, 0);
        }
    }
    const bool act = t < ntiles && (!CAUSAL || t * kBK <= wq_hi);
    if (act) {
      const bf16* k = sK + (t & 1) * kBK * D;
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const bf16x8 a = *(const bf16x8*)(k + k_off<D>(kb * 32 + c32, 2 * ks + hf));
          S[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], ks ? S[kb] : f32x16{}, 0, 0, 0);
        }
    }
    __syncthreads();
    if (t == ntiles && grp == 1) break;
    // ---------------- V phase: softmax of tile t --------------------------
    if (act) {
      const int k0 = t * kBK;
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
      const float tmax = tile_max(S[0], S[1]);
      const bool grow = (tmax - m_run) * c2 > kRescaleThr;
      float alpha = 1.f;
      if (__builtin_amdgcn_ballot_w64(grow)) {
        const float m_new = fmaxf(m_run, tmax);
        alpha = (m_run == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f((m_run - m_new) * c2);
        m_run = m_new;
      }
#pragma unroll
      for (int i = 0; i < DB; ++i) O[i] *= alpha;
      L *= alpha;
      const float mc = (m_run == -INFINITY) ? 0.f : m_run * c2;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) pf[2 * kb + s] = softmax_frag(S[kb], s, c2, -mc);
    }
    __syncthreads();
  }

  const float l_tot = L[0];
  const float inv_l = 1.f / l_tot;
  if (my_q < N) {
    const ORow Og = o_row(p, b, hh, my_q);
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(Og, db * 32 + 8 * g + 4 * hf, O[db][4 * g] * inv_l, O[db][4 * g + 1] * inv_l,
               O[db][4 * g + 2] * inv_l, O[db][4 * g + 3] * inv_l);
    if (hf == 0) {
      const int64_t row = (int64_t)bh * N + my_q;
      if (p.m) p.m[row] = m_run * p.scale;
      if (p.l) p.l[row] = l_tot;
    }
  }
}

#undef PP_LD1
#undef PP_STAGE_LOAD
#undef PP_STAGE_STORE

template <int D, bool CAUSAL>
static hipError_t launch_pp_t(const AttnArgs& a, hipStream_t st) {
  const size_t smem = 4 * (size_t)kBK * D * sizeof(bf16);
  auto kfn = fa_fwd_bf16_pp<D, CAUSAL>;
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)smem);
  if (e != hipSuccess) return e;
  const int nqb = (a.N + kBQ - 1) / kBQ;
  const int64_t nblk = (int64_t)nqb * a.B * a.H;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kfn, dim3((unsigned)nblk), dim3(kThreads), smem, st, a, nqb);
  return hipGetLastError();
}

#undef SP_LD1
#undef SP_ST1
#undef SP_LOAD
#undef SP_STORE

template <int D, bool CAUSAL, int NW, int ABL = 0>
static hipError_t launch_fast_t(const AttnArgs& a, hipStream_t st) {
  const size_t smem = 4 * (size_t)kBK * D * sizeof(bf16);
  auto kfn = fa_fwd_bf16_fast<D, CAUSAL, NW, ABL>;
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)smem);
  if (e != hipSuccess) return e;
  const int nqb = (a.N + 32 * NW - 1) / (32 * NW);
  const int64_t nblk = (int64_t)nqb * a.B * a.H;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kfn, dim3((unsigned)nblk), dim3(64 * NW), smem, st, a, nqb);
  return hipGetLastError();
}

// Variant map (mt_flash_set_kernel_policy): 0 = default = single-phase 4-wave kernel
// (fastest measured: r01 A/B in profiles/), 2 = single-phase 8-wave, 3 = same as 0,
// 4 / 5 = software-pipelined 8 / 4-wave, 6 = ping-pong 8-wave, 10..15 = ablation builds
// (MT_DIAGNOSTICS only: wrong results, timing only).
hipError_t launch_fwd_fast(const AttnArgs& a, bool causal, int variant, hipStream_t st,
                           bool* handled) {
  *handled = true;
  const int d = a.d;
  if (d != 64 && d != 128) {
    *handled = false;
    return hipSuccess;
  }
#define MT_DISPATCH(LAUNCH, ...)                                                         \
  return d == 64 ? (causal ? LAUNCH<64, true, ##__VA_ARGS__>(a, st)                      \
                           : LAUNCH<64, false, ##__VA_ARGS__>(a, st))                    \
                 : (causal ? LAUNCH<128, true, ##__VA_ARGS__>(a, st)                     \
                           : LAUNCH<128, false, ##__VA_ARGS__>(a, st));
#ifndef MT_DIAGNOSTICS
  // product build: the single-phase 8-wave kernel (the default fallback); the others are A/B
  (void)variant;
  MT_DISPATCH(launch_fast_t, 8)
#else
  switch (variant) {
    case 2: MT_DISPATCH(launch_fast_t, 8)
    case 4: MT_DISPATCH(launch_sp2_t, 8)
    case 5: MT_DISPATCH(launch_sp2_t, 4)
    case 6: MT_DISPATCH(launch_pp_t)
    default: break;
  }
  if (variant >= 10 && variant <= 15 && d == 64 && !causal) {  // diagnostics
    switch (variant) {
      case 10: return launch_fast_t<64, false, 8, 0>(a, st);
      case 11: return launch_fast_t<64, false, 8, 1>(a, st);
      case 12: return launch_fast_t<64, false, 8, 2>(a, st);
      case 13: return launch_fast_t<64, false, 8, 3>(a, st);
      case 14: return launch_fast_t<64, false, 8, 4>(a, st);
      default: return launch_fast_t<64, false, 8, 5>(a, st);
    }
  }
  MT_DISPATCH(launch_fast_t, 4)
#endif
#undef MT_DISPATCH
}

}  // namespace mt
