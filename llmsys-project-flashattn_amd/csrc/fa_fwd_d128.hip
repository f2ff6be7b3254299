// FlashAttention forward, bf16 MFMA kernel for d = 128 (BASELINE config 4's head size).
//
// Same scheme as the d = 64 kernel v4 (fa_fwd_v4.hip): query-on-lane Sᵀ = K·Qᵀ with the
// accumulator reused as the PV B operand, K/V tiles of 64 keys double-buffered in LDS, a
// software pipeline in which QKᵀ of tile t+1 overlaps the softmax of tile t, and a frozen
// first-tile softmax reference in the mask-free bulk tiles (a workgroup whose row-sum share
// leaves 2^64 recomputes with the per-tile deferred-max path). At d = 128 a tile costs 32
// MFMAs per wave (16 QKᵀ over 8 k-steps, 16 PV over 4 d-blocks) against the same 32
// exponentials per lane as at d = 64, so the softmax VALU work per MFMA halves and the
// MFMA pipe, not the VALU issue, is the intended bound.
//
// Bulk iteration issue order (sched_barrier-fenced):
//    8 x [K read (2 ahead), QKᵀ(t+1) MFMA (key block 0), 2 exponentials of key block 0 of t]
//    8 x [K read (2 ahead), QKᵀ(t+1) MFMA (key block 1), 1 exponential of key block 1 of t]
//    8 x [Vᵀ reads (2 ahead), PV MFMA (key block 0), 1 exponential of key block 1]
//    8 x [Vᵀ reads (2 ahead), PV MFMA (key block 1)]
// Reference semantics: forward_kernel, src/flashattention_kernel.cu:9-112 (non-causal) and
// forward_kernel_causal :438-545; same (O, m, l) contract as every forward kernel here.
#include "fa_fwd_bf16.h"

namespace mt {

namespace {

using namespace fwdbf16;
constexpr int D = 128;
constexpr int kBK = 64;
constexpr int TILE = kBK * D;
constexpr int CPR = D / 8;                     // 16-B chunks per row
constexpr float kThr = 8.0f;                   // log2 units: deferred-rescale threshold
constexpr float kBulkLimit = 1.8446744e19f;    // 2^64: bound on a lane's row-sum share

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

template <int NW>
struct C6 {
  static constexpr int kThreads = 64 * NW;
  static constexpr int kBQ = 32 * NW;
  static constexpr int RSTEP = kThreads / CPR;
  static constexpr int LPT = kBK / RSTEP;      // staging chunks per thread per tile
};

template <int LPT>
struct Ctx6 {
  int koff[8];   // K row-image offset of this lane's A fragment per k-step (key block 0)
  int voff[4];   // Vᵀ transpose-read offset per 32-wide d block (16-key step 0)
  int kgo[LPT], vgo[LPT], kso[LPT], vso[LPT];
  int kdo[LPT], vdo[LPT];  // LDS-DMA per-lane source offsets
};

__device__ __forceinline__ bf16x8 vt_read(const bf16* a1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1 + 8 * D));
  const s16x8 av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, av);
}

// S = K(tile at sk)·Qᵀ (32 queries x 64 keys as two 32-key blocks)
template <int LPT>
__device__ __forceinline__ void qk6(const bf16* sk, const Ctx6<LPT>& c, const bf16x8 (&qf)[8],
                                    f32x16 (&S)[2]) {
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const bf16x8 a = *(const bf16x8*)(sk + kb * 32 * D + c.koff[ks]);
      S[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], ks ? S[kb] : f32x16{}, 0, 0, 0);
    }
}

// O += Vᵀ(key block KB of the tile at sv)·Pᵀ
template <int KB, int LPT>
__device__ __forceinline__ void pv6(const bf16* sv, const Ctx6<LPT>& c, const bf16x8& p0,
                                    const bf16x8& p1, f32x16 (&O)[4]) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int db = 0; db < 4; ++db)
      O[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vt_read(sv + (KB * 32 + 16 * s) * D + c.voff[db]),
                                                      s ? p1 : p0, O[db], 0, 0, 0);
}

__device__ __forceinline__ void exp6(const f32x16& s, float c2, float nmc, bf16x8& p0, bf16x8& p1,
                                     float& l) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(s[j], c2, nmc));
    l += e;
    if (j < 8) p0[j] = (bf16)e;
    else p1[j - 8] = (bf16)e;
  }
}

template <bool CAUSAL>
__device__ __forceinline__ void mask6(f32x16 (&S)[2], int k0, int N, int my_q, int hf) {
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = k0 + kb * 32 + acc_row(r, hf);
      if (key >= N || (CAUSAL && key > my_q)) S[kb][r] = -INFINITY;
    }
}

// Deferred-max bookkeeping of the general path; returns -m*c2.
__device__ __forceinline__ float max6(const f32x16 (&S)[2], f32x16 (&O)[4], float& l, float& m_run,
                                      float c2) {
  const float tmax = row_max32(S[0], S[1]);
  if (__builtin_amdgcn_ballot_w64((tmax - m_run) * c2 > kThr)) {
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m_run - m_new) * c2);
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) O[i][r] *= alpha;
    l *= alpha;
  }
  return -(m_run * c2);
}

template <int LPT>
__device__ __forceinline__ void load6(uint4 (&r)[LPT], __amdgpu_buffer_rsrc_t rs, const int (&go)[LPT],
                                      int step) {
#pragma unroll
  for (int i = 0; i < LPT; ++i)
    r[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, go[i] + step, 0, 0));
}

template <int LPT>
__device__ __forceinline__ void store6(bf16* dst, const uint4 (&r)[LPT], const int (&so)[LPT]) {
#pragma unroll
  for (int i = 0; i < LPT; ++i) *(uint4*)(dst + so[i]) = r[i];
}

// LDS-DMA (DMA = true): one buffer_load_dwordx4 ... lds writes 1 KiB = 4 rows of 256 B in
// lane order; lane l of rows R0..R0+3 fetches the chunk the swizzle puts at slot l % 16 of
// row R0 + l / 16 (the XOR swizzles are involutions).
__device__ __forceinline__ void dma6(bf16* dst_rows, __amdgpu_buffer_rsrc_t rs, int go, int step) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst_rows, 16,
                                           go + step, 0, 0, 0);
}

__device__ __forceinline__ bf16 exp1(float s, float c2, float nmc, float& l) {
  const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(s, c2, nmc));
  l += e;
  return (bf16)e;
}

// One bulk iteration (see the file comment): QKᵀ(t+1) from sk into SN, exp of SC, PV(t)
// from sv into O.
template <int LPT>
__device__ __forceinline__ void bulk6(const bf16* sk, const bf16* sv, const Ctx6<LPT>& c,
                                      const bf16x8 (&qf)[8], const f32x16 (&SC)[2], f32x16 (&SN)[2],
                                      f32x16 (&O)[4], float& l, float c2, float nmc) {
  bf16x8 kf[16];
  bf16x8 pf[4];
  float l0 = 0.f, l1 = 0.f;
  // QKᵀ MFMA i: key block i >> 3, k-step i & 7 (block 0's chain completes first, so SC[0]
  // is dead before SN[1] starts: 48 score registers live instead of 64)
#define D6_KREAD(I_) kf[I_] = *(const bf16x8*)(sk + ((I_) >> 3) * 32 * D + c.koff[(I_) & 7]);
  D6_KREAD(0)
  D6_KREAD(1)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i + 2 < 16) D6_KREAD(i + 2)
    SN[i >> 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[i], qf[i & 7], (i & 7) ? SN[i >> 3] : f32x16{},
                                                        0, 0, 0);
    if (i < 8) {  // 2 exponentials of SC[0] per MFMA
      pf[i >> 2][(2 * i) & 7] = exp1(SC[0][2 * i], c2, nmc, l0);
      pf[i >> 2][(2 * i + 1) & 7] = exp1(SC[0][2 * i + 1], c2, nmc, l1);
    } else {      // then SC[1], one per MFMA
      const int j = i - 8;
      pf[2 + (j >> 3)][j & 7] = exp1(SC[1][j], c2, nmc, (j & 1) ? l1 : l0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#undef D6_KREAD
  bf16x8 vf[8];
  // PV MFMA n of key block KB: 16-key step n >> 2, d block n & 3
#define D6_VREAD(KB_, N_) vf[N_] = vt_read(sv + ((KB_) * 32 + 16 * ((N_) >> 2)) * D + c.voff[(N_) & 3]);
  D6_VREAD(0, 0)
  D6_VREAD(0, 1)
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    if (n + 2 < 8) D6_VREAD(0, n + 2)
    O[n & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[n], pf[n >> 2], O[n & 3], 0, 0, 0);
    pf[3][n] = exp1(SC[1][8 + n], c2, nmc, (n & 1) ? l1 : l0);  // the rest of SC[1]
    __builtin_amdgcn_sched_barrier(0);
  }
  D6_VREAD(1, 0)
  D6_VREAD(1, 1)
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    if (n + 2 < 8) D6_VREAD(1, n + 2)
    O[n & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[n], pf[2 + (n >> 2)], O[n & 3], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
#undef D6_VREAD
  l += l0 + l1;
}

}  // namespace

// PAIR (causal): a workgroup owns query blocks nqb-1-u and u of one head (heaviest, then
// lightest; PAIR = 2: lightest first), so every workgroup walks nqb + 1 key tiles
// (fa_fwd_v4.hip, same scheme).
template <bool CAUSAL, int NW, bool DMA = false, int PAIR = 0>
__global__ __launch_bounds__(64 * NW, 8 / NW) void fa_fwd_bf16_d128(AttnArgs p, int nqb) {
  using C = C6<NW>;
  constexpr int LPT = C::LPT;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* const sK0 = (bf16*)smem_raw;
  bf16* const sK1 = sK0 + TILE;
  bf16* const sV0 = sK0 + 2 * TILE;
  bf16* const sV1 = sK0 + 3 * TILE;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;

  // XCD-aware bijective block remap: consecutive logical blocks (same head) share an XCD's L2
  const int nblk = gridDim.x, hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3, qd = nblk >> 3, rm = nblk & 7;
  const int logical = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + slot;
  const int nunit = PAIR ? (nqb + 1) / 2 : nqb;  // work units per head
  const int bh = logical / nunit;
  const int unit = logical % nunit;
  const int b = bh / p.H, hh = bh % p.H;
  for (int rep = 0; rep < (PAIR ? 2 : 1); ++rep) {
  int qb = unit;
  if (PAIR) {
    qb = (rep == (PAIR == 2 ? 0 : 1)) ? unit : nqb - 1 - unit;
    if (rep && unit == nqb - 1 - unit) break;  // odd nqb: the middle block has no partner
  } else if (CAUSAL) {
    qb = nqb - 1 - qb;  // heaviest first
  }
  const int q0 = qb * C::kBQ;

  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Kg = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1];
  const bf16* Vg = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1];
  const int skn = (int)p.sk[2], svn = (int)p.sv[2];
  const __amdgpu_buffer_rsrc_t rk =
      __builtin_amdgcn_make_buffer_rsrc((void*)Kg, (short)0, ((N - 1) * skn + D) * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv =
      __builtin_amdgcn_make_buffer_rsrc((void*)Vg, (short)0, ((N - 1) * svn + D) * 2, 0x00020000);

  const int my_q = q0 + wave * 32 + c32;
  const int wq_hi = q0 + wave * 32 + 31;

  bf16x8 qf[8];
  {
    const bf16* qrow = Qg + (int64_t)min(my_q, N - 1) * p.sq[2];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = *(const bf16x8*)(qrow + ks * 16 + 8 * hf);
  }

  Ctx6<LPT> c;
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) c.koff[ks] = k_swz<D>(c32, 2 * ks + hf);
  {
    const int i16 = lane & 15, g = (lane >> 4) & 1;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const int col = db * 32 + 16 * g + 4 * (i16 & 3);
      c.voff[db] = v_swz<D>(4 * hf + (i16 >> 2), col >> 3) + (col & 7);
    }
    const int st_r = tid / CPR, st_c = tid % CPR;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int r = st_r + i * C::RSTEP;
      c.kgo[i] = (r * skn + st_c * 8) * 2;
      c.vgo[i] = (r * svn + st_c * 8) * 2;
      c.kso[i] = k_swz<D>(r, st_c);
      c.vso[i] = v_swz<D>(r, st_c);
      // DMA: wave w's instruction i fills rows 4 * (LPT * w + i) .. + 3
      const int dr = 4 * (LPT * wave + i) + (lane >> 4), dc = lane & 15;
      c.kdo[i] = (dr * skn + (dc ^ (dr & 15)) * 8) * 2;
      c.vdo[i] = (dr * svn + (dc ^ ((dr & 3) << 2)) * 8) * 2;
    }
  }
  const float c2 = p.scale_log2;
  const int kend = CAUSAL ? min(N, q0 + C::kBQ) : N;
  const int ntiles = (kend + kBK - 1) / kBK;
  const int ktile_b = kBK * skn * 2, vtile_b = kBK * svn * 2;
  const int nfull = CAUSAL ? min(N / kBK, q0 / kBK) : N / kBK;  // mask-free tiles

  // staging: issue (global -> registers, or LDS-DMA straight into the slot) and write
  // (registers -> slot; nothing with DMA, whose writes land by the barrier's vmcnt(0))
#define D6_ISSUE_K(SLOT_, STEP_)                                                             \
  {                                                                                          \
    if (DMA) {                                                                               \
      _Pragma("unroll") for (int i = 0; i < LPT; ++i)                                        \
        dma6((SLOT_) + 4 * (LPT * wave + i) * D, rk, c.kdo[i], (STEP_));                     \
    } else load6(rK, rk, c.kgo, (STEP_));                                                    \
  }
#define D6_ISSUE_V(SLOT_, STEP_)                                                             \
  {                                                                                          \
    if (DMA) {                                                                               \
      _Pragma("unroll") for (int i = 0; i < LPT; ++i)                                        \
        dma6((SLOT_) + 4 * (LPT * wave + i) * D, rv, c.vdo[i], (STEP_));                     \
    } else load6(rV, rv, c.vgo, (STEP_));                                                    \
  }
#define D6_WRITE_K(SLOT_) { if (!DMA) store6((SLOT_), rK, c.kso); }
#define D6_WRITE_V(SLOT_) { if (!DMA) store6((SLOT_), rV, c.vso); }
  f32x16 O[4];
  float l_part, m_run;
  uint4 rK[LPT], rV[LPT];
  f32x16 SA[2], SB[2];

  // Pass 0: frozen-reference bulk loop. Pass 1 (only if a lane's row-sum share left the
  // safe range): the whole workgroup recomputes with the deferred-max path throughout.
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int i = 0; i < 4; ++i) O[i] = f32x16{};
    l_part = 0.f;
    m_run = -INFINITY;
    D6_ISSUE_K(sK0, 0)
    D6_ISSUE_V(sV0, 0)
    D6_WRITE_K(sK0)
    D6_WRITE_V(sV0)
    D6_ISSUE_K(sK1, ktile_b)
    D6_WRITE_K(sK1)
    __syncthreads();
    qk6(sK0, c, qf, SA);
    __syncthreads();  // iteration 0 overwrites K slot 0, which every wave just read

    // General iteration t (deferred max, masks, per-wave causal skipping); S(t) in SA,
    // QK(t+1) after PV(t) into SA. LDS slots by runtime parity.
#define D6_GENERAL(T_)                                                                       \
  {                                                                                          \
    const int t_ = (T_);                                                                     \
    const int par = t_ & 1;                                                                  \
    const bool next = t_ + 1 < ntiles;                                                       \
    if (t_ + 2 < ntiles) D6_ISSUE_K(par ? sK1 : sK0, (t_ + 2) * ktile_b)                     \
    if (next) D6_ISSUE_V(par ? sV0 : sV1, (t_ + 1) * vtile_b)                                \
    if (!CAUSAL || t_ * kBK <= wq_hi) {                                                      \
      if (t_ >= nfull) mask6<CAUSAL>(SA, t_ * kBK, N, my_q, hf);                             \
      const float nmc = max6(SA, O, l_part, m_run, c2);                                      \
      bf16x8 p0, p1, p2, p3;                                                                 \
      exp6(SA[0], c2, nmc, p0, p1, l_part);                                                  \
      exp6(SA[1], c2, nmc, p2, p3, l_part);                                                  \
      const bf16* sv = par ? sV1 : sV0;                                                      \
      pv6<0>(sv, c, p0, p1, O);                                                              \
      pv6<1>(sv, c, p2, p3, O);                                                              \
    }                                                                                        \
    if (next && (!CAUSAL || (t_ + 1) * kBK <= wq_hi)) qk6(par ? sK0 : sK1, c, qf, SA);       \
    if (t_ + 2 < ntiles) D6_WRITE_K(par ? sK1 : sK0)                                         \
    if (next) D6_WRITE_V(par ? sV0 : sV1)                                                    \
    __syncthreads();                                                                         \
  }

    D6_GENERAL(0)  // tile 0 sets the reference max
    int t = 1;
    if (pass == 0) {
      const float nmc = -(m_run * c2);
      // Bulk iteration t (tiles t, t+1, t+2 mask-free and active for every wave); staging
      // of K(t+2) / V(t+1) is unconditional (past the end it reads zeros or unused rows
      // into a slot nobody reads).
#define D6_BULK(SC_, SN_, SKN_, SVC_, SKW_, SVW_, T_)                                        \
  {                                                                                         \
    D6_ISSUE_K(SKW_, ((T_) + 2) * ktile_b)                                                  \
    D6_ISSUE_V(SVW_, ((T_) + 1) * vtile_b)                                                  \
    bulk6(SKN_, SVC_, c, qf, SC_, SN_, O, l_part, c2, nmc);                                 \
    D6_WRITE_K(SKW_)                                                                        \
    D6_WRITE_V(SVW_)                                                                        \
    __syncthreads();                                                                        \
  }
      // t odd: S(t) in SA, K(t+1) in slot 0, V(t) in slot 1; writes K(t+2) -> slot 1,
      // V(t+1) -> slot 0. t+1 even: mirror.
      for (; t + 2 < nfull; t += 2) {
        D6_BULK(SA, SB, sK0, sV1, sK1, sV0, t)
        D6_BULK(SB, SA, sK1, sV0, sK0, sV1, t + 1)
      }
#undef D6_BULK
    }
    for (; t < ntiles; ++t) D6_GENERAL(t)
#undef D6_GENERAL
#undef D6_ISSUE_K
#undef D6_ISSUE_V
#undef D6_WRITE_K
#undef D6_WRITE_V
    const bool bad = !(l_part <= kBulkLimit);
    if (pass == 1 || !__syncthreads_or(bad)) break;
  }

  const auto lsw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_part), __float_as_uint(l_part),
                                                    false, false);
  const float l_tot = __uint_as_float(lsw[0]) + __uint_as_float(lsw[1]);
  const float inv_l = 1.f / l_tot;
  if (my_q < N) {
    bf16* Og = (bf16*)p.out + b * p.so[0] + hh * p.so[1] + (int64_t)my_q * p.so[2];
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(Og + db * 32 + 8 * g + 4 * hf, O[db][4 * g] * inv_l, O[db][4 * g + 1] * inv_l,
               O[db][4 * g + 2] * inv_l, O[db][4 * g + 3] * inv_l, true);
    if (hf == 0) {
      const int64_t row = (int64_t)bh * N + my_q;
      if (p.m) p.m[row] = m_run * p.scale;
      if (p.l) p.l[row] = l_tot;
    }
  }
  }  // rep
}

template <bool CAUSAL, int NW, bool DMA = false, int PAIR = 0>
static hipError_t launch_d128_t(const AttnArgs& a, hipStream_t st) {
  const size_t smem = 4 * (size_t)TILE * sizeof(bf16);
  auto kfn = fa_fwd_bf16_d128<CAUSAL, NW, DMA, PAIR>;
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)smem);
  if (e != hipSuccess) return e;
  const int nqb = (a.N + 32 * NW - 1) / (32 * NW);
  const int64_t nblk = (int64_t)(PAIR ? (nqb + 1) / 2 : nqb) * a.B * a.H;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kfn, dim3((unsigned)nblk), dim3(64 * NW), smem, st, a, nqb);
  return hipGetLastError();
}

// d = 128, bf16, unit d-stride (the caller's vec check); every per-head K/V byte offset up
// to two tiles past N must fit the 31-bit buffer offset (the bulk loop stages one tile
// ahead of the last one it needs).
hipError_t launch_fwd_d128(const AttnArgs& a, bool causal, int nw, bool dma, hipStream_t st,
                           bool* handled, int pair) {
  *handled = false;
  // an fp32 O (MT_BF16_F32OUT) takes the generic kernels: the epilogue's extra store path
  // moved this kernel's register allocation into spills inside its main loop
  if (a.d != D || a.o_f32) return hipSuccess;
  const int64_t lim = (int64_t)1 << 31;
  if (((int64_t)a.N + 2 * kBK) * a.sk[2] * 2 >= lim || ((int64_t)a.N + 2 * kBK) * a.sv[2] * 2 >= lim)
    return hipSuccess;
  *handled = true;
#ifndef MT_DIAGNOSTICS
  // product build: 8 waves, causal paired light-first (the defaults); the rest are A/B policies
  (void)nw;
  (void)dma;
  (void)pair;
  return causal ? launch_d128_t<true, 8, false, 2>(a, st) : launch_d128_t<false, 8>(a, st);
#else
  if (causal && pair == 2)
    return nw == 8 ? launch_d128_t<true, 8, false, 2>(a, st) : launch_d128_t<true, 4, false, 2>(a, st);
  if (causal && pair)
    return nw == 8 ? launch_d128_t<true, 8, false, 1>(a, st) : launch_d128_t<true, 4, false, 1>(a, st);
  if (dma) {
    if (nw == 8) return causal ? launch_d128_t<true, 8, true>(a, st) : launch_d128_t<false, 8, true>(a, st);
    return causal ? launch_d128_t<true, 4, true>(a, st) : launch_d128_t<false, 4, true>(a, st);
  }
  if (nw == 8) return causal ? launch_d128_t<true, 8>(a, st) : launch_d128_t<false, 8>(a, st);
  return causal ? launch_d128_t<true, 4>(a, st) : launch_d128_t<false, 4>(a, st);
#endif
}

}  // namespace mt
