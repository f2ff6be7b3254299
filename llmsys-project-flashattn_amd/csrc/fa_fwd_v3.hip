// FlashAttention forward, bf16 MFMA kernel v3: software-pipelined tile loop (d = 64).
//
// Same contract, LDS images and MFMA layout as v2 (fa_fwd_v2.hip). v2's tile is a serial
// chain inside one wave — QKᵀ(t) → row max → exp → PVᵀ(t) — so a wave's softmax VALU can
// only overlap the matrix pipe through the other wave on its SIMD. v3 skews the chain
// by one tile: iteration t runs
//     row max(t) ; [rare rescale] ; QKᵀ(t+1) ‖ exp(t, keys 0-31) ; PV(t, keys 0-31) ‖
//     exp(t, keys 32-63) ; PV(t, keys 32-63)
// so the MFMAs of the next tile's scores and of this tile's first half of PV are
// independent of the exponentials issued between them, and one wave keeps the matrix
// pipe fed on its own. K and V are staged one tile apart (iteration t stages K(t+2) and
// V(t+1)); both still double-buffer in LDS with one barrier per iteration, because every
// slot written in iteration t was last read in iteration t-1.
#include "fa_fwd_bf16.h"

namespace mt {

namespace {

using namespace fwdbf16;
constexpr int kBK = 64;
constexpr float kThr = 8.0f;  // log2 units: deferred-rescale threshold

template <int D, int NW>
struct V3 {
  static constexpr int kThreads = 64 * NW;
  static constexpr int kBQ = 32 * NW;
  static constexpr int CPR = D / 8;
  static constexpr int LPT = kBK * CPR / kThreads;  // 16-B chunks per thread per tile
  static constexpr int RSTEP = kThreads / CPR;
  static constexpr int KSTEPS = D / 16;
  static constexpr int DB = D / 32;
  static constexpr int TILE = kBK * D;  // elements per K (or V) tile
};

struct Ctx {
  int koff[4];    // per-lane K operand offsets per k-step (elements, slot 0, kb 0)
  int voff[2];    // per-lane Vᵀ tr-read offsets per 32-wide d block (slot 0, row block 0)
  int kgo[4], vgo[4];  // staging: per-thread global byte offsets of tile 0
  int kso[4], vso[4];  // staging: per-thread LDS element offsets (slot 0)
};

// S = K(tile in slot KS)·Qᵀ for one wave (32 queries x 64 keys).
template <int D, int NW, int KS>
__device__ __forceinline__ void v3_qk(const bf16* smem, const Ctx& c, const bf16x8 (&qf)[D / 16],
                                      f32x16 (&S)[2]) {
  using C = V3<D, NW>;
  const bf16* sk = smem + KS * C::TILE;
#pragma unroll
  for (int ks = 0; ks < C::KSTEPS; ++ks)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const bf16x8 a = *(const bf16x8*)(sk + kb * 32 * D + c.koff[ks]);
      S[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], ks ? S[kb] : f32x16{}, 0, 0, 0);
    }
}

// bf16 P fragments (B operands of PV) of one 32-key block: p = exp2(s*c2 - m*c2); the
// fp32 p also go into the lane's partial row sum (the two lane halves hold different
// keys of the same query and are combined once, at the end).
template <bool LM>
__device__ __forceinline__ void v3_exp(const f32x16& s, float c2, float nmc, bf16x8& p0, bf16x8& p1,
                                       float& l) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(s[j], c2, nmc));
    if (!LM) l += e;
    p0[j] = (bf16)e;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(s[8 + j], c2, nmc));
    if (!LM) l += e;
    p1[j] = (bf16)e;
  }
}

// Row sum on the matrix pipe: L += 1·Pᵀ (every row of L holds the sum; 4 MFMAs a tile
// instead of 32 VALU adds).
__device__ __forceinline__ void v3_lsum(f32x16& L, const bf16x8& p) {
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;
  L = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, p, L, 0, 0, 0);
}

// O += Vᵀ(key block kb of the tile in slot VS)·Pᵀ.
template <int D, int NW, int VS, int KB>
__device__ __forceinline__ void v3_pv(const bf16* smem, const Ctx& c, const bf16x8& p0,
                                      const bf16x8& p1, f32x16 (&O)[D / 32]) {
  using C = V3<D, NW>;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  const bf16* sv = smem + 2 * C::TILE + VS * C::TILE;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const bf16x8& pf = s ? p1 : p0;
#pragma unroll
    for (int db = 0; db < C::DB; ++db) {
      const bf16* a1 = sv + (KB * 32 + 16 * s) * D + c.voff[db];
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1 + 8 * D));
      const s16x8 av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      O[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av), pf, O[db], 0, 0, 0);
    }
  }
}

template <int D, bool CAUSAL>
__device__ __forceinline__ void v3_mask(f32x16 (&S)[2], int k0, int N, int my_q, int hf) {
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = k0 + kb * 32 + acc_row(r, hf);
      if (key >= N || (CAUSAL && key > my_q)) S[kb][r] = -INFINITY;
    }
}

// Deferred-max online-softmax bookkeeping for one tile; returns -m*c2 for the exponent.
template <int D>
__device__ __forceinline__ float v3_max(const f32x16 (&S)[2], f32x16 (&O)[D / 32], float& l,
                                        f32x16& L, float& m_run, float c2) {
  const float tmax = row_max32(S[0], S[1]);
  if (__builtin_amdgcn_ballot_w64((tmax - m_run) * c2 > kThr)) {
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m_run - m_new) * c2);
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < D / 32; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) O[i][r] *= alpha;
    l *= alpha;
#pragma unroll
    for (int r = 0; r < 16; ++r) L[r] *= alpha;
  }
  return -(m_run * c2);
}

template <int D, int NW>
__device__ __forceinline__ void v3_load(uint4 (&r)[4], __amdgpu_buffer_rsrc_t rs, const int (&go)[4],
                                        int step) {
#pragma unroll
  for (int i = 0; i < V3<D, NW>::LPT; ++i)
    r[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, go[i] + step, 0, 0));
}

template <int D, int NW>
__device__ __forceinline__ void v3_store(bf16* dst, const uint4 (&r)[4], const int (&so)[4]) {
#pragma unroll
  for (int i = 0; i < V3<D, NW>::LPT; ++i) *(uint4*)(dst + so[i]) = r[i];
}

// One bulk iteration after the row max, in an explicit issue order fenced by
// sched_barrier(0) (the compiler otherwise clusters the MFMAs and the exponentials):
//   8 x [K read (2 ahead), QKᵀ(t+1) MFMA, exp(t) slice: 2 keys of block 0]
//   4 x [Vᵀ reads, PV(t, block 0) MFMA, exp(t) slice: 4 keys of block 1]
//   4 x [Vᵀ reads, PV(t, block 1) MFMA]
template <int D, int NW, int KSN, int VS, bool LM>
__device__ __forceinline__ void v3_bulk(const bf16* smem, const Ctx& c, const bf16x8 (&qf)[D / 16],
                                        const f32x16 (&SC)[2], f32x16 (&SN)[2], f32x16 (&O)[D / 32],
                                        float& l, f32x16& L, float c2, float nmc) {
  using C = V3<D, NW>;
  static_assert(C::KSTEPS == 4 && C::DB == 2, "d = 64 schedule");
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  const bf16* sk = smem + KSN * C::TILE;
  const bf16* sv = smem + 2 * C::TILE + VS * C::TILE;
  bf16x8 kf[8];
  bf16x8 pf[4];
  // MFMA i of QKᵀ: k-step i/2, key block i%2
#define V3_KREAD(I_) kf[I_] = *(const bf16x8*)(sk + ((I_) & 1) * 32 * D + c.koff[(I_) >> 1]);
  V3_KREAD(0)
  V3_KREAD(1)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i + 2 < 8) V3_KREAD(i + 2)
    SN[i & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[i], qf[i >> 1], i < 2 ? f32x16{} : SN[i & 1],
                                                       0, 0, 0);
#pragma unroll
    for (int j = 2 * i; j < 2 * i + 2; ++j) {
      const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(SC[0][j], c2, nmc));
      if (!LM) l += e;
      pf[j >> 3][j & 7] = (bf16)e;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#undef V3_KREAD
  // PV: MFMA (kb, s, db) reads Vᵀ rows kb*32+16s.. of d block db
  s16x4 vlo[4], vhi[4];
#define V3_VREAD(KB_, N_)                                                                  \
  {                                                                                        \
    const bf16* a1 = sv + ((KB_) * 32 + 16 * ((N_) >> 1)) * D + c.voff[(N_) & 1];          \
    vlo[N_] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);                     \
    vhi[N_] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1 + 8 * D));           \
  }
#define V3_PVMMA(N_, PF_)                                                                  \
  {                                                                                        \
    const s16x8 av = {vlo[N_][0], vlo[N_][1], vlo[N_][2], vlo[N_][3],                      \
                      vhi[N_][0], vhi[N_][1], vhi[N_][2], vhi[N_][3]};                     \
    O[(N_) & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av),  \
                                                          PF_, O[(N_) & 1], 0, 0, 0);      \
  }
  V3_VREAD(0, 0)
  V3_VREAD(0, 1)
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    if (n + 2 < 4) V3_VREAD(0, n + 2)
    V3_PVMMA(n, pf[n >> 1])
    if (LM && (n & 1)) v3_lsum(L, pf[n >> 1]);
#pragma unroll
    for (int j = 4 * n; j < 4 * n + 4; ++j) {
      const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(SC[1][j], c2, nmc));
      if (!LM) l += e;
      pf[2 + (j >> 3)][j & 7] = (bf16)e;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  V3_VREAD(1, 0)
  V3_VREAD(1, 1)
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    if (n + 2 < 4) V3_VREAD(1, n + 2)
    V3_PVMMA(n, pf[2 + (n >> 1)])
    if (LM && (n & 1)) v3_lsum(L, pf[2 + (n >> 1)]);
  }
#undef V3_VREAD
#undef V3_PVMMA
}

}  // namespace

template <int D, bool CAUSAL, int NW, bool SCHED, bool LM>
__global__ __launch_bounds__(64 * NW, 2) void fa_fwd_bf16_v3(AttnArgs p, int nqb) {
  using C = V3<D, NW>;
  static_assert(D == 64, "v3 is the d = 64 kernel");
  static_assert(C::LPT >= 1 && C::LPT <= 4, "staging layout");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* smem = (bf16*)smem_raw;  // K[2][TILE], V[2][TILE]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;

  // XCD-aware bijective block remap (see fa_fwd_fast.hip).
  const int nblk = gridDim.x;
  const int hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3;
  const int qd = nblk >> 3, rm = nblk & 7;
  const int logical = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + slot;
  const int bh = logical / nqb;
  int qb = logical % nqb;
  if (CAUSAL) qb = nqb - 1 - qb;  // heaviest first
  const int b = bh / p.H, hh = bh % p.H;
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

  bf16x8 qf[C::KSTEPS];
  {
    const int qr = min(my_q, N - 1);
    const bf16* qrow = Qg + (int64_t)qr * p.sq[2];
#pragma unroll
    for (int ks = 0; ks < C::KSTEPS; ++ks) qf[ks] = *(const bf16x8*)(qrow + ks * 16 + 8 * hf);
  }

  Ctx c;
#pragma unroll
  for (int ks = 0; ks < C::KSTEPS; ++ks) c.koff[ks] = k_swz<D>(c32, 2 * ks + hf);
  {
    const int i16 = lane & 15, g = (lane >> 4) & 1;
#pragma unroll
    for (int db = 0; db < C::DB; ++db) {
      const int col = db * 32 + 16 * g + 4 * (i16 & 3);
      c.voff[db] = v_swz<D>(4 * hf + (i16 >> 2), col >> 3) + (col & 7);
    }
  }
  const int st_r = tid / C::CPR, st_c = tid % C::CPR;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = st_r + i * C::RSTEP;
    c.kgo[i] = (r * skn + st_c * 8) * 2;
    c.vgo[i] = (r * svn + st_c * 8) * 2;
    c.kso[i] = k_swz<D>(r, st_c);
    c.vso[i] = v_swz<D>(r, st_c);
  }
  const int ktile_b = kBK * skn * 2, vtile_b = kBK * svn * 2;
  bf16* const sK0 = smem;
  bf16* const sK1 = smem + C::TILE;
  bf16* const sV0 = smem + 2 * C::TILE;
  bf16* const sV1 = smem + 3 * C::TILE;

  f32x16 O[C::DB];
#pragma unroll
  for (int i = 0; i < C::DB; ++i) O[i] = f32x16{};
  float l_part = 0.f;  // this lane's share of the row sum (!LM)
  f32x16 L = f32x16{};  // row sum on the matrix pipe (LM)
  float m_run = -INFINITY;
  const float c2 = p.scale_log2;

  const int kend = CAUSAL ? min(N, q0 + C::kBQ) : N;
  const int ntiles = (kend + kBK - 1) / kBK;
  const int nfull = CAUSAL ? min(N / kBK, q0 / kBK) : N / kBK;  // mask-free tiles

  // Prologue: K(0), V(0) -> slot 0, K(1) -> slot 1; S(0).
  uint4 rK[4], rV[4];
  v3_load<D, NW>(rK, rk, c.kgo, 0);
  v3_load<D, NW>(rV, rv, c.vgo, 0);
  v3_store<D, NW>(sK0, rK, c.kso);
  v3_store<D, NW>(sV0, rV, c.vso);
  v3_load<D, NW>(rK, rk, c.kgo, ktile_b);  // tile 1 (zeros / unused when ntiles == 1)
  v3_store<D, NW>(sK1, rK, c.kso);
  __syncthreads();
  f32x16 SA[2], SB[2];
  v3_qk<D, NW, 0>(smem, c, qf, SA);
  __syncthreads();  // iteration 0 overwrites K slot 0, which every wave just read

  // Bulk iteration t (tile t and t+1 mask-free, QK(t+1) exists for every wave): staging
  // of K(t+2) / V(t+1) is unconditional (a K tile past the end is read from memory past
  // the causal bound or as zeros past N, and lands in a slot nobody reads).
#define V3_BULK(T_, SC_, SN_, KSN_, VS_)                                                   \
  {                                                                                        \
    v3_load<D, NW>(rK, rk, c.kgo, ((T_) + 2) * ktile_b);                                   \
    v3_load<D, NW>(rV, rv, c.vgo, ((T_) + 1) * vtile_b);                                   \
    const float nmc = v3_max<D>(SC_, O, l_part, L, m_run, c2);                                \
    if (SCHED) {                                                                           \
      v3_bulk<D, NW, KSN_, VS_, LM>(smem, c, qf, SC_, SN_, O, l_part, L, c2, nmc);                \
    } else {                                                                               \
      bf16x8 p0, p1, p2, p3;                                                               \
      v3_qk<D, NW, KSN_>(smem, c, qf, SN_);                                                \
      v3_exp<LM>(SC_[0], c2, nmc, p0, p1, l_part);                                         \
      v3_pv<D, NW, VS_, 0>(smem, c, p0, p1, O);                                            \
      v3_exp<LM>(SC_[1], c2, nmc, p2, p3, l_part);                                         \
      v3_pv<D, NW, VS_, 1>(smem, c, p2, p3, O);                                            \
      if (LM) { v3_lsum(L, p0); v3_lsum(L, p1); v3_lsum(L, p2); v3_lsum(L, p3); }          \
    }                                                                                      \
    v3_store<D, NW>((VS_) ? sK1 : sK0, rK, c.kso);                                         \
    v3_store<D, NW>((VS_) ? sV0 : sV1, rV, c.vso);                                         \
    __syncthreads();                                                                       \
  }

  int t = 0;
  for (; t + 2 < nfull; t += 2) {
    V3_BULK(t, SA, SB, 1, 0)
    V3_BULK(t + 1, SB, SA, 0, 1)
  }
#undef V3_BULK

  // General iterations (mask, causal per-wave skipping, end of the tile range): not
  // pipelined; S(t) arrives in SA (the bulk loop leaves on an even t) and QK(t+1) is
  // computed after PV(t) into SA again. LDS slots by runtime parity.
  for (; t < ntiles; ++t) {
    const int par = t & 1;
    const bool next = t + 1 < ntiles;
    if (t + 2 < ntiles) v3_load<D, NW>(rK, rk, c.kgo, (t + 2) * ktile_b);
    if (next) v3_load<D, NW>(rV, rv, c.vgo, (t + 1) * vtile_b);
    if (!CAUSAL || t * kBK <= wq_hi) {
      if (t >= nfull) v3_mask<D, CAUSAL>(SA, t * kBK, N, my_q, hf);
      const float nmc = v3_max<D>(SA, O, l_part, L, m_run, c2);
      bf16x8 p0, p1, p2, p3;
      v3_exp<LM>(SA[0], c2, nmc, p0, p1, l_part);
      v3_exp<LM>(SA[1], c2, nmc, p2, p3, l_part);
      if (LM) { v3_lsum(L, p0); v3_lsum(L, p1); v3_lsum(L, p2); v3_lsum(L, p3); }
      const bf16* sv = smem + (2 + par) * C::TILE;
      v3_pv<D, NW, 0, 0>(sv - 2 * C::TILE, c, p0, p1, O);
      v3_pv<D, NW, 0, 1>(sv - 2 * C::TILE, c, p2, p3, O);
    }
    if (next && (!CAUSAL || (t + 1) * kBK <= wq_hi))
      v3_qk<D, NW, 0>(smem + (par ^ 1) * C::TILE, c, qf, SA);
    if (t + 2 < ntiles) v3_store<D, NW>(par ? sK1 : sK0, rK, c.kso);
    if (next) v3_store<D, NW>(par ? sV0 : sV1, rV, c.vso);
    __syncthreads();
  }

  float l_tot;
  if (LM) {
    l_tot = L[0];
  } else {
    const auto lsw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_part), __float_as_uint(l_part),
                                                      false, false);
    l_tot = __uint_as_float(lsw[0]) + __uint_as_float(lsw[1]);
  }
  const float inv_l = 1.f / l_tot;
  if (my_q < N) {
    bf16* Og = (bf16*)p.out + b * p.so[0] + hh * p.so[1] + (int64_t)my_q * p.so[2];
#pragma unroll
    for (int db = 0; db < C::DB; ++db)
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
}

template <int D, bool CAUSAL, int NW, bool SCHED, bool LM>
static hipError_t launch_v3_t(const AttnArgs& a, hipStream_t st) {
  const size_t smem = 4 * (size_t)kBK * D * sizeof(bf16);
  auto kfn = fa_fwd_bf16_v3<D, CAUSAL, NW, SCHED, LM>;
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)smem);
  if (e != hipSuccess) return e;
  const int nqb = (a.N + 32 * NW - 1) / (32 * NW);
  const int64_t nblk = (int64_t)nqb * a.B * a.H;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kfn, dim3((unsigned)nblk), dim3(64 * NW), smem, st, a, nqb);
  return hipGetLastError();
}

// d = 64 only; every per-head K/V byte offset up to two tiles past N must fit the 31-bit
// buffer offset (the bulk loop stages one tile ahead of the last one it needs).
hipError_t launch_fwd_v3(const AttnArgs& a, bool causal, int variant, hipStream_t st,
                         bool* handled) {
  *handled = false;
  if (a.d != 64) return hipSuccess;
  const int64_t lim = (int64_t)1 << 31;
  if (((int64_t)a.N + 2 * kBK) * a.sk[2] * 2 >= lim || ((int64_t)a.N + 2 * kBK) * a.sv[2] * 2 >= lim)
    return hipSuccess;
  *handled = true;
#define V3_DISPATCH(NW_, SCHED_, LM_)                                                   \
  return causal ? launch_v3_t<64, true, NW_, SCHED_, LM_>(a, st)                       \
                : launch_v3_t<64, false, NW_, SCHED_, LM_>(a, st);
  switch (variant) {
    case 0: V3_DISPATCH(4, true, false)
    case 1: V3_DISPATCH(8, true, false)
    case 2: V3_DISPATCH(4, false, false)
    case 3: V3_DISPATCH(4, true, true)
    default: V3_DISPATCH(8, true, true)
  }
#undef V3_DISPATCH
}

}  // namespace mt
