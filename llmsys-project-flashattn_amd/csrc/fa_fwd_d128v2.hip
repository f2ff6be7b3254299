// FlashAttention forward, bf16, d = 128, non-causal, N % 64 == 0: the config-4 kernel on the
// 16x16x32 MFMA.
//
// fa_fwd_d128.hip runs d = 128 on v_mfma_f32_32x32x16_bf16 with register-staged K/V. At d =
// 128 a 64-key tile costs 64 16x16x32 MFMAs per 32-query wave against the same 32
// exponentials per lane as at d = 64, so the loop has issue slack, and the chip holds a
// ≈12-15 % higher clock on the 16x16x32 shape at equal cycles per FLOP (MI355X_MICROARCH.md,
// 'DVFS give-back' item 7; v6 at d = 64 spent that gain on issue, here there is room for it).
// What else changes against fa_fwd_d128.hip:
//  * K/V tiles arrive by LDS-DMA issued from inline asm (no staging registers, no ds_write,
//    no compiler vmcnt wait mid-tile), two slots each, one barrier per tile;
//  * the row sums run on the MFMA pipe (R += ones·Pᵀ after each P operand's first PV MFMA,
//    as v6's policy 102): no v_add per score;
//  * the softmax of one 64-key tile is spread evenly over the four 16-MFMA phases of the
//    next: P1 QKᵀ(t+1) keys 0-31 ‖ exp S(t) keys 32-47, P2 QKᵀ(t+1) keys 32-63 ‖ exp S(t)
//    keys 48-63, P3 PV(t) keys 0-31 ‖ exp S(t+1) keys 0-15, P4 PV(t) keys 32-63 ‖ exp
//    S(t+1) keys 16-31: 8 exponentials per phase, one every other MFMA slot.
// Same frozen first-tile reference, spike fallback (serial deferred-max recompute when a row
// sum leaves 2^64), XCD-aware block order and (O, m, l) contract as every forward kernel here
// (reference semantics: forward_kernel, src/flashattention_kernel.cu:9-112).
//
// Layouts (v6's, cdna_hip_programming.md §3, 16x16x32 bf16): lane l, g = l >> 4, i = l & 15.
//  * Sᵀ(16 keys x 16 queries) = K·Qᵀ: A = K rows (key 16kb + i, d 32ks + 8g ..), B = Q of
//    query 16qh + i (register resident, 4 k-steps), C: keys 16kb + 4g + r, query 16qh + i.
//  * Oᵀ(16 d x 16 queries) += Vᵀ·Pᵀ per 32-key half hv: B = the lane's keys 32hv + 4g + 0..3
//    and 32hv + 16 + 4g + 0..3 of query 16qh + i; A = Vᵀ of d 16db + i in the same key order
//    (two ds_read_b64_tr_b16). C: d 16db + 4g + r, query 16qh + i.
//  * K image (256-B rows): chunk c of row r at c ^ (r & 15) (fa_fwd_bf16.h): the 16 rows x
//    2 chunks of a ds_read_b128 lane group land on distinct banks.
//  * V image: chunk c of row r at c ^ ((r & 7) << 1): a half-wave's transposed read covers
//    rows 4g + 0..3 (g = 0, 1) x chunks {2db, 2db + 1} x two 8-B halves, 64 distinct banks.
#include "fa_fwd_bf16.h"

namespace mt {

namespace {

constexpr int D = 128;
constexpr int kBK = 64;
constexpr int TILE = kBK * D;           // elements of one K or V tile (16 KiB)
constexpr float kLimit = 1.8446744e19f; // 2^64
constexpr float kThr = 8.0f;

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

struct Sc {
  f32x4 s[4][2];  // scores of a 64-key tile: [16-key block kb][query half qh]
};
struct Pf {
  bf16x8 p[2];    // Pᵀ B operands of one 32-key half: [query half qh]
};

__device__ __forceinline__ int kswz(int r, int c) { return r * D + ((c ^ (r & 15)) << 3); }
__device__ __forceinline__ int vswz(int r, int c) { return r * D + ((c ^ ((r & 7) << 1)) << 3); }

__device__ __forceinline__ f32x4 mma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// K fragment of 16-key block kb, k-step ks (d 32ks + 8g ..)
__device__ __forceinline__ bf16x8 kread(const bf16* sk, const int (&ko)[4], int kb, int ks) {
  return *(const bf16x8*)(sk + kb * 16 * D + ko[ks]);
}
// Vᵀ fragment of key half hv, d block db
__device__ __forceinline__ bf16x8 vread(const bf16* sv, const int (&vo)[8], int hv, int db) {
  const bf16* a = sv + hv * 32 * D + vo[db];
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 16 * D));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Pair j (0..3) of 16-key block kb: query half j >> 1, rows 2(j & 1), 2(j & 1) + 1.
__device__ __forceinline__ f32x2 exp_pair(const Sc& s, int kb, int j, float c2, const float (&nmc)[2]) {
  const int qh = j >> 1, r0 = 2 * (j & 1);
  const float x0 = __builtin_fmaf(s.s[kb][qh][r0], c2, nmc[qh]);
  const float x1 = __builtin_fmaf(s.s[kb][qh][r0 + 1], c2, nmc[qh]);
  return f32x2{__builtin_amdgcn_exp2f(x0), __builtin_amdgcn_exp2f(x1)};
}
// Pack pair j of block kb into the P operand of its half (slots 4(kb & 1) + r0 ..); VS: and
// add it to the lane's row-sum shares acc (the VALU row-sum form).
template <bool VS = false>
__device__ __forceinline__ void fin_pair(const f32x2& e, int kb, int j, Pf& pf, f32x2* acc = nullptr) {
  const int qh = j >> 1, r0 = 2 * (j & 1);
  if (VS) acc[qh] += e;
  pf.p[qh][4 * (kb & 1) + r0] = (bf16)e[0];
  pf.p[qh][4 * (kb & 1) + r0 + 1] = (bf16)e[1];
}
// The softmax work of MFMA slot m (0..15) of a phase over 16-key block kb: the two
// exponentials of pair m / 4 in slot 4j, their pack in slot 4j + 2.
template <bool VS>
__device__ __forceinline__ void sm_slot(int m, const Sc& s, int kb, float c2, const float (&nmc)[2],
                                        Pf& pf, f32x2& ep, f32x2* acc) {
  if ((m & 3) == 0) ep = exp_pair(s, kb, m >> 2, c2, nmc);
  else if ((m & 3) == 2) fin_pair<VS>(ep, kb, m >> 2, pf, acc);
}

// QKᵀ phase over 16-key blocks kb0, kb0 + 1 of the tile at sk into S (16 MFMAs: fragment f =
// m >> 1 = (block, k-step), query half m & 1), beside the softmax of block skb of s_in.
template <bool SOFT, bool VS = false, int AH = 2>
__device__ __forceinline__ void qk_phase(const bf16* sk, const int (&ko)[4], const bf16x8 (&qf)[2][4],
                                         Sc& S, int kb0, const Sc& s_in, int skb, float c2,
                                         const float (&nmc)[2], Pf& pf, f32x2* acc = nullptr) {
  bf16x8 kf[8];
#pragma unroll
  for (int f = 0; f < AH; ++f) kf[f] = kread(sk, ko, kb0 + (f >> 2), f & 3);
  f32x2 ep;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int f = m >> 1, kb = kb0 + (f >> 2), ks = f & 3, qh = m & 1;
    if (!(m & 1) && f + AH < 8) kf[f + AH] = kread(sk, ko, kb0 + ((f + AH) >> 2), (f + AH) & 3);
    S.s[kb][qh] = mma16(kf[f], qf[qh][ks], ks ? S.s[kb][qh] : f32x4{});
    if (SOFT) sm_slot<VS>(m, s_in, skb, c2, nmc, pf, ep, acc);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// PV phase of key half hv of the tile at sv with P operand pp (16 MFMAs: Vᵀ fragment f = m >> 1
// = d block, query half m & 1; plus, unless VS, the two row-sum MFMAs R[qh] += ones·Pᵀ),
// beside the softmax of block skb of s_in.
template <bool SOFT, bool VS = false, int AH = 2>
__device__ __forceinline__ void pv_phase(const bf16* sv, const int (&vo)[8], f32x4 (&O)[8][2], const Pf& pp,
                                         int hv, f32x4 (&R)[2], const Sc& s_in, int skb, float c2,
                                         const float (&nmc)[2], Pf& pf, f32x2* acc = nullptr) {
  const bf16x8 ones = __builtin_bit_cast(bf16x8, s16x8{0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80});
  bf16x8 vf[8];
#pragma unroll
  for (int f = 0; f < AH; ++f) vf[f] = vread(sv, vo, hv, f);
  f32x2 ep;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int db = m >> 1, qh = m & 1;
    if (!(m & 1) && db + AH < 8) vf[db + AH] = vread(sv, vo, hv, db + AH);
    O[db][qh] = mma16(vf[db], pp.p[qh], O[db][qh]);
    if (!VS && db == 0) R[qh] = mma16(ones, pp.p[qh], R[qh]);
    if (SOFT) sm_slot<VS>(m, s_in, skb, c2, nmc, pf, ep, acc);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// max over the four lanes that share a query (i, i + 16, i + 32, i + 48)
__device__ __forceinline__ float quad_max(float x) {
  x = fmaxf(x, __shfl_xor(x, 16));
  return fmaxf(x, __shfl_xor(x, 32));
}
__device__ __forceinline__ float quad_sum(float x) {
  x += __shfl_xor(x, 16);
  return x + __shfl_xor(x, 32);
}
__device__ __forceinline__ float lane_max(const Sc& s, int qh) {
  float m = fmaxf(fmaxf(s.s[0][qh][0], s.s[0][qh][1]), s.s[0][qh][2]);
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = (kb ? 0 : 3); r < 4; ++r) m = fmaxf(m, s.s[kb][qh][r]);
  return m;
}

// LDS-DMA of 64 x 16 B to the LDS byte address lds (wave-uniform), from inline asm so that
// hipcc's waitcnt pass puts no vmcnt wait on it inside the tile (fa_fwd_v6.hip, dma6).
__device__ __forceinline__ void dma(uint32_t lds, __amdgpu_buffer_rsrc_t rs, int go, int step) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(go + step), "s"(lds), "s"(rs)
      : "memory");
}

}  // namespace

// grid: ceil(N / (32 NW)) query blocks x B·H, XCD-aware order; 64 NW threads; 64 KiB LDS
// (K slots 0, 1 then V slots 0, 1). NW = 8: one workgroup per CU; NW = 4: two (the two waves
// of a SIMD from different workgroups, not tied to one barrier). VAR 1: row sums by VALU adds
// instead of MFMAs; VAR 2: s_setprio 1 for the second half of the waves (MI355X_MICROARCH.md,
// 'Two waves per SIMD' item 4); VAR 4 / 8: operand fragments read 3 / 4 fragments (6 / 8
// MFMAs) ahead instead of 2; VAR 32: causal, a workgroup runs query block u (light) and then
// nqb - 1 - u (heavy) of one head, as v6's causal form.
template <int NW, int VAR>
__global__ __launch_bounds__(64 * NW, 8 / NW) void fa_fwd_bf16_d128v2(AttnArgs p, int nqb) {
  constexpr int kBQ = 32 * NW;
  constexpr int LPT = TILE * 2 / 1024 / NW;  // 1-KiB LDS-DMA pieces per wave per tile and tensor
  constexpr bool VS = VAR & 1, CAUSAL = VAR & 32;
  // VAR 128 (diagnostics, timing only, may read stale tiles): no staging wait before the tile
  // barrier (what the DMA latency costs); VAR 256 (the same, racy): no tile barrier
  constexpr int AH = (VAR & 4) ? 3 : (VAR & 8) ? 4 : 2;  // operand fragments read ahead
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* const sK = (bf16*)smem_raw;  // [2][TILE]
  bf16* const sV = sK + 2 * TILE;    // [2][TILE]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  const int N = p.N;

  const int nblk = gridDim.x, hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3, qd = nblk >> 3, rm = nblk & 7;
  const int logical = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + slot;
  const int nunit = CAUSAL ? (nqb + 1) / 2 : nqb;  // causal: light / heavy block pairs
  const int bh = logical / nunit, qb = logical % nunit;
  const int b = bh / p.H, hh = bh % p.H;

  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Kg = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1];
  const bf16* Vg = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1];
  const int skn = (int)p.sk[2], svn = (int)p.sv[2];
  const __amdgpu_buffer_rsrc_t rk =
      __builtin_amdgcn_make_buffer_rsrc((void*)Kg, (short)0, ((N - 1) * skn + D) * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv =
      __builtin_amdgcn_make_buffer_rsrc((void*)Vg, (short)0, ((N - 1) * svn + D) * 2, 0x00020000);

  int ko[4], vo[8];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) ko[ks] = kswz(i16, 4 * ks + g);
  {
    const int q = i16 >> 2, pp = i16 & 3, row = 4 * g + q;
#pragma unroll
    for (int db = 0; db < 8; ++db) vo[db] = vswz(row, 2 * db + (pp >> 1)) + 4 * (pp & 1);
  }
  // LDS-DMA: piece i of wave w fills rows 4 (LPT w + i) .. + 3 of a tile in lane order; lane l
  // fetches the source chunk the swizzle puts at chunk l % 16 of row 4 (LPT w + i) + l / 16
  int kdo[LPT], vdo[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    const int dr = 4 * (LPT * wave + i) + (lane >> 4), dc = lane & 15;
    kdo[i] = (dr * skn + ((dc ^ (dr & 15)) << 3)) * 2;
    vdo[i] = (dr * svn + ((dc ^ ((dr & 7) << 1)) << 3)) * 2;
  }
  const int ktile_b = kBK * skn * 2, vtile_b = kBK * svn * 2;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem_raw);
  auto dma_k = [&](int s, int step) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < LPT; ++i)
      dma(lds0 + (uint32_t)(s * TILE + 4 * (LPT * wave + i) * D) * 2, rk, kdo[i], step);
  };
  auto dma_v = [&](int s, int step) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < LPT; ++i)
      dma(lds0 + (uint32_t)((2 + s) * TILE + 4 * (LPT * wave + i) * D) * 2, rv, vdo[i], step);
  };
  const float c2 = p.scale_log2;
  if ((VAR & 2) && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);

  const int ntiles_all = N / kBK;

  // One query block [q0, q0 + kBQ) of head bh. Causal: wave w's queries qw .. qw + 31 see the
  // keys up to their own, so it computes tiles 0 .. tD = qw / 64 (the last one masked in
  // registers); the workgroup stages the tiles its last wave needs, and a wave that is done
  // keeps staging its share and joins every barrier (fa_fwd_v6.hip's causal scheme).
  auto run_block = [&](const int q0) __attribute__((always_inline)) {
  const int qw = q0 + wave * 32;  // this wave's first query
  bf16x8 qf[2][4];                // [qh][ks]
#pragma unroll
  for (int qh = 0; qh < 2; ++qh) {
    const bf16* qr = Qg + (int64_t)min(qw + 16 * qh + i16, N - 1) * p.sq[2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[qh][ks] = *(const bf16x8*)(qr + 32 * ks + 8 * g);
  }
  const int ntiles = CAUSAL ? min(N, q0 + kBQ) / kBK : ntiles_all;  // tiles the workgroup stages
  const int tD = qw / kBK;
  const int nbulk = CAUSAL ? (qw < N ? tD + 1 : 0) : ntiles;      // tiles this wave computes
  // causal: key 16 kb + 4 g + r of the wave's diagonal tile tD is after query 16 qh + i of the
  // wave when 64 tD + 16 kb + 4 g + r > qw + 16 qh + i
  auto mask_diag = [&](Sc& S) __attribute__((always_inline)) {
    const int off = kBK * tD - qw;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (off + 16 * kb + 4 * g + r > 16 * qh + i16) S.s[kb][qh][r] = -INFINITY;
  };

  f32x4 O[8][2];
  auto zero_o = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int db = 0; db < 8; ++db) { O[db][0] = f32x4{}; O[db][1] = f32x4{}; }
  };
  zero_o();
  float m[2] = {0.f, 0.f}, l[2] = {0.f, 0.f};

  // ---- pass 0: the pipelined loop with the frozen first-tile reference ------------------
  dma_k(0, 0);
  dma_v(0, 0);
  dma_k(1, ktile_b);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  Sc SA, SB;
  Pf dpf, pl0, pl1, ph;
  if (nbulk >= 1) {
    const float z[2] = {0.f, 0.f};
    qk_phase<false>(sK, ko, qf, SA, 0, SA, 0, c2, z, dpf);
    qk_phase<false>(sK, ko, qf, SA, 2, SA, 0, c2, z, dpf);
  }
  __syncthreads();  // every wave is done with K slot 0 (iteration 0 stages K(2) into it)
  if (nbulk >= 1) {
    if (CAUSAL && tD == 0) mask_diag(SA);  // tile 0 is the wave's diagonal: the reference over visible keys
    float nmc[2];
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      m[qh] = quad_max(lane_max(SA, qh));
      nmc[qh] = -(m[qh] * c2);
    }
    f32x4 R[2] = {f32x4{}, f32x4{}};
    f32x2 acc[2] = {f32x2{0.f, 0.f}, f32x2{0.f, 0.f}};  // VS: the lane's row-sum shares
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      fin_pair<VS>(exp_pair(SA, 0, j, c2, nmc), 0, j, pl0, acc);
      fin_pair<VS>(exp_pair(SA, 1, j, c2, nmc), 1, j, pl0, acc);
    }

    // iteration t: S(t) in SC with P(t) keys 0-31 in PC; K(t + 1) in slot (t + 1) & 1, V(t) in
    // slot t & 1; stages K(t + 2) into slot t & 1 and V(t + 1) into slot (t + 1) & 1. MASK:
    // S(t + 1) is the wave's diagonal tile, masked before its first exponentials (P3).
    auto iter = [&](int t, int par, const Sc& SC, Sc& SN, const Pf& PC, Pf& PN, bool mask) __attribute__((always_inline)) {
      __builtin_amdgcn_sched_barrier(0);
      dma_k(par, (t + 2) * ktile_b);
      dma_v(par ^ 1, (t + 1) * vtile_b);
      const bf16* skn_ = sK + (par ^ 1) * TILE;
      const bf16* svc = sV + par * TILE;
      qk_phase<true, VS, AH>(skn_, ko, qf, SN, 0, SC, 2, c2, nmc, ph, acc);    // P1
      qk_phase<true, VS, AH>(skn_, ko, qf, SN, 2, SC, 3, c2, nmc, ph, acc);    // P2
      if (CAUSAL && mask) mask_diag(SN);
      pv_phase<true, VS, AH>(svc, vo, O, PC, 0, R, SN, 0, c2, nmc, PN, acc);   // P3
      pv_phase<true, VS, AH>(svc, vo, O, ph, 1, R, SN, 1, c2, nmc, PN, acc);   // P4
      if (!(VAR & 128)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (!(VAR & 256)) __syncthreads();
    };
    // iterations 0 .. nbulk - 2 (causal: the last computes QKᵀ of the diagonal tile)
    const int L = nbulk - 1, Lu = CAUSAL ? L - 1 : L;
    int t = 0;
    for (; t + 2 <= Lu; t += 2) {
      iter(t, 0, SA, SB, pl0, pl1, false);
      iter(t + 1, 1, SB, SA, pl1, pl0, false);
    }
    if (t < Lu) {
      iter(t, 0, SA, SB, pl0, pl1, false);
      ++t;
      SA = SB;
      pl0 = pl1;
    }
    if (CAUSAL && t < L) {  // runtime slot parity
      iter(t, t & 1, SA, SB, pl0, pl1, true);
      ++t;
      SA = SB;
      pl0 = pl1;
    }
    {  // the last tile t: S(t) in SA, P(t) keys 0-31 in pl0, V(t) in slot t & 1
      const bf16* svc = sV + (t & 1) * TILE;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        fin_pair<VS>(exp_pair(SA, 2, j, c2, nmc), 2, j, ph, acc);
        fin_pair<VS>(exp_pair(SA, 3, j, c2, nmc), 3, j, ph, acc);
      }
      pv_phase<false, VS>(svc, vo, O, pl0, 0, R, SA, 0, c2, nmc, dpf);
      pv_phase<false, VS>(svc, vo, O, ph, 1, R, SA, 0, c2, nmc, dpf);
    }
    if (VS) {
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) R[qh][0] = quad_sum(acc[qh][0] + acc[qh][1]);
    }
    // every lane of a query's column group holds its whole row sum
    l[0] = R[0][0];
    l[1] = R[1][0];
  }
  if (CAUSAL) {
    // tail: this wave's share of the staging of the tiles the other waves still need
    for (int t = nbulk > 0 ? nbulk - 1 : 0; t + 1 < ntiles; ++t) {
      dma_k(t & 1, (t + 2) * ktile_b);
      dma_v((t + 1) & 1, (t + 1) * vtile_b);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  // ---- serial path: every tile again with the per-tile deferred-max bookkeeping, when a
  // row sum left 2^64 (the workgroup starts over) ----------------------------------------
  const bool bad = nbulk > 0 && (!(l[0] <= kLimit) || !(l[1] <= kLimit));
  if (__syncthreads_or(bad)) {
    zero_o();
    f32x2 acc[2] = {f32x2{0.f, 0.f}, f32x2{0.f, 0.f}};
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) m[qh] = -INFINITY;
    for (int t = 0; t < ntiles; ++t) {
      __syncthreads();  // every wave is done with the previous tile
      dma_k(0, t * ktile_b);
      dma_v(0, t * vtile_b);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t >= nbulk) continue;  // causal: past this wave's diagonal (or its queries past N)
      Sc S;
      Pf plo, phi, dpf2;
      const float z[2] = {0.f, 0.f};
      qk_phase<false>(sK, ko, qf, S, 0, S, 0, c2, z, dpf2);
      qk_phase<false>(sK, ko, qf, S, 2, S, 0, c2, z, dpf2);
      if (CAUSAL && t == tD) mask_diag(S);
      float nmc[2];
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        const float tmax = quad_max(lane_max(S, qh));
        if (__builtin_amdgcn_ballot_w64((tmax - m[qh]) * c2 > kThr)) {
          const float m_new = fmaxf(m[qh], tmax);
          const float alpha = m[qh] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m[qh] - m_new) * c2);
          m[qh] = m_new;
#pragma unroll
          for (int db = 0; db < 8; ++db) O[db][qh] *= alpha;
          acc[qh] *= alpha;
        }
        nmc[qh] = -(m[qh] * c2);
      }
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x2 e = exp_pair(S, kb, j, c2, nmc);
          acc[j >> 1] += e;
          fin_pair(e, kb, j, kb < 2 ? plo : phi);
        }
      f32x4 dR[2] = {f32x4{}, f32x4{}};
      pv_phase<false>(sV, vo, O, plo, 0, dR, S, 0, c2, nmc, dpf2);
      pv_phase<false>(sV, vo, O, phi, 1, dR, S, 0, c2, nmc, dpf2);
    }
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) l[qh] = quad_sum(acc[qh][0] + acc[qh][1]);
  }

  // ---- epilogue ------------------------------------------------------------------------
#pragma unroll
  for (int qh = 0; qh < 2; ++qh) {
    const int q = qw + 16 * qh + i16;
    const float inv = 1.f / l[qh];
    if (q < N) {
      const ORow Og = o_row(p, b, hh, q);
#pragma unroll
      for (int db = 0; db < 8; ++db)
        store4(Og, 16 * db + 4 * g, O[db][qh][0] * inv, O[db][qh][1] * inv, O[db][qh][2] * inv,
               O[db][qh][3] * inv);
      if (g == 0) {
        const int64_t row = (int64_t)bh * N + q;
        if (p.m) p.m[row] = m[qh] * p.scale;
        if (p.l) p.l[row] = l[qh];
      }
    }
  }
  };  // run_block

  if (CAUSAL) {  // the light query block first, then the heavy one of the same head
    const int heavy = nqb - 1 - qb;
    run_block(qb * kBQ);
    if (heavy != qb) {
      __syncthreads();  // every wave is done with the light block's LDS tiles
      run_block(heavy * kBQ);
    }
  } else {
    run_block(qb * kBQ);
  }
}

template <int NW, int VAR>
static hipError_t launch_v2_t(const AttnArgs& a, hipStream_t st) {
  const size_t smem = 4 * (size_t)TILE * sizeof(bf16);
  auto kfn = fa_fwd_bf16_d128v2<NW, VAR>;
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  const int nqb = (a.N + 32 * NW - 1) / (32 * NW);
  const int64_t nblk = (int64_t)((VAR & 32) ? (nqb + 1) / 2 : nqb) * a.B * a.H;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kfn, dim3((unsigned)nblk), dim3(64 * NW), smem, st, a, nqb);
  return hipGetLastError();
}

// d = 128, non-causal, N % 64 == 0, N >= 128, every per-head K/V byte offset up to two tiles
// past N inside the 31-bit buffer range. var: bit 4 = 4 waves (two workgroups per CU), bits
// 0-1 the kernel's VAR.
hipError_t launch_fwd_d128v2(const AttnArgs& a, bool causal, int var, hipStream_t st, bool* handled) {
  *handled = false;
  if (causal != ((var & 32) != 0) || a.d != D || a.N % kBK != 0 || a.N < 2 * kBK) return hipSuccess;
  const int64_t lim = (int64_t)1 << 31;
  if (((int64_t)a.N + 2 * kBK) * a.sk[2] * 2 >= lim || ((int64_t)a.N + 2 * kBK) * a.sv[2] * 2 >= lim)
    return hipSuccess;
  *handled = true;
  switch (var) {  // product build: the defaults 0 / 32; the rest are A/B policies
    case 0: return launch_v2_t<8, 0>(a, st);
    case 32: return launch_v2_t<8, 32>(a, st);
#ifdef MT_DIAGNOSTICS
    case 1: return launch_v2_t<8, 1>(a, st);
    case 2: return launch_v2_t<8, 2>(a, st);
    case 16: return launch_v2_t<4, 0>(a, st);
    case 17: return launch_v2_t<4, 1>(a, st);
    case 4: return launch_v2_t<8, 4>(a, st);
    case 8: return launch_v2_t<8, 8>(a, st);
    case 128: return launch_v2_t<8, 128>(a, st);
    case 256: return launch_v2_t<8, 256>(a, st);
#endif
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mt
