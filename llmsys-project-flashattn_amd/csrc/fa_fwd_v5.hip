// FlashAttention forward, bf16 MFMA kernel v5 (d = 64, N % 64 == 0): two 32-query blocks
// per wave, skewed by half a tile. Causal: a workgroup takes a light and a heavy query block
// of one head in turn; each wave runs the pipelined loop over the key tiles up to its own
// diagonal tile (the peeled last tile, masked), then keeps staging and joining barriers for
// the waves whose diagonal lies further on.
//
// v4 gives each wave one 32-query block and relies on the second wave of its SIMD to
// overlap one wave's softmax with the other's MFMAs. v5 gives each wave two blocks, A and
// B, and interleaves them inside the wave's own instruction stream: block B runs half a
// tile behind block A, so every phase pairs 8 MFMAs of one block with the softmax of a
// 32-key half of the other:
//     P1: Sᵀ_A(t)   = K(t)·Q_Aᵀ        ‖ softmax B(t), keys 32-63
//     P2: Oᵀ_B     += Vᵀ(t)·P_Bᵀ(t)    ‖ softmax A(t), keys 0-31
//     P3: Sᵀ_B(t+1) = K(t+1)·Q_Bᵀ      ‖ softmax A(t), keys 32-63
//     P4: Oᵀ_A     += Vᵀ(t)·P_Aᵀ(t)    ‖ softmax B(t+1), keys 0-31
// Each phase is 8 x [MFMA, two scores' pk_fma / 2 exp / pk_add / cvt], fenced with
// sched_barrier(0). Only S_B(t+1)'s upper half and P_B(t+1)'s lower half cross an
// iteration, so a wave holds 64 queries in about the registers v4 needs for 32 and still
// runs two waves per SIMD. K uses a 4-slot LDS ring (an iteration reads K(t) and K(t+1)
// and writes K(t+2)), V a 2-slot ring; one barrier per iteration.
// Softmax: v4's frozen first-tile reference (row max of tile 0 per block); a lane whose
// row-sum share leaves 2^64 sends its workgroup through a serial deferred-max recompute.
#include <type_traits>

#include "fa_fwd_bf16.h"

namespace mt {

namespace {

using namespace fwdbf16;
constexpr int D = 64;
constexpr int kBK = 64;
constexpr int TILE = kBK * D;              // elements per K or V tile
constexpr int kKSlots = 4, kVSlots = 2;
template <int NW>
constexpr int lpt() { return kBK * (D / 8) / (64 * NW); }  // 16-B staging chunks per thread per tile
constexpr float kLimit = 1.8446744e19f;   // 2^64
constexpr float kThr = 8.0f;

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(2))) float f32x2;

template <int LPT>
struct Ctx5 {
  int koff[4];  // per-lane K row-image offsets per k-step (slot 0, key block 0)
  int voff[2];  // per-lane Vᵀ transpose-read offsets per d block (slot 0, row block 0)
  int kgo[LPT], vgo[LPT], kso[LPT], vso[LPT];
  int kdo[LPT], vdo[LPT];  // LDS-DMA per-lane source offsets (rows R0(i) + lane / 8)
};

// Softmax of one 32-key half of a block: pair i (0..7) of the 16 scores of S_half.
// VAR bit 1 (diagnostic timing builds only, wrong results): no scale-and-shift.
// (A v_dot2c_f32_bf16 row sum of the bf16-rounded pair was tried as VAR bit 0: slower,
// 962 vs 978 TF/s, and it failed the 150x spike test; removed.)
// VAR bit 2: the tile loop unrolled by 4 (see iter in the kernel).
// VAR bit 1024: K/V staged by LDS-DMA (dma5) instead of through registers.
// Diagnostic ablation bits (timing only, wrong results; policies 80-86): 8 no K/V staging,
// 16 no barrier either, 64 no Vᵀ operand reads, 128 no exponential, 256 no row-sum add.
// (Replacing the K operand reads with Q fragments is not a valid ablation: the QKᵀ
// products become loop-invariant and the compiler hoists them out of the loop.)
// VAR bit 8192: single-issue f32 VALU only (v_fma_f32 / v_add_f32 pinned by inline asm, so
// neither SLP nor the vector types form v_pk_fma_f32 / v_pk_add_f32 beside the MFMAs).
__device__ __forceinline__ float fma1(float a, float b, float c) {
  float r;
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float add1(float a, float b) {
  float r;
  asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// VAR bit 262144 (RS): the row sums come from the MFMA pipe (phase_pv), not from VALU adds.
template <int VAR>
__device__ __forceinline__ void sm_pair(const f32x16& s, int i, float c2, float nmc, f32x2& acc,
                                        bf16x8 (&pf)[2]) {
  constexpr bool RS = (VAR & 262144) != 0;
  const int j = 2 * i;
  if (VAR & 8192) {
    const float e0 = __builtin_amdgcn_exp2f(__builtin_fmaf(s[j], c2, nmc));
    const float e1 = __builtin_amdgcn_exp2f(__builtin_fmaf(s[j + 1], c2, nmc));
    acc[0] += e0;
    acc[1] += e1;
    pf[j >> 3][j & 7] = (bf16)e0;
    pf[j >> 3][(j & 7) + 1] = (bf16)e1;
    return;
  }
  f32x2 x;
  if (VAR & 2)
    x = f32x2{s[j], s[j + 1]};
  else
    x = f32x2{s[j], s[j + 1]} * f32x2{c2, c2} + f32x2{nmc, nmc};
  const float e0 = (VAR & 128) ? x[0] : __builtin_amdgcn_exp2f(x[0]);
  const float e1 = (VAR & 128) ? x[1] : __builtin_amdgcn_exp2f(x[1]);
  if (!(VAR & 256) && !RS) acc += f32x2{e0, e1};
  pf[j >> 3][j & 7] = (bf16)e0;
  pf[j >> 3][(j & 7) + 1] = (bf16)e1;
}

// VAR bit 65536: the softmax of pair i is split in two: its scale-and-shift and
// exponentials in MFMA slot i, its row-sum add and bf16 pack in slot i + 1 (the last pair's
// after the phase's last MFMA). A v_exp_f32 result read by the very next VALU instruction
// costs an s_nop (trans-use hazard); one slot of distance removes it.
__device__ __forceinline__ f32x2 sm_exp(const f32x16& s, int i, float c2, float nmc) {
  const f32x2 x = f32x2{s[2 * i], s[2 * i + 1]} * f32x2{c2, c2} + f32x2{nmc, nmc};
  return f32x2{__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
}
template <bool RS = false>
__device__ __forceinline__ void sm_fin(const f32x2& e, int i, f32x2& acc, bf16x8 (&pf)[2]) {
  const int j = 2 * i;
  if (!RS) acc += e;
  pf[j >> 3][j & 7] = (bf16)e[0];
  pf[j >> 3][(j & 7) + 1] = (bf16)e[1];
}

// VAR bit 1048576 (diagnostic timing builds only, wrong results): every 32x32x16 MFMA of the
// two phases replaced by two 16x16x32 MFMAs of the same MACs on half of the accumulator, to
// price the MFMA shape (MI355X_MICROARCH.md 'DVFS give-back' item 7) under this kernel's
// VALU and LDS load; the softmax then reads stale registers.
template <int VAR>
__device__ __forceinline__ f32x16 mfma_sh(const bf16x8& a, const bf16x8& b, const f32x16& c) {
#ifdef MT_DIAGNOSTICS
  if (VAR & 1048576) {
    typedef __attribute__((ext_vector_type(4))) float f32x4;
    f32x4 lo = {c[0], c[1], c[2], c[3]}, hi = {c[4], c[5], c[6], c[7]};
    lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, lo, 0, 0, 0);
    hi = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, hi, 0, 0, 0);
    f32x16 r = c;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
#endif
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 kread(const bf16* sk, const int (&ko)[4], int i) {
  // MFMA i of a QKᵀ phase: key block i/4, k-step i%4 (block 0's chain completes first)
  return *(const bf16x8*)(sk + (i >> 2) * 32 * D + ko[i & 3]);
}

__device__ __forceinline__ bf16x8 vread(const bf16* sv, const int (&vo)[2], int n) {
  // MFMA n of a PV phase: key block n/4, 16-key step (n/2)%2, d block n%2
  const bf16* a1 = sv + ((n >> 2) * 32 + 16 * ((n >> 1) & 1)) * D + vo[n & 1];
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1 + 8 * D));
  const s16x8 av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, av);
}

// QKᵀ phase (8 MFMAs into S) interleaved with the softmax of s_in (8 pairs) -> pf.
// SOFT = false: MFMAs only.
template <bool SOFT, int kAhead, int VAR>
__device__ __forceinline__ void phase_qk(const bf16* sk, const int (&ko)[4], const bf16x8 (&qf)[4],
                                         f32x16 (&S)[2], const f32x16& s_in, float c2, float nmc,
                                         f32x2& acc, bf16x8 (&pf)[2]) {
  bf16x8 kf[8];
  f32x2 ep;
#pragma unroll
  for (int i = 0; i < kAhead; ++i) kf[i] = kread(sk, ko, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i + kAhead < 8) kf[i + kAhead] = kread(sk, ko, i + kAhead);
    S[i >> 2] = mfma_sh<VAR>(kf[i], qf[i & 3], (i & 3) ? S[i >> 2] : f32x16{});
    if (SOFT && (VAR & 65536)) {
      const f32x2 e = sm_exp(s_in, i, c2, nmc);
      if (i) sm_fin<(VAR & 262144) != 0>(ep, i - 1, acc, pf);
      ep = e;
    } else if (SOFT) {
      sm_pair<VAR>(s_in, i, c2, nmc, acc, pf);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (SOFT && (VAR & 65536)) sm_fin<(VAR & 262144) != 0>(ep, 7, acc, pf);
}

// PV phase (8 MFMAs into O with P fragments p_lo (keys 0-31) and p_hi (keys 32-63))
// interleaved with the softmax of s_in (8 pairs) -> pf.
// KEEP (VAR bit 32768): 1 = read the Vᵀ fragments and leave them in vk, 2 = take them from
// vk (P2 and P4 of an iteration multiply the same V(t): the second phase reads no LDS).
// RS (VAR bit 262144): R += ones·Pᵀ after each P fragment's second PV MFMA (every row of
// the 32 x 32 R tile is the running row sum of the block's queries, lane = query), so the
// softmax issues no row-sum adds; R must be given (R_ON) wherever P fragments are consumed.
template <bool SOFT, int kAhead, int VAR, int KEEP = 0>
__device__ __forceinline__ void phase_pv(const bf16* sv, const int (&vo)[2], f32x16 (&O)[2],
                                         const bf16x8 (&p_lo)[2], const bf16x8 (&p_hi)[2],
                                         const f32x16& s_in, float c2, float nmc, f32x2& acc,
                                         bf16x8 (&pf)[2], bf16x8 (&vk)[8], f32x16* R = nullptr) {
  constexpr bool RS = (VAR & 262144) != 0;
  typedef __attribute__((ext_vector_type(8))) short s16x8o;
  const bf16x8 ones = __builtin_bit_cast(bf16x8, s16x8o{0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80});
  bf16x8 vf_own[8];
  f32x2 ep;
  bf16x8 (&vf)[8] = KEEP ? vk : vf_own;
  if (KEEP != 2) {
#pragma unroll
    for (int n = 0; n < kAhead; ++n) vf[n] = (VAR & 64) ? p_lo[n & 1] : vread(sv, vo, n);
  }
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    if (KEEP != 2 && n + kAhead < 8) vf[n + kAhead] = (VAR & 64) ? p_hi[n & 1] : vread(sv, vo, n + kAhead);
    const bf16x8& p = (n >> 2) ? p_hi[(n >> 1) & 1] : p_lo[(n >> 1) & 1];
    O[n & 1] = mfma_sh<VAR>(vf[n], p, O[n & 1]);
    if (RS && (n & 1)) *R = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, p, *R, 0, 0, 0);
    if (SOFT && (VAR & 65536)) {
      const f32x2 e = sm_exp(s_in, n, c2, nmc);
      if (n) sm_fin<RS>(ep, n - 1, acc, pf);
      ep = e;
    } else if (SOFT) {
      sm_pair<VAR>(s_in, n, c2, nmc, acc, pf);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (SOFT && (VAR & 65536)) sm_fin<RS>(ep, 7, acc, pf);
}

template <int LPT>
__device__ __forceinline__ void load5(uint4 (&r)[LPT], __amdgpu_buffer_rsrc_t rs, const int (&go)[LPT],
                                      int step) {
#pragma unroll
  for (int i = 0; i < LPT; ++i)
    r[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, go[i] + step, 0, 0));
}

template <int LPT>
__device__ __forceinline__ void store5(bf16* dst, const uint4 (&r)[LPT], const int (&so)[LPT]) {
#pragma unroll
  for (int i = 0; i < LPT; ++i) *(uint4*)(dst + so[i]) = r[i];
}

// LDS-DMA staging (VAR bit 1024): buffer_load_dwordx4 ... lds writes each lane's 16 B at
// (wave-uniform base + lane * 16), so a wave instruction fills 8 consecutive 128-B rows of
// the image in lane order; the swizzle moves to the per-lane global source (lane l of
// rows R0..R0+7 fetches chunk (l % 8) ^ swz(row) of row R0 + l / 8). No VGPRs hold the
// tile and there are no ds_write instructions. dst: the slot image + R0 rows.
// VAR bit 524288: the same instruction from inline asm. hipcc tracks builtin LDS-DMA as an
// LDS store of unknown address and puts an s_waitcnt vmcnt(0) before the first Vᵀ read of
// every tile (the DMA then has to land within P1); the asm form is invisible to its waitcnt
// pass, and the explicit vmcnt(0) before each tile barrier is the only wait. M0 is
// compiler-reserved: saved and restored inside the statement (cdna_hip_programming.md §5.7).
template <int VAR>
__device__ __forceinline__ void dma5(bf16* dst_rows, __amdgpu_buffer_rsrc_t rs, int go, int step) {
  if (VAR & 524288) {
    const unsigned lds = __builtin_amdgcn_readfirstlane(
        (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)dst_rows);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(go + step), "s"(lds), "s"(rs)
        : "memory");
  } else {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst_rows, 16,
                                             go + step, 0, 0, 0);
  }
}

__device__ __forceinline__ float lane_pair_sum(float x) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
}

}  // namespace

// AHEAD: LDS operand reads are issued this many MFMAs ahead of their use. VAR: see sm_pair.
template <int AHEAD, int VAR, bool CAUSAL, int NW = 4>
__global__ __launch_bounds__(64 * NW, 8 / NW) void fa_fwd_bf16_v5(AttnArgs p, int nqb) {
#ifndef MT_DIAGNOSTICS
  static_assert((VAR & (2 | 8 | 16 | 64 | 128 | 256 | 1048576)) == 0,
                "wrong-result ablation variants exist only in the MT_DIAGNOSTICS build");
#endif
  // VAR bit 131072 (8 waves, non-causal, LDS-DMA): split keys inside the workgroup. Waves
  // 0-3 and 4-7 take the same 256 queries (wave w and w + 4 the same 64) over the first and
  // the second half of the keys, each half with its own K/V rings and its own share of the
  // staging, both under the same barriers; at the end the second half hands (m, l, O) to the
  // first through LDS, which merges the two and stores. A grid of B·H·N / 256 workgroups
  // then runs two waves per SIMD where the unsplit 8-wave form has fewer workgroups than CUs.
  constexpr bool SPLIT = (VAR & 131072) != 0;
  static_assert(!SPLIT || (NW == 8 && !CAUSAL && (VAR & 1024)), "split keys: 8 waves, non-causal, LDS-DMA");
  constexpr int NWQ = SPLIT ? 4 : NW;  // waves sharing one query block and its key tiles
  constexpr int LPT = lpt<NWQ>();
  constexpr int kBQ = 64 * NWQ;  // queries per workgroup
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  // VAR bit 16384 (8 waves): waves 4-7 (the second wave of each SIMD) take the tile barrier
  // after P2 instead of after P4, so they run half a tile behind waves 0-3 and the two
  // waves of a SIMD stop reaching their MFMA / VALU bursts in lockstep
  // (MI355X_MICROARCH.md, two waves per SIMD, item 9). V then needs a 4-slot ring: a
  // lagging wave still reads V(t) in P4 while the others stage V(t+2).
  constexpr int kVS = (VAR & 16384) ? 4 : kVSlots;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;
  const int half = SPLIT ? (__builtin_amdgcn_readfirstlane(wave) >> 2) : 0;
  const int wq = SPLIT ? (wave & 3) : wave;  // this wave's 64 queries within the block
  const int Nk = SPLIT ? N / 2 : N;          // keys this wave's half walks
  bf16* const sK = (bf16*)smem_raw + half * (kKSlots + kVS) * TILE;  // [kKSlots][TILE]
  bf16* const sV = sK + kKSlots * TILE;                              // [kVS][TILE]
  const bool late = (VAR & 16384) && NW == 8 && __builtin_amdgcn_readfirstlane(wave) >= 4;

  const int nblk = gridDim.x, hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3, qd = nblk >> 3, rm = nblk & 7;
  const int logical = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + slot;
  // Non-causal: one query block per workgroup. Causal: a pair of query blocks of one head,
  // the light block u first, then the heavy block nqb-1-u (every workgroup walks about
  // nqb + 1 blocks' worth of key tiles; the heavy block finds the light block's tiles still
  // in the XCD's L2).
  const int nunit = CAUSAL ? (nqb + 1) / 2 : nqb;
  const int bh = logical / nunit, unit = logical % nunit;
  const int b = bh / p.H, hh = bh % p.H;

  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Kg = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1] + (int64_t)half * Nk * p.sk[2];
  const bf16* Vg = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1] + (int64_t)half * Nk * p.sv[2];
  const int skn = (int)p.sk[2], svn = (int)p.sv[2];
  const __amdgpu_buffer_rsrc_t rk =
      __builtin_amdgcn_make_buffer_rsrc((void*)Kg, (short)0, ((Nk - 1) * skn + D) * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv =
      __builtin_amdgcn_make_buffer_rsrc((void*)Vg, (short)0, ((Nk - 1) * svn + D) * 2, 0x00020000);

  Ctx5<LPT> c;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) c.koff[ks] = k_swz<D>(c32, 2 * ks + hf);
  {
    const int i16 = lane & 15, g = (lane >> 4) & 1;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const int col = db * 32 + 16 * g + 4 * (i16 & 3);
      c.voff[db] = v_swz<D>(4 * hf + (i16 >> 2), col >> 3) + (col & 7);
    }
    const int tq = SPLIT ? (tid & 255) : tid;  // thread index within the half
    const int st_r = tq / (D / 8), st_c = tq % (D / 8);
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int r = st_r + i * (64 * NWQ / (D / 8));
      c.kgo[i] = (r * skn + st_c * 8) * 2;
      c.vgo[i] = (r * svn + st_c * 8) * 2;
      c.kso[i] = k_swz<D>(r, st_c);
      c.vso[i] = v_swz<D>(r, st_c);
      // DMA: wave w's instruction i fills rows 8 * (LPT * w + i) .. + 7
      const int dr = 8 * (LPT * wq + i) + (lane >> 3), dc = lane & 7;
      c.kdo[i] = (dr * skn + (dc ^ ((dr >> 1) & 7)) * 8) * 2;
      c.vdo[i] = (dr * svn + (dc ^ (((dr >> 1) & 1) << 2)) * 8) * 2;
    }
  }
  const int ktile_b = kBK * skn * 2, vtile_b = kBK * svn * 2;
  const float c2 = p.scale_log2;

  auto dma_k = [&](bf16* slot, int step) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) dma5<VAR>(slot + 8 * (LPT * wq + i) * D, rk, c.kdo[i], step);
  };
  auto dma_v = [&](bf16* slot, int step) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) dma5<VAR>(slot + 8 * (LPT * wq + i) * D, rv, c.vdo[i], step);
  };

  // VAR bit 4096 (8 waves): the younger half of the workgroup (waves 4-7) runs at issue
  // priority 1 for the whole kernel, so it does not lose VALU arbitration to the older
  // half at every phase start (cdna_hip_programming.md T5, static form).
  if (NW == 8 && (VAR & 4096) && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256)
    __builtin_amdgcn_s_setprio(1);

  // One query block [q0, q0 + kBQ) of head bh.
  auto run_block = [&](const int q0) __attribute__((always_inline)) {
  const int qw = q0 + wq * 64;                // first query of this wave (block A; B = +32)
  const int qA = qw + c32;                    // this lane's query in block A; B = qA + 32

  bf16x8 qfA[4], qfB[4];
  {
    const bf16* ra = Qg + (int64_t)min(qA, N - 1) * p.sq[2];
    const bf16* rb = Qg + (int64_t)min(qA + 32, N - 1) * p.sq[2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      qfA[ks] = *(const bf16x8*)(ra + ks * 16 + 8 * hf);
      qfB[ks] = *(const bf16x8*)(rb + ks * 16 + 8 * hf);
    }
  }
  // Tiles the workgroup stages: non-causal all N / 64; causal the keys below its last query.
  // Tiles this wave computes: non-causal all; causal [0, tD] with tD = qw / 64 its diagonal
  // tile (the last, masked; none when the wave's queries are past N). A causal wave that
  // is done keeps staging its share of the later tiles and joins every barrier (the tail
  // loop), so all waves of the workgroup take the same barriers.
  const int ntiles = CAUSAL ? min(N, q0 + kBQ) / kBK : Nk / kBK;
  const int tD = qw / kBK;
  const int nbulk = CAUSAL ? (qw < N ? tD + 1 : 0) : ntiles;

  f32x16 OA[2], OB[2];
  f32x16 RA = f32x16{}, RB = f32x16{};  // MFMA row sums (VAR bit 262144)
  bf16x8 vk[8];  // Vᵀ fragments kept from P2 to P4 (VAR bit 32768)
  constexpr int kKeep = (VAR & 32768) ? 1 : 0;
  float mA = -INFINITY, mB = -INFINITY;
  float pA = 0.f, pB = 0.f;  // this lane's share of each block's row sum
#pragma unroll
  for (int i = 0; i < 2; ++i) { OA[i] = f32x16{}; OB[i] = f32x16{}; }

  // causal diagonal tile of a wave (keys qw .. qw + 63): key row r of a 32-key block is
  // masked for this lane's query when it lies above it (row > c32 within the same block)
  auto mask_tri = [&](f32x16& s) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (acc_row(r, hf) > c32) s[r] = -INFINITY;
  };
  auto mask_all = [&](f32x16& s) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = -INFINITY;
  };

  // ---- pass 0: the pipelined loop with the frozen first-tile reference over the tiles
  //      [0, nbulk); causal: its last tile is the wave's masked diagonal -------------------
  uint4 rK[LPT], rV[LPT];
  if (VAR & 1024) {
    dma_k(sK, 0);
    dma_v(sV, 0);
    dma_k(sK + TILE, ktile_b);
    if (VAR & 524288) __builtin_amdgcn_s_waitcnt(0x0F70);  // asm DMA: hipcc does not wait
  } else {
    load5(rK, rk, c.kgo, 0);
    load5(rV, rv, c.vgo, 0);
    store5(sK, rK, c.kso);
    store5(sV, rV, c.vso);
    load5(rK, rk, c.kgo, ktile_b);
    store5(sK + TILE, rK, c.kso);
  }
  __syncthreads();

  if (nbulk >= 1) {  // non-causal: the launcher guarantees N >= 128
    // reference maxima from tile 0; S_B(0) kept for the pipeline, P_B(0) keys 0-31 computed
    f32x16 SA[2], SB[2];
    {
      int ko[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) ko[ks] = c.koff[ks];
      f32x2 dummy = {0.f, 0.f};
      bf16x8 dpf[2];
      phase_qk<false, AHEAD, VAR>(sK, ko, qfA, SA, SA[0], c2, 0.f, dummy, dpf);
      phase_qk<false, AHEAD, VAR>(sK, ko, qfB, SB, SB[0], c2, 0.f, dummy, dpf);
    }
    if (CAUSAL && tD == 0) {  // tile 0 is this wave's diagonal: reference over visible keys
      mask_tri(SA[0]);
      mask_all(SA[1]);
      mask_tri(SB[1]);
    }
    mA = row_max32(SA[0], SA[1]);
    mB = row_max32(SB[0], SB[1]);
    const float nmcA = -(mA * c2), nmcB = -(mB * c2);
    f32x2 accA = {0.f, 0.f}, accB = {0.f, 0.f};
    bf16x8 pB0[2], pB1[2], pA0[2], pA1[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) sm_pair<VAR>(SB[0], i, c2, nmcB, accB, pB0);
#pragma unroll
    for (int i = 0; i < 2; ++i) { OA[i] = f32x16{}; OB[i] = f32x16{}; }

    // iteration t: K(t) in slot t%4, K(t+1) in slot (t+1)%4, V(t) in slot t%2; stages
    // K(t+2) -> slot (t+2)%4 and V(t+1) -> slot (t+1)%2. The last tile is peeled.
    // One iteration; s0 = t & 3. With VAR bit 2 the loop is unrolled by the K ring size so
    // that every slot offset is a compile-time constant (folded into the LDS instructions'
    // immediate offsets instead of per-iteration address VALU).
    auto iter = [&](int t, int s0, auto late_tag) __attribute__((always_inline)) {
      constexpr bool kLate = decltype(late_tag)::value;
      __builtin_amdgcn_sched_barrier(0);
      if (VAR & 1024) {
        // K(t+2) -> slot (t+2)%4 and V(t+1) -> slot (t+1)%2, both free since the last barrier
        dma_k(sK + ((s0 + 2) & 3) * TILE, (t + 2) * ktile_b);
        dma_v(sV + ((s0 + 1) & (kVS - 1)) * TILE, (t + 1) * vtile_b);
      } else if (!(VAR & 8)) {
        load5(rK, rk, c.kgo, (t + 2) * ktile_b);
        load5(rV, rv, c.vgo, (t + 1) * vtile_b);
      }
      int koA[4], koB[4], vo[2];
      const int kslA = s0 * TILE, kslB = ((s0 + 1) & 3) * TILE, vsl = (s0 & (kVS - 1)) * TILE;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        koA[ks] = c.koff[ks] + kslA;
        koB[ks] = c.koff[ks] + kslB;
      }
      vo[0] = c.voff[0] + vsl;
      vo[1] = c.voff[1] + vsl;
      phase_qk<true, AHEAD, VAR>(sK, koA, qfA, SA, SB[1], c2, nmcB, accB, pB1);             // P1
      phase_pv<true, AHEAD, VAR, kKeep>(sV, vo, OB, pB0, pB1, SA[0], c2, nmcA, accA, pA0, vk, &RB);  // P2
      if (kLate) {
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();
      }
      phase_qk<true, AHEAD, VAR>(sK, koB, qfB, SB, SA[1], c2, nmcA, accA, pA1);             // P3
      phase_pv<true, AHEAD, VAR, 2 * kKeep>(sV, vo, OA, pA0, pA1, SB[0], c2, nmcB, accB, pB0, vk, &RA);  // P4
      if (!(VAR & 8) && !(VAR & 1024)) {
        store5(sK + ((s0 + 2) & 3) * TILE, rK, c.kso);
        store5(sV + ((s0 + 1) & 1) * TILE, rV, c.vso);
      }
      if (!kLate) {
        if (VAR & 1024) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the DMA has landed
        if (!(VAR & 16)) __syncthreads();
      }
    };
    // The staggered half runs its own copy of the loop (straight-line bodies; a branch on
    // `late` inside the body splits it and the register allocator then spills).
    auto loop = [&](auto late_tag) __attribute__((always_inline)) {
      int t = 0;
      if (VAR & 4)
        for (; t + 4 < nbulk; t += 4) {
          iter(t, 0, late_tag);
          iter(t + 1, 1, late_tag);
          iter(t + 2, 2, late_tag);
          iter(t + 3, 3, late_tag);
        }
      for (; t + 1 < nbulk; ++t) iter(t, t & 3, late_tag);
    };
    if ((VAR & 16384) && late)
      loop(std::integral_constant<bool, true>{});
    else
      loop(std::integral_constant<bool, false>{});
    {
      const int t = nbulk - 1;
      int koA[4], vo[2];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) koA[ks] = c.koff[ks] + (t & 3) * TILE;
      vo[0] = c.voff[0] + (t & (kVS - 1)) * TILE;
      vo[1] = c.voff[1] + (t & (kVS - 1)) * TILE;
      if (CAUSAL) mask_tri(SB[1]);  // S_B(tD), keys 32-63: the diagonal of block B
      phase_qk<true, AHEAD, VAR>(sK, koA, qfA, SA, SB[1], c2, nmcB, accB, pB1);
      if (CAUSAL) {  // S_A(tD): keys 0-31 the diagonal of block A, keys 32-63 above it
        mask_tri(SA[0]);
        mask_all(SA[1]);
      }
      phase_pv<true, AHEAD, VAR, kKeep>(sV, vo, OB, pB0, pB1, SA[0], c2, nmcA, accA, pA0, vk, &RB);
#pragma unroll
      for (int i = 0; i < 8; ++i) sm_pair<VAR>(SA[1], i, c2, nmcA, accA, pA1);
      f32x2 d2 = {0.f, 0.f};
      bf16x8 dpf[2];
      phase_pv<false, AHEAD, VAR, 2 * kKeep>(sV, vo, OA, pA0, pA1, SA[0], c2, 0.f, d2, dpf, vk, &RA);
    }
    if (VAR & 262144) {  // every lane holds its query's whole sum; lane_pair_sum adds two
      pA = 0.5f * RA[0];
      pB = 0.5f * RB[0];
    } else {
      pA = accA[0] + accA[1];
      pB = accB[0] + accB[1];
    }
  }
  if (CAUSAL) {
    // tail: this wave's share of the staging of the tiles the other waves still need
    for (int t = nbulk > 0 ? nbulk - 1 : 0; t + 1 < ntiles; ++t) {
      if (VAR & 1024) {
        dma_k(sK + ((t + 2) & 3) * TILE, (t + 2) * ktile_b);
        dma_v(sV + ((t + 1) & (kVS - 1)) * TILE, (t + 1) * vtile_b);
        __builtin_amdgcn_s_waitcnt(0x0F70);
      } else {
        load5(rK, rk, c.kgo, (t + 2) * ktile_b);
        load5(rV, rv, c.vgo, (t + 1) * vtile_b);
        store5(sK + ((t + 2) & 3) * TILE, rK, c.kso);
        store5(sV + ((t + 1) & 1) * TILE, rV, c.vso);
      }
      __syncthreads();
    }
  }

  // ---- serial path: every tile again with the per-tile deferred-max bookkeeping, when a
  // lane's row-sum share left 2^64 (the workgroup starts over) ----------------------------
  auto serial = [&](int t0) {
    int ko[4], vo[2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) ko[ks] = c.koff[ks];
    vo[0] = c.voff[0];
    vo[1] = c.voff[1];
    for (int t = t0; t < ntiles; ++t) {
      uint4 rK2[LPT], rV2[LPT];
      load5(rK2, rk, c.kgo, t * ktile_b);
      load5(rV2, rv, c.vgo, t * vtile_b);
      __syncthreads();
      store5(sK, rK2, c.kso);
      store5(sV, rV2, c.vso);
      __syncthreads();
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        const int qf0 = qw + 32 * blk;  // the block's first query (wave-uniform)
        if (CAUSAL && qf0 + 31 < t * kBK) continue;  // every key of the tile is masked
        f32x16 S[2];
        f32x2 acc = {0.f, 0.f};
        bf16x8 plo[2], phi[2], dpf[2];
        phase_qk<false, AHEAD, VAR>(sK, ko, blk ? qfB : qfA, S, S[0], c2, 0.f, acc, dpf);
        if (CAUSAL && t * kBK + kBK - 1 > qf0) {
          const int q = qf0 + c32;
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (t * kBK + kb * 32 + acc_row(r, hf) > q) S[kb][r] = -INFINITY;
        }
        float& m = blk ? mB : mA;
        float& l = blk ? pB : pA;
        f32x16(&O)[2] = blk ? OB : OA;
        const float tmax = row_max32(S[0], S[1]);
        if (__builtin_amdgcn_ballot_w64((tmax - m) * c2 > kThr)) {
          const float m_new = fmaxf(m, tmax);
          const float alpha = m == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m - m_new) * c2);
          m = m_new;
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) O[i][r] *= alpha;
          l *= alpha;
        }
        const float nmc = -(m * c2);
#pragma unroll
        for (int i = 0; i < 8; ++i) sm_pair<(VAR & ~262144)>(S[0], i, c2, nmc, acc, plo);
#pragma unroll
        for (int i = 0; i < 8; ++i) sm_pair<(VAR & ~262144)>(S[1], i, c2, nmc, acc, phi);
        l += acc[0] + acc[1];
        phase_pv<false, AHEAD, (VAR & ~262144)>(sV, vo, O, plo, phi, S[0], c2, 0.f, acc, dpf, vk);
      }
    }
  };
  if (__syncthreads_or(!(pA <= kLimit) || !(pB <= kLimit))) {
    mA = mB = -INFINITY;
    pA = pB = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) { OA[i] = f32x16{}; OB[i] = f32x16{}; }
    serial(0);
  }
  if (SPLIT) {  // merge the second half's (m, row-sum share, O) into the first half's
    __syncthreads();  // every wave is done with its half's LDS tiles
    float4* xch = (float4*)smem_raw + wq * 17 * 64 + lane;
    if (half) {
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          xch[(4 * db + g) * 64] = make_float4(OA[db][4 * g], OA[db][4 * g + 1], OA[db][4 * g + 2], OA[db][4 * g + 3]);
          xch[(8 + 4 * db + g) * 64] = make_float4(OB[db][4 * g], OB[db][4 * g + 1], OB[db][4 * g + 2], OB[db][4 * g + 3]);
        }
      xch[16 * 64] = make_float4(mA, mB, pA, pB);
    }
    __syncthreads();
    if (half) return;
    const float4 t = xch[16 * 64];
    const float nA = fmaxf(mA, t.x), nB = fmaxf(mB, t.y);
    const float a0 = __builtin_amdgcn_exp2f((mA - nA) * c2), a1 = __builtin_amdgcn_exp2f((t.x - nA) * c2);
    const float b0 = __builtin_amdgcn_exp2f((mB - nB) * c2), b1 = __builtin_amdgcn_exp2f((t.y - nB) * c2);
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 u = xch[(4 * db + g) * 64], w = xch[(8 + 4 * db + g) * 64];
        OA[db][4 * g] = OA[db][4 * g] * a0 + u.x * a1;
        OA[db][4 * g + 1] = OA[db][4 * g + 1] * a0 + u.y * a1;
        OA[db][4 * g + 2] = OA[db][4 * g + 2] * a0 + u.z * a1;
        OA[db][4 * g + 3] = OA[db][4 * g + 3] * a0 + u.w * a1;
        OB[db][4 * g] = OB[db][4 * g] * b0 + w.x * b1;
        OB[db][4 * g + 1] = OB[db][4 * g + 1] * b0 + w.y * b1;
        OB[db][4 * g + 2] = OB[db][4 * g + 2] * b0 + w.z * b1;
        OB[db][4 * g + 3] = OB[db][4 * g + 3] * b0 + w.w * b1;
      }
    pA = pA * a0 + t.z * a1;
    pB = pB * b0 + t.w * b1;
    mA = nA;
    mB = nB;
  }
  const float lA = lane_pair_sum(pA), lB = lane_pair_sum(pB);

#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const int q = qA + 32 * blk;
    const float l = blk ? lB : lA, m = blk ? mB : mA;
    const f32x16(&O)[2] = blk ? OB : OA;
    const float inv = 1.f / l;
    // Widened store: lane (c32, hf) holds columns 8g + 4hf .. +3 of each 32-column block;
    // one v_permlane32_swap per dword pairs groups (g, g+1) so lanes 0-31 hold the 16
    // contiguous bytes of group g and lanes 32-63 those of group g+1: 4 dwordx4 stores
    // per block instead of 8 dwordx2 (every lane takes part in the swap; stores are guarded).
    bf16* Og = (bf16*)p.out + b * p.so[0] + hh * p.so[1] + (int64_t)min(q, N - 1) * p.so[2];
    if (p.o_f32) {  // fp32 output: plain 16-B stores of the lane's four columns
      const ORow Of = o_row(p, b, hh, q);
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          if (q < N)
            store4(Of, db * 32 + 8 * g + 4 * hf, O[db][4 * g] * inv, O[db][4 * g + 1] * inv,
                   O[db][4 * g + 2] * inv, O[db][4 * g + 3] * inv);
    } else {
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      uint2 u[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        const bf16x4 v = {(bf16)(O[db][4 * g] * inv), (bf16)(O[db][4 * g + 1] * inv),
                          (bf16)(O[db][4 * g + 2] * inv), (bf16)(O[db][4 * g + 3] * inv)};
        u[g] = __builtin_bit_cast(uint2, v);
      }
#pragma unroll
      for (int k = 0; k < 4; k += 2) {
        const auto rx = __builtin_amdgcn_permlane32_swap(u[k].x, u[k + 1].x, false, false);
        const auto ry = __builtin_amdgcn_permlane32_swap(u[k].y, u[k + 1].y, false, false);
        if (q < N)
          *(uint4*)(Og + db * 32 + 8 * k + 8 * hf) = uint4{rx[0], ry[0], rx[1], ry[1]};
      }
    }
    }
    if (q < N) {
      if (hf == 0) {
        const int64_t row = (int64_t)bh * N + q;
        if (p.m) p.m[row] = m * p.scale;
        if (p.l) p.l[row] = l;
      }
    }
  }
  };  // run_block

  if (CAUSAL) {
    const int heavy = nqb - 1 - unit;
    run_block(unit * kBQ);
    if (heavy != unit) {
      __syncthreads();  // every wave is done with the light block's LDS tiles
      run_block(heavy * kBQ);
    }
  } else {
    run_block(unit * kBQ);
  }
}

// d = 64, N a multiple of 64 (no ragged tile) and at least two tiles, and all per-head K/V
// offsets (two tiles past N) inside the 31-bit buffer range. Causal runs the mask-free
// prefix through the pipelined loop and the diagonal tiles through the serial path.
hipError_t launch_fwd_v5(const AttnArgs& a, bool causal, int ahead, int var, hipStream_t st,
                         bool* handled) {
  *handled = false;
  if (a.d != 64 || a.N % kBK != 0 || a.N < 2 * kBK) return hipSuccess;
  const bool split = (var & 131072) != 0;  // split keys: each half needs two whole tiles
  if (split && (causal || a.N % (2 * kBK) != 0 || a.N < 4 * kBK)) return hipSuccess;
  const int64_t lim = (int64_t)1 << 31;
  if (((int64_t)a.N + 2 * kBK) * a.sk[2] * 2 >= lim || ((int64_t)a.N + 2 * kBK) * a.sv[2] * 2 >= lim)
    return hipSuccess;
  *handled = true;
  const size_t smem = (size_t)(split ? 2 : 1) * (kKSlots + ((var & 16384) ? 4 : kVSlots)) * TILE * sizeof(bf16);
  void (*kfn)(AttnArgs, int);
  const int nw = (var & 2048) ? 8 : 4;  // VAR bit 2048 (launcher only): 8 waves per workgroup
  var &= ~2048;
#ifndef MT_DIAGNOSTICS
  // product build: the default forms only (causal paired 8-wave; non-causal 8-wave, its
  // split-keys form, the 4-wave LDS-DMA form of small grids); the rest are A/B policies
  (void)ahead;
  if (causal)
    kfn = fa_fwd_bf16_v5<2, 99332, true, 8>;
  else if (nw == 8)
    kfn = split ? fa_fwd_bf16_v5<2, 230404, false, 8> : fa_fwd_bf16_v5<2, 99332, false, 8>;
  else
    kfn = fa_fwd_bf16_v5<2, 1028, false>;
#else
  if (causal)  // paired query blocks, pipelined diagonal (8 or 4 waves), or the 4-wave forms
    kfn = var == 99332 ? (nw == 8 ? fa_fwd_bf16_v5<2, 99332, true, 8> : fa_fwd_bf16_v5<2, 99332, true, 4>)
          : var == 4   ? fa_fwd_bf16_v5<2, 4, true>
                       : fa_fwd_bf16_v5<2, 0, true>;
  else if (nw == 8 && ahead == 3)  // LDS operand reads 3 / 4 MFMAs ahead (policies 57 / 58)
    kfn = fa_fwd_bf16_v5<3, 99332, false, 8>;
  else if (nw == 8 && ahead == 4)
    kfn = fa_fwd_bf16_v5<4, 99332, false, 8>;
  else if (nw == 8)
    kfn = var == 1028   ? fa_fwd_bf16_v5<2, 1028, false, 8>
          : var == 5124 ? fa_fwd_bf16_v5<2, 5124, false, 8>
          : var == 9220 ? fa_fwd_bf16_v5<2, 9220, false, 8>
          : var == 17412 ? fa_fwd_bf16_v5<2, 17412, false, 8>
          : var == 25604 ? fa_fwd_bf16_v5<2, 25604, false, 8>
          : var == 21508 ? fa_fwd_bf16_v5<2, 21508, false, 8>
          : var == 33796 ? fa_fwd_bf16_v5<2, 33796, false, 8>
          : var == 37892 ? fa_fwd_bf16_v5<2, 37892, false, 8>
          : var == 99332 ? fa_fwd_bf16_v5<2, 99332, false, 8>
          : var == 230404 ? fa_fwd_bf16_v5<2, 230404, false, 8>
#ifdef MT_DIAGNOSTICS
          : var == 1147908 ? fa_fwd_bf16_v5<2, 1147908, false, 8>  // MFMA-shape ablation
#endif
          : var == 361476 ? fa_fwd_bf16_v5<2, 361476, false, 8>
          : var == 328708 ? fa_fwd_bf16_v5<2, 328708, false, 8>
          : var == 623620 ? fa_fwd_bf16_v5<2, 623620, false, 8>
                        : fa_fwd_bf16_v5<2, 4, false, 8>;
  else if (var == 1028)
    kfn = fa_fwd_bf16_v5<2, 1028, false>;
#ifdef MT_DIAGNOSTICS
  else if (var >= 8 || var == 2)  // diagnostic ablations (wrong results, timing only)
    kfn = var == 12    ? fa_fwd_bf16_v5<2, 12, false>
          : var == 28  ? fa_fwd_bf16_v5<2, 28, false>
          : var == 68  ? fa_fwd_bf16_v5<2, 68, false>
          : var == 132 ? fa_fwd_bf16_v5<2, 132, false>
          : var == 260 ? fa_fwd_bf16_v5<2, 260, false>
          : var == 2   ? fa_fwd_bf16_v5<2, 2, false>
                       : fa_fwd_bf16_v5<2, 6, false>;
#endif
  else
    kfn = var == 4   ? fa_fwd_bf16_v5<2, 4, false>
          : ahead >= 6 ? fa_fwd_bf16_v5<6, 0, false>
          : ahead >= 4 ? fa_fwd_bf16_v5<4, 0, false>
                       : fa_fwd_bf16_v5<2, 0, false>;
#endif
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  const int kBQ = split ? 256 : 64 * nw;
  const int nqb = (a.N + kBQ - 1) / kBQ;
  // causal: one workgroup per (light, heavy) pair of query blocks
  const int64_t nblk = (int64_t)(causal ? (nqb + 1) / 2 : nqb) * a.B * a.H;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kfn, dim3((unsigned)nblk), dim3(64 * nw), smem, st, a, nqb);
  return hipGetLastError();
}

}  // namespace mt
