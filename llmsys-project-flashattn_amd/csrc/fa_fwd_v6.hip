// FlashAttention forward, bf16 MFMA kernel v6 (d = 64, non-causal, N % 64 == 0): v5's
// schedule (fa_fwd_v5.hip) on the 16x16x32 MFMA instead of the 32x32x16 one.
//
// The two shapes take the same cycles per FLOP, but the chip holds a higher clock on the
// 16x16x32 loop (MI355X_MICROARCH.md, 'DVFS give-back' item 7); priced under v5's own VALU and
// LDS load by the diagnostic ablation 98 (profiles/r2_ab_v5_mfma_shape.txt). Everything else
// is v5's: 8 waves, two 32-query blocks A and B per wave skewed by half a tile, the softmax of
// one block's 32-key half beside each 16-MFMA phase of the other block, K by LDS-DMA two tiles
// ahead into a 4-slot ring and V one tile ahead into a 2-slot ring, one barrier per tile, the
// Vᵀ fragments of P2 kept for P4, exponentials one MFMA slot ahead of their use, the frozen
// first-tile softmax reference with the serial deferred-max recompute when a lane's row-sum
// share leaves 2^64, and the XCD-aware block order.
//
// Layouts (cdna_hip_programming.md §3, 16x16x32 bf16): lane l, g = l >> 4, i = l & 15.
//  * Sᵀ(16 keys x 16 queries) = K·Qᵀ: A = K rows (key 16kb + i, d 32ks + 8g ..), B = Q
//    fragment of query 16qh + i (register resident), C: keys 16kb + 4g + r, query 16qh + i.
//    A block's 64 x 32 scores are s[kb = 0..3][qh = 0..1] (f32x4): a lane holds 16 keys of
//    two queries; the four lanes i, i+16, i+32, i+48 share a query.
//  * Oᵀ(16 d x 16 queries) += Vᵀ·Pᵀ over 32-key halves kk: the B operand of half kk takes
//    the lane's own eight keys of it in k-slot order (keys 32kk + 4g + 0..3, then
//    32kk + 16 + 4g + 0..3), and the A operand (two ds_read_b64_tr_b16 of four keys each)
//    reads Vᵀ in the same key order. C: d 16db + 4g + r, query 16qh + i.
//  * K image: chunk c of row r at c ^ ((r >> 1) & 7) (conflict-free for the 16-row A reads);
//    V image: chunk c of row r at c ^ (((r >> 1) & 3) << 1) (conflict-free for the
//    transposed reads of rows 4g .. 4g + 3 by the 32 lanes of a half-wave).
#include "fa_fwd_bf16.h"

// Timing-only ablations of the bulk loop (WRONG results by construction), built into separate
// A/B libraries with -DV6ABL=n (scripts/build_abl.sh fa_fwd_v6 V6ABL n), never into the product: 1 half
// the K fragment reads (key blocks 2, 3 take blocks 0, 1's fragments with the k-steps swapped, so
// no MFMA chain repeats another), 2 no row-sum MFMAs, 4 no exponentials, 8 half the Vᵀ fragment
// reads (profiles/r5_abl_fwd.txt), 16 no O stores (the epilogue's store tail, round 6).
#ifndef V6ABL
#define V6ABL 0
#endif
// The epilogue's O stores are non-temporal (round 6): O is written once and never read by
// this kernel, and the 'nt' policy keeps it from displacing the K/V tiles other workgroups of
// the XCD are still streaming through L2. Same-process A/B against the plain stores
// (profiles/r6_ab_fwd_nt_store.txt): C3 fp32 O 1121 -> 1142 TF/s, (16,16,2048,64) fp32 O
// 1049 -> 1062, bf16 O +0.3 % / +1.1 %.
#ifndef V6NT
#define V6NT 1
#endif

namespace mt {

namespace {

using namespace fwdbf16;
constexpr int D = 64;
constexpr int kBK = 64;
constexpr int TILE = kBK * D;
constexpr int kKSlots = 4, kVSlots = 2;
constexpr int kNW = 8;                    // waves per workgroup
constexpr int kBQ = 64 * kNW;             // queries per workgroup
constexpr float kLimit = 1.8446744e19f;   // 2^64
constexpr float kThr = 8.0f;

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

struct Blk6 {
  f32x4 s[4][2];  // scores of one 32-query block and 64-key tile: [16-key block kb][query half qh]
};
struct Pf6 {
  bf16x8 p[2];  // Pᵀ B operands of one 32-key half: [query half qh]
};

__device__ __forceinline__ f32x4 mma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// The PV product: bf16, or with H fp16 operands (the Vᵀ fragments read from an image the
// kernel converted to fp16, the P operand packed as fp16) held in the same registers.
template <bool H>
__device__ __forceinline__ f32x4 mma_pv(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  if (!H) return mma16(a, b, c);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// H: the in-LDS bf16 -> fp16 conversion of a staged V tile, 16 B per thread of the workgroup
// (exact for |v| < 65520; larger values become inf and send the block to the bf16 serial pass).
__device__ __forceinline__ u32x4 vcvt_read(const bf16* tile, int tid) {
  return *(const u32x4*)((const char*)tile + tid * 16);
}
__device__ __forceinline__ void vcvt_write(bf16* tile, int tid, const u32x4& x) {
  u32x4 y;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x2 f = {__uint_as_float(x[j] << 16), __uint_as_float(x[j] & 0xffff0000u)};
    y[j] = __builtin_bit_cast(unsigned, __builtin_convertvector(f, f16x2));
  }
  *(u32x4*)((char*)tile + tid * 16) = y;
}

// K fragment f of a tile: 16-key block f >> 1, k-step f & 1 (d 32ks + 8g ..)
__device__ __forceinline__ bf16x8 kread6(const bf16* sk, const int (&ko)[2], int f) {
  return *(const bf16x8*)(sk + (f >> 1) * 16 * D + ko[f & 1]);
}

// Vᵀ fragment f of a tile: key half f >> 2, d block f & 3; keys 4g..4g+3 and 16+4g..16+4g+3
// of the half (rows), d 16db + i (the lane's A row)
__device__ __forceinline__ bf16x8 vread6(const bf16* sv, const int (&vo)[4], int f) {
  const bf16* a1 = sv + (f >> 2) * 32 * D + vo[f & 3];
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1 + 16 * D));
  const s16x8 av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, av);
}

// Softmax pair i (0..7) of half kk of a block: 16-key block 2kk + (i >> 2), query half
// (i >> 1) & 1, rows 2(i & 1), 2(i & 1) + 1. Exponentials in one MFMA slot, the row-sum add
// and bf16 pack in the next (no transcendental-to-use stall). PS: the scores already are
// c2 s - reference (Q pre-scaled, the shift in the MFMA's C operand): no scale-and-shift.
template <bool PS, bool PK = false, bool ABL = false>
__device__ __forceinline__ f32x2 sm6_exp(const Blk6& s, int kk, int i, float c2, const float (&nmc)[2]) {
  const int kbl = i >> 2, qh = (i >> 1) & 1, r0 = 2 * (i & 1);
  const f32x4& v = s.s[2 * kk + kbl][qh];
  if ((V6ABL & 4) && ABL && !PS)
    return f32x2{__builtin_fmaf(v[r0], c2, nmc[qh]), __builtin_fmaf(v[r0 + 1], c2, nmc[qh])};
  if (PS) return f32x2{__builtin_amdgcn_exp2f(v[r0]), __builtin_amdgcn_exp2f(v[r0 + 1])};
  if (PK) {  // diagnostics (VAR 32768): the pair's scale-and-shift as one v_pk_fma_f32
    const f32x2 x = __builtin_elementwise_fma(f32x2{v[r0], v[r0 + 1]}, f32x2{c2, c2}, f32x2{nmc[qh], nmc[qh]});
    return f32x2{__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
  }
  // scalar f32 arithmetic: packed v_pk_fma_f32 / v_pk_add_f32 beside the MFMAs cost issue
  // cycles the scalar forms do not (MI355X_MICROARCH.md, 'price of one filler')
  const float x0 = __builtin_fmaf(v[r0], c2, nmc[qh]), x1 = __builtin_fmaf(v[r0 + 1], c2, nmc[qh]);
  return f32x2{__builtin_amdgcn_exp2f(x0), __builtin_amdgcn_exp2f(x1)};
}
// RS: no row-sum adds (the PV phase sums the packed P on the MFMA pipe)
// H: P packed as fp16 (v_cvt_pk_f16_f32, round to nearest even: 11 significant bits).
template <bool RS = false, bool H = false>
__device__ __forceinline__ void sm6_fin(const f32x2& e, int i, f32x2 (&acc)[2], Pf6& pf) {
  const int kbl = i >> 2, qh = (i >> 1) & 1, r0 = 2 * (i & 1);
  if (!RS) {
    acc[qh][0] += e[0];
    acc[qh][1] += e[1];
  }
  if (H) {
    u32x4 w = __builtin_bit_cast(u32x4, pf.p[qh]);
    w[2 * kbl + (i & 1)] = __builtin_bit_cast(unsigned, __builtin_convertvector(e, f16x2));
    pf.p[qh] = __builtin_bit_cast(bf16x8, w);
    return;
  }
  pf.p[qh][4 * kbl + r0] = (bf16)e[0];
  pf.p[qh][4 * kbl + r0 + 1] = (bf16)e[1];
}

// The softmax work of MFMA slot m (0..15) of a phase. Default: the two exponentials of pair
// m / 2 in the even slot, its row-sum adds and bf16 pack in the odd one. EV (with RS only):
// one exponential per slot, and in odd slots the pack of the previous pair (the last pair is
// packed after the phase's last MFMA): 12 / 16 cycles of issue per slot instead of 24 / 4.
template <bool PS, bool RS, bool EV, bool H = false, bool PK = false>
__device__ __forceinline__ void sm6_slot(int m, const Blk6& s_in, int kk, float c2, const float (&nmc)[2],
                                         f32x2 (&acc)[2], Pf6& pf, f32x2& ep, f32x2& ec) {
  if (!EV) {
    if (m & 1) sm6_fin<RS, H>(ep, m >> 1, acc, pf);
    else ep = sm6_exp<PS, PK, true>(s_in, kk, m >> 1, c2, nmc);
    return;
  }
  const int i = m >> 1, j = m & 1, kbl = i >> 2, qh = (i >> 1) & 1, r = 2 * (i & 1) + j;
  const float v = s_in.s[2 * kk + kbl][qh][r];
  ec[j] = __builtin_amdgcn_exp2f(PS ? v : __builtin_fmaf(v, c2, nmc[qh]));
  if (j) {
    if (i) sm6_fin<true, H>(ep, i - 1, acc, pf);
    ep = ec;
  }
}

// QKᵀ phase: 16 MFMAs into S (16-key blocks in order, so keys 0-31 finish first), beside the
// softmax of half kk of s_in. MFMA m: fragment f = m >> 1 (block f >> 1, k-step f & 1),
// query half m & 1. The chains start from ci[qh] (zero, or the PS shift).
template <bool SOFT, bool PS, bool RS = false, bool EV = false, bool H = false, bool PK = false>
__device__ __forceinline__ void qk6(const bf16* sk, const int (&ko)[2], const bf16x8 (&qf)[2][2], Blk6& S,
                                    const f32x4 (&ci)[2], const Blk6& s_in, int kk, float c2,
                                    const float (&nmc)[2], f32x2 (&acc)[2], Pf6& pf) {
  bf16x8 kf[8];
  kf[0] = kread6(sk, ko, 0);
  kf[1] = kread6(sk, ko, 1);
  f32x2 ep, ec;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int f = m >> 1, kb = f >> 1, ks = f & 1, qh = m & 1;
    if (!(m & 1) && f + 2 < 8) kf[f + 2] = ((V6ABL & 1) && SOFT && f + 2 >= 4) ? kf[(f - 2) ^ 1] : kread6(sk, ko, f + 2);
    S.s[kb][qh] = mma16(kf[f], qf[qh][ks], ks ? S.s[kb][qh] : ci[qh]);
    if (SOFT) sm6_slot<PS, RS, EV, H, PK>(m, s_in, kk, c2, nmc, acc, pf, ep, ec);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (SOFT && EV) sm6_fin<true, H>(ep, 7, acc, pf);
}

// PV phase: 16 MFMAs into O with the P operands of halves 0 (plo) and 1 (phi), beside the
// softmax of half kk of s_in. MFMA m: Vᵀ fragment f = m >> 1 (half f >> 2, d block f & 3),
// query half m & 1. KEEP: 1 = read the Vᵀ fragments and leave them in vk, 2 = take them
// from vk (P2 and P4 multiply the same V(t)). RS: R[qh] += ones·Pᵀ right after each P
// operand's first MFMA (every element of R[qh] is then the running row sum of its query).
template <bool SOFT, int KEEP, bool PS, bool RS = false, bool EV = false, bool H = false, bool PK = false>
__device__ __forceinline__ void pv6(const bf16* sv, const int (&vo)[4], f32x4 (&O)[4][2], const Pf6& plo,
                                    const Pf6& phi, const Blk6& s_in, int kk, float c2,
                                    const float (&nmc)[2], f32x2 (&acc)[2], Pf6& pf, bf16x8 (&vk)[8],
                                    f32x4 (&R)[2]) {
  constexpr short one = H ? 0x3c00 : 0x3f80;  // 1.0 in fp16 / bf16
  const bf16x8 ones = __builtin_bit_cast(bf16x8, s16x8{one, one, one, one, one, one, one, one});
  bf16x8 vf_own[8];
  bf16x8(&vf)[8] = KEEP ? vk : vf_own;
  if (KEEP != 2) {
    vf[0] = vread6(sv, vo, 0);
    vf[1] = vread6(sv, vo, 1);
  }
  f32x2 ep, ec;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int f = m >> 1, hv = f >> 2, db = f & 3, qh = m & 1;
    if (KEEP != 2 && !(m & 1) && f + 2 < 8) vf[f + 2] = ((V6ABL & 8) && SOFT && f + 2 >= 4) ? vf[f - 2] : vread6(sv, vo, f + 2);
    O[db][qh] = mma_pv<H>(vf[f], (hv ? phi : plo).p[qh], O[db][qh]);
    if (RS && db == 0 && !((V6ABL & 2) && SOFT)) R[qh] = mma_pv<H>(ones, (hv ? phi : plo).p[qh], R[qh]);
    if (SOFT) sm6_slot<PS, RS, EV, H, PK>(m, s_in, kk, c2, nmc, acc, pf, ep, ec);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (SOFT && EV) sm6_fin<true, H>(ep, 7, acc, pf);
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
// a lane's max over its 16 keys of query half qh
__device__ __forceinline__ float lane_max6(const Blk6& s, int qh) {
  float m = fmaxf(fmaxf(s.s[0][qh][0], s.s[0][qh][1]), s.s[0][qh][2]);
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = (kb ? 0 : 3); r < 4; ++r) m = fmaxf(m, s.s[kb][qh][r]);
  return m;
}

// LDS-DMA of 64 x 16 B to the LDS byte address lds (wave-uniform). Issued from inline asm:
// with the builtin, hipcc's waitcnt pass cannot tell the destination slot from the slots the
// phase reads and put an s_waitcnt vmcnt(0) in front of the first Vᵀ read of every tile,
// waiting mid-tile for the K(t+2) / V(t+1) staging issued at its start. The slots are
// published by the tile's closing vmcnt(0) + barrier, which the loop issues itself.
__device__ __forceinline__ void dma6(uint32_t lds, __amdgpu_buffer_rsrc_t rs, int go, int step) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(go + step), "s"(lds), "s"(rs)
      : "memory");
}

// dma6 with a scalar byte offset on top of the per-lane one (soffset): the W4 form's second
// piece reuses the first piece's address VGPR
__device__ __forceinline__ void dma6s(uint32_t lds, __amdgpu_buffer_rsrc_t rs, int go, int soff) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(go), "s"(lds), "s"(rs), "s"(soff)
      : "memory");
}

}  // namespace

// PS (policy 101): Q pre-scaled by c2 = log2(e) / sqrt(d) (rounded to bf16 once, in
// registers) and the frozen reference subtracted through the QKᵀ chains' C operand, so the
// exponent needs no scale-and-shift (one v_fma_f32 per score fewer). The returned m is the
// reference / log2(e); the bf16 rounding of c2 Q adds a relative score error of 2^-9, past
// the (m, l) tolerance of the parity tests, so it exists only in the diagnostics build.
// RS (VAR 2): row sums on the MFMA pipe (pv6). NK (VAR 4): no Vᵀ reuse (P4 re-reads V).
// EV (VAR 8, with RS): one exponential per MFMA slot (sm6_slot).
// CAUSAL (VAR 32): v5's causal schedule (paired light / heavy query blocks, each wave's
// masked diagonal tile peeled from its own pipelined loop, finished waves keep staging).
// SPLIT (VAR 16): the keys split between the two halves of the workgroup (v5's VAR 131072):
// waves w and w + 4 take the same 64 queries over the first and the second half of the keys,
// each half with its own K/V rings and staging under the same barriers; the second half
// hands (m, row-sum share, O) to the first through LDS at the end. 256 queries per
// workgroup, for grids with fewer 8-wave workgroups than CUs.
template <int VAR>
__global__ __launch_bounds__(64 * kNW, 1) void fa_fwd_bf16_v6(AttnArgs p, int nqb) {
  constexpr bool PS = VAR & 1, RS = VAR & 2, EV = RS && (VAR & 8), SPLIT = VAR & 16, CAUSAL = VAR & 32;
  constexpr bool WIDE = VAR & 64;  // 16-B epilogue stores (T21)
  constexpr bool NOBAR = VAR & 128;  // diagnostics, timing only, racy: no tile barrier in the bulk loop
  // causal, two 4-wave halves: each half walks its own light / heavy pair of 256-query blocks
  // through its own K/V rings (the halves' pairs have equal tile counts, so their barriers
  // line up); wave-tile utilisation 95.6 % instead of 90.3 % at C3
  constexpr bool DUAL = VAR & 256;
  // causal, fp16 PV (VAR 512, the fp32-output default): V tiles are staged two ahead into a
  // 4-slot ring and converted to fp16 in LDS the tile before use; P is packed as fp16 (11
  // significant bits instead of 8) for the PV and row-sum MFMAs, which takes the rounding
  // of P, the error that dominates rows with few keys, down 8x
  constexpr bool H = VAR & 512;
  // diagnostics (VAR 1024): s_memtime stamps at the phase boundaries of the bulk loop; per wave
  // the cycle sums of [DMA issue, P1, P2, P3, P4, vmcnt(0), barrier] go to p.dbg
  constexpr bool STAMP = VAR & 1024;
  // diagnostics (VAR 2048): the older half of the workgroup (waves 0-3, which win the SIMDs'
  // issue arbitration and then wait at the tile barrier) issues all of the tile's LDS-DMA, two
  // pieces each, and the younger half (the pole) none
  constexpr bool ODMA = (VAR & 2048) && !SPLIT && !DUAL;
  // diagnostics (VAR 4096 / 8192): the younger half (waves 4-7) at issue priority 1 from the
  // tile's start to P3 (4096) or to P2 (8192), priority 0 for the rest of the tile (the older
  // half wins the arbitration of P1-P2 otherwise and then waits at the barrier)
  constexpr int PFLIP = (VAR & 4096) ? 3 : (VAR & 8192) ? 2 : 0;
  // W4 (VAR 16384; the bf16-output causal default since round 4): 4-wave workgroups (256
  // queries), two per CU, so the two waves of a SIMD belong to different workgroups and share
  // no barrier (the 8-wave form's older half waits at every tile barrier for the younger half,
  // which loses the SIMDs' issue arbitration); each workgroup stages its own K/V tiles (two
  // LDS-DMA pieces per wave)
  constexpr bool W4 = (VAR & 16384) && !SPLIT && !DUAL;
  constexpr bool PK = (VAR & 32768) && !PS;  // diagnostics: packed scale-and-shift (sm6_exp)
  // RG (VAR 65536): any N >= 128, not only multiples of 64. The last key tile is partial: its
  // rows past N arrive as zeros (the buffer range check). Non-causal (8-wave form), their
  // scores are masked in registers, S_B's right after the last bulk iteration's P3 computes
  // them (its P4 starts their softmax), S_A's in the peeled last tile. Causal, the diagonal
  // mask already hides them (a key past N is past every query below N), so only the tile
  // count changes. Queries past N are loaded clamped and not stored, as everywhere.
  constexpr bool RG = VAR & 65536;
  static_assert(!RG || (!SPLIT && !DUAL && !PS && (CAUSAL || !W4)), "ragged N: the 8-wave non-causal and the causal forms");
  constexpr bool RGM = RG && !CAUSAL;  // the key mask of the partial tile
  // H with W4: 256 threads convert a V tile (8 KiB) in two 16-B chunks each
  constexpr int NCV = W4 ? 2 : 1;
  static_assert(!(SPLIT && CAUSAL), "split keys: non-causal");
  static_assert(!DUAL || CAUSAL, "dual halves: causal");
  static_assert(!H || (CAUSAL && !DUAL && !PS && RS && !EV), "fp16 PV: the causal default form");
  constexpr int VS = H ? 4 : kVSlots;  // V ring slots
  constexpr int K1 = (VAR & 4) ? 0 : 1, K2 = (VAR & 4) ? 0 : 2;
  constexpr int NWQ = (SPLIT || DUAL || W4) ? 4 : kNW;  // waves sharing one query block and its key tiles
  constexpr int LPT = ODMA ? 2 : kNW / NWQ;  // LDS-DMA instructions per (issuing) wave per tile
  constexpr int BQ = 64 * NWQ;          // queries per workgroup
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loop control
  const int g = lane >> 4, i16 = lane & 15;
  const int N = p.N;
  const int half = (SPLIT || DUAL) ? (wave >> 2) : 0;
  const int wq = (SPLIT || DUAL) ? (wave & 3) : wave;  // this wave's 64 queries within the block
  const int Nk = SPLIT ? N / 2 : N;          // keys this wave's half walks
  bf16* const sK = (bf16*)smem_raw + half * (kKSlots + VS) * TILE;  // [kKSlots][TILE]
  bf16* const sV = sK + kKSlots * TILE;                             // [VS][TILE]

  const int nblk = gridDim.x, hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3, qd = nblk >> 3, rm = nblk & 7;
  const int logical = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + slot;
  // Non-causal: one query block per workgroup. Causal: a pair of query blocks of one head,
  // the light block u first, then the heavy block nqb - 1 - u (every workgroup walks about
  // nqb + 1 blocks' worth of key tiles; the heavy block finds the light block's tiles still
  // in the XCD's L2).
  const int nunit = DUAL ? nqb / 4 : CAUSAL ? (nqb + 1) / 2 : nqb;
  const int bh = logical / nunit, qb = logical % nunit;
  const int b = bh / p.H, hh = bh % p.H;

  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Kg = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1] + (int64_t)(SPLIT ? half : 0) * Nk * p.sk[2];
  const bf16* Vg = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1] + (int64_t)(SPLIT ? half : 0) * Nk * p.sv[2];
  const int skn = (int)p.sk[2], svn = (int)p.sv[2];
  const __amdgpu_buffer_rsrc_t rk =
      __builtin_amdgcn_make_buffer_rsrc((void*)Kg, (short)0, ((Nk - 1) * skn + D) * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv =
      __builtin_amdgcn_make_buffer_rsrc((void*)Vg, (short)0, ((Nk - 1) * svn + D) * 2, 0x00020000);

  int ko[2], vo[4];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) ko[ks] = k_swz<D>(i16, 4 * ks + g);
  {
    const int q = i16 >> 2, pp = i16 & 3, row = 4 * g + q;
#pragma unroll
    for (int db = 0; db < 4; ++db)
      vo[db] = row * D + (((2 * db + (pp >> 1)) ^ (((row >> 1) & 3) << 1)) * 8) + 4 * (pp & 1);
  }
  // LDS-DMA: instruction i of wave w fills rows 8 (LPT w + i) .. + 7 of a tile in lane
  // order, so lane l fetches the source chunk the swizzle puts at chunk l % 8 of row
  // 8 (LPT w + i) + l / 8
  // W4: piece i of wave w fills rows 8 (w + 4 i) ..: rows 32 apart take the same swizzle, so
  // piece 1's source offset is piece 0's plus a scalar (one address VGPR per tensor)
  auto prow = [&](int i) __attribute__((always_inline)) { return W4 ? 8 * (wq + 4 * i) : 8 * (LPT * wq + i); };
  constexpr int NDO = W4 ? 1 : LPT;
  int kdo[NDO], vdo[NDO];
#pragma unroll
  for (int i = 0; i < NDO; ++i) {
    const int dr = prow(i) + (lane >> 3), dc = lane & 7;
    kdo[i] = (dr * skn + (dc ^ ((dr >> 1) & 7)) * 8) * 2;
    vdo[i] = (dr * svn + (dc ^ (((dr >> 1) & 3) << 1)) * 8) * 2;
  }
  const int ktile_b = kBK * skn * 2, vtile_b = kBK * svn * 2;
  // the workgroup's LDS base as a wave-uniform byte address; slot pointers become constant
  // offsets from it
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem_raw);
  auto lds_of = [&](const bf16* sl, int i) __attribute__((always_inline)) {
    return lds0 + (uint32_t)((sl - (const bf16*)smem_raw) + prow(i) * D) * 2;
  };
  auto dma_k = [&](bf16* sl, int step) __attribute__((always_inline)) {
    if (ODMA && wave >= 4) return;
    if (W4) {
      const int go = kdo[0] + step;
      dma6s(lds_of(sl, 0), rk, go, 0);
      dma6s(lds_of(sl, 1), rk, go, 64 * skn);
      return;
    }
#pragma unroll
    for (int i = 0; i < LPT; ++i) dma6(lds_of(sl, i), rk, kdo[i], step);
  };
  auto dma_v = [&](bf16* sl, int step) __attribute__((always_inline)) {
    if (ODMA && wave >= 4) return;
    if (W4) {
      const int go = vdo[0] + step;
      dma6s(lds_of(sl, 0), rv, go, 0);
      dma6s(lds_of(sl, 1), rv, go, 64 * svn);
      return;
    }
#pragma unroll
    for (int i = 0; i < LPT; ++i) dma6(lds_of(sl, i), rv, vdo[i], step);
  };
  const float c2 = p.scale_log2;

  // One query block [q0, q0 + BQ) of head bh. mode 0: the pipelined pass, then the serial
  // pass when a row sum left 2^64; 1 (DUAL): the pipelined pass only, returning whether the
  // serial pass is needed; 2 (DUAL): the serial pass only.
  auto run_block = [&](const int q0, const int mode) __attribute__((always_inline)) -> bool {
  const int qw = q0 + wq * 64;  // first query of this wave (block A; block B = +32)
  bf16x8 qfA[2][2], qfB[2][2];  // [qh][ks]
#pragma unroll
  for (int qh = 0; qh < 2; ++qh) {
    const bf16* ra = Qg + (int64_t)min(qw + 16 * qh + i16, N - 1) * p.sq[2];
    const bf16* rb = Qg + (int64_t)min(qw + 32 + 16 * qh + i16, N - 1) * p.sq[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qfA[qh][ks] = *(const bf16x8*)(ra + 32 * ks + 8 * g);
      qfB[qh][ks] = *(const bf16x8*)(rb + 32 * ks + 8 * g);
      if (PS) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          qfA[qh][ks][j] = (bf16)((float)qfA[qh][ks][j] * c2);
          qfB[qh][ks][j] = (bf16)((float)qfB[qh][ks][j] * c2);
        }
      }
    }
  }
  const float c2e = PS ? 1.f : c2;  // the factor from an MFMA score to log2 units
  const f32x4 ci0[2] = {f32x4{}, f32x4{}};
  // Tiles the workgroup stages: non-causal all Nk / 64; causal the keys below its last
  // query. Tiles this wave computes: non-causal all; causal [0, tD] with tD = qw / 64 its
  // diagonal tile (the last, masked; none when the wave's queries are past N). A causal wave
  // that is done keeps staging its share of the later tiles and joins every barrier (the
  // tail loop), so all waves of the workgroup take the same barriers.
  const int ntiles = RG ? (min(Nk, CAUSAL ? q0 + BQ : Nk) + kBK - 1) / kBK : CAUSAL ? min(N, q0 + BQ) / kBK : Nk / kBK;
  const int nlast = Nk - (ntiles - 1) * kBK;  // RG: the keys of the last tile (1 .. 64)
  const int tD = qw / kBK;
  const int nbulk = CAUSAL ? (qw < N ? tD + 1 : 0) : ntiles;

  f32x4 OA[4][2], OB[4][2];
  auto zero_o = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) { OA[db][qh] = f32x4{}; OB[db][qh] = f32x4{}; }
  };
  zero_o();
  // per query half: reference max, row-sum share
  float mA[2] = {0.f, 0.f}, mB[2] = {0.f, 0.f}, pA[2] = {0.f, 0.f}, pB[2] = {0.f, 0.f};
  bf16x8 vk[8];
  // causal: the wave's diagonal tile holds keys qw .. qw + 63; key 16 kb + 4 g + r of it is
  // above query lq0 + 16 qh + i16 of the wave (lq0 = 0 for block A, 32 for block B) when
  // larger
  // RG: keys at or past nlast of the last tile
  auto mask_tail = [&](Blk6& S) __attribute__((always_inline)) {
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (16 * kb + 4 * g + r >= nlast) S.s[kb][qh][r] = -INFINITY;
  };
  auto mask_diag = [&](Blk6& S, int lq0) __attribute__((always_inline)) {
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (16 * kb + 4 * g + r > lq0 + 16 * qh + i16) S.s[kb][qh][r] = -INFINITY;
  };

  // ---- pass 0: the pipelined loop with the frozen first-tile reference over the tiles
  //      [0, nbulk); causal: its last tile is the wave's masked diagonal --------------------
  if (mode != 2) {
  dma_k(sK, 0);
  dma_v(sV, 0);
  dma_k(sK + TILE, ktile_b);
  if (H) dma_v(sV + TILE, vtile_b);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (H) {  // V(0) to fp16 (V(1) is converted in iteration 0)
#pragma unroll
    for (int c = 0; c < NCV; ++c) vcvt_write(sV, tid + 256 * c, vcvt_read(sV, tid + 256 * c));
    __syncthreads();
  }
  if (nbulk >= 1) {  // non-causal: the launcher guarantees N >= 128
    Blk6 SA, SB;
    {
      f32x2 dacc[2];
      Pf6 dpf;
      const float z[2] = {0.f, 0.f};
      qk6<false, false>(sK, ko, qfA, SA, ci0, SA, 0, c2, z, dacc, dpf);
      qk6<false, false>(sK, ko, qfB, SB, ci0, SB, 0, c2, z, dacc, dpf);
    }
    if (CAUSAL && tD == 0) {  // tile 0 is this wave's diagonal: reference over visible keys
      mask_diag(SA, 0);
      mask_diag(SB, 32);
    }
    float nmcA[2], nmcB[2];
    f32x4 ciA[2], ciB[2];
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      mA[qh] = quad_max(lane_max6(SA, qh));
      mB[qh] = quad_max(lane_max6(SB, qh));
      nmcA[qh] = -(mA[qh] * c2);
      nmcB[qh] = -(mB[qh] * c2);
      ciA[qh] = f32x4{-mA[qh], -mA[qh], -mA[qh], -mA[qh]};
      ciB[qh] = f32x4{-mB[qh], -mB[qh], -mB[qh], -mB[qh]};
      if (PS) {  // tile 0's scores were computed from zero
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          SA.s[kb][qh] += ciA[qh];
          SB.s[kb][qh] += ciB[qh];
        }
      }
    }
    f32x2 accA[2] = {f32x2{0.f, 0.f}, f32x2{0.f, 0.f}}, accB[2] = {f32x2{0.f, 0.f}, f32x2{0.f, 0.f}};
    Pf6 pB0, pB1, pA0, pA1;
#pragma unroll
    for (int i = 0; i < 8; ++i) sm6_fin<RS, H>(sm6_exp<PS>(SB, 0, i, c2, nmcB), i, accB, pB0);
    f32x4 RA[2] = {f32x4{}, f32x4{}}, RB[2] = {f32x4{}, f32x4{}};

    // iteration t: K(t) in slot t % 4, K(t + 1) in slot (t + 1) % 4, V(t) in slot t % 2;
    // stages K(t + 2) and V(t + 1). Unrolled by the K ring size (slot offsets immediate).
    // H: V(t + 2) is staged (4-slot V ring) and V(t + 1), landed by the previous tile's
    // barrier, is converted to fp16 beside P1 (read before it, written after it).
    unsigned long long seg[7] = {0, 0, 0, 0, 0, 0, 0}, tprev = 0;
    auto stamp = [&](int k) __attribute__((always_inline)) {
      if (!STAMP) return;
      unsigned long long tnow;
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tnow) :: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (k >= 0) seg[k] += tnow - tprev;
      tprev = tnow;
    };
    // last_b (RG): the last bulk iteration, whose P3 computes S_B of the partial last tile
    auto iter = [&](int t, int s0, bool last_b = false) __attribute__((always_inline)) {
      __builtin_amdgcn_sched_barrier(0);
      if (PFLIP && wave >= 4) __builtin_amdgcn_s_setprio(1);
      stamp(-1);
      dma_k(sK + ((s0 + 2) & 3) * TILE, (t + 2) * ktile_b);
      if (H) dma_v(sV + ((s0 + 2) & 3) * TILE, (t + 2) * vtile_b);
      else dma_v(sV + ((s0 + 1) & 1) * TILE, (t + 1) * vtile_b);
      u32x4 vraw[NCV];
#pragma unroll
      for (int c = 0; c < NCV; ++c)
        if (H) vraw[c] = vcvt_read(sV + ((s0 + 1) & 3) * TILE, tid + 256 * c);
      int koA[2], koB[2], vv[4];
      const int kslA = s0 * TILE, kslB = ((s0 + 1) & 3) * TILE, vsl = (s0 & (VS - 1)) * TILE;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        koA[ks] = ko[ks] + kslA;
        koB[ks] = ko[ks] + kslB;
      }
#pragma unroll
      for (int db = 0; db < 4; ++db) vv[db] = vo[db] + vsl;
      stamp(0);
      qk6<true, PS, RS, EV, H, PK>(sK, koA, qfA, SA, PS ? ciA : ci0, SB, 1, c2, nmcB, accB, pB1);  // P1
#pragma unroll
      for (int c = 0; c < NCV; ++c)
        if (H) vcvt_write(sV + ((s0 + 1) & 3) * TILE, tid + 256 * c, vraw[c]);
      stamp(1);
      if (PFLIP == 2 && wave >= 4) __builtin_amdgcn_s_setprio(0);
      pv6<true, K1, PS, RS, EV, H, PK>(sV, vv, OB, pB0, pB1, SA, 0, c2, nmcA, accA, pA0, vk, RB);  // P2
      stamp(2);
      if (PFLIP == 3 && wave >= 4) __builtin_amdgcn_s_setprio(0);
      qk6<true, PS, RS, EV, H, PK>(sK, koB, qfB, SB, PS ? ciB : ci0, SA, 1, c2, nmcA, accA, pA1);  // P3
      if (RGM && last_b) mask_tail(SB);  // S_B of the partial last tile (before P4 starts its softmax)
      stamp(3);
      pv6<true, K2, PS, RS, EV, H, PK>(sV, vv, OA, pA0, pA1, SB, 0, c2, nmcB, accB, pB0, vk, RA);  // P4
      stamp(4);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stamp(5);
      if (!NOBAR) __syncthreads();
      stamp(6);
    };
    int t = 0;
    const int nloop = RGM ? nbulk - 1 : nbulk;  // RGM: the last bulk iteration peeled (its S_B mask)
    for (; t + 4 < nloop; t += 4) {
      iter(t, 0);
      iter(t + 1, 1);
      iter(t + 2, 2);
      iter(t + 3, 3);
    }
    for (; t + 1 < nloop; ++t) iter(t, t & 3);
    if (RGM) {
      iter(t, t & 3, true);
      ++t;
    }
    {  // the last tile (causal: the wave's diagonal)
      int koA[2], vv[4];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) koA[ks] = ko[ks] + (t & 3) * TILE;
#pragma unroll
      for (int db = 0; db < 4; ++db) vv[db] = vo[db] + (t & (VS - 1)) * TILE;
      if (CAUSAL) mask_diag(SB, 32);  // S_B(tD): keys 32-63 are block B's diagonal
      qk6<true, PS, RS, EV, H, PK>(sK, koA, qfA, SA, PS ? ciA : ci0, SB, 1, c2, nmcB, accB, pB1);
      if (CAUSAL) mask_diag(SA, 0);  // S_A(tD): keys 0-31 its diagonal, 32-63 above it
      if (RGM && nlast < kBK) mask_tail(SA);
      pv6<true, K1, PS, RS, EV, H, PK>(sV, vv, OB, pB0, pB1, SA, 0, c2, nmcA, accA, pA0, vk, RB);
#pragma unroll
      for (int i = 0; i < 8; ++i) sm6_fin<RS, H>(sm6_exp<PS>(SA, 1, i, c2, nmcA), i, accA, pA1);
      f32x2 d2[2];
      Pf6 dpf;
      pv6<false, K2, PS, RS, false, H>(sV, vv, OA, pA0, pA1, SA, 0, c2, nmcA, d2, dpf, vk, RA);
    }
    if (STAMP && lane == 0) {
      unsigned long long* o = p.dbg + ((int64_t)blockIdx.x * kNW + wave) * 8;
#pragma unroll
      for (int k = 0; k < 7; ++k) o[k] = seg[k];
      o[7] = (unsigned long long)max(nbulk - 1, 0);
    }
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      // RS: every lane holds its query's whole row sum; a quarter each for the epilogue's
      // sum over the four lanes of a query (exact)
      pA[qh] = RS ? 0.25f * RA[qh][0] : accA[qh][0] + accA[qh][1];
      pB[qh] = RS ? 0.25f * RB[qh][0] : accB[qh][0] + accB[qh][1];
    }
    if (H) {
      // fp16 P must stay below 65504: a row sum past 2^15 (a quarter share past 2^13), or a
      // non-finite O (a V value past the fp16 range), sends the block to the serial pass
      float om = 0.f;
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh)
#pragma unroll
          for (int r = 0; r < 4; ++r) om = fmaxf(om, fmaxf(fabsf(OA[db][qh][r]), fabsf(OB[db][qh][r])));
      if (!(om <= 3.0e38f)) pA[0] = INFINITY;
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        if (!(pA[qh] <= 8192.f)) pA[qh] = INFINITY;
        if (!(pB[qh] <= 8192.f)) pB[qh] = INFINITY;
      }
    }
  }
  if (CAUSAL) {
    // tail: this wave's share of the staging of the tiles the other waves still need
    for (int t = nbulk > 0 ? nbulk - 1 : 0; t + 1 < ntiles; ++t) {
      dma_k(sK + ((t + 2) & 3) * TILE, (t + 2) * ktile_b);
      if (H) {  // and its share of the conversion of V(t + 1)
        dma_v(sV + ((t + 2) & 3) * TILE, (t + 2) * vtile_b);
#pragma unroll
        for (int c = 0; c < NCV; ++c)
          vcvt_write(sV + ((t + 1) & 3) * TILE, tid + 256 * c, vcvt_read(sV + ((t + 1) & 3) * TILE, tid + 256 * c));
      } else {
        dma_v(sV + ((t + 1) & 1) * TILE, (t + 1) * vtile_b);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  }  // mode != 2

  // ---- serial path: every tile again with the per-tile deferred-max bookkeeping, when a
  // lane's row-sum share left 2^64 (the workgroup starts over) -----------------------------
  const bool bad = mode != 2 &&
                   (!(pA[0] <= kLimit) || !(pA[1] <= kLimit) || !(pB[0] <= kLimit) || !(pB[1] <= kLimit));
  if (mode == 0 ? __syncthreads_or(bad) : mode == 2) {
    zero_o();
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      mA[qh] = mB[qh] = -INFINITY;
      pA[qh] = pB[qh] = 0.f;
    }
    for (int t = 0; t < ntiles; ++t) {
      __syncthreads();  // every wave is done with the previous tile
      dma_k(sK, t * ktile_b);
      dma_v(sV, t * vtile_b);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        const int qf0 = qw + 32 * blk;  // the block's first query (wave-uniform)
        if (CAUSAL && (qf0 + 31 < t * kBK || qf0 >= N)) continue;  // all masked / past N
        Blk6 S;
        f32x2 acc[2] = {f32x2{0.f, 0.f}, f32x2{0.f, 0.f}};
        Pf6 plo, phi, dpf;
        const float z[2] = {0.f, 0.f};
        qk6<false, false>(sK, ko, blk ? qfB : qfA, S, ci0, S, 0, c2, z, acc, dpf);
        if (RGM && t * kBK + kBK > Nk) {
#pragma unroll
          for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int qh = 0; qh < 2; ++qh)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (t * kBK + 16 * kb + 4 * g + r >= Nk) S.s[kb][qh][r] = -INFINITY;
        }
        if (CAUSAL && t * kBK + kBK - 1 > qf0) {
#pragma unroll
          for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int qh = 0; qh < 2; ++qh)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (t * kBK + 16 * kb + 4 * g + r > qf0 + 16 * qh + i16) S.s[kb][qh][r] = -INFINITY;
        }
        float(&m)[2] = blk ? mB : mA;
        float(&l)[2] = blk ? pB : pA;
        f32x4(&O)[4][2] = blk ? OB : OA;
        float nmc[2];
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          const float tmax = quad_max(lane_max6(S, qh));
          if (__builtin_amdgcn_ballot_w64((tmax - m[qh]) * c2e > kThr)) {
            const float m_new = fmaxf(m[qh], tmax);
            const float alpha = m[qh] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m[qh] - m_new) * c2e);
            m[qh] = m_new;
#pragma unroll
            for (int db = 0; db < 4; ++db) O[db][qh] *= alpha;
            l[qh] *= alpha;
          }
          nmc[qh] = -(m[qh] * c2e);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) sm6_fin(sm6_exp<false>(S, 0, i, c2e, nmc), i, acc, plo);
#pragma unroll
        for (int i = 0; i < 8; ++i) sm6_fin(sm6_exp<false>(S, 1, i, c2e, nmc), i, acc, phi);
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) l[qh] += acc[qh][0] + acc[qh][1];
        f32x2 d2[2];
        f32x4 dR[2];
        pv6<false, 0, false>(sV, vo, O, plo, phi, S, 0, c2, nmc, d2, dpf, vk, dR);
      }
    }
  }
  if (SPLIT) {  // merge the second half's (m, row-sum share, O) into the first half's
    __syncthreads();  // every wave is done with its half's LDS tiles
    float4* xch = (float4*)smem_raw + wq * 18 * 64 + lane;
    if (half) {
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          const f32x4 a = OA[db][qh], o = OB[db][qh];
          xch[(2 * db + qh) * 64] = make_float4(a[0], a[1], a[2], a[3]);
          xch[(8 + 2 * db + qh) * 64] = make_float4(o[0], o[1], o[2], o[3]);
        }
      xch[16 * 64] = make_float4(mA[0], mA[1], mB[0], mB[1]);
      xch[17 * 64] = make_float4(pA[0], pA[1], pB[0], pB[1]);
    }
    __syncthreads();
    if (half) return false;  // (non-causal only: one block per workgroup)
    const float4 tm = xch[16 * 64], tp = xch[17 * 64];
    const float om[4] = {tm.x, tm.y, tm.z, tm.w}, op[4] = {tp.x, tp.y, tp.z, tp.w};
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        float& m = blk ? mB[qh] : mA[qh];
        float& l = blk ? pB[qh] : pA[qh];
        const float n = fmaxf(m, om[2 * blk + qh]);
        const float a0 = __builtin_amdgcn_exp2f((m - n) * c2e), a1 = __builtin_amdgcn_exp2f((om[2 * blk + qh] - n) * c2e);
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          const float4 u = xch[((blk ? 8 : 0) + 2 * db + qh) * 64];
          f32x4& o = (blk ? OB : OA)[db][qh];
          o = o * a0 + f32x4{u.x, u.y, u.z, u.w} * a1;
        }
        l = l * a0 + op[2 * blk + qh] * a1;
        m = n;
      }
  }

  // ---- epilogue ------------------------------------------------------------------------
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      const int q = qw + 32 * blk + 16 * qh + i16;
      const float l = quad_sum(blk ? pB[qh] : pA[qh]);
      const float m = blk ? mB[qh] : mA[qh];
      const float inv = 1.f / l;
      const f32x4(&O)[4][2] = blk ? OB : OA;
      if (V6ABL & 16) {  // timing-only: no O stores (kept live through an improbable store)
        float t = 0.f;
#pragma unroll
        for (int db = 0; db < 4; ++db) t += O[db][qh][0] * inv + O[db][qh][1] + O[db][qh][2] + O[db][qh][3];
        if (t == 1.2345e-30f) p.l[0] = t;
        if (q < N && g == 0) {
          const int64_t row = (int64_t)bh * N + q;
          if (p.m) p.m[row] = m * p.scale;
          if (p.l) p.l[row] = l;
        }
        continue;
      }
      if (WIDE && !p.o_f32) {
        // Widened store (cdna_hip_programming.md T21): lane (i, g) holds d 16db + 4g .. + 3;
        // one v_permlane16_swap per dword pairs the 16-lane rows g, g + 1 (even g keeps d block
        // 2k and takes its partner's next four d, odd g the same for block 2k + 1), so every
        // lane stores 16 contiguous bytes: 4 dwordx4 instead of 8 dwordx2 per query half.
        bf16* Ob = (bf16*)p.out + b * p.so[0] + hh * p.so[1] + (int64_t)min(q, N - 1) * p.so[2];
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const f32x4 &x = O[2 * k][qh], &y = O[2 * k + 1][qh];
          const uint2 ux = __builtin_bit_cast(uint2, bf16x4{(bf16)(x[0] * inv), (bf16)(x[1] * inv), (bf16)(x[2] * inv), (bf16)(x[3] * inv)});
          const uint2 uy = __builtin_bit_cast(uint2, bf16x4{(bf16)(y[0] * inv), (bf16)(y[1] * inv), (bf16)(y[2] * inv), (bf16)(y[3] * inv)});
          const auto rx = __builtin_amdgcn_permlane16_swap(ux.x, uy.x, false, false);
          const auto ry = __builtin_amdgcn_permlane16_swap(ux.y, uy.y, false, false);
          if (q < N) {
            u32x4* dst = (u32x4*)(Ob + 32 * k + 16 * (g & 1) + 4 * (g & 2));
            const u32x4 val = {rx[0], ry[0], rx[1], ry[1]};
            if (V6NT) __builtin_nontemporal_store(val, dst);
            else *dst = val;
          }
        }
      }
      if (q < N) {
        const ORow Og = o_row(p, b, hh, q);
        if (V6NT && p.o_f32) {
#pragma unroll
          for (int db = 0; db < 4; ++db)
            __builtin_nontemporal_store(f32x4{O[db][qh][0] * inv, O[db][qh][1] * inv, O[db][qh][2] * inv,
                                              O[db][qh][3] * inv}, (f32x4*)((float*)Og.p + 16 * db + 4 * g));
        } else if (!WIDE || p.o_f32) {
#pragma unroll
          for (int db = 0; db < 4; ++db)
            store4(Og, 16 * db + 4 * g, O[db][qh][0] * inv, O[db][qh][1] * inv, O[db][qh][2] * inv,
                   O[db][qh][3] * inv);
        }
        if (g == 0) {
          const int64_t row = (int64_t)bh * N + q;
          if (p.m) p.m[row] = m * (PS ? p.scale / c2 : p.scale);
          if (p.l) p.l[row] = l;
        }
      }
    }
  }
  return bad;
  };  // run_block

  if (DUAL) {  // this half's pair (the launcher guarantees nqb % 4 == 0: light != heavy)
    const int light = 2 * qb + half, heavy = nqb - 1 - light;
    bool bad = run_block(light * BQ, 1);
    __syncthreads();
    bad = run_block(heavy * BQ, 1) || bad;
    // both halves arrive here after the same number of barriers; a row sum past 2^64 in
    // either sends both halves through the serial pass of both their blocks (equal barrier
    // counts again), which rewrites O, m and l
    if (__syncthreads_or(bad)) {
      run_block(light * BQ, 2);
      __syncthreads();
      run_block(heavy * BQ, 2);
    }
  } else if (CAUSAL) {  // the light query block first, then the heavy one of the same head
    const int heavy = nqb - 1 - qb;
    run_block(qb * BQ, 0);
    if (heavy != qb) {
      __syncthreads();  // every wave is done with the light block's LDS tiles
      run_block(heavy * BQ, 0);
    }
  } else {
    run_block(qb * BQ, 0);
  }
}

// d = 64, N % 64 == 0, N >= 128, causal only with VAR 32 (split keys: N % 128 == 0, N >= 256, so each
// half walks two whole tiles or more), every per-head K/V offset (two tiles past N) inside
// the 31-bit buffer range.
hipError_t launch_fwd_v6(const AttnArgs& a, bool causal, int var, hipStream_t st, bool* handled) {
  *handled = false;
  // diagnostics (launch bit 1 << 20): the workgroup's LDS padded to 96 KiB, so one workgroup
  // fits a CU: with W4 that is one wave per SIMD (round 6 A/B of the one-wave form)
  const bool one_wg = (var & (1 << 20)) != 0;
  var &= ~(1 << 20);
  const bool split = (var & 16) != 0;  // (var & 64: the widened epilogue stores)
  const bool dual = (var & 256) != 0;   // causal, two 4-wave halves with a pair each
  const bool rg = (var & 65536) != 0;  // any N >= 128
  if (causal != ((var & 32) != 0) || a.d != 64 || (!rg && a.N % kBK != 0) || a.N < 2 * kBK) return hipSuccess;
  if (split && (a.N % (2 * kBK) != 0 || a.N < 4 * kBK)) return hipSuccess;
  if (dual && a.N % (4 * kBQ / 2) != 0) return hipSuccess;  // whole pairs of 256-query blocks per half
  const int64_t lim = (int64_t)1 << 31;
  if (((int64_t)a.N + 2 * kBK) * a.sk[2] * 2 >= lim || ((int64_t)a.N + 2 * kBK) * a.sv[2] * 2 >= lim)
    return hipSuccess;
  *handled = true;
  const size_t smem = (size_t)(split || dual ? 2 : 1) * (kKSlots + (var & 512 ? 4 : kVSlots)) * TILE * sizeof(bf16);
  void (*kern)(AttnArgs, int) = nullptr;
  switch (var) {  // product build: the defaults 16450 / 66 / 18 / 98 / 610 / 16482; the rest are A/B policies
    case 66: kern = fa_fwd_bf16_v6<66>; break;
    case 18: kern = fa_fwd_bf16_v6<18>; break;
    case 98: kern = fa_fwd_bf16_v6<98>; break;
    case 610: kern = fa_fwd_bf16_v6<610>; break;  // 98 with fp16 PV (the fp32-output causal default)
    case 16482: kern = fa_fwd_bf16_v6<16482>; break;  // 98 with 4-wave workgroups (the causal default)
    case 16450: kern = fa_fwd_bf16_v6<16450>; break;  // 66 with 4-wave workgroups (the non-causal default, round 6)
    case 65602: kern = fa_fwd_bf16_v6<65602>; break;  // 66 for any N (the non-causal default for N % 64 != 0)
    case 65634: kern = fa_fwd_bf16_v6<65634>; break;  // 98 for any N
    case 82018: kern = fa_fwd_bf16_v6<82018>; break;  // 16482 for any N (the causal default for N % 64 != 0)
#ifdef MT_DIAGNOSTICS
    case 354: kern = fa_fwd_bf16_v6<354>; break;
    case 1090: kern = fa_fwd_bf16_v6<1090>; break;  // 66 with stamps
    case 2114: kern = fa_fwd_bf16_v6<2114>; break;  // 66 with the tile's DMA by waves 0-3
    case 3138: kern = fa_fwd_bf16_v6<3138>; break;  // 2114 with stamps
    case 4162: kern = fa_fwd_bf16_v6<4162>; break;  // 66, waves 4-7 at priority 1 for P1-P2
    case 8258: kern = fa_fwd_bf16_v6<8258>; break;  // 66, waves 4-7 at priority 1 for P1
    case 5186: kern = fa_fwd_bf16_v6<5186>; break;  // 4162 with stamps
    case 32834: kern = fa_fwd_bf16_v6<32834>; break;  // 66 with packed scale-and-shift
    case 102: kern = fa_fwd_bf16_v6<102>; break;  // 98 without the Vᵀ reuse (32 VGPRs fewer)
    case 16994: kern = fa_fwd_bf16_v6<16994>; break;  // 610 with 4-wave workgroups
    case 16486: kern = fa_fwd_bf16_v6<16486>; break;  // 16482 without the Vᵀ reuse
    case 16998: kern = fa_fwd_bf16_v6<16998>; break;  // 16994 without the Vᵀ reuse
    case 614: kern = fa_fwd_bf16_v6<614>; break;  // 610 without the Vᵀ reuse
    case 194: kern = fa_fwd_bf16_v6<194>; break;
    case 2: kern = fa_fwd_bf16_v6<2>; break;
    case 34: kern = fa_fwd_bf16_v6<34>; break;
    case 82: kern = fa_fwd_bf16_v6<82>; break;
    case 0: kern = fa_fwd_bf16_v6<0>; break;
    case 6: kern = fa_fwd_bf16_v6<6>; break;
    case 10: kern = fa_fwd_bf16_v6<10>; break;
    case 1: kern = fa_fwd_bf16_v6<1>; break;
#endif
    default: return hipErrorInvalidValue;
  }
  const size_t smem_launch = one_wg && smem < 96 * 1024 ? (size_t)96 * 1024 : smem;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem_launch);
  if (e != hipSuccess) return e;
  const bool w4 = (var & 16384) != 0;
  const int bq = split || dual || w4 ? kBQ / 2 : kBQ;
  const int nqb = (a.N + bq - 1) / bq;
  const int64_t nblk = (int64_t)(dual ? nqb / 4 : causal ? (nqb + 1) / 2 : nqb) * a.B * a.H;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(w4 ? 32 * kNW : 64 * kNW), smem_launch, st, a, nqb);
  return hipGetLastError();
}

}  // namespace mt
