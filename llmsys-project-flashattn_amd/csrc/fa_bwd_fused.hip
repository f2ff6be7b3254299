// FlashAttention backward with dQ folded into the dK/dV pass: bf16 I/O, head dim 64.
//
// The split backward (fa_bwd_bf16.hip) runs dK/dV and dQ as two kernels, so the dQ pass
// recomputes S = Q·Kᵀ and dP = dO·Vᵀ: 7 matrix products where the algorithm needs 5. Here
// one pass computes all five, as the reference's backward_kernel does
// (src/flashattention_kernel.cu:115-255; it accumulates dQ in HBM at :228-235):
//     P = exp2(c2·S'),  dV += Pᵀ·dO,  dS = P ∘ dP',  dK += dSᵀ·Q,  dQ += dS·K
// (S' and dP' start from the row constants −lse2/c2 and −δ, see fa_bwd_prep_bf16).
//
// Workgroup = 8 waves = 256 keys, a wave owns 32 keys (K, V rows as register-resident B
// operands, the dKᵀ/dVᵀ accumulators), exactly like the split kernel's dK/dV pass. Step t =
// 64 queries (two 32-query sub-tiles), staged by LDS-DMA one step ahead into a two-slot ring,
// one barrier per step. dQ needs a sum over the key, which is the lane index of the S/dP
// accumulators, so dS crosses LDS once:
//  * every wave writes its bf16 dS (32 keys x 64 queries of the step) into a [key][query]
//    image (double-buffered by step parity);
//  * in step t + 1 every wave computes its 16-query x 32-d strip of dQᵀ(step t) = Kᵀ·dSᵀ
//    over the workgroup's 256 keys (two 16x16x32 MFMA tiles, 8 k-steps of 32 keys: 16
//    MFMAs, a quarter of the wave's step), interleaved with its dK/dV sub-tiles in the same
//    basic block, from the dS image and a K image [key][d] written once at the start, both
//    read with ds_read_b64_tr_b16;
//  * the strip is a partial sum over this workgroup's keys: it goes to a bf16 slab
//    [bh][step][key block][wave][lane][8] in the accumulator's own register order (one 16-B
//    store per lane, sc1: written through, not held in this XCD's L2);
//  * the last workgroup to finish a (head, query step) sums that step's partials and writes
//    dQ, inside this launch (round 4; round 3 ran a separate reduce kernel over the whole
//    slab, ≈ 170 µs at C3). The hand-off is MI355X_MICROARCH.md 'Valid forms' row 1: every
//    storing wave waits for its partial store, the workgroup barrier follows, then one lane
//    adds 1 to the step's arrival counter (agent scope) and the add's return value names the
//    last arriver, which reads the partials with sc1 loads. Every sum runs in key-block
//    order in f32 (deterministic, the round-3 reduce's arithmetic), and no workgroup ever
//    waits for another (no spin, so no co-residency assumption). The adds are issued a step
//    late and their return values read a step later still, by when they have long returned;
//    a workgroup that turns out last for some steps reduces them after its pass (their
//    partials are then fresh in the Infinity Cache). The key blocks of a head walk the query
//    steps in rotated orders (VAR 32), so each is last for about nstep / nkb steps: walked in
//    one order, the head's slowest block was last almost everywhere and reduced the whole
//    head alone after its pass (1.77 ms at C3 against 1.48 rotated).
//    That form is the non-causal default; causal and masked heads (ragged N, kv_len) keep
//    the round-3 hand-off (plain partial stores, fa_bwd_dq_reduce after the pass), which the
//    in-kernel forms did not beat there (profiles/r4_ab_fused_forms.txt).
// Why slabs and not float atomics: at 256 keys per workgroup dQ is summed over N/256
// workgroups, 2.1 GB of f32 adds at C3, whose floor at the chip's ≈1.3 TB/s atomic rate
// (MI355X_MICROARCH.md, Global float atomics) is 1.65 ms, longer than the whole split
// backward. A bf16 partial adds one rounding of 2^-9 of the partial, inside tests/bounds.py's
// 2^-7 (three roundings: dS, partial, output). The slab of one launch is capped at
// kSlabCap; longer sequences and bigger batches run the pass over groups of heads.
//
// LDS images are single copies read both by rows (ds_read_b128: the A operands of S, dP)
// and by columns (ds_read_b64_tr_b16: dVᵀ, dKᵀ, dQᵀ), with the chunk swizzle
// c ^ f(r), f(r) = x ^ ((x & 1) << 2), x = (r >> 1) & 7: f takes 8 distinct values on the
// same-parity rows of every ds_read_b128 lane group (row reads conflict-free), and bit 2 of
// f flips between rows 4m, 4m+1 and 4m+2, 4m+3 (transposed reads conflict-free); f(r + 8) =
// f(r) ^ 4, so the transposed read of rows +8 takes its own offset (tlo / thi).
#include "fa_bwd_bf16.h"

#include <algorithm>

// Timing-only ablations of the pass (WRONG results by construction), built into separate A/B
// libraries with -DBWDABL=n (scripts/build_abl.sh fa_bwd_fused BWDABL n), never into the
// product: 1 no dQ strips (their operand reads and MFMAs), 2 no exponentials, 4 the dQ strips'
// second K fragment read taken from another k-step's first, 8 the dVᵀ / dKᵀ transposed
// fragments of k-step 1 taken from k-step 0, 16 no step barrier in the walk, 32 no Q / dO
// staging in the walk (profiles/r5_abl_bwd.txt).
#ifndef BWDABL
#define BWDABL 0
#endif


namespace mt {

using namespace bwdbf16;

namespace {
constexpr int kQT = 32;                             // queries per sub-tile
constexpr int kStep = 64;                           // queries per barrier step
constexpr int kKB = 256;                            // keys per workgroup
constexpr int kImg = kQT * D;                       // elements of one sub-tile image
constexpr int kSub = 2 * kImg * 2 + 2 * kQT * 4;    // bytes: Q image, dO image, row constants
constexpr int kRingB = 4 * kSub;                    // 2 slots x 2 sub-tiles
constexpr int kKImgB = kKB * D * 2;                 // K image [256][64]
constexpr int kDsB = kKB * kStep * 2;               // dS image [256][64]
constexpr int kSmemFused = kRingB + kKImgB + 2 * kDsB;
constexpr int kMaxRed = 1024;                       // query steps (of 64) a pass can own: N <= 65536
constexpr int kSmemAll = kSmemFused + (kMaxRed + 4) * 4;  // + the pass's list of steps to reduce
static_assert(kSmemAll <= 160 * 1024, "LDS budget");
constexpr int kSc1 = 16;                            // buffer cache policy bits: sc1
constexpr int64_t kSlabCap = (int64_t)1 << 30;      // dQ partial bytes per launch (C3: exactly 1 GiB)
// the product's dQ hand-off forms (the kernel's VAR; same-box A/B of every form at C3,
// profiles/r4_ab_fused_forms.txt): non-causal with mask-free heads (N % 64 == 0, no kv_len) the
// rotated walks with the in-kernel reduce (32), everything else the round-3 form (16: plain
// partial stores and the ordered reduce kernel after the pass)
constexpr int kFormRot = 32, kFormR3 = 16;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
static_assert(kSub % 16 == 0, "16-B aligned sub-tiles");

__device__ __forceinline__ int swf(int r) {
  const int x = (r >> 1) & 7;
  return x ^ ((x & 1) << 2);
}
__device__ __forceinline__ int sw(int r, int c) { return r * D + ((c ^ swf(r)) << 3); }

struct FCtx {
  bf16x8 kf[4], vf[4];   // B operands: K / V rows of this lane's key
  int roff[4];           // row reads: row c32, chunk 2ks + hf
  int tlo[2], thi[2];    // transposed reads of column block db: rows 4hf.. / 8 + 4hf..
};

// Transposed fragment (ds_read_b64_tr_b16 x 2) of rows row0 + {0..15 in the accumulator
// k order}, row0 a multiple of 16.
__device__ __forceinline__ bf16x8 trf(const bf16* img, int row0, int lo, int hi) {
  const bf16* a = img + row0 * D;
  const s16x4 l = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + lo));
  const s16x4 h = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + hi));
  const s16x8 v = {l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ void tr_offsets(int lane, int db, int& lo, int& hi) {
  const int hf = lane >> 5, i16 = lane & 15, g = (lane >> 4) & 1;
  const int col = db * 32 + 16 * g + 4 * (i16 & 3), row = 4 * hf + (i16 >> 2);
  lo = sw(row, col >> 3) + (col & 7);
  hi = sw(row + 8, col >> 3) + (col & 7);
}

// One 32-query sub-tile u of the step: S, dP, P, dS, dVᵀ, dKᵀ, and dS into the dS image.
// MASK: queries past N, keys at or past Nk (N, or the batch row's kv_len) and, causal,
// keys after the query get p = 0; a workgroup whose block holds a key >= Nk runs every step
// masked.
// Unmasked tiles issue operand reads a phase ahead of their MFMAs (the row fragments of S
// and dP before the first of those products, the transposed fragments of dVᵀ and dKᵀ right
// after them, so they land during the softmax), fenced by sched_barrier: left to itself
// hipcc issues each MFMA's reads right before it and waits lgkmcnt(0), which serialises the
// LDS latency into every product. Masked tiles (causal diagonal, ragged tail, padding) read
// at use: the mask's registers on top of sixteen live fragments spill.
template <bool CAUSAL, bool MASK, bool PF, bool PKM = false>
__device__ __forceinline__ void fdkv_tile(const char* sub, const FCtx& c, f32x16 (&dK)[2],
                                          f32x16 (&dV)[2], float c2, int qt, int N, int Nk,
                                          int my_k, int hf, bf16* dsrow, int fk, int u) {
  const bf16* Qi = (const bf16*)sub;
  const bf16* Oi = Qi + kImg;
  const float* nl = (const float*)(Qi + 2 * kImg);
  const float* nd = nl + kQT;
  bf16x8 aq[4], ao[4];
  if (PF) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      aq[ks] = *(const bf16x8*)(Qi + c.roff[ks]);
      ao[ks] = *(const bf16x8*)(Oi + c.roff[ks]);
    }
  }
  f32x16 S, dP;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 a = *(const float4*)(nl + 8 * g + 4 * hf);
    const float4 e = *(const float4*)(nd + 8 * g + 4 * hf);
    S[4 * g] = a.x; S[4 * g + 1] = a.y; S[4 * g + 2] = a.z; S[4 * g + 3] = a.w;
    dP[4 * g] = e.x; dP[4 * g + 1] = e.y; dP[4 * g + 2] = e.z; dP[4 * g + 3] = e.w;
  }
  if (PF) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(!PF ? *(const bf16x8*)(Qi + c.roff[ks]) : aq[ks],
                                                c.kf[ks], S, 0, 0, 0);
    dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(!PF ? *(const bf16x8*)(Oi + c.roff[ks]) : ao[ks],
                                                 c.vf[ks], dP, 0, 0, 0);
  }
  bf16x8 tv[2][2], tk[2][2];  // [s][db]: dOᵀ and Qᵀ fragments of dVᵀ and dKᵀ
  if (PF) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        tv[s][db] = ((BWDABL & 8) && s) ? tv[0][db] : trf(Oi, 16 * s, c.tlo[db], c.thi[db]);
        tk[s][db] = ((BWDABL & 8) && s) ? tk[0][db] : trf(Qi, 16 * s, c.tlo[db], c.thi[db]);
      }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (MASK) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = qt + acc_row(r, hf);
      if (q >= N || my_k >= Nk || (CAUSAL && my_k > q)) S[r] = -INFINITY;
    }
  }
  if (PKM) {  // diagnostics (VAR 64): the scale and the dS product as v_pk_mul_f32 pairs
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const f32x2 x = f32x2{S[r], S[r + 1]} * f32x2{c2, c2};
      const f32x2 pv = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
      const f32x2 ds = pv * f32x2{dP[r], dP[r + 1]};
      S[r] = pv[0]; S[r + 1] = pv[1];
      dP[r] = ds[0]; dP[r + 1] = ds[1];
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pv = (BWDABL & 2) ? S[r] * c2 : __builtin_amdgcn_exp2f(S[r] * c2);
      S[r] = pv;
      dP[r] = pv * dP[r];
    }
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const bf16x8 pf = to_bf16x8(S, s);
    const bf16x8 sf = to_bf16x8(dP, s);
    // dS rows of this lane's key: queries 32u + 16s + 4hf + 0..3 and + 8 (chunks 4u + 2s, +1)
    const uint4 w = __builtin_bit_cast(uint4, sf);
    *(uint2*)(dsrow + (((4 * u + 2 * s) ^ fk) << 3) + 4 * hf) = make_uint2(w.x, w.y);
    *(uint2*)(dsrow + (((4 * u + 2 * s + 1) ^ fk) << 3) + 4 * hf) = make_uint2(w.z, w.w);
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      dV[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(!PF ? trf(Oi, 16 * s, c.tlo[db], c.thi[db]) : tv[s][db],
                                                       pf, dV[db], 0, 0, 0);
      dK[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(!PF ? trf(Qi, 16 * s, c.tlo[db], c.thi[db]) : tk[s][db],
                                                       sf, dK[db], 0, 0, 0);
    }
  }
}

// dQ operands of a 16x16x32 MFMA from a [key][64] image: lane group G = l >> 4 supplies the
// keys 4G + 0..3 (read 1) and 16 + 4G + 0..3 (read 2) of a 32-key step, the same k order
// for the Kᵀ (A) and dSᵀ (B) fragments; lane l & 15 = column. Within a 32-lane half the
// rows of one read are 8 consecutive rows, on which f is a bijection: conflict-free.
__device__ __forceinline__ int dq_off(int lane, int col0) {
  const int G = lane >> 4, i16 = lane & 15;
  const int col = col0 + 4 * (i16 & 3);
  return sw(4 * G + (i16 >> 2), col >> 3) + (col & 7);
}
__device__ __forceinline__ bf16x8 dq_frag(const bf16* p) {
  const s16x4 l = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
  const s16x4 h = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 16 * D));
  const s16x8 v = {l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
  return __builtin_bit_cast(bf16x8, v);
}
typedef __attribute__((ext_vector_type(4))) float f32x4;
// k-steps [s0, s1) (32 keys each) of this wave's dQᵀ strip: d 32·d32 + 16t + .., q 16·q16 + ..
// All the range's operand reads first (fenced), then the MFMAs.
template <int S0, int S1, bool PF = true>
__device__ __forceinline__ void dq_ksteps(const bf16* kimg, const bf16* si, int oa0, int oa1, int ob,
                                          f32x4 (&acc)[2]) {
  if (BWDABL & 1) return;
  if (!PF) {
#pragma unroll
    for (int s = S0; s < S1; ++s) {
      const bf16x8 bq = dq_frag(si + 32 * s * kStep + ob);
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dq_frag(kimg + 32 * s * D + oa0), bq, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dq_frag(kimg + 32 * s * D + oa1), bq, acc[1], 0, 0, 0);
    }
    return;
  }
  bf16x8 a0[S1 - S0], a1[S1 - S0], bq[S1 - S0];
#pragma unroll
  for (int s = S0; s < S1; ++s) {
    bq[s - S0] = dq_frag(si + 32 * s * kStep + ob);
    a0[s - S0] = dq_frag(kimg + 32 * s * D + oa0);
    if (!(BWDABL & 4)) a1[s - S0] = dq_frag(kimg + 32 * s * D + oa1);
  }
  if (BWDABL & 4) {  // (a rotated copy, so that no two MFMA chains are identical)
#pragma unroll
    for (int s = 0; s < S1 - S0; ++s) a1[s] = a0[(s + 1) % (S1 - S0)];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < S1 - S0; ++s) {
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[s], bq[s], acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[s], bq[s], acc[1], 0, 0, 0);
  }
}
}  // namespace

// grid: (N / 256 key blocks) x the ngrp heads [bh0, bh0 + ngrp), XCD-aware order (one head's
// blocks on one XCD); 512 threads; kSmemAll bytes of LDS. nsa = ceil(N / 64) query steps of the
// whole sequence (the slab's and the counters' step axis). ws_bytes: the arrival counters
// (slab_off bytes) and the group's slab behind them, one buffer resource over both.
// PAIR (causal): a workgroup owns key blocks nkb - 1 - u (light: the fewest query steps) and
// then u (heavy) of one head, so every workgroup walks about nkb + 1 blocks' worth of steps
// (the split kernels' pairing, fa_bwd_bf16.hip); the two blocks are two passes of one body.
// VAR (A/B forms of the dQ hand-off; the product runs 32 or 16, kFormRot): 1 no in-kernel reduction, 2 no
// arrivals (both: wrong dQ, timing only), 4 plain instead of sc1 partial stores, 8 the arrival
// add as a global atomic (its return register is not its data register), 16 the round-3 form
// (plain stores, no arrivals, fa_bwd_dq_reduce after the pass), 32 rotated walks (non-causal,
// no masked steps: key block kb starts its walk over the query steps at kb·nstep/nkb, so the
// blocks of a head pass any given step at evenly spread times and each arrives last at about
// nstep/nkb steps, instead of the head's slowest block arriving last almost everywhere).
template <bool CAUSAL, bool PAIR = false, int VAR = 0>
__global__ __launch_bounds__(512, 2) void fa_bwd_fused_bf16(AttnArgs p, int nkb, int nsa, int bh0,
                                                             int slab_off, int ws_bytes) {
  constexpr bool R3 = VAR & 16;
  constexpr bool NORED = (VAR & 1) || R3, NOARR = (VAR & 2) || R3, PLAIN = (VAR & 4) || R3, GATOM = VAR & 8;
  constexpr bool ROT = VAR & 32;
  constexpr bool PKM = VAR & 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar branches)
  // operand prefetch in the unmasked steps: the dQ strips' (dq_ksteps) in every kernel, the
  // sub-tiles' (fdkv_tile) in the non-causal kernel only: in the causal kernels those extra
  // live fragments spill around the masked head loop (measured: causal 0.991 -> 1.020 ms with
  // it, non-causal 1.643 -> 1.559 ms); the dQ prefetch alone took C3 causal 0.905 -> 0.875 ms
  // (round 5, profiles/r5_ab_bwd_dq.txt)
  constexpr bool kPF = !CAUSAL;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int nslot = PAIR ? (nkb + 1) / 2 : nkb;
  const int bhl = logical / nslot, u_ = logical % nslot;  // head within the group
  const int bh = bh0 + bhl;
  const int b = bh / p.H, hh = bh % p.H;
  // the dQ hand-off: one buffer resource over the arrival counters (atomics) and the group's
  // slab (sc1 stores and loads), and the pass's list of steps this workgroup reduces
  const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(p.dq_cnt, (short)0, ws_bytes, 0x00020000);
  int* const red = (int*)(smem + kSmemFused);  // [0]: count, [1 ..]: query steps
#pragma nounroll
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
  const int kb = PAIR ? (pass == 0 ? nkb - 1 - u_ : u_) : u_;
  if (PAIR && pass == 1) {
    if (kb == nkb - 1 - u_) break;  // odd nkb: the middle block has no partner
    __syncthreads();                 // the first block's last LDS reads are done
  }
  const int k0 = kb * kKB;
  const int krow = wave * 32 + c32;  // this lane's key row in the block
  const int my_k = k0 + krow;
  const int Nk = kv_keys(p, b);      // keys >= Nk are padding (zero dK, dV; no dQ share)
  bf16* kimg = (bf16*)(smem + kRingB);
  bf16* dsimg = (bf16*)(smem + kRingB + kKImgB);
  const int fk = swf(krow);
  bf16* const dsrow0 = dsimg + krow * kStep;  // step parity 0; parity 1 is + kKB * kStep

  FCtx c;
  {
    const bool kval = my_k < Nk;
    const int kr = min(my_k, N - 1);
    const bf16* krp = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1] + (int64_t)kr * p.sk[2];
    const bf16* vrp = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1] + (int64_t)kr * p.sv[2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      c.kf[ks] = *(const bf16x8*)(krp + 16 * ks + 8 * hf);
      c.vf[ks] = *(const bf16x8*)(vrp + 16 * ks + 8 * hf);
      c.roff[ks] = sw(c32, 2 * ks + hf);
      // the K image for dQ (zero rows past N)
      *(bf16x8*)(kimg + sw(krow, 2 * ks + hf)) = kval ? c.kf[ks] : bf16x8{};
    }
    tr_offsets(lane, 0, c.tlo[0], c.thi[0]);
    tr_offsets(lane, 1, c.tlo[1], c.thi[1]);
  }
  // this wave's dQᵀ strip: queries 16·(wave & 3) .., d 32·(wave >> 2) ..
  const int q16 = wave & 3, d32 = wave >> 2;
  const int oa0 = dq_off(lane, 32 * d32), oa1 = dq_off(lane, 32 * d32 + 16), ob = dq_off(lane, 16 * q16);
  // byte offsets in the group's slab: this wave's partial of step s at slab_w + s · slab_step
  const int slab_w = slab_off + ((bhl * nsa * nkb + kb) * 8 + wave) * 1024 + lane * 16;
  const int slab_step = nkb * 8 * 1024;
  const int nkv = (Nk + kKB - 1) / kKB;  // key blocks holding keys that attend

  // LDS-DMA staging: wave w fills rows 8(w & 3) .. + 7 of sub-tile w >> 2's Q and dO images
  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Og = (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const int sqn = (int)p.sq[2], son = (int)p.sdo[2];
  const __amdgpu_buffer_rsrc_t rq = head_rsrc(Qg, N, sqn), ro = head_rsrc(Og, N, son);
  const int wq = wave & 3, wu = wave >> 2;
  const uint32_t lds0 = lds_base(smem) + __builtin_amdgcn_readfirstlane(wq) * 8 * D * 2 +
                        __builtin_amdgcn_readfirstlane(wu) * kSub;
  int gq, go;
  {
    const int r = 8 * wq + (lane >> 3), pc = lane & 7;
    const int cs = pc ^ swf(r);  // the logical chunk that lands in LDS chunk pc
    gq = (r * sqn + cs * 8) * 2;
    go = (r * son + cs * 8) * 2;
  }
  // Row constants of sub-tile wu (its 32 queries' −lse2/c2, then their −δ) by one LDS-DMA
  // instruction of wave 4·wu: lanes 0-31 read lse2, lanes 32-63 δ, both from one buffer over
  // the workspace (δ follows lse2, fused_bwd_applies keeps it under 2^31 bytes); a query past
  // N gets an out-of-range offset, which reads 0.
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.lse2, (short)0, (int)(2 * (int64_t)p.B * p.H * N * 4), 0x00020000);
  const int crow = (lane >= kQT ? p.B * p.H * N : 0) + bh * N;  // + query

  const int qt0 = CAUSAL ? k0 : 0;
  const int step0 = qt0 / kStep;
  // a block of padding keys only (k0 >= Nk) stores zero dK / dV and no dQ partials
  const int nstep = N > qt0 && k0 < Nk ? (N - qt0 + kStep - 1) / kStep : 0;
  // steps: [0, nhead) causal diagonal (masked), [nhead, nfull) mask-free, [nfull, nstep) tail.
  const int nhead = k0 + kKB > Nk ? nstep : CAUSAL ? min(nstep, kKB / kStep) : 0;
  const int nfull = min(nstep, max(nhead, (N - qt0) / kStep));
  // the walk: local step t covers query step step0 + sq(t); rotated where the head has no
  // padding keys and N % 64 == 0: non-causal over all steps, causal over the mask-free steps
  // only (the diagonal steps come first, as the masked head loop needs)
  const int nrot = nfull - nhead;
  const int rot = ROT && N % kStep == 0 && Nk == N && nrot > 1 ? (kb * nrot) / nkb : 0;
  auto sq = [&](int t) __attribute__((always_inline)) {
    if (rot == 0 || t < nhead || t >= nfull) return t;
    const int r = t + rot;
    return r >= nfull ? r - nrot : r;
  };
  auto stage = [&](int t, int slot) __attribute__((always_inline)) {
    const int qs = qt0 + sq(t) * kStep + wu * kQT;
    const uint32_t img = lds0 + slot * 2 * kSub;
    dma_rows(img, rq, gq + qs * sqn * 2);
    dma_rows(img + kImg * 2, ro, go + qs * son * 2);
    if (wq == 0) {
      const int q = qs + (lane & (kQT - 1));
      dma_dwords(img + 2 * kImg * 2, rc, q < N ? (crow + q) * 4 : 0x7ffffff0);  // wq = 0
    }
  };
  // after_store: the step issued its dQ partial store after the staging loads. vmcnt retires
  // in issue order, so vmcnt(1) waits for the staging and leaves that store in flight; a
  // vmcnt(0) here had every step wait for the store's write acknowledgement before the
  // barrier (it was issued a few instructions earlier).
  auto publish = [&](bool after_store) __attribute__((always_inline)) {
    if (after_store) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  auto dq_store = [&](const f32x4 (&acc)[2], int tl) __attribute__((always_inline)) {
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[i] = (bf16)acc[0][i]; o[4 + i] = (bf16)acc[1][i]; }
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rsl, slab_w + (step0 + tl) * slab_step, 0,
                                           PLAIN ? 0 : kSc1);
  };
  // Arrivals (wave 0; the add by lane 0): arrive(s) first settles the previous add, whose
  // return value the caller has waited for (the next step's vmcnt, or settle's own wait at the
  // end), then adds 1 to step s's counter. The contributors of step s are the key blocks below
  // nkv (keys that attend) and, causal, at or before it (4 kb <= s).
  int pend_s = -1, nred = 0;  // wave-uniform
  int pend_old = 0;           // lane 0
  auto settle = [&]() __attribute__((always_inline)) {
    if (pend_s >= 0) {
      const int tgt = CAUSAL ? min(nkv, pend_s / (kKB / kStep) + 1) : nkv;
      if (__builtin_amdgcn_readfirstlane(pend_old) + 1 == tgt) {
        if (lane == 0) red[1 + nred] = pend_s;
        ++nred;
      }
      pend_s = -1;
    }
  };
  auto arrive = [&](int s) __attribute__((always_inline)) {
    if (NOARR) return;
    if (wave == 0) {
      settle();
      if (lane == 0) {
        if (GATOM)
          pend_old = (int)__hip_atomic_fetch_add(p.dq_cnt + (int64_t)bh * nsa + s, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
        else
          pend_old = __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, rsl, (bh * nsa + s) * 4, 0, 0);
      }
      pend_s = s;
    }
  };

  f32x16 dK[2], dV[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) { dK[i] = f32x16{}; dV[i] = f32x16{}; }
  const float c2 = p.scale_log2;

  if (nstep > 0) {
    stage(0, 0);
    publish(false);
  }
  __syncthreads();
  // Step t > 0 also computes the dQ strip of step t - 1 (its dS image, the other parity):
  // half its k-steps before each sub-tile. Masked sub-tiles are computed in full, also when
  // every score of the wave is masked (causal, before the wave's keys; past N): their dS is
  // then exactly zero, as the dS image needs, and a wave-level skip would be a branch around
  // the accumulators (copies and spills in the masked steps).
#define FSUB(MASK_, SLOT_, T_, U_)                                                       \
  {                                                                                      \
    const int qt_ = qt0 + sq(T_) * kStep + (U_) * kQT;                                   \
    bf16* dsr_ = dsrow0 + (SLOT_) * (kKB * kStep);                                       \
    fdkv_tile<CAUSAL, MASK_, kPF && !(MASK_), PKM>(smem + (2 * (SLOT_) + (U_)) * kSub, c, dK, dV, c2, qt_, N,  \
                             Nk, my_k, hf, dsr_, fk, U_);                                \
  }
#define FSTEP(MASK_, SLOT_, T_, DQ_)                                                     \
  {                                                                                      \
    const int t_ = (T_);                                                                 \
    const bool more_ = t_ + 1 < nstep;                                                   \
    if (more_ && !(BWDABL & 32)) stage(t_ + 1, (SLOT_) ^ 1);                             \
    f32x4 qa_[2] = {f32x4{}, f32x4{}};                                                   \
    const bf16* si_ = dsimg + ((SLOT_) ^ 1) * (kKB * kStep);                             \
    if (DQ_) dq_ksteps<0, 4, !(MASK_)>(kimg, si_, oa0, oa1, ob, qa_);                     \
    FSUB(MASK_, SLOT_, t_, 0)                                                            \
    if (DQ_) dq_ksteps<4, 8, !(MASK_)>(kimg, si_, oa0, oa1, ob, qa_);                     \
    FSUB(MASK_, SLOT_, t_, 1)                                                            \
    if (DQ_) dq_store(qa_, sq(t_ - 1));                                                  \
    if (more_ || (DQ_)) publish(DQ_);  /* DQ_: the store of step t - 2 has completed */  \
    if (!(BWDABL & 16)) __syncthreads();                                                 \
    if (t_ >= 2) arrive(step0 + sq(t_ - 2));                                             \
  }
  if (nstep > 0) {
    if (nhead > 0 || nfull == 0) FSTEP(true, 0, 0, false) else FSTEP(false, 0, 0, false)
  }
  int t = 1;
  for (; t < nhead; ++t) {
    if (t & 1) FSTEP(true, 1, t, true) else FSTEP(true, 0, t, true)
  }
  if ((t & 1) && t < nfull) {
    FSTEP(false, 1, t, true)
    ++t;
  }
  for (; t + 1 < nfull; t += 2) {
    FSTEP(false, 0, t, true)
    FSTEP(false, 1, t + 1, true)
  }
  for (; t < nstep; ++t) {
    if (t < nfull) {
      if (t & 1) FSTEP(false, 1, t, true) else FSTEP(false, 0, t, true)
    } else {
      if (t & 1) FSTEP(true, 1, t, true) else FSTEP(true, 0, t, true)
    }
  }
#undef FSTEP
#undef FSUB
  if (nstep > 0) {  // the last step's dQ strip
    f32x4 qa[2] = {f32x4{}, f32x4{}};
    dq_ksteps<0, 4>(kimg, dsimg + ((nstep - 1) & 1) * (kKB * kStep), oa0, oa1, ob, qa);
    dq_ksteps<4, 8>(kimg, dsimg + ((nstep - 1) & 1) * (kKB * kStep), oa0, oa1, ob, qa);
    dq_store(qa, sq(nstep - 1));
  }
  // the last two steps' arrivals: every wave's stores complete, the barrier, the adds
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nstep >= 2) arrive(step0 + sq(nstep - 2));
  if (nstep >= 1) arrive(step0 + sq(nstep - 1));
  if (wave == 0) {
    settle();
    if (lane == 0) red[0] = nred;
  }

  if (my_k < N) {
    bf16* dKg = (bf16*)p.dk + b * p.sdk[0] + hh * p.sdk[1] + (int64_t)my_k * p.sdk[2];
    bf16* dVg = (bf16*)p.dv + b * p.sdv[0] + hh * p.sdv[1] + (int64_t)my_k * p.sdv[2];
    const float sc = p.scale;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = db * 32 + 8 * g + 4 * hf;
        store4(dKg + col, dK[db][4 * g] * sc, dK[db][4 * g + 1] * sc, dK[db][4 * g + 2] * sc,
               dK[db][4 * g + 3] * sc, true);
        store4(dVg + col, dV[db][4 * g], dV[db][4 * g + 1], dV[db][4 * g + 2], dV[db][4 * g + 3], true);
      }
  }

  // dQ of the steps this workgroup arrived last at: wave w sums its strip's partials over the
  // step's contributing key blocks in key-block order (fp32, one rounding at the end: the
  // round-3 reduce kernel's arithmetic), from sc1 loads, eight 16-B loads in flight per lane.
  // Lane l holds d = 32 (w >> 2) + 4 (l >> 4) + 0..3 (+ 16) of query 64 s + 16 (w & 3) + (l & 15).
  __syncthreads();  // red[] is written
  const int nr = NORED ? 0 : red[0];
  bf16* const dQh = (bf16*)p.dq + b * p.sdq[0] + hh * p.sdq[1] + 32 * (wave >> 2) + 4 * (lane >> 4);
  const float sc = p.scale;
  for (int i = 0; i < nr; ++i) {
    const int st = red[1 + i];
    const int nk = CAUSAL ? min(nkv, st / (kKB / kStep) + 1) : nkv;
    const int src = slab_off + ((bhl * nsa + st) * nkb * 8 + wave) * 1024 + lane * 16;
    float a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = 0.f;
    int k = 0;
    for (; k + 16 <= nk; k += 16) {  // sixteen 16-B loads in flight per lane (the pass's registers are free here)
      u32x4 x[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) x[u] = __builtin_amdgcn_raw_buffer_load_b128(rsl, src + (k + u) * 8192, 0, kSc1);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const bf16x8 y = __builtin_bit_cast(bf16x8, x[u]);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += (float)y[j];
      }
    }
    for (; k + 8 <= nk; k += 8) {
      u32x4 x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = __builtin_amdgcn_raw_buffer_load_b128(rsl, src + (k + u) * 8192, 0, kSc1);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bf16x8 y = __builtin_bit_cast(bf16x8, x[u]);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += (float)y[j];
      }
    }
    for (; k < nk; ++k) {
      const bf16x8 y = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsl, src + k * 8192, 0, kSc1));
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += (float)y[j];
    }
    const int q = st * kStep + 16 * (wave & 3) + (lane & 15);
    if (q < N) {
      bf16* dst = dQh + (int64_t)q * p.sdq[2];
      store4(dst, a[0] * sc, a[1] * sc, a[2] * sc, a[3] * sc, true);
      store4(dst + 16, a[4] * sc, a[5] * sc, a[6] * sc, a[7] * sc, true);
    }
  }
  // a head whose keys are all padding (kv_len = 0): nothing arrives, its dQ is zero
  if (!R3 && nkv == 0 && kb == 0) {
    bf16* dQz = (bf16*)p.dq + b * p.sdq[0] + hh * p.sdq[1];
    for (int r = tid >> 3; r < N; r += 64) *(uint4*)(dQz + (int64_t)r * p.sdq[2] + 8 * (tid & 7)) = uint4{0, 0, 0, 0};
  }
  }  // pass
}

// The round-3 reduce (VAR 16): dQ = scale · Σ_kb slab[bh][step][kb] in key-block order, one wave
// per (bh, step, strip w), after the pass; the slab of the launch's heads, offsets as above.
__global__ __launch_bounds__(256) void fa_bwd_dq_reduce(AttnArgs p, int nkb, int nsa, int bh0, int ngrp,
                                                        int slab_off, int ws_bytes, int causal) {
  const int lane = threadIdx.x & 63;
  const int64_t unit = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (unit >= (int64_t)ngrp * nsa * 8) return;
  const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(p.dq_cnt, (short)0, ws_bytes, 0x00020000);
  const int w = (int)(unit & 7);
  const int64_t bs = unit >> 3;
  const int s = (int)(bs % nsa);
  const int bhl = (int)(bs / nsa), bh = bh0 + bhl;
  const int q = s * kStep + 16 * (w & 3) + (lane & 15);
  const int nkv = (kv_keys(p, bh / p.H) + kKB - 1) / kKB;
  const int nk = min(nkv, causal ? min(nkb, s / (kKB / kStep) + 1) : nkb);
  const int src = slab_off + ((bhl * nsa + s) * nkb * 8 + w) * 1024 + lane * 16;
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = 0.f;
  int k = 0;
  for (; k + 16 <= nk; k += 16) {
    u32x4 x[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) x[u] = __builtin_amdgcn_raw_buffer_load_b128(rsl, src + (k + u) * 8192, 0, 2);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const bf16x8 y = __builtin_bit_cast(bf16x8, x[u]);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] += (float)y[i];
    }
  }
  for (; k + 8 <= nk; k += 8) {
    u32x4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = __builtin_amdgcn_raw_buffer_load_b128(rsl, src + (k + u) * 8192, 0, 2);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bf16x8 y = __builtin_bit_cast(bf16x8, x[u]);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] += (float)y[i];
    }
  }
  for (; k < nk; ++k) {
    const bf16x8 y = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsl, src + k * 8192, 0, 2));
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] += (float)y[i];
  }
  if (q >= p.N) return;
  const int b = bh / p.H, hh = bh % p.H;
  bf16* dst = (bf16*)p.dq + b * p.sdq[0] + hh * p.sdq[1] + (int64_t)q * p.sdq[2] + 32 * (w >> 2) + 4 * (lane >> 4);
  const float sc = p.scale;
  store4(dst, a[0] * sc, a[1] * sc, a[2] * sc, a[3] * sc, true);
  store4(dst + 16, a[4] * sc, a[5] * sc, a[6] * sc, a[7] * sc, true);
}

// The fused backward's workspace beyond the prep rows: the arrival counters ([B·H][nsa] u32,
// 256-B padded) and the slab of one head group (at most kSlabCap bytes); 0 when a single
// head's slab exceeds the cap (N > 46340: the split backward runs instead).
static int64_t fused_head_slab(int64_t N) {
  return ((N + kStep - 1) / kStep) * ((N + kKB - 1) / kKB) * 8 * 512 * 2;
}
static int64_t fused_counter_bytes(int64_t B, int64_t H, int64_t N) {
  return (B * H * ((N + kStep - 1) / kStep) * 4 + 255) / 256 * 256;
}
static int64_t fused_group_heads(int64_t B, int64_t H, int64_t N) {
  return std::min<int64_t>(B * H, kSlabCap / fused_head_slab(N));
}
// what ABI 2 (rounds 3) reserved beyond the prep rows for d = 64, N <= 8192: the whole
// unsplit slab, no counters (the legacy unchecked entry points use the fused pass only where
// the current layout fits inside that)
int64_t bwd_fused_abi2_bytes(int64_t B, int64_t H, int64_t N) { return B * H * fused_head_slab(N); }
int64_t bwd_fused_ws_bytes(int64_t B, int64_t H, int64_t N) {
  // (one buffer resource with 32-bit offsets spans the counters and the slab)
  if (fused_head_slab(N) > kSlabCap || fused_counter_bytes(B, H, N) + kSlabCap > 0x7fffffff) return 0;
  return fused_counter_bytes(B, H, N) + fused_group_heads(B, H, N) * fused_head_slab(N);
}

// The fused pass (after fa_bwd_prep_bf16, which zeroes the arrival counters), launched once
// per group of at most fused_group_heads heads so that the partials of a launch stay within
// kSlabCap (C3: one launch of 128 heads); the groups reuse the slab in stream order. ws: the
// bwd_fused_ws_bytes region of the workspace, 256-B aligned.
hipError_t launch_bwd_fused(const AttnArgs& a0, bool causal, void* ws, hipStream_t st) {
  AttnArgs a = a0;
  const int64_t B = a.B, H = a.H, N = a.N;
  if (fused_head_slab(N) > kSlabCap || fused_counter_bytes(B, H, N) + kSlabCap > 0x7fffffff)
    return hipErrorInvalidValue;
  a.dq_cnt = (unsigned*)ws;
  const int nkb = (a.N + kKB - 1) / kKB, nsa = (a.N + kStep - 1) / kStep;
  int64_t grp = fused_group_heads(B, H, N);
#ifdef MT_DIAGNOSTICS
  // A/B: smaller head groups (MT_FUSED_GROUP heads per launch), so a group's partials stay in
  // the Infinity Cache between their store and the last arriver's read
  if (const char* e = getenv("MT_FUSED_GROUP")) grp = std::max<int64_t>(1, std::min<int64_t>(grp, atoll(e)));
#endif
  // causal: light/heavy pairs while the paired grid still has a workgroup per CU
  const bool pair = causal && (int64_t)((nkb + 1) / 2) * grp >= 256;
  // the product form (an A/B form of the kernel's VAR, see kFormRot)
  const bool rot = !causal && N % kStep == 0 && !a.kv_len;
  void (*kfn)(AttnArgs, int, int, int, int, int) =
      pair ? fa_bwd_fused_bf16<true, true, kFormR3> : causal ? fa_bwd_fused_bf16<true, false, kFormR3>
      : rot ? fa_bwd_fused_bf16<false, false, kFormRot> : fa_bwd_fused_bf16<false, false, kFormR3>;
  int form = rot ? kFormRot : kFormR3;
#ifdef MT_DIAGNOSTICS
  // A/B forms of the dQ hand-off (MT_KNOB, see the kernel's VAR)
#define MT_FVAR(V) \
  if (a.knob == V) { kfn = pair ? fa_bwd_fused_bf16<true, true, V> : causal ? fa_bwd_fused_bf16<true, false, V> : fa_bwd_fused_bf16<false, false, V>; form = V; }
  MT_FVAR(1) MT_FVAR(2) MT_FVAR(3) MT_FVAR(4) MT_FVAR(7) MT_FVAR(8) MT_FVAR(16) MT_FVAR(32) MT_FVAR(40)
  MT_FVAR(33) MT_FVAR(80) MT_FVAR(96)
#undef MT_FVAR
  if (a.knob == 64) {  // the round-4 first form: in-kernel reduce, unrotated walks
    kfn = pair ? fa_bwd_fused_bf16<true, true, 0> : causal ? fa_bwd_fused_bf16<true, false, 0> : fa_bwd_fused_bf16<false, false, 0>;
    form = 0;
  }
#endif
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, kSmemAll);
  if (e != hipSuccess) return e;
  for (int64_t bh0 = 0; bh0 < B * H; bh0 += grp) {
    const int64_t ng = std::min<int64_t>(grp, B * H - bh0);
    const int64_t nblk = (int64_t)(pair ? (nkb + 1) / 2 : nkb) * ng;
    if (nblk > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kfn, dim3((unsigned)nblk), dim3(512), kSmemAll, st, a, nkb, nsa, (int)bh0,
                       (int)fused_counter_bytes(B, H, N),
                       (int)(fused_counter_bytes(B, H, N) + ng * fused_head_slab(N)));
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (form & 16) {
      const int64_t nunit = ng * nsa * 8;
      hipLaunchKernelGGL(fa_bwd_dq_reduce, dim3((unsigned)((nunit + 3) / 4)), dim3(256), 0, st, a, nkb, nsa,
                         (int)bh0, (int)ng, (int)fused_counter_bytes(B, H, N),
                         (int)(fused_counter_bytes(B, H, N) + ng * fused_head_slab(N)), causal ? 1 : 0);
      e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

}  // namespace mt
