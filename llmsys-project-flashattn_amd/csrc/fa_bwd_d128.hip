// FlashAttention backward, bf16 I/O, head dim 128 (BASELINE config 4's head dim): the split
// form (a dK/dV pass and a dQ pass) on the 16x16x32 MFMA. Two kernel bodies: the two-wave form
// (16 stationary rows per wave, 8 waves; described below) and the product's one-wave-per-SIMD
// form (32 stationary rows per wave, 4 waves; fa_bwd_d128w_bf16), same layouts and slot stream.
//
// Same mathematics as every backward here (reference backward_kernel,
// src/flashattention_kernel.cu:115-255, with its dV term corrected):
//     P = exp2(c2·S'),  dV = Pᵀ·dO,  dS = P ∘ dP',  dK = dSᵀ·Q / √d,  dQ = dS·K / √d
// where S' = Q·Kᵀ − lse2/c2 and dP' = dO·Vᵀ − δ start from the prep kernel's pre-negated row
// constants (C-init), as in fa_bwd_bf16.hip.
//
// Why this form at d = 128. The d = 64 kernels give each wave 32 keys (32x32x16 MFMA); at d =
// 128 a wave's dKᵀ/dVᵀ for 32 keys is 128 accumulator registers and its K/V operands another
// 64, past the two-waves-per-SIMD budget. With 16 keys per wave the accumulators are 64
// registers, and the 16x16x32 MFMA has the lane dimension 16. The fused form (dQ inside the
// dK/dV pass) would sum dQ over N/128 key blocks per query step: at (8,16,4096,128) 4.3 GB of
// bf16 partials written and read back, ≈ 0.7 ms at HBM rate, as long as the extra dQ pass's
// S and dP products, so the split (7 products, no slab, no cross-workgroup sum) is kept.
//
// One kernel body serves both passes (MODE): a workgroup of 8 waves owns 128 "stationary" rows
// (16 per wave, in registers as MFMA B operands) and walks 64-row tiles of the "streamed"
// operands through a two-slot LDS ring (LDS-DMA staging, one barrier per tile):
//   MODE 0 (dK/dV): stationary K, V (keys); streamed Q, dO (+ the queries' row constants);
//                   S[q][key] = Q·Kᵀ, dP[q][key] = dO·Vᵀ; dVᵀ += dOᵀ·P, dKᵀ += Qᵀ·dS.
//   MODE 1 (dQ):    stationary Q, dO (queries, row constants in registers); streamed K, V;
//                   Sᵀ[key][q] = K·Qᵀ, dPᵀ[key][q] = V·dOᵀ; dQᵀ += Kᵀ·dSᵀ.
// Layouts (16x16x32: lane l, g = l >> 4, i = l & 15; A lane holds row i, k = 8g .. 8g + 7; B
// lane holds column i, k = 8g ..; C lane holds rows 4g + 0..3 of column i):
//  * T = Y·Xᵀ per streamed 16-row tile rt: A = Y rows 16 rt + i (ds_read_b128 of the image),
//    B = X row i of the wave (k-step ks: d 32 ks + 8 g ..), C: streamed rows 16 rt + 4 g + r
//    of stationary row i. So the stationary row is the lane, and for a 32-row k-step kq the
//    lane holds the streamed rows 32 kq + 4 g + r and 32 kq + 16 + 4 g + r: eight values of one
//    stationary row, which are directly the B operand of the accumulate products in that k
//    order (v6's P fragment, transposed roles).
//  * The accumulate products take A = Yᵀ (d 16 dt + i, the same streamed rows in the same k
//    order) by two ds_read_b64_tr_b16 of four rows each, as fa_fwd_d128v2.hip's Vᵀ.
//  * One image per streamed tensor serves both reads: chunk c of row r at c ^ ((r & 7) << 1).
//    A ds_read_b128 lane group ({0-3, 12-15 | 20-27} and its three siblings: rows i of two
//    k-chunks) and a half-wave's transposed read (rows 4 g + 0..3, g = 0, 1, chunks 2 dt,
//    2 dt + 1) both land on 16 distinct chunk slots (64 banks).
// Each MFMA has one LDS operand and one register operand, so the LDS array delivers operands
// at the MFMA's own rate (256 B per clock per CU against 1 KiB per 16-cycle MFMA per SIMD).
// No masks for ragged N: rows past N read as zero through the buffer range check, and every
// product they enter is zero (their Q / dO rows in the dK/dV pass, their K / V rows in the dQ
// pass); causal masks on the diagonal tiles only.
#include "fa_bwd_bf16.h"

namespace mt {

namespace {

constexpr int D = 128;
constexpr int kT = 64;                 // streamed rows per tile
constexpr int kW = 16;                 // stationary rows per wave
constexpr int kNW = 8;                 // waves per workgroup
constexpr int kBR = kW * kNW;          // stationary rows per workgroup
// a ring slot of a KT-row staging step: Y1, Y2 images (KT x 128 bf16 each) + the row constants
// (MODE 0: KT of -lse2/c2, then KT of -δ)
constexpr int img_bytes(int kt) { return kt * D * 2; }
constexpr int slot_bytes(int kt) { return 2 * img_bytes(kt) + 2 * kt * 4; }
constexpr int smem_bytes(int kt) { return 2 * slot_bytes(kt); }
static_assert(smem_bytes(128) <= 160 * 1024, "LDS budget");

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

__device__ __forceinline__ int swz(int r, int c) { return r * D + ((c ^ ((r & 7) << 1)) << 3); }

__device__ __forceinline__ f32x4 mma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// dst += a·b on the 16x16x32 MFMA with the accumulator pinned to AGPRs (the one-wave form: its
// score tiles take the VGPR form, file flag -amdgpu-mfma-vgpr-form, so the softmax reads them
// directly; pinning keeps hipcc from parking loop-carried accumulators in VGPRs and copying
// them over for every product). Only ever followed by its own next product, tiles later.
__device__ __forceinline__ void mma16a(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

__device__ __forceinline__ void mma32a(f32x16& c, const bf16x8& a, const bf16x8& b) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

// Yᵀ fragment of the 32x32x16 form: two transposed reads at rows row0 + lo-offset / hi-offset
__device__ __forceinline__ bf16x8 trf(const bf16* img, int row0, int lo, int hi) {
  const bf16* a = img + row0 * D;
  const s16x4 l = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + lo));
  const s16x4 h = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + hi));
  const s16x8 v = {l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Yᵀ fragment (A operand of an accumulate product): d block dt, streamed rows 32 kq + 4 g + 0..3
// and + 16, at the lane's transposed-read offset to[dt]
__device__ __forceinline__ bf16x8 trread(const bf16* img, const int (&to)[8], int kq, int dt) {
  const bf16* a = img + kq * 32 * D + to[dt];
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 16 * D));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// the eight values of k-step kq of a score tile set (tiles 2 kq, 2 kq + 1, rows r) as bf16
__device__ __forceinline__ bf16x8 pack8(const f32x4 (&t)[4], int kq) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = (bf16)t[2 * kq][j];
    r[4 + j] = (bf16)t[2 * kq + 1][j];
  }
  return r;
}

__device__ __forceinline__ void dma16(uint32_t lds, __amdgpu_buffer_rsrc_t rs, int go) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(go), "s"(lds), "s"(rs)
      : "memory");
}
__device__ __forceinline__ void dma4(uint32_t lds, __amdgpu_buffer_rsrc_t rs, int go) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "buffer_load_dword %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(go), "s"(lds), "s"(rs)
      : "memory");
}

}  // namespace

// grid: ceil(N / 128) blocks of stationary rows x B·H, XCD-aware order (one head's blocks on
// one XCD, where its streamed tiles stay in L2); 512 threads; smem_bytes(KT) of LDS.
// PAIR (causal): a workgroup runs a light and a heavy block of one head as two passes (MODE 0:
// key blocks nblk - 1 - u, then u; MODE 1: query blocks u, then nblk - 1 - u), so every
// workgroup walks about nblk + 1 blocks' worth of tiles (the d = 64 kernels' pairing).
// KT: streamed rows staged per barrier step (64, or 128 = two 64-row halves computed in turn
// between one pair of barriers: half the barriers and staging waits, twice the LDS)
template <int MODE, bool CAUSAL, bool PAIR = false, int AHEAD = 3, int KT = 64>
__global__ __launch_bounds__(512, 2) void fa_bwd_d128_bf16(AttnArgs p, int nblk_head) {
  constexpr int kImgB = img_bytes(KT), kSlotB = slot_bytes(KT);
  constexpr int NP = KT / 32;  // LDS-DMA pieces of 4 rows per wave per image
  constexpr int NH = KT / kT;  // 64-row halves per staging step
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  const int N = p.N;
  const int logical = bwdbf16::xcd_remap(blockIdx.x, gridDim.x);
  const int nslot = PAIR ? (nblk_head + 1) / 2 : nblk_head;
  const int bh = logical / nslot, u_ = logical % nslot;
  const int b = bh / p.H, hh = bh % p.H;

  // streamed operands: images of 64-row tiles, staged by LDS-DMA: piece j of wave w fills rows
  // 4 (2 w + j) .. + 3 in lane order, lane l fetching the source chunk the swizzle puts at
  // chunk l % 16
  const bf16* Y1 = MODE == 0 ? (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1]
                             : (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1];
  const bf16* Y2 = MODE == 0 ? (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1]
                             : (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1];
  const int sy1 = (int)(MODE == 0 ? p.sq[2] : p.sk[2]), sy2 = (int)(MODE == 0 ? p.sdo[2] : p.sv[2]);
  const __amdgpu_buffer_rsrc_t ry1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)Y1, (short)0, ((N - 1) * sy1 + D) * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t ry2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)Y2, (short)0, ((N - 1) * sy2 + D) * 2, 0x00020000);
  int yo1[NP], yo2[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int dr = 4 * (NP * wave + j) + (lane >> 4), dc = lane & 15;
    const int cs = dc ^ ((dr & 7) << 1);
    yo1[j] = (dr * sy1 + cs * 8) * 2;
    yo2[j] = (dr * sy2 + cs * 8) * 2;
  }
  const uint32_t lds0 = bwdbf16::lds_base(smem);
  // MODE 0 row constants: KT / 64 waves per tensor each move 64 dwords (−lse2/c2, then −δ) per
  // staging step; a query past N reads an out-of-range offset, i.e. 0
  const __amdgpu_buffer_rsrc_t rcl = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.lse2 + (int64_t)bh * N), (short)0, N * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rcd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.delta + (int64_t)bh * N), (short)0, N * 4, 0x00020000);
  auto stage = [&](int t, int slot) __attribute__((always_inline)) {
    const uint32_t base = lds0 + slot * kSlotB;
    const int row0 = t * KT;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const uint32_t off = (uint32_t)(4 * (NP * wave + j) * D * 2);
      dma16(base + off, ry1, yo1[j] + row0 * sy1 * 2);
      dma16(base + kImgB + off, ry2, yo2[j] + row0 * sy2 * 2);
    }
    if (MODE == 0 && wave < 2 * (KT / 64)) {
      const int tsel = wave / (KT / 64), ch = wave % (KT / 64);  // tensor (lse2, δ), 64-row chunk
      const int q = row0 + 64 * ch + lane;
      dma4(base + 2 * kImgB + (tsel * KT + 64 * ch) * 4, tsel ? rcd : rcl, q < N ? q * 4 : 0x7ffffff0);
    }
  };

  // operand offsets: row reads (A of T = Y·Xᵀ): row i, chunk 4 ks + g; transposed reads (A of
  // the accumulate products): rows 4 g + (i >> 2) (+ 16), chunk 2 dt + ((i & 3) >> 1), half i & 1
  int ro[4], to[8];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) ro[ks] = swz(i16, 4 * ks + g);
  {
    const int q = i16 >> 2, pp = i16 & 3, row = 4 * g + q;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) to[dt] = swz(row, 2 * dt + (pp >> 1)) + 4 * (pp & 1);
  }

#pragma nounroll
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
  const int light = MODE == 0 ? nblk_head - 1 - u_ : u_, heavy = nblk_head - 1 - light;
  const int blk = PAIR ? (pass == 0 ? light : heavy) : u_;
  if (PAIR && pass == 1 && heavy == light) break;  // odd block count: the middle block alone
  const int r0 = blk * kBR;               // first stationary row of the workgroup
  const int rw = r0 + wave * kW;          // first stationary row of this wave
  const int my = rw + i16;                // this lane's stationary row
  const float c2 = p.scale_log2;

  // stationary operands (B fragments): X1, X2 row `my`, k-step ks = d 32 ks + 8 g ..
  const bf16* X1 = MODE == 0 ? (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1]
                             : (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* X2 = MODE == 0 ? (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1]
                             : (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const int64_t sx1 = MODE == 0 ? p.sk[2] : p.sq[2], sx2 = MODE == 0 ? p.sv[2] : p.sdo[2];
  bf16x8 xf1[4], xf2[4];
  {
    const int rr = min(my, N - 1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      xf1[ks] = *(const bf16x8*)(X1 + (int64_t)rr * sx1 + 32 * ks + 8 * g);
      xf2[ks] = *(const bf16x8*)(X2 + (int64_t)rr * sx2 + 32 * ks + 8 * g);
    }
  }
  // MODE 1: the row constants of the lane's query (C-init of Sᵀ and dPᵀ)
  float nl = 0.f, nd = 0.f;
  if (MODE == 1 && my < N) {
    nl = p.lse2[(int64_t)bh * N + my];
    nd = p.delta[(int64_t)bh * N + my];
  }
  // Wait for these loads here: left to itself hipcc waits for them at their first use, inside
  // the tile loop, with vmcnt counts that also cover the staging issued from inline asm at the
  // top of every tile (which it does not count), and so stalls each tile mid-way for the next
  // tile's staging.
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) asm volatile("" ::"v"(xf1[ks]), "v"(xf2[ks]));
  asm volatile("" ::"v"(nl), "v"(nd));

  // the tiles this workgroup walks: MODE 0 queries (causal: from the block's first key), MODE 1
  // keys (causal: up to the block's last query)
  const int ntile_all = (N + KT - 1) / KT;
  const int t0 = (MODE == 0 && CAUSAL) ? r0 / KT : 0;
  const int t1 = (MODE == 1 && CAUSAL) ? min(ntile_all, (min(r0 + kBR, N) + KT - 1) / KT) : ntile_all;

  f32x4 acc1[8], acc2[8];  // MODE 0: dKᵀ, dVᵀ [d block]; MODE 1: dQᵀ in acc1
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) { acc1[dt] = f32x4{}; acc2[dt] = f32x4{}; }

  if (t0 < t1) {
    stage(t0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  for (int t = t0; t < t1; ++t) {
    const int slot = (t - t0) & 1;
    if (t + 1 < t1) stage(t + 1, slot ^ 1);
#pragma unroll
    for (int hh2 = 0; hh2 < NH; ++hh2) {  // the step's 64-row halves
    const bf16* I1 = (const bf16*)(smem + slot * kSlotB) + hh2 * kT * D;
    const bf16* I2 = (const bf16*)(smem + slot * kSlotB + kImgB) + hh2 * kT * D;
    const float* cstl = (const float*)(smem + slot * kSlotB + 2 * kImgB) + hh2 * kT;
    // T1 = Y1·X1ᵀ, T2 = Y2·X2ᵀ over the tile's four 16-row blocks, from the row constants
    f32x4 T1[4], T2[4];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      if (MODE == 0) {
        T1[rt] = *(const f32x4*)(cstl + 16 * rt + 4 * g);
        T2[rt] = *(const f32x4*)(cstl + KT + 16 * rt + 4 * g);
      } else {
        T1[rt] = f32x4{nl, nl, nl, nl};
        T2[rt] = f32x4{nd, nd, nd, nd};
      }
    }
    // causal: the diagonal tiles (a streamed row on the wrong side of the lane's row)
    const int y0 = t * KT + hh2 * kT;  // first streamed row of the half
    const bool diag = CAUSAL && (MODE == 0 ? y0 < rw + kW : y0 + kT - 1 > rw);
    bf16x8 pf[2], sf[2];  // P and dS of k-steps 0, 1 (B operands of the accumulate products)
    // The tile as one unrolled stream of MFMA slots (sched_barrier after each, so the source
    // order is the issue order): [0, 32) the T products, rows 0-31 (k-step 0) first; then
    // the accumulate products of k-step 0 and of k-step 1 (16 + 16 in MODE 0: dVᵀ and dKᵀ
    // alternating; 8 + 8 in MODE 1). Every MFMA's LDS operand is read kAhead slots before it
    // (a ring of register fragments; hipcc's own order read each operand right before its
    // MFMA and waited lgkmcnt(0) there, exposing the LDS latency in every slot). The softmax
    // of k-step 0 runs beside the T products of k-step 1, that of k-step 1 beside the
    // accumulate products of k-step 0.
    constexpr int kNA = MODE == 0 ? 16 : 8;  // accumulate products per k-step
    constexpr int kL = 32 + 2 * kNA;
    constexpr int kAhead = AHEAD;  // (diagnostics A/B: 2, 4, 5)
    auto operand = [&](int m) __attribute__((always_inline)) -> bf16x8 {
      if (m < 32) {  // T slot: tensor m & 1, 16-row block rt, k-step ks (chains alternate)
        const int idx = m >> 1, rt = 2 * (idx >> 3) + (idx & 1), ks = (idx >> 1) & 3;
        return *(const bf16x8*)(((m & 1) ? I2 : I1) + 16 * rt * D + ro[ks]);
      }
      const int j = m - 32, kq = j / kNA, jj = j % kNA;
      if (MODE == 0) return trread((jj & 1) ? I1 : I2, to, kq, jj >> 1);  // dVᵀ (I2), dKᵀ (I1)
      return trread(I1, to, kq, jj);
    };
    // softmax item it (0..7) of k-step kq: score (rt = 2 kq + (it >> 2), r = it & 3)
    auto item = [&](int kq, int it) __attribute__((always_inline)) {
      const int rt = 2 * kq + (it >> 2), r = it & 3;
      float x = T1[rt][r];
      if (diag) {
        const int y = y0 + 16 * rt + 4 * g + r;
        if (MODE == 0 ? my > y : y > my) x = -INFINITY;  // MODE 0: key after query; 1: the reverse
      }
      const float pv = __builtin_amdgcn_exp2f(x * c2);
      T1[rt][r] = pv;
      T2[rt][r] = pv * T2[rt][r];
    };
    // pack piece k (0..3) of k-step kq: elements 2k, 2k + 1 of P (MODE 0) and dS
    auto piece = [&](int kq, int k) __attribute__((always_inline)) {
      const int rt = 2 * kq + (k >> 1), r = 2 * (k & 1);
      if (MODE == 0) {
        pf[kq][2 * k] = (bf16)T1[rt][r];
        pf[kq][2 * k + 1] = (bf16)T1[rt][r + 1];
      }
      sf[kq][2 * k] = (bf16)T2[rt][r];
      sf[kq][2 * k + 1] = (bf16)T2[rt][r + 1];
    };
    bf16x8 ring[kAhead + 1];
#pragma unroll
    for (int m = 0; m < kAhead; ++m) ring[m] = operand(m);
#pragma unroll
    for (int m = 0; m < kL; ++m) {
      if (m + kAhead < kL) ring[(m + kAhead) % (kAhead + 1)] = operand(m + kAhead);
      const bf16x8 a = ring[m % (kAhead + 1)];
      if (m < 32) {
        const int idx = m >> 1, rt = 2 * (idx >> 3) + (idx & 1), ks = (idx >> 1) & 3;
        if (m & 1) T2[rt] = mma16(a, xf2[ks], T2[rt]);
        else T1[rt] = mma16(a, xf1[ks], T1[rt]);
      } else {
        const int j = m - 32, kq = j / kNA, jj = j % kNA;
        if (MODE == 0) {
          if (jj & 1) acc1[jj >> 1] = mma16(a, sf[kq], acc1[jj >> 1]);  // dKᵀ += Qᵀ·dS
          else acc2[jj >> 1] = mma16(a, pf[kq], acc2[jj >> 1]);        // dVᵀ += dOᵀ·P
        } else {
          acc1[jj] = mma16(a, sf[kq], acc1[jj]);  // dQᵀ += Kᵀ·dSᵀ
        }
      }
      // the softmax beside the MFMAs: k-step 0 in slots [16, 32), k-step 1 in [32, 32 + kNA)
      const int kq = m < 32 ? 0 : 1, w = m < 32 ? m - 16 : m - 32;
      const int wl = kq == 0 ? 16 : kNA;  // window length
      if (w >= 0 && w < wl) {
        if (wl == 16) {
          if (w < 8) item(kq, w);
          else if (w < 12) piece(kq, w - 8);
        } else {
          item(kq, w);
        }
      }
      if (m == 32 + kNA - 1 && kNA == 8) {  // MODE 1: k-step 1's packs after its window
#pragma unroll
        for (int k = 0; k < 4; ++k) piece(1, k);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    }  // half
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // outputs: lane (i, g) holds rows d = 16 dt + 4 g + r of stationary row `my`
  if (my < N) {
    const float sc = p.scale;
    if (MODE == 0) {
      bf16* dKg = (bf16*)p.dk + b * p.sdk[0] + hh * p.sdk[1] + (int64_t)my * p.sdk[2];
      bf16* dVg = (bf16*)p.dv + b * p.sdv[0] + hh * p.sdv[1] + (int64_t)my * p.sdv[2];
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        const int col = 16 * dt + 4 * g;
        store4(dKg + col, acc1[dt][0] * sc, acc1[dt][1] * sc, acc1[dt][2] * sc, acc1[dt][3] * sc, true);
        store4(dVg + col, acc2[dt][0], acc2[dt][1], acc2[dt][2], acc2[dt][3], true);
      }
    } else {
      bf16* dQg = (bf16*)p.dq + b * p.sdq[0] + hh * p.sdq[1] + (int64_t)my * p.sdq[2];
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        const int col = 16 * dt + 4 * g;
        store4(dQg + col, acc1[dt][0] * sc, acc1[dt][1] * sc, acc1[dt][2] * sc, acc1[dt][3] * sc, true);
      }
    }
  }
  }  // pass
}

// The one-wave-per-SIMD form of the same two passes: 4 waves of 32 stationary rows (two 16-row
// groups sg, both in registers) per 128-row block, so every streamed operand read from LDS
// feeds two MFMAs (half the LDS traffic per product of the form above) and no second wave
// competes for the SIMD's issue port; the price is registers (the accumulators live in AGPRs)
// and a barrier every SIMD waits at with nothing else to run. So the barrier step is hidden:
// a three-slot ring staged two tiles ahead keeps the next tile published during the current
// one, and the operand ring runs across the tile boundary (the last kAhead slots of a tile read
// the first operands of the next, and its row constants load during the last accumulate
// products), so the first MFMAs after the barrier find their operands in registers.
// PK: the softmax on score pairs (packed multiplies: two scores per VALU instruction)
// ABL (timing-only ablations, WRONG results, diagnostics build): 1 no barrier in the tile loop,
// 2 no softmax (scores packed as they are), 4 no staging in the tile loop
// NWV: waves per workgroup (4: one per SIMD; 8: two per SIMD, 256 stationary rows, for a
// kernel that fits 256 registers)
// PREP (MODE 1): the pass forms the row constants of its stationary queries itself (the prep
// kernel's −lse2/c2 and −δ = −rowsum(dO ∘ O)) and writes them for the dK/dV pass, which then
// runs second; no prep launch
template <int MODE, bool CAUSAL, bool PAIR = false, bool PK = true, int ABL = 0, int AH = 7, int NWV = 4,
          bool PREP = false>
__global__ __launch_bounds__(64 * NWV, NWV / 4) void fa_bwd_d128w_bf16(AttnArgs p, int nblk_head) {
  constexpr int kImgB = img_bytes(kT), kSlotB = slot_bytes(kT);
  constexpr int kWw = 32;     // stationary rows per wave
  constexpr int NP = 16 / NWV;  // LDS-DMA pieces of 4 rows per wave per image
  constexpr int kBRw = kWw * NWV;  // stationary rows per workgroup
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  const int N = p.N;
  const int logical = bwdbf16::xcd_remap(blockIdx.x, gridDim.x);
  const int nslot = PAIR ? (nblk_head + 1) / 2 : nblk_head;
  const int bh = logical / nslot, u_ = logical % nslot;
  const int b = bh / p.H, hh = bh % p.H;

  const bf16* Y1 = MODE == 0 ? (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1]
                             : (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1];
  const bf16* Y2 = MODE == 0 ? (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1]
                             : (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1];
  const int sy1 = (int)(MODE == 0 ? p.sq[2] : p.sk[2]), sy2 = (int)(MODE == 0 ? p.sdo[2] : p.sv[2]);
  const __amdgpu_buffer_rsrc_t ry1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)Y1, (short)0, ((N - 1) * sy1 + D) * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t ry2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)Y2, (short)0, ((N - 1) * sy2 + D) * 2, 0x00020000);
  int yo1[NP], yo2[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int dr = 4 * (NP * wave + j) + (lane >> 4), dc = lane & 15;
    const int cs = dc ^ ((dr & 7) << 1);
    yo1[j] = (dr * sy1 + cs * 8) * 2;
    yo2[j] = (dr * sy2 + cs * 8) * 2;
  }
  const uint32_t lds0 = bwdbf16::lds_base(smem);
  const __amdgpu_buffer_rsrc_t rcl = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.lse2 + (int64_t)bh * N), (short)0, N * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rcd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.delta + (int64_t)bh * N), (short)0, N * 4, 0x00020000);
  auto stage = [&](int t, int slot) __attribute__((always_inline)) {
    const uint32_t base = lds0 + slot * kSlotB;
    const int row0 = t * kT;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const uint32_t off = (uint32_t)(4 * (NP * wave + j) * D * 2);
      dma16(base + off, ry1, yo1[j] + row0 * sy1 * 2);
      dma16(base + kImgB + off, ry2, yo2[j] + row0 * sy2 * 2);
    }
    if (MODE == 0 && wave < 2) {  // wave 0: −lse2/c2, wave 1: −δ
      const int q = row0 + lane;
      dma4(base + 2 * kImgB + wave * kT * 4, wave ? rcd : rcl, q < N ? q * 4 : 0x7ffffff0);
    }
  };
  int ro[4], to[8];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) ro[ks] = swz(i16, 4 * ks + g);
  {
    const int q = i16 >> 2, pp = i16 & 3, row = 4 * g + q;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) to[dt] = swz(row, 2 * dt + (pp >> 1)) + 4 * (pp & 1);
  }

#pragma nounroll
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
  const int light = MODE == 0 ? nblk_head - 1 - u_ : u_, heavy = nblk_head - 1 - light;
  const int blk = PAIR ? (pass == 0 ? light : heavy) : u_;
  if (PAIR && pass == 1 && heavy == light) break;
  const int r0 = blk * kBRw;
  const int rw = r0 + wave * kWw;
  int my[2];
  my[0] = rw + i16;
  my[1] = rw + 16 + i16;
  const float c2 = p.scale_log2;

  const bf16* X1 = MODE == 0 ? (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1]
                             : (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* X2 = MODE == 0 ? (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1]
                             : (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const int64_t sx1 = MODE == 0 ? p.sk[2] : p.sq[2], sx2 = MODE == 0 ? p.sv[2] : p.sdo[2];
  bf16x8 xf1[2][4], xf2[2][4];
  float nl[2] = {0.f, 0.f}, nd[2] = {0.f, 0.f};
#pragma unroll
  for (int sg = 0; sg < 2; ++sg) {
    const int rr = min(my[sg], N - 1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      xf1[sg][ks] = *(const bf16x8*)(X1 + (int64_t)rr * sx1 + 32 * ks + 8 * g);
      xf2[sg][ks] = *(const bf16x8*)(X2 + (int64_t)rr * sx2 + 32 * ks + 8 * g);
    }
    if (MODE == 1 && !PREP && my[sg] < N) {
      nl[sg] = p.lse2[(int64_t)bh * N + my[sg]];
      nd[sg] = p.delta[(int64_t)bh * N + my[sg]];
    }
  }
  // PREP: the forward's O rows and (m, l) of the stationary queries, in flight across the first
  // tiles' staging; the row constants are formed after it (below)
  bf16x8 of[2][4];
  float pm[2] = {0.f, 0.f}, pl[2] = {1.f, 1.f};
  if (MODE == 1 && PREP) {
    const bf16* Og = (const bf16*)p.o + b * p.so[0] + hh * p.so[1];
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
      const int rr = min(my[sg], N - 1);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) of[sg][ks] = *(const bf16x8*)(Og + (int64_t)rr * p.so[2] + 32 * ks + 8 * g);
      pm[sg] = p.m[(int64_t)bh * N + rr];
      pl[sg] = p.l[(int64_t)bh * N + rr];
    }
  }
  // (waited here, not at first use inside the loop: see the form above)
#pragma unroll
  for (int sg = 0; sg < 2; ++sg) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) asm volatile("" ::"v"(xf1[sg][ks]), "v"(xf2[sg][ks]));
    if (!PREP) asm volatile("" ::"v"(nl[sg]), "v"(nd[sg]));
  }

  const int ntile_all = (N + kT - 1) / kT;
  const int t0 = (MODE == 0 && CAUSAL) ? r0 / kT : 0;
  const int t1 = (MODE == 1 && CAUSAL) ? min(ntile_all, (min(r0 + kBRw, N) + kT - 1) / kT) : ntile_all;

  f32x4 acc1[2][8], acc2[2][8];
#pragma unroll
  for (int sg = 0; sg < 2; ++sg)
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) { acc1[sg][dt] = f32x4{}; acc2[sg][dt] = f32x4{}; }

  if (t0 < t1) {
    stage(t0, 0);
    if (t0 + 1 < t1) stage(t0 + 1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (MODE == 1 && PREP) {
    // the prep kernel's row constants from the stationary dO fragments: the four lanes g of a
    // row hold its columns 32 ks + 8 g .. + 7, so δ is their sum over ks, then across g; written
    // for the dK/dV pass, which runs after this one
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
      float acc = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += (float)of[sg][ks][j] * (float)xf2[sg][ks][j];
      acc += __shfl_xor(acc, 16);
      acc += __shfl_xor(acc, 32);
      if (my[sg] < N) {
        nd[sg] = -acc;
        nl[sg] = -(pm[sg] * kLog2e + log2f(pl[sg])) / p.scale_log2;
        if (g == 0) {
          const int64_t row = (int64_t)bh * N + my[sg];
          p.delta[row] = nd[sg];
          p.lse2[row] = nl[sg];
        }
      }
    }
  }

  constexpr int kNA = MODE == 0 ? 16 : 8;
  constexpr int kL = 32 + 2 * kNA;
  constexpr int kAhead = AH, kR = kAhead + 1;  // (diagnostics A/B: 3, 15)
  static_assert(kL % kR == 0, "the operand ring runs across tiles");
  auto operand = [&](const bf16* I1, const bf16* I2, int m) __attribute__((always_inline)) -> bf16x8 {
    if (m < 32) {
      const int idx = m >> 1, rt = 2 * (idx >> 3) + (idx & 1), ks = (idx >> 1) & 3;
      return *(const bf16x8*)(((m & 1) ? I2 : I1) + 16 * rt * D + ro[ks]);
    }
    const int j = m - 32, kq = j / kNA, jj = j % kNA;
    if (MODE == 0) return trread((jj & 1) ? I1 : I2, to, kq, jj >> 1);
    return trread(I1, to, kq, jj);
  };
  f32x4 T1[2][4], T2[2][4];
  auto tinit = [&](int slot) __attribute__((always_inline)) {
    const float* cst = (const float*)(smem + slot * kSlotB + 2 * kImgB);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      if (MODE == 0) {
        const f32x4 l = *(const f32x4*)(cst + 16 * rt + 4 * g);
        const f32x4 d = *(const f32x4*)(cst + kT + 16 * rt + 4 * g);
        T1[0][rt] = l; T1[1][rt] = l;
        T2[0][rt] = d; T2[1][rt] = d;
      } else {
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
          T1[sg][rt] = f32x4{nl[sg], nl[sg], nl[sg], nl[sg]};
          T2[sg][rt] = f32x4{nd[sg], nd[sg], nd[sg], nd[sg]};
        }
      }
    }
  };
  bf16x8 ring[kR];
  tinit(0);
  {
    const bf16* I1 = (const bf16*)smem;
    const bf16* I2 = (const bf16*)(smem + kImgB);
#pragma unroll
    for (int m = 0; m < kAhead; ++m) ring[m] = operand(I1, I2, m);
  }
  int cur = 0;
  for (int t = t0; t < t1; ++t) {
    const int nxt = cur == 2 ? 0 : cur + 1, nn = nxt == 2 ? 0 : nxt + 1;
    if (!(ABL & 4) && t + 2 < t1) stage(t + 2, nn);
    const bf16* I1 = (const bf16*)(smem + cur * kSlotB);
    const bf16* I2 = (const bf16*)(smem + cur * kSlotB + kImgB);
    const bf16* N1 = (const bf16*)(smem + nxt * kSlotB);
    const bf16* N2 = (const bf16*)(smem + nxt * kSlotB + kImgB);
    const int y0 = t * kT;
    const bool diag = CAUSAL && (MODE == 0 ? y0 < rw + kWw : y0 + kT - 1 > rw);
    bf16x8 pf[2][2], sf[2][2];  // [k-step][sg]
    auto item = [&](int kq, int sg, int it) __attribute__((always_inline)) {
      const int rt = 2 * kq + (it >> 2), r = it & 3;
      float x = T1[sg][rt][r];
      if (diag) {
        const int y = y0 + 16 * rt + 4 * g + r;
        if (MODE == 0 ? my[sg] > y : y > my[sg]) x = -INFINITY;
      }
      const float pv = __builtin_amdgcn_exp2f(x * c2);
      T1[sg][rt][r] = pv;
      T2[sg][rt][r] = pv * T2[sg][rt][r];
    };
    auto piece = [&](int kq, int sg, int k) __attribute__((always_inline)) {
      const int rt = 2 * kq + (k >> 1), r = 2 * (k & 1);
      if (MODE == 0) {
        pf[kq][sg][2 * k] = (bf16)T1[sg][rt][r];
        pf[kq][sg][2 * k + 1] = (bf16)T1[sg][rt][r + 1];
      }
      sf[kq][sg][2 * k] = (bf16)T2[sg][rt][r];
      sf[kq][sg][2 * k + 1] = (bf16)T2[sg][rt][r + 1];
    };
    // scores (rt, r), (rt, r + 1) of pair ip (0..3) of k-step kq
    auto item2 = [&](int kq, int sg, int ip) __attribute__((always_inline)) {
      const int rt = 2 * kq + (ip >> 1), r = 2 * (ip & 1);
      f32x2 x = f32x2{T1[sg][rt][r], T1[sg][rt][r + 1]} * f32x2{c2, c2};
      if (diag) {
        const int y = y0 + 16 * rt + 4 * g + r;
        if (MODE == 0 ? my[sg] > y : y > my[sg]) x[0] = -INFINITY;
        if (MODE == 0 ? my[sg] > y + 1 : y + 1 > my[sg]) x[1] = -INFINITY;
      }
      const f32x2 pv = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
      const f32x2 ds = pv * f32x2{T2[sg][rt][r], T2[sg][rt][r + 1]};
      T1[sg][rt][r] = pv[0]; T1[sg][rt][r + 1] = pv[1];
      T2[sg][rt][r] = ds[0]; T2[sg][rt][r + 1] = ds[1];
    };
    // softmax action a of k-step kq: items (sg alternating), then packs (24 actions; PK: 16)
    constexpr int kAct = PK ? 16 : 24;
    auto action = [&](int kq, int a) __attribute__((always_inline)) {
      if (ABL & 2) {
        if (a < 8) piece(kq, a & 1, a >> 1);
      } else if (PK) {
        if (a < 8) item2(kq, a & 1, a >> 1);
        else piece(kq, (a - 8) & 1, (a - 8) >> 1);
      } else {
        if (a < 16) item(kq, a & 1, a >> 1);
        else piece(kq, (a - 16) & 1, (a - 16) >> 1);
      }
    };
#pragma unroll
    for (int m = 0; m < kL; ++m) {
      const int mp = m + kAhead;
      ring[mp % kR] = mp < kL ? operand(I1, I2, mp) : operand(N1, N2, mp - kL);
      const bf16x8 a = ring[m % kR];
      if (m < 32) {
        const int idx = m >> 1, rt = 2 * (idx >> 3) + (idx & 1), ks = (idx >> 1) & 3;
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
          if (m & 1) T2[sg][rt] = mma16(a, xf2[sg][ks], T2[sg][rt]);
          else T1[sg][rt] = mma16(a, xf1[sg][ks], T1[sg][rt]);
        }
      } else {
        const int j = m - 32, kq = j / kNA, jj = j % kNA;
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
          if (MODE == 0) {
            if (jj & 1) mma16a(acc1[sg][jj >> 1], a, sf[kq][sg]);
            else mma16a(acc2[sg][jj >> 1], a, pf[kq][sg]);
          } else if (NWV == 8) {  // all in VGPRs (the 256-register budget of two waves)
            acc1[sg][jj] = mma16(a, sf[kq][sg], acc1[sg][jj]);
          } else {
            mma16a(acc1[sg][jj], a, sf[kq][sg]);
          }
        }
      }
      // softmax of k-step 0 beside the T products of k-step 1 (slots [16, 32)), of k-step 1
      // beside the accumulate products of k-step 0 (slots [32, 32 + kNA))
      const int kq = m < 32 ? 0 : 1, w = m < 32 ? m - 16 : m - 32;
      const int wl = kq == 0 ? 16 : kNA;
      if (w >= 0 && w < wl) {
#pragma unroll
        for (int a2 = w * kAct / wl; a2 < (w + 1) * kAct / wl; ++a2) action(kq, a2);
      }
      // the next tile's row constants, once k-step 1's scores are packed
      if (m == 32 + kNA) tinit(nxt);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!(ABL & 1)) __syncthreads();
    cur = nxt;
  }

  if (true) {
    const float sc = p.scale;
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
      if (my[sg] >= N) continue;
      if (MODE == 0) {
        bf16* dKg = (bf16*)p.dk + b * p.sdk[0] + hh * p.sdk[1] + (int64_t)my[sg] * p.sdk[2];
        bf16* dVg = (bf16*)p.dv + b * p.sdv[0] + hh * p.sdv[1] + (int64_t)my[sg] * p.sdv[2];
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          const int col = 16 * dt + 4 * g;
          store4(dKg + col, acc1[sg][dt][0] * sc, acc1[sg][dt][1] * sc, acc1[sg][dt][2] * sc,
                 acc1[sg][dt][3] * sc, true);
          store4(dVg + col, acc2[sg][dt][0], acc2[sg][dt][1], acc2[sg][dt][2], acc2[sg][dt][3], true);
        }
      } else {
        bf16* dQg = (bf16*)p.dq + b * p.sdq[0] + hh * p.sdq[1] + (int64_t)my[sg] * p.sdq[2];
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          const int col = 16 * dt + 4 * g;
          store4(dQg + col, acc1[sg][dt][0] * sc, acc1[sg][dt][1] * sc, acc1[sg][dt][2] * sc,
                 acc1[sg][dt][3] * sc, true);
        }
      }
    }
  }
  }  // pass
}

// The one-wave form on the 32x32x16 MFMA (round 4 late): the 32 stationary rows of a wave are
// one 32-wide B operand, so a 64-row tile is 64 products (MODE 0; 48 in MODE 1) of 32 cycles
// instead of 128 of 16. An MFMA holds the SIMD's vector issue for 8 cycles whatever its shape
// (MI355X_MICROARCH.md, issue costs), so the softmax, the LDS reads and the staging of a
// one-wave kernel get 24 free cycles per 32-cycle product here against 8 per 16-cycle one.
// Layouts (32x32x16: c32 = lane & 31, hf = lane >> 5; A lane: row c32, k 8 hf ..; B lane:
// column c32, k 8 hf ..; C value v: row 8 (v >> 2) + 4 hf + (v & 3), column c32):
//  * T[u] = Y·Xᵀ per 32-row block u of the tile: A = Y row 32 u + c32 (ds_read_b128, chunk
//    2 ks + hf), B = the lane's stationary row (k-step ks: d 16 ks + 8 hf ..);
//  * the accumulate products take A = Yᵀ (d 32 db + c32; streamed rows 16 s + 4 hf + 0..3 and
//    + 8, the C order of T's values 8 s .. 8 s + 7) by two ds_read_b64_tr_b16, B = P or dS of
//    values 8 s ..;
//  * image swizzle: chunk c of row r at c ^ f(r), f(r) = ((r & 3) << 2) | ((r >> 2) & 3): on
//    the 16 rows of a ds_read_b128 lane group f is a bijection, and on the 4 rows x 4 chunks
//    of a half-wave's transposed read it moves every row to its own chunk quad.
template <int MODE, bool CAUSAL, bool PAIR = false, int ABL = 0>
__global__ __launch_bounds__(256, 1) void fa_bwd_d128x_bf16(AttnArgs p, int nblk_head) {
  constexpr int kImgB = img_bytes(kT), kSlotB = slot_bytes(kT);
  constexpr int kWw = 32, NP = 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c32 = lane & 31, hf = lane >> 5;
  const int N = p.N;
  const int logical = bwdbf16::xcd_remap(blockIdx.x, gridDim.x);
  const int nslot = PAIR ? (nblk_head + 1) / 2 : nblk_head;
  const int bh = logical / nslot, u_ = logical % nslot;
  const int b = bh / p.H, hh = bh % p.H;
  auto fsw = [](int r) { return ((r & 3) << 2) | ((r >> 2) & 3); };
  auto sw2 = [&](int r, int c) { return r * D + ((c ^ fsw(r)) << 3); };

  const bf16* Y1 = MODE == 0 ? (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1]
                             : (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1];
  const bf16* Y2 = MODE == 0 ? (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1]
                             : (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1];
  const int sy1 = (int)(MODE == 0 ? p.sq[2] : p.sk[2]), sy2 = (int)(MODE == 0 ? p.sdo[2] : p.sv[2]);
  const __amdgpu_buffer_rsrc_t ry1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)Y1, (short)0, ((N - 1) * sy1 + D) * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t ry2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)Y2, (short)0, ((N - 1) * sy2 + D) * 2, 0x00020000);
  int yo1[NP], yo2[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int dr = 4 * (NP * wave + j) + (lane >> 4), dc = lane & 15;
    const int cs = dc ^ fsw(dr);
    yo1[j] = (dr * sy1 + cs * 8) * 2;
    yo2[j] = (dr * sy2 + cs * 8) * 2;
  }
  const uint32_t lds0 = bwdbf16::lds_base(smem);
  const __amdgpu_buffer_rsrc_t rcl = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.lse2 + (int64_t)bh * N), (short)0, N * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rcd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.delta + (int64_t)bh * N), (short)0, N * 4, 0x00020000);
  auto stage = [&](int t, int slot) __attribute__((always_inline)) {
    const uint32_t base = lds0 + slot * kSlotB;
    const int row0 = t * kT;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const uint32_t off = (uint32_t)(4 * (NP * wave + j) * D * 2);
      dma16(base + off, ry1, yo1[j] + row0 * sy1 * 2);
      dma16(base + kImgB + off, ry2, yo2[j] + row0 * sy2 * 2);
    }
    if (MODE == 0 && wave < 2) {  // wave 0: −lse2/c2, wave 1: −δ
      const int q = row0 + lane;
      dma4(base + 2 * kImgB + wave * kT * 4, wave ? rcd : rcl, q < N ? q * 4 : 0x7ffffff0);
    }
  };
  int ro[8], tlo[4], thi[4];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) ro[ks] = sw2(c32, 2 * ks + hf);
  {
    const int i16 = lane & 15, g = (lane >> 4) & 1;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const int col = 32 * db + 16 * g + 4 * (i16 & 3), row = 4 * hf + (i16 >> 2);
      tlo[db] = sw2(row, col >> 3) + (col & 7);
      thi[db] = sw2(row + 8, col >> 3) + (col & 7);
    }
  }

#pragma nounroll
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
  const int light = MODE == 0 ? nblk_head - 1 - u_ : u_, heavy = nblk_head - 1 - light;
  const int blk = PAIR ? (pass == 0 ? light : heavy) : u_;
  if (PAIR && pass == 1 && heavy == light) break;
  const int r0 = blk * kBR;
  const int rw = r0 + wave * kWw;
  const int my = rw + c32;
  const float c2 = p.scale_log2;

  const bf16* X1 = MODE == 0 ? (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1]
                             : (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* X2 = MODE == 0 ? (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1]
                             : (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const int64_t sx1 = MODE == 0 ? p.sk[2] : p.sq[2], sx2 = MODE == 0 ? p.sv[2] : p.sdo[2];
  bf16x8 xf1[8], xf2[8];
  float nl = 0.f, nd = 0.f;
  {
    const int rr = min(my, N - 1);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      xf1[ks] = *(const bf16x8*)(X1 + (int64_t)rr * sx1 + 16 * ks + 8 * hf);
      xf2[ks] = *(const bf16x8*)(X2 + (int64_t)rr * sx2 + 16 * ks + 8 * hf);
    }
    if (MODE == 1 && my < N) {
      nl = p.lse2[(int64_t)bh * N + my];
      nd = p.delta[(int64_t)bh * N + my];
    }
  }
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) asm volatile("" ::"v"(xf1[ks]), "v"(xf2[ks]));
  asm volatile("" ::"v"(nl), "v"(nd));

  const int ntile_all = (N + kT - 1) / kT;
  const int t0 = (MODE == 0 && CAUSAL) ? r0 / kT : 0;
  const int t1 = (MODE == 1 && CAUSAL) ? min(ntile_all, (min(r0 + kBR, N) + kT - 1) / kT) : ntile_all;

  f32x16 acc1[4], acc2[4];  // MODE 0: dKᵀ, dVᵀ [d block]; MODE 1: dQᵀ in acc1
#pragma unroll
  for (int db = 0; db < 4; ++db) { acc1[db] = f32x16{}; acc2[db] = f32x16{}; }

  if (t0 < t1) {
    stage(t0, 0);
    if (t0 + 1 < t1) stage(t0 + 1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  // slot stream of a tile (one MFMA per slot): [0, 32) T products (block u = m >> 4, k-step
  // (m >> 1) & 7, tensor m & 1); then the accumulate products of block 0 and of block 1 (kNA
  // each: s, d block, and in MODE 0 the tensor). Softmax of block 0 beside the T products of
  // block 1, of block 1 beside the accumulate products of block 0.
  constexpr int kNA = MODE == 0 ? 16 : 8;
  constexpr int kL = 32 + 2 * kNA;
  constexpr int kAhead = 5, kR = 8;
  static_assert(kL % kR == 0, "the operand ring runs across tiles");
  auto operand = [&](const bf16* I1, const bf16* I2, int m) __attribute__((always_inline)) -> bf16x8 {
    if (m < 32) {
      const int u = m >> 4, ks = (m >> 1) & 7;
      return *(const bf16x8*)(((m & 1) ? I2 : I1) + 32 * u * D + ro[ks]);
    }
    const int j = m - 32, u = j / kNA, jj = j % kNA;
    const int s = MODE == 0 ? jj >> 3 : jj >> 2, db = MODE == 0 ? (jj >> 1) & 3 : jj & 3;
    const bf16* img = MODE == 0 ? ((jj & 1) ? I1 : I2) : I1;  // MODE 0: dVᵀ (I2), dKᵀ (I1)
    return trf(img, 32 * u + 16 * s, tlo[db], thi[db]);
  };
  f32x16 T1[2], T2[2];
  auto tinit = [&](int slot) __attribute__((always_inline)) {
    const float* cst = (const float*)(smem + slot * kSlotB + 2 * kImgB);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (MODE == 0) {
          const f32x4 l = *(const f32x4*)(cst + 32 * u + 8 * j + 4 * hf);
          const f32x4 d = *(const f32x4*)(cst + kT + 32 * u + 8 * j + 4 * hf);
#pragma unroll
          for (int r = 0; r < 4; ++r) { T1[u][4 * j + r] = l[r]; T2[u][4 * j + r] = d[r]; }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) { T1[u][4 * j + r] = nl; T2[u][4 * j + r] = nd; }
        }
      }
    }
  };
  bf16x8 ring[kR];
  tinit(0);
  {
    const bf16* I1 = (const bf16*)smem;
    const bf16* I2 = (const bf16*)(smem + kImgB);
#pragma unroll
    for (int m = 0; m < kAhead; ++m) ring[m] = operand(I1, I2, m);
  }
  int cur = 0;
  for (int t = t0; t < t1; ++t) {
    const int nxt = cur == 2 ? 0 : cur + 1, nn = nxt == 2 ? 0 : nxt + 1;
    if (!(ABL & 4) && t + 2 < t1) stage(t + 2, nn);
    const bf16* I1 = (const bf16*)(smem + cur * kSlotB);
    const bf16* I2 = (const bf16*)(smem + cur * kSlotB + kImgB);
    const bf16* N1 = (const bf16*)(smem + nxt * kSlotB);
    const bf16* N2 = (const bf16*)(smem + nxt * kSlotB + kImgB);
    const int y0 = t * kT;
    const bool diag = CAUSAL && (MODE == 0 ? y0 < rw + kWw : y0 + kT - 1 > rw);
    bf16x8 pf[2][2], sf[2][2];  // [u][s]
    // values 2 ip, 2 ip + 1 of block u
    auto item2 = [&](int u, int ip) __attribute__((always_inline)) {
      const int v = 2 * ip;
      f32x2 x = f32x2{T1[u][v], T1[u][v + 1]} * f32x2{c2, c2};
      if (diag) {
        const int y = y0 + 32 * u + 8 * (v >> 2) + 4 * hf + (v & 3);
        if (MODE == 0 ? my > y : y > my) x[0] = -INFINITY;
        if (MODE == 0 ? my > y + 1 : y + 1 > my) x[1] = -INFINITY;
      }
      const f32x2 pv = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
      const f32x2 ds = pv * f32x2{T2[u][v], T2[u][v + 1]};
      T1[u][v] = pv[0]; T1[u][v + 1] = pv[1];
      T2[u][v] = ds[0]; T2[u][v + 1] = ds[1];
    };
    // packs of block u: MODE 0 P(s = 0), dS(0), P(1), dS(1); MODE 1 dS(0), dS(1)
    auto piece = [&](int u, int k) __attribute__((always_inline)) {
      if (MODE == 0) {
        if (k & 1) sf[u][k >> 1] = bwdbf16::to_bf16x8(T2[u], k >> 1);
        else pf[u][k >> 1] = bwdbf16::to_bf16x8(T1[u], k >> 1);
      } else {
        sf[u][k] = bwdbf16::to_bf16x8(T2[u], k);
      }
    };
    constexpr int kNP = MODE == 0 ? 4 : 2;
    constexpr int kAct = 8 + kNP;
    auto action = [&](int u, int a) __attribute__((always_inline)) {
      if (ABL & 2) {
        if (a < kNP) piece(u, a);
      } else if (a < 8) {
        item2(u, a);
      } else {
        piece(u, a - 8);
      }
    };
#pragma unroll
    for (int m = 0; m < kL; ++m) {
      const int mp = m + kAhead;
      ring[mp % kR] = mp < kL ? operand(I1, I2, mp) : operand(N1, N2, mp - kL);
      const bf16x8 a = ring[m % kR];
      if (m < 32) {
        const int u = m >> 4, ks = (m >> 1) & 7;
        if (m & 1) T2[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, xf2[ks], T2[u], 0, 0, 0);
        else T1[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, xf1[ks], T1[u], 0, 0, 0);
      } else {
        const int j = m - 32, u = j / kNA, jj = j % kNA;
        const int s = MODE == 0 ? jj >> 3 : jj >> 2, db = MODE == 0 ? (jj >> 1) & 3 : jj & 3;
        if (MODE == 0) {
          if (jj & 1) mma32a(acc1[db], a, sf[u][s]);  // dKᵀ += Qᵀ·dS
          else mma32a(acc2[db], a, pf[u][s]);         // dVᵀ += dOᵀ·P
        } else {
          mma32a(acc1[db], a, sf[u][s]);  // dQᵀ += Kᵀ·dSᵀ
        }
      }
      const int u = m < 32 ? 0 : 1, w = m < 32 ? m - 16 : m - 32;
      const int wl = u == 0 ? 16 : kNA;
      if (w >= 0 && w < wl) {
#pragma unroll
        for (int a2 = w * kAct / wl; a2 < (w + 1) * kAct / wl; ++a2) action(u, a2);
      }
      if (m == 32 + kNA) tinit(nxt);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!(ABL & 1)) __syncthreads();
    cur = nxt;
  }

  if (my < N) {
    const float sc = p.scale;
    if (MODE == 0) {
      bf16* dKg = (bf16*)p.dk + b * p.sdk[0] + hh * p.sdk[1] + (int64_t)my * p.sdk[2];
      bf16* dVg = (bf16*)p.dv + b * p.sdv[0] + hh * p.sdv[1] + (int64_t)my * p.sdv[2];
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = 32 * db + 8 * j + 4 * hf;
          store4(dKg + col, acc1[db][4 * j] * sc, acc1[db][4 * j + 1] * sc, acc1[db][4 * j + 2] * sc,
                 acc1[db][4 * j + 3] * sc, true);
          store4(dVg + col, acc2[db][4 * j], acc2[db][4 * j + 1], acc2[db][4 * j + 2], acc2[db][4 * j + 3], true);
        }
    } else {
      bf16* dQg = (bf16*)p.dq + b * p.sdq[0] + hh * p.sdq[1] + (int64_t)my * p.sdq[2];
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = 32 * db + 8 * j + 4 * hf;
          store4(dQg + col, acc1[db][4 * j] * sc, acc1[db][4 * j + 1] * sc, acc1[db][4 * j + 2] * sc,
                 acc1[db][4 * j + 3] * sc, true);
        }
    }
  }
  }  // pass
}

hipError_t launch_prep_d128(const AttnArgs& a, hipStream_t st);  // fa_bwd_bf16.hip

// The d = 128 backward: the dQ pass (forming the row constants) then the dK/dV pass, or, for the
// diagnostics forms without PREP, the prep kernel (fa_bwd_prep_bf16<128>) and the two passes.
// bf16, d = 128, 16-B rows, every per-head row offset (plus one tile past N) inside the 31-bit
// buffer range.
hipError_t launch_bwd_d128_passes(const AttnArgs& a, bool causal, hipStream_t st) {
  const int nbh = (a.N + kBR - 1) / kBR;
  // causal: light / heavy pairs while the paired grid keeps a workgroup per CU
  bool pair = causal && (int64_t)((nbh + 1) / 2) * a.B * a.H >= 256;
#ifdef MT_DIAGNOSTICS
  if (a.knob == 1) pair = false;
#endif
  const int64_t nblk = (int64_t)(pair ? (nbh + 1) / 2 : nbh) * a.B * a.H;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  // the one-wave-per-SIMD form for both passes (round 4: 3.40 -> 3.30 ms non-causal, 2.08 ->
  // 1.99 ms causal at (8,16,4096,128) against the two-wave form)
  void (*kd)(AttnArgs, int) = pair ? fa_bwd_d128w_bf16<0, true, true>
                              : causal ? fa_bwd_d128w_bf16<0, true> : fa_bwd_d128w_bf16<0, false>;
  // the dQ pass in 8-wave workgroups of the same form, two waves per SIMD (256 query rows per
  // workgroup, the accumulators in VGPRs: 244 registers non-causal with the operand ring 3 slots
  // ahead; causal with light / heavy pairs of 256-row blocks and the ring 2 ahead, 9 registers
  // spilled), while the grid still holds a workgroup per CU: (8,16,4096,128) 3.31 -> 3.09 ms,
  // causal 1.96 -> 1.86 ms; at (2,8,1024,128), 64 workgroups, the 8-wave pass was 0.084
  // against 0.071 ms
  const int nbh8 = (a.N + 255) / 256;
  bool q8 = !causal && (int64_t)nbh8 * a.B * a.H >= 256;
  bool q8p = causal && (int64_t)((nbh8 + 1) / 2) * a.B * a.H >= 256;
  // the product's dQ pass forms the row constants itself (PREP) and runs first, the dK/dV pass
  // reads them second: no prep launch (its 51 µs at (8,16,4096,128) read O and dO once more)
  void (*kq)(AttnArgs, int) = q8p ? fa_bwd_d128w_bf16<1, true, true, true, 0, 2, 8, true>
                              : pair ? fa_bwd_d128w_bf16<1, true, true, true, 0, 7, 4, true>
                              : causal ? fa_bwd_d128w_bf16<1, true, false, true, 0, 7, 4, true>
                              : q8 ? fa_bwd_d128w_bf16<1, false, false, true, 0, 3, 8, true>
                                   : fa_bwd_d128w_bf16<1, false, false, true, 0, 7, 4, true>;
  void (*const kq_prep)(AttnArgs, int) = kq;
  bool wd = true, wq = true;
  int kt_d = 64, kt_q = 64;
#ifdef MT_DIAGNOSTICS
  // knob 54: the round-4 order (prep kernel, dK/dV pass, dQ pass without PREP)
  if (a.knob == 54)
    kq = q8p ? fa_bwd_d128w_bf16<1, true, true, true, 0, 2, 8>
         : pair ? fa_bwd_d128w_bf16<1, true, true>
         : causal ? fa_bwd_d128w_bf16<1, true>
         : q8 ? fa_bwd_d128w_bf16<1, false, false, true, 0, 3, 8> : fa_bwd_d128w_bf16<1, false>;
  void (*const kq_product)(AttnArgs, int) = a.knob == 54 ? kq : kq_prep;
  // knob 50: the dQ pass in the 4-wave form at any grid
  if (a.knob == 50) kq = pair ? fa_bwd_d128w_bf16<1, true, true> : causal ? fa_bwd_d128w_bf16<1, true> : fa_bwd_d128w_bf16<1, false>;
  // the two-wave form (knob 34: both passes; 12 / 14 / 15: with operand reads 2 / 4 / 5 MFMA
  // slots ahead, non-causal; 17 / 18 / 19: 128-row staging steps in both passes / the dQ pass
  // / the dK/dV pass, the other pass in the one-wave form)
  if (a.knob == 34 || a.knob == 12 || a.knob == 14 || a.knob == 15) {
    kd = pair ? fa_bwd_d128_bf16<0, true, true> : causal ? fa_bwd_d128_bf16<0, true> : fa_bwd_d128_bf16<0, false>;
    kq = pair ? fa_bwd_d128_bf16<1, true, true> : causal ? fa_bwd_d128_bf16<1, true> : fa_bwd_d128_bf16<1, false>;
    wd = wq = false;
  }
#define MT_AH(K, A)                                                       \
  if (!causal && a.knob == K) {                                           \
    kd = fa_bwd_d128_bf16<0, false, false, A>;                            \
    kq = fa_bwd_d128_bf16<1, false, false, A>;                            \
  }
  MT_AH(12, 2) MT_AH(14, 4) MT_AH(15, 5)
#undef MT_AH
  if (a.knob == 17 || a.knob == 19) {
    kd = pair ? fa_bwd_d128_bf16<0, true, true, 3, 128> : causal ? fa_bwd_d128_bf16<0, true, false, 3, 128>
                                                          : fa_bwd_d128_bf16<0, false, false, 3, 128>;
    kt_d = 128;
    wd = false;
  }
  if (a.knob == 17 || a.knob == 18) {
    kq = pair ? fa_bwd_d128_bf16<1, true, true, 3, 128> : causal ? fa_bwd_d128_bf16<1, true, false, 3, 128>
                                                          : fa_bwd_d128_bf16<1, false, false, 3, 128>;
    kt_q = 128;
    wq = false;
  }
  // the one-wave form without the packed softmax (knob 20), and its timing-only ablations
  // (29 / 30 / 31: ABL 1 / 2 / 4)
#define MT_W(PK, ABL)                                                                              \
  {                                                                                                \
    kd = pair ? fa_bwd_d128w_bf16<0, true, true, PK, ABL> : causal ? fa_bwd_d128w_bf16<0, true, false, PK, ABL> \
                                                          : fa_bwd_d128w_bf16<0, false, false, PK, ABL>; \
    kq = pair ? fa_bwd_d128w_bf16<1, true, true, PK, ABL> : causal ? fa_bwd_d128w_bf16<1, true, false, PK, ABL> \
                                                          : fa_bwd_d128w_bf16<1, false, false, PK, ABL>; \
  }
  if (a.knob == 20) MT_W(false, 0)
  if (a.knob == 29) MT_W(true, 1)
  if (a.knob == 30) MT_W(true, 2)
  if (a.knob == 31) MT_W(true, 4)
#undef MT_W
  // the 32x32x16 form (knob 36: both passes, 37: the dQ pass, 38: the dK/dV pass; 39 / 40 /
  // 41: both passes with the ablations ABL 1 / 2 / 4)
#define MT_X(ABL)                                                                                \
  {                                                                                              \
    if (a.knob != 37)                                                                            \
      kd = pair ? fa_bwd_d128x_bf16<0, true, true, ABL> : causal ? fa_bwd_d128x_bf16<0, true, false, ABL> \
                                                        : fa_bwd_d128x_bf16<0, false, false, ABL>; \
    if (a.knob != 38)                                                                            \
      kq = pair ? fa_bwd_d128x_bf16<1, true, true, ABL> : causal ? fa_bwd_d128x_bf16<1, true, false, ABL> \
                                                        : fa_bwd_d128x_bf16<1, false, false, ABL>; \
  }
  if (a.knob >= 36 && a.knob <= 38) MT_X(0)
  // the one-wave form's operand ring 3 / 15 slots ahead (knobs 43 / 44)
#define MT_A(K, AH)                                                                               \
  if (a.knob == K) {                                                                              \
    kd = pair ? fa_bwd_d128w_bf16<0, true, true, true, 0, AH> : causal ? fa_bwd_d128w_bf16<0, true, false, true, 0, AH> \
                                                              : fa_bwd_d128w_bf16<0, false, false, true, 0, AH>; \
    kq = pair ? fa_bwd_d128w_bf16<1, true, true, true, 0, AH> : causal ? fa_bwd_d128w_bf16<1, true, false, true, 0, AH> \
                                                              : fa_bwd_d128w_bf16<1, false, false, true, 0, AH>; \
  }
  MT_A(43, 3) MT_A(44, 15)
#undef MT_A
  if (a.knob == 39) MT_X(1)
  if (a.knob == 40) MT_X(2)
  if (a.knob == 41) MT_X(4)
#undef MT_X
#endif
#ifdef MT_DIAGNOSTICS
  if (kq != kq_product) q8 = q8p = false;  // a diagnostics form replaced the dQ kernel
  // the 8-wave dQ pass with the operand ring 2 (knob 48) / 5 (knob 49) slots ahead, and causal
  // ones (47: 3 ahead, 9 registers spilled; 48: 2 ahead)
  if (a.knob == 53 && causal) {  // the paired causal 8-wave dQ pass with the ring 3 ahead
    kq = fa_bwd_d128w_bf16<1, true, true, true, 0, 3, 8>;
    q8p = true;
  }
  if (a.knob == 47 || a.knob == 48 || (a.knob == 49 && !causal)) {
    kq = a.knob == 49 ? fa_bwd_d128w_bf16<1, false, false, true, 0, 5, 8>
         : a.knob == 48 ? (causal ? fa_bwd_d128w_bf16<1, true, false, true, 0, 2, 8> : fa_bwd_d128w_bf16<1, false, false, true, 0, 2, 8>)
         : causal ? fa_bwd_d128w_bf16<1, true, false, true, 0, 3, 8> : fa_bwd_d128w_bf16<1, false, false, true, 0, 3, 8>;
    q8 = true;
  }
#endif
  const int nbh_q = (q8 || q8p) ? nbh8 : nbh;
  const int64_t nblk_q = q8 ? (int64_t)nbh8 * a.B * a.H : q8p ? (int64_t)((nbh8 + 1) / 2) * a.B * a.H : nblk;
  const bool prep_in_dq = kq == kq_prep;
  if (!prep_in_dq) {
    const hipError_t e = launch_prep_d128(a, st);
    if (e != hipSuccess) return e;
  }
  for (int step = 0; step < 2; ++step) {
    const int pass = prep_in_dq ? 1 - step : step;  // 1 = the dQ pass
    void (*k)(AttnArgs, int) = pass ? kq : kd;
    const bool w = pass ? wq : wd;
    const int smem = w ? 3 * slot_bytes(kT) : smem_bytes(pass ? kt_q : kt_d);
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    if (e != hipSuccess) return e;
    const int thr = (pass && (q8 || q8p)) ? 512 : w ? 256 : 512;
    hipLaunchKernelGGL(k, dim3((unsigned)(pass ? nblk_q : nblk)), dim3(thr), smem, st, a, pass ? nbh_q : nbh);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace mt
