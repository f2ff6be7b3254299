// FlashAttention forward, generic tiled kernel (fp32 and bf16, any head dim).
//
// Replaces the reference forward_kernel / forward_kernel_causal
// (src/flashattention_kernel.cu:9-112, :438-545). Same contract: O = softmax(QKᵀ/√d) V
// per (b, h) slice, plus the row statistics m (max of the scaled logits) and
// l = Σ exp(s − m), so that P = exp(s − m)/l (:194). Causal masks key > query.
//
// MI355X design (not the reference's FA-1 loop order):
//  * Q-tile outer loop; a 256-thread workgroup (4 waves) owns BQ = 128 queries,
//    32 per wave, and streams K/V tiles of BK keys through LDS.
//  * "Query on the lane": Sᵀ = K·Qᵀ on MFMA puts one query per lane column, so the
//    online softmax (row max / row sum / rescale) is lane-local except for one
//    cross-half shuffle, and Sᵀ feeds Oᵀ = Vᵀ·Pᵀ directly as the MFMA B operand
//    (no LDS round trip for P). V is read transposed with ds_read_b64_tr_b16.
//  * exp2 with log2(e)/√d folded into one scale; m, l kept in registers; O written
//    once (the reference read-modify-writes O in HBM for every K tile, :92-104).
//  * Head dims above the tile DT are handled by a d-chunked QKᵀ and a grid.z split
//    of the O columns (each z-slice recomputes S; exact, only slower).
//  * int64 addressing throughout (the reference overflows at 2^31 elements).
#include <type_traits>

#include "fa_common.h"

namespace mt {

template <typename T, int DT, int KB, bool VEC, bool CAUSAL>
__global__ __launch_bounds__(256, 3) void fa_fwd_generic(AttnArgs p) {
  constexpr int BQ = 128, BK = 32 * KB;
  constexpr int PAD = 16 / sizeof(T);
  constexpr int LD = DT + PAD;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* sQ = (T*)smem;
  T* sK = sQ + BQ * LD;
  T* sV = sK + BK * LD;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N, d = p.d;
  // XCD-aware block order: the grid is flattened and dealt out so that all query blocks of
  // one (b,h) run on one XCD and find its K/V in that XCD's L2 (the hardware hands
  // consecutive workgroups to the 8 XCDs in turn)
  const int nqb = gridDim.x, nbh = gridDim.y;
  const int hw = blockIdx.y * nqb + blockIdx.x, nblk = nqb * nbh;
  const int xcd = hw & 7, slot = hw >> 3, qd = nblk >> 3, rm = nblk & 7;
  const int logical = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + slot;
  const int q0 = (logical % nqb) * BQ;
  const int bh = logical / nqb, b = bh / p.H, hh = bh % p.H;
  const int oc = blockIdx.z * DT;  // first output column of this slice
  const T* Qg = (const T*)p.q + b * p.sq[0] + hh * p.sq[1];
  const T* Kg = (const T*)p.k + b * p.sk[0] + hh * p.sk[1];
  const T* Vg = (const T*)p.v + b * p.sv[0] + hh * p.sv[1];
  const int dpad = (d + 15) & ~15;
  const int nch = (dpad + DT - 1) / DT;
  const int my_q = q0 + wave * 32 + c32;
  const int wave_qmax = q0 + wave * 32 + 31;
  const int Nk = kv_keys(p, b);  // keys >= Nk are padding

  float m_run = -INFINITY, l_run = 0.f;
  f32x16 O[DT / 32];
#pragma unroll
  for (int i = 0; i < DT / 32; ++i) O[i] = f32x16{};

  const int kend = CAUSAL ? min(Nk, q0 + BQ) : Nk;
  const int ntiles = (kend + BK - 1) / BK;

  // One d-chunk with 16-B rows: the K / V tile t + 1 is loaded into registers while tile t
  // computes and written to LDS after the next barrier, so no global-load latency is exposed
  // after the first tile. Otherwise: K (per d-chunk), then V, staged in place.
  const bool pref = VEC && nch == 1;
  constexpr int EPC = 16 / sizeof(T), CPR = DT / EPC, NCK = BK * CPR / 256;
  uint4 pk[NCK], pv[NCK];
  auto pre_load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NCK; ++i) {
      const int ch = tid + 256 * i, r = ch / CPR, cc = (ch % CPR) * EPC, gr = k0 + r;
      pk[i] = pv[i] = make_uint4(0, 0, 0, 0);
      if (gr < N && cc < d) pk[i] = *(const uint4*)(Kg + (int64_t)gr * p.sk[2] + cc);
      if (gr < N && oc + cc < d) pv[i] = *(const uint4*)(Vg + (int64_t)gr * p.sv[2] + oc + cc);
    }
  };
  auto pre_store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NCK; ++i) {
      const int ch = tid + 256 * i, r = ch / CPR, cc = (ch % CPR) * EPC;
      *(uint4*)(sK + r * LD + cc) = pk[i];
      *(uint4*)(sV + r * LD + cc) = pv[i];
    }
  };
  if (nch == 1) stage_tile<T, BQ, DT, 256, VEC>(sQ, LD, Qg, p.sq[2], q0, N, 0, d);
  if (pref) pre_load(0);

  for (int t = 0; t < ntiles; ++t) {
    const int k0 = t * BK;
    const bool active = !(CAUSAL && k0 > wave_qmax);
    f32x16 S[KB];
#pragma unroll
    for (int i = 0; i < KB; ++i) S[i] = f32x16{};
    for (int c = 0; c < nch; ++c) {
      __syncthreads();
      if (pref) {
        pre_store();
        if (t + 1 < ntiles) pre_load(k0 + BK);
      } else {
        if (nch > 1) stage_tile<T, BQ, DT, 256, VEC>(sQ, LD, Qg, p.sq[2], q0, N, c * DT, d);
        stage_tile<T, BK, DT, 256, VEC>(sK, LD, Kg, p.sk[2], k0, N, c * DT, d);
      }
      __syncthreads();
      const int ksteps = min(DT, dpad - c * DT) / 16;
      if (active) {
        for (int ks = 0; ks < ksteps; ++ks) {
          Frag<T> bq = row_frag<T>(sQ + (wave * 32 + c32) * LD + ks * 16 + 8 * hf);
#pragma unroll
          for (int kb = 0; kb < KB; ++kb) {
            Frag<T> ak = row_frag<T>(sK + (kb * 32 + c32) * LD + ks * 16 + 8 * hf);
            mma(S[kb], ak, bq);
          }
        }
      }
    }
    // V rows k0.., output columns oc..oc+DT (sV is not read by the QKᵀ phase).
    if (!pref) stage_tile<T, BK, DT, 256, VEC>(sV, LD, Vg, p.sv[2], k0, N, oc, d);

    if (active) {
      // Online softmax in the log2 domain; lane (c32, hf) holds 16*KB keys of query my_q.
      float smax = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + kb * 32 + acc_row(r, hf);
          float x = S[kb][r] * p.scale_log2;
          if (key >= Nk || (CAUSAL && key > my_q)) x = -INFINITY;
          S[kb][r] = x;
          smax = fmaxf(smax, x);
        }
      smax = fmaxf(smax, __shfl_xor(smax, 32));
      const float m_new = fmaxf(m_run, smax);
      const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
      float rs = 0.f;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = __builtin_amdgcn_exp2f(S[kb][r] - m_use);
          S[kb][r] = e;
          rs += e;
        }
      l_run = l_run * alpha + rs;
      m_run = m_new;
#pragma unroll
      for (int i = 0; i < DT / 32; ++i) O[i] *= alpha;
    }
    if (!pref) __syncthreads();  // the V tile staged above
    if (active) {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          Frag<T> bp = acc_frag<T>(S[kb], s);
#pragma unroll
          for (int db = 0; db < DT / 32; ++db) {
            Frag<T> av = col_frag<T>(sV, LD, kb * 32 + 16 * s + 4 * hf, db * 32, lane);
            mma(O[db], av, bp);
          }
        }
    }
  }

  // Epilogue: combine the two lane halves' partial row sums, normalise, store (a row with no
  // key, kv_len = 0, stores O = 0, m = -inf, l = 0).
  const float l_tot = l_run + __shfl_xor(l_run, 32);
  const float inv_l = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (my_q < N) {
    const int64_t oe = b * p.so[0] + hh * p.so[1] + (int64_t)my_q * p.so[2];
    T* Og = (T*)p.out + oe;
    float* Of = (float*)p.out + oe;  // bf16 inputs with an fp32 output (o_f32)
    const bool f32o = !std::is_same<T, float>::value && p.o_f32;
#pragma unroll
    for (int db = 0; db < DT / 32; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = oc + db * 32 + 8 * g + 4 * hf;
        const float a[4] = {O[db][4 * g] * inv_l, O[db][4 * g + 1] * inv_l,
                            O[db][4 * g + 2] * inv_l, O[db][4 * g + 3] * inv_l};
        if (f32o) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col + e < d) Of[col + e] = a[e];
        } else if (VEC && col + 3 < d) {
          store4(Og + col, a[0], a[1], a[2], a[3], true);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col + e < d) Og[col + e] = from_f32<T>(a[e]);
        }
      }
    if (blockIdx.z == 0 && hf == 0) {
      const int64_t row = (int64_t)bh * N + my_q;
      if (p.m) p.m[row] = m_run * kLn2;
      if (p.l) p.l[row] = l_tot;
    }
  }
}


// One d-chunk with 16-B rows (the fp32 path of minitorch's MHA at d <= 64, config 2): the
// wave's Q fragments live in registers for the whole launch and K/V go through a two-slot
// LDS ring, so a tile takes one barrier instead of two. Tile t + 1 was loaded into
// registers during tile t - 1 and is written to the other slot after tile t computes (that
// slot was last read in tile t - 1, before the previous barrier); tile t + 2 is then loaded.
// Same math, masks, m/l contract and block order as fa_fwd_generic.
// PAIR: a workgroup runs query blocks u and nqb - 1 - u of one head in turn (causal: a
// light and a heavy block, every workgroup walks nqb + 1 key-tile pairs' worth; non-causal:
// half the workgroups, each filling the ring for its second block while it drains the first).
// (32-key slots at four workgroups per CU, 128 VGPRs with 9 spilled, measured 4.8 % slower
// non-causal and 22 % slower causal: profiles/r2m_ab_fp32_fwd_ring32.txt; not kept.)
// X3 (fp32 only): both products on the bf16 MFMA with every fp32 operand in three bf16 pieces
// (fa_common.h mma_x3: six 32x32x16 bf16 MFMAs per 16-deep k step, fp32 accuracy, 2.67x the
// v_mfma_f32_32x32x2_f32 rate). Q is split once into registers; each K / V tile is split once
// when it is written to the ring, into three bf16 planes ([BK][DT + 8] each, read like the bf16
// kernel's tiles); P is split per tile in registers.
template <typename T, int DT, int KB, bool CAUSAL, bool PAIR, bool X3 = false>
__global__ __launch_bounds__(256, 2) void fa_fwd_generic_ring(AttnArgs p) {
  static_assert(!X3 || std::is_same<T, float>::value, "x3: fp32 inputs");
  constexpr int BQ = 128, BK = 32 * KB;
  constexpr int PAD = 16 / sizeof(T);
  constexpr int LD = DT + PAD;
  constexpr int SLOT = 2 * BK * LD;  // K then V
  constexpr int LDB = DT + 8;        // X3: a bf16 plane's row (elements)
  constexpr int PLANE = BK * LDB;    // X3: one bf16 plane (elements); a slot is K h, m, l, V h, m, l
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* ring = (T*)smem;
  bf16* ring3 = (bf16*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N, d = p.d;
  int u, bh;
  if (CAUSAL && !PAIR)
    xcd_order_heavy_first(u, bh);
  else
    xcd_order(u, bh);
  const int nqb = (N + BQ - 1) / BQ;
  const int b = bh / p.H, hh = bh % p.H;
  const T* Qg = (const T*)p.q + b * p.sq[0] + hh * p.sq[1];
  const T* Kg = (const T*)p.k + b * p.sk[0] + hh * p.sk[1];
  const T* Vg = (const T*)p.v + b * p.sv[0] + hh * p.sv[1];
  constexpr int EPC = 16 / sizeof(T), CPR = DT / EPC, NCK = BK * CPR / 256;
#pragma nounroll
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
  if (PAIR && pass == 1 && nqb - 1 - u == u) break;  // odd nqb: the middle block runs alone
  const int q0 = (pass == 0 ? u : nqb - 1 - u) * BQ;
  const int my_q = q0 + wave * 32 + c32;
  const int wave_qmax = q0 + wave * 32 + 31;
  const int Nk = kv_keys(p, b);  // keys >= Nk are padding

  // Q row my_q (clamped; rows past N are computed but not stored), k-step ks: elements
  // 16 ks + 8 hf .. +7, zero past d (d is a multiple of 16 B here)
  Frag<T> bq[X3 ? 1 : DT / 16];
  X3Frag bq3[X3 ? DT / 16 : 1];
  {
    const T* qrow = Qg + (int64_t)min(my_q, N - 1) * p.sq[2];
#pragma unroll
    for (int ks = 0; ks < DT / 16; ++ks) {
      uint4 ch[8 / EPC];
#pragma unroll
      for (int j = 0; j < 8 / EPC; ++j) {
        const int col = 16 * ks + 8 * hf + j * EPC;
        ch[j] = col < d ? *(const uint4*)(qrow + col) : make_uint4(0, 0, 0, 0);
      }
      if constexpr (X3)
        bq3[ks] = x3_split(__builtin_bit_cast(f32x8, ch));
      else
        bq[ks] = __builtin_bit_cast(Frag<T>, ch);
    }
  }

  float m_run = -INFINITY, l_run = 0.f;
  f32x16 O[DT / 32];
#pragma unroll
  for (int i = 0; i < DT / 32; ++i) O[i] = f32x16{};

  const int kend = CAUSAL ? min(Nk, q0 + BQ) : Nk;
  const int ntiles = (kend + BK - 1) / BK;

  uint4 pk[NCK], pv[NCK];
  auto pre_load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NCK; ++i) {
      const int ch = tid + 256 * i, r = ch / CPR, cc = (ch % CPR) * EPC, gr = k0 + r;
      pk[i] = pv[i] = make_uint4(0, 0, 0, 0);
      if (gr < N && cc < d) {
        pk[i] = *(const uint4*)(Kg + (int64_t)gr * p.sk[2] + cc);
        pv[i] = *(const uint4*)(Vg + (int64_t)gr * p.sv[2] + cc);
      }
    }
  };
  auto pre_store = [&](int s) __attribute__((always_inline)) {
    if constexpr (X3) {  // three bf16 planes per tensor: 8 B of each per 16-B chunk
      bf16* sl = ring3 + s * 6 * PLANE;
#pragma unroll
      for (int i = 0; i < NCK; ++i) {
        const int ch = tid + 256 * i, r = ch / CPR, cc = (ch % CPR) * EPC;
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2) {
          const float4 f = __builtin_bit_cast(float4, t2 ? pv[i] : pk[i]);
          unsigned h0, m0, l0, h1, m1, l1;
          x3_split2(f.x, f.y, h0, m0, l0);
          x3_split2(f.z, f.w, h1, m1, l1);
          bf16* pl = sl + 3 * t2 * PLANE + r * LDB + cc;
          *(uint2*)(pl) = make_uint2(h0, h1);
          *(uint2*)(pl + PLANE) = make_uint2(m0, m1);
          *(uint2*)(pl + 2 * PLANE) = make_uint2(l0, l1);
        }
      }
      return;
    }
    T* sK = ring + s * SLOT;
    T* sV = sK + BK * LD;
#pragma unroll
    for (int i = 0; i < NCK; ++i) {
      const int ch = tid + 256 * i, r = ch / CPR, cc = (ch % CPR) * EPC;
      *(uint4*)(sK + r * LD + cc) = pk[i];
      *(uint4*)(sV + r * LD + cc) = pv[i];
    }
  };
  if (ntiles > 0) {
    pre_load(0);
    pre_store(0);
    if (ntiles > 1) pre_load(BK);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int k0 = t * BK;
    const T* sK = ring + (t & 1) * SLOT;
    const T* sV = sK + BK * LD;
    const bf16* sK3 = ring3 + (t & 1) * 6 * PLANE;  // X3: K h, m, l planes, then V's
    const bf16* sV3 = sK3 + 3 * PLANE;
    if (!(CAUSAL && k0 > wave_qmax)) {
      f32x16 S[KB];
#pragma unroll
      for (int i = 0; i < KB; ++i) S[i] = f32x16{};
      // all DT / 16 k-steps, unrolled: bq[] indexed by a constant (a runtime index makes hipcc
      // move each fragment through s_set_gpr_idx, and a runtime trip count copies S between
      // branches); columns past d are zero in both Q and K, so they add nothing
#pragma unroll
      for (int ks = 0; ks < DT / 16; ++ks) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
          if constexpr (X3) {
            const int o = (kb * 32 + c32) * LDB + ks * 16 + 8 * hf;
            X3Frag ak;
            ak.h = *(const bf16x8*)(sK3 + o);
            ak.m = *(const bf16x8*)(sK3 + PLANE + o);
            ak.l = *(const bf16x8*)(sK3 + 2 * PLANE + o);
            mma_x3(S[kb], ak, bq3[ks]);
          } else {
            Frag<T> ak = row_frag<T>(sK + (kb * 32 + c32) * LD + ks * 16 + 8 * hf);
            mma(S[kb], ak, bq[ks]);
          }
        }
      }
      // masks only on the ragged last tile and on tiles that reach past the wave's first
      // query (causal); the row max is taken on the raw scores (the scale c2 > 0), and
      // exp2(c2·s − m) is one fma into one v_exp_f32
      const float c2 = p.scale_log2;
      if (k0 + BK > Nk || (CAUSAL && k0 + BK - 1 > q0 + wave * 32)) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + kb * 32 + acc_row(r, hf);
            if (key >= Nk || (CAUSAL && key > my_q)) S[kb][r] = -INFINITY;
          }
      }
      float smax = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) smax = fmaxf(smax, S[kb][r]);
      smax = fmaxf(smax, __shfl_xor(smax, 32));
      const float m_new = fmaxf(m_run, smax * c2);
      const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
      float rs = 0.f;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(S[kb][r], c2, -m_use));
          S[kb][r] = e;
          rs += e;
        }
      l_run = l_run * alpha + rs;
      m_run = m_new;
      // X3: the tile's PV in its own accumulator, added to the running O by a VALU fma: the
      // bf16 MFMA's accumulation is not a round-to-nearest fp32 add chain, and over thousands
      // of keys its error compounds into a bias (1.2e-5 relative in a dW_out at N = 4096, where
      // the fp32 MFMA's chain stayed within 1e-6); within one 32-key tile it stays below 1e-6
      f32x16 Ot[X3 ? DT / 32 : 1];
      if constexpr (X3) {
#pragma unroll
        for (int i = 0; i < DT / 32; ++i) Ot[i] = f32x16{};
      } else {
#pragma unroll
        for (int i = 0; i < DT / 32; ++i) O[i] *= alpha;
      }
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if constexpr (X3) {
            const X3Frag bp = x3_split(acc_frag<float>(S[kb], s));
#pragma unroll
            for (int db = 0; db < DT / 32; ++db) {
              const int k0v = kb * 32 + 16 * s + 4 * hf;
              X3Frag av;
              av.h = col_frag<bf16>(sV3, LDB, k0v, db * 32, lane);
              av.m = col_frag<bf16>(sV3 + PLANE, LDB, k0v, db * 32, lane);
              av.l = col_frag<bf16>(sV3 + 2 * PLANE, LDB, k0v, db * 32, lane);
              mma_x3(Ot[db], av, bp);
            }
            continue;
          }
          Frag<T> bp = acc_frag<T>(S[kb], s);
#pragma unroll
          for (int db = 0; db < DT / 32; ++db) {
            Frag<T> av = col_frag<T>(sV, LD, kb * 32 + 16 * s + 4 * hf, db * 32, lane);
            mma(O[db], av, bp);
          }
        }
      if constexpr (X3) {
#pragma unroll
        for (int i = 0; i < DT / 32; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) O[i][r] = __builtin_fmaf(O[i][r], alpha, Ot[i][r]);
      }
    }
    if (t + 1 < ntiles) {
      pre_store((t + 1) & 1);
      if (t + 2 < ntiles) pre_load(k0 + 2 * BK);
    }
    __syncthreads();
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32);
  const float inv_l = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (my_q < N) {
    const int64_t oe = b * p.so[0] + hh * p.so[1] + (int64_t)my_q * p.so[2];
    T* Og = (T*)p.out + oe;
    float* Of = (float*)p.out + oe;  // bf16 inputs with an fp32 output (o_f32)
    const bool f32o = !std::is_same<T, float>::value && p.o_f32;
#pragma unroll
    for (int db = 0; db < DT / 32; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = db * 32 + 8 * g + 4 * hf;
        if (col < d && f32o)  // d is a multiple of 4 here
          store4(Of + col, O[db][4 * g] * inv_l, O[db][4 * g + 1] * inv_l, O[db][4 * g + 2] * inv_l,
                 O[db][4 * g + 3] * inv_l, true);
        else if (col < d)
          store4(Og + col, O[db][4 * g] * inv_l, O[db][4 * g + 1] * inv_l, O[db][4 * g + 2] * inv_l,
                 O[db][4 * g + 3] * inv_l, true);
      }
    if (hf == 0) {
      const int64_t row = (int64_t)bh * N + my_q;
      if (p.m) p.m[row] = m_run * kLn2;
      if (p.l) p.l[row] = l_tot;
    }
  }
  }  // pass
}

template <typename T, int DT, int KB, bool CAUSAL, bool PAIR, bool X3 = false>
static hipError_t launch_fwd_ring_t(const AttnArgs& a, hipStream_t st) {
  // two slots of K and V: fp32 / bf16 rows, or (X3) three bf16 planes each
  const size_t smem = X3 ? (size_t)2 * 6 * 32 * KB * (DT + 8) * 2
                         : sizeof(T) * (size_t)(DT + 16 / sizeof(T)) * 4 * 32 * KB;
  auto kfn = fa_fwd_generic_ring<T, DT, KB, CAUSAL, PAIR, X3>;
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)smem);
  if (e != hipSuccess) return e;
  const int nqb = (a.N + 127) / 128;
  dim3 grid(PAIR ? (nqb + 1) / 2 : nqb, a.B * a.H, 1);
  hipLaunchKernelGGL(kfn, grid, dim3(256), smem, st, a);
  return hipGetLastError();
}


template <typename T, int DT, int KB>
static size_t fwd_generic_smem() {
  constexpr int LD = DT + 16 / sizeof(T);
  return sizeof(T) * (size_t)LD * (128 + 2 * 32 * KB);
}

template <typename T, int DT, int KB, bool VEC, bool CAUSAL>
static hipError_t launch_fwd_generic_t(const AttnArgs& a, hipStream_t st) {
  const size_t smem = fwd_generic_smem<T, DT, KB>();
  auto kfn = fa_fwd_generic<T, DT, KB, VEC, CAUSAL>;
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)smem);
  if (e != hipSuccess) return e;
  dim3 grid((a.N + 127) / 128, a.B * a.H, (a.d + DT - 1) / DT);
  hipLaunchKernelGGL(kfn, grid, dim3(256), smem, st, a);
  return hipGetLastError();
}

template <typename T, int DT, int KB>
static hipError_t dispatch_fwd_generic(const AttnArgs& a, bool vec, bool causal, hipStream_t st) {
  if (vec)
    return causal ? launch_fwd_generic_t<T, DT, KB, true, true>(a, st)
                  : launch_fwd_generic_t<T, DT, KB, true, false>(a, st);
  return causal ? launch_fwd_generic_t<T, DT, KB, false, true>(a, st)
                : launch_fwd_generic_t<T, DT, KB, false, false>(a, st);
}

hipError_t launch_fwd_generic(const AttnArgs& a, bool bf16_io, bool vec, bool causal,
                              hipStream_t st, int ring) {
  // fp32 with 16-B rows and d <= 64 (one d-chunk): the register-Q / two-slot ring kernel;
  // ring = 1 unpaired, 2 paired query blocks, 3 paired when the paired grid keeps two
  // workgroups per CU (0: fa_fwd_generic)
  // bf16 reaches this function only for head dims the MFMA fast paths do not take (d != 64,
  // 128) or strided rows; d < 64 with 16-B rows takes the same ring kernel
  if (ring && vec && bf16_io && (a.d < 64 || (a.kv_len && a.d == 64))) {
    const bool pair = ring == 2 || (ring == 3 && (int64_t)((a.N + 255) / 256) * a.B * a.H >= 512);
    if (a.d <= 32)
      return causal ? (pair ? launch_fwd_ring_t<bf16, 32, 2, true, true>(a, st)
                            : launch_fwd_ring_t<bf16, 32, 2, true, false>(a, st))
                    : (pair ? launch_fwd_ring_t<bf16, 32, 2, false, true>(a, st)
                            : launch_fwd_ring_t<bf16, 32, 2, false, false>(a, st));
    return causal ? (pair ? launch_fwd_ring_t<bf16, 64, 2, true, true>(a, st)
                          : launch_fwd_ring_t<bf16, 64, 2, true, false>(a, st))
                  : (pair ? launch_fwd_ring_t<bf16, 64, 2, false, true>(a, st)
                          : launch_fwd_ring_t<bf16, 64, 2, false, false>(a, st));
  }
  if (ring && vec && !bf16_io && a.d <= 64) {
    const bool pair = ring == 2 || (ring == 3 && (int64_t)((a.N + 255) / 256) * a.B * a.H >= 512);
    // round 6: the products on the bf16 MFMA, every fp32 operand in three bf16 pieces (X3,
    // fp32 accuracy: C2 0.277 -> 0.184 ms, causal 0.163 -> 0.108 ms, O within 6.9e-7 of the C
    // oracle on every head against 8.0e-7 for the fp32 MFMA; profiles/r6_ab_fp32_fwd_x3.txt),
    // 32-key slots (three planes per tensor: the 64-key form leaves one workgroup per CU and ran
    // 0.246 ms)
    bool x3 = true;
#ifdef MT_DIAGNOSTICS
    if (a.knob == 65) x3 = false;  // A/B: the v_mfma_f32_32x32x2_f32 ring
    if (a.knob == 64)  // A/B: X3 with 64-key slots (one workgroup per CU)
      return causal ? (pair ? launch_fwd_ring_t<float, 64, 2, true, true, true>(a, st)
                            : launch_fwd_ring_t<float, 64, 2, true, false, true>(a, st))
                    : (pair ? launch_fwd_ring_t<float, 64, 2, false, true, true>(a, st)
                            : launch_fwd_ring_t<float, 64, 2, false, false, true>(a, st));
#endif
    if (x3) {
      if (a.d <= 32)
        return causal ? (pair ? launch_fwd_ring_t<float, 32, 1, true, true, true>(a, st)
                              : launch_fwd_ring_t<float, 32, 1, true, false, true>(a, st))
                      : (pair ? launch_fwd_ring_t<float, 32, 1, false, true, true>(a, st)
                              : launch_fwd_ring_t<float, 32, 1, false, false, true>(a, st));
      return causal ? (pair ? launch_fwd_ring_t<float, 64, 1, true, true, true>(a, st)
                            : launch_fwd_ring_t<float, 64, 1, true, false, true>(a, st))
                    : (pair ? launch_fwd_ring_t<float, 64, 1, false, true, true>(a, st)
                            : launch_fwd_ring_t<float, 64, 1, false, false, true>(a, st));
    }
    if (a.d <= 32)  // 32-column tiles: no zero-padded half of the QKᵀ and PV work (minitorch's
                    // MHA at config 5 has d = 256 / 8 = 32)
      return causal ? (pair ? launch_fwd_ring_t<float, 32, 2, true, true>(a, st)
                            : launch_fwd_ring_t<float, 32, 2, true, false>(a, st))
                    : (pair ? launch_fwd_ring_t<float, 32, 2, false, true>(a, st)
                            : launch_fwd_ring_t<float, 32, 2, false, false>(a, st));
    if (causal)
      return pair ? launch_fwd_ring_t<float, 64, 2, true, true>(a, st)
                  : launch_fwd_ring_t<float, 64, 2, true, false>(a, st);
    return pair ? launch_fwd_ring_t<float, 64, 2, false, true>(a, st)
                : launch_fwd_ring_t<float, 64, 2, false, false>(a, st);
  }
  // fp32 64 < d <= 128: 128-column ring with 32-key slots, unpaired (the paired form spills
  // 36-38 VGPRs at 256); causal grids go heaviest block first
  if (ring && vec && !bf16_io && a.d <= 128)
    return causal ? launch_fwd_ring_t<float, 128, 1, true, false>(a, st)
                  : launch_fwd_ring_t<float, 128, 1, false, false>(a, st);
  if (bf16_io) {
    if (a.d <= 64) return dispatch_fwd_generic<bf16, 64, 2>(a, vec, causal, st);
    return dispatch_fwd_generic<bf16, 128, 2>(a, vec, causal, st);
  }
  if (a.d <= 64) return dispatch_fwd_generic<float, 64, 2>(a, vec, causal, st);
  return dispatch_fwd_generic<float, 128, 1>(a, vec, causal, st);
}

}  // namespace mt
