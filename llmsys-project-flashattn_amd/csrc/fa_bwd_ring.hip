// fp32 (d <= 64) and bf16 (d < 64) backward for one zero-padded d-chunk of 16-B rows: the FA-2 split of
// fa_bwd.hip (dK/dV with the key on the lane, dQ with the query on the lane; same math, same
// masks, same block order and causal pairing) with the workgroup's own rows in registers.
//
// fa_bwd.hip keeps the workgroup's 128 K/V rows (dK/dV) or Q/dO rows (dQ) in LDS next to
// the streamed tile: 87 KiB, one workgroup per CU, one wave per SIMD. Those rows are only
// ever read by the wave that owns them, so here each lane keeps its row's four k-step
// fragments (f32x8 each) in VGPRs and only the streamed 32-row tiles go through LDS, in a
// two-slot ring (35 KiB) with one barrier per tile: tile t + 1 is written to the free slot
// after tile t computes (that slot was last read in tile t - 1, before the previous
// barrier) and tile t + 2 is then loaded into registers. Two workgroups per CU, two waves
// per SIMD. Replaces the reference backward_kernel / backward_kernel_causal
// (src/flashattention_kernel.cu:115-255, :547-690) on the fp32 path minitorch's
// MultiHeadAttention runs.
#include "fa_common.h"

#include <algorithm>

namespace mt {

namespace {

// the KS k-step fragments of row r (zero past d, which is a multiple of 16 B here)
template <typename T, int KS>
__device__ __forceinline__ void row_frags(Frag<T> (&f)[KS], const T* row, int d, int hf) {
  constexpr int EPC = 16 / sizeof(T);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    uint4 ch[8 / EPC];
#pragma unroll
    for (int j = 0; j < 8 / EPC; ++j) {
      const int col = 16 * ks + 8 * hf + j * EPC;
      ch[j] = col < d ? *(const uint4*)(row + col) : make_uint4(0, 0, 0, 0);
    }
    f[ks] = __builtin_bit_cast(Frag<T>, ch);
  }
}

}  // namespace

// dK, dV: grid (nkb or ceil(nkb / 2) when PAIR, B*H); 4 waves x 32 keys; Q/dO tiles of 32
// queries (with their lse2 / delta) streamed through the ring.
// X3 (fp32): the four products on the bf16 MFMA in three pieces per operand (fa_common.h
// mma_x3): the Q / dO tiles split once when written to the ring (three bf16 planes each), the
// register K / V rows per use, P and dS per tile; dK and dV take each k-step's products in a
// fresh sum added with a VALU fp32 add (x3_tile_sum). 1.28-1.43x the fp32-MFMA form, closer to
// float64 on the MHA test's inputs (profiles/r6_x3_split_ring.txt).
template <typename T, int DT, bool CAUSAL, bool PAIR, bool X3 = false>
__global__ __launch_bounds__(256, 2) void fa_bwd_dkv_ring(AttnArgs p) {
  // DT = 64, or 32 for d <= 32; rows padded by 16 B; NCK 16-B chunks per thread per 32-row tile
  constexpr int EPC = 16 / sizeof(T), kLD = DT + EPC, kCPR = DT / EPC;
  constexpr int NCK = (32 * kCPR + 255) / 256, KS = DT / 16, NDB = DT / 32;
  constexpr int BKV = 128, BQ = 32;
  // Q, dO, lse2, delta (bytes); X3: Q and dO as three bf16 planes each ([32][DT + 8])
  constexpr int LDB = DT + 8, PLANE = BQ * LDB;
  constexpr int SLOT = X3 ? 6 * PLANE * 2 + 2 * BQ * 4 : 2 * BQ * kLD * (int)sizeof(T) + 2 * BQ * 4;
  static_assert(!X3 || sizeof(T) == 4, "X3 splits fp32 operands");
  extern __shared__ __attribute__((aligned(16))) char ring[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N, d = p.d;
  int ublk, bh;
  xcd_order(ublk, bh);
  const int b = bh / p.H, hh = bh % p.H;
  const int nkb = (N + BKV - 1) / BKV;
  const T* Qg = (const T*)p.q + b * p.sq[0] + hh * p.sq[1];
  const T* Kg = (const T*)p.k + b * p.sk[0] + hh * p.sk[1];
  const T* Vg = (const T*)p.v + b * p.sv[0] + hh * p.sv[1];
  const T* dOg = (const T*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const float* lse2 = p.lse2 + (int64_t)bh * N;
  const float* delta = p.delta + (int64_t)bh * N;
  const float c2 = p.scale_log2;

#pragma nounroll
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
    const int kblk = !PAIR ? ublk : pass == 0 ? nkb - 1 - ublk : ublk;
    if (PAIR && pass == 1) {
      if (kblk == nkb - 1 - ublk) break;  // odd nkb: the middle block runs alone
      __syncthreads();                     // the first block's LDS reads are done
    }
    const int k0 = kblk * BKV;
    const int my_k = k0 + wave * 32 + c32;
    const int wave_kmin = k0 + wave * 32;
    // the causal skip bound; X3 non-causal: -1 behind an opaque copy, so the tile body stays a
    // branch (as a branch-free body, hipcc 7.2 scheduled it into 200 spilled VGPRs at d = 64)
    int skip_lim = CAUSAL ? wave_kmin : -1;
    if (X3 && !CAUSAL) asm volatile("" : "+s"(skip_lim));
    const int Nk = kv_keys(p, b);  // keys >= Nk are padding: zero gradients
    Frag<T> bk[KS], bv[KS];
    {
      const int kr = min(my_k, N - 1);
      row_frags(bk, Kg + (int64_t)kr * p.sk[2], d, hf);
      row_frags(bv, Vg + (int64_t)kr * p.sv[2], d, hf);
    }
    f32x16 dK[NDB], dV[NDB];
#pragma unroll
    for (int i = 0; i < NDB; ++i) { dK[i] = f32x16{}; dV[i] = f32x16{}; }

    const int qstart = CAUSAL ? k0 : 0;  // k0 is a multiple of BQ
    const int ntile = N > qstart && k0 < Nk ? (N - qstart + BQ - 1) / BQ : 0;
    uint4 pq[NCK], po[NCK];
    float pl = 0.f, pd = 0.f;
    auto pre_load = [&](int qt) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < NCK; ++i) {
        const int ch = tid + 256 * i, r = ch / kCPR, cc = (ch % kCPR) * EPC, gr = qt + r;
        pq[i] = po[i] = make_uint4(0, 0, 0, 0);
        if (ch < 32 * kCPR && gr < N && cc < d) {
          pq[i] = *(const uint4*)(Qg + (int64_t)gr * p.sq[2] + cc);
          po[i] = *(const uint4*)(dOg + (int64_t)gr * p.sdo[2] + cc);
        }
      }
      if (tid < BQ) {
        const int q = qt + tid;
        pl = q < N ? lse2[q] : 0.f;
        pd = q < N ? delta[q] : 0.f;
      }
    };
    auto pre_store = [&](int s) __attribute__((always_inline)) {
      T* sQ = (T*)(ring + s * SLOT);
      T* sO = sQ + BQ * kLD;
#pragma unroll
      for (int i = 0; i < NCK; ++i) {
        const int ch = tid + 256 * i, r = ch / kCPR, cc = (ch % kCPR) * EPC;
        if (ch < 32 * kCPR) {
          if constexpr (X3) {
            bf16* q3 = (bf16*)(ring + s * SLOT) + r * LDB + cc;
            x3_store4(q3, PLANE, pq[i]);
            x3_store4(q3 + 3 * PLANE, PLANE, po[i]);
          } else {
            *(uint4*)(sQ + r * kLD + cc) = pq[i];
            *(uint4*)(sO + r * kLD + cc) = po[i];
          }
        }
      }
      if (tid < BQ) {
        float* sRow = X3 ? (float*)((bf16*)(ring + s * SLOT) + 6 * PLANE) : (float*)(sO + BQ * kLD);
        sRow[tid] = pl;
        sRow[BQ + tid] = pd;
      }
    };
    if (ntile > 0) {
      pre_load(qstart);
      pre_store(0);
      if (ntile > 1) pre_load(qstart + BQ);
    }
    __syncthreads();

#pragma nounroll
    for (int t = 0; t < ntile; ++t) {
      const int qt = qstart + t * BQ;
      const T* sQ = (const T*)(ring + (t & 1) * SLOT);
      const T* sO = sQ + BQ * kLD;
      const bf16* sQ3 = (const bf16*)(ring + (t & 1) * SLOT);  // X3: Q planes, then dO's
      const bf16* sO3 = sQ3 + 3 * PLANE;
      const float* sLse = X3 ? (const float*)(sQ3 + 6 * PLANE) : (const float*)(sO + BQ * kLD);
      const float* sDel = sLse + BQ;
      if (!((CAUSAL || X3) && qt + BQ - 1 < skip_lim)) {
        // Sᵀ and dPᵀ: the lane's column is key my_k, rows are queries qt + acc_row(r, hf)
        f32x16 S = f32x16{}, dP = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int col = ks * 16 + 8 * hf;
          if constexpr (X3) {
            // (an opaque use per tile keeps hipcc from hoisting the loop-invariant splits)
            asm volatile("" : "+v"(bk[ks]), "+v"(bv[ks]));
            mma_x3(S, x3_rows(sQ3 + c32 * LDB + col, PLANE), x3_split(bk[ks]));
            mma_x3(dP, x3_rows(sO3 + c32 * LDB + col, PLANE), x3_split(bv[ks]));
          } else {
            mma(S, row_frag<T>(sQ + c32 * kLD + col), bk[ks]);
            mma(dP, row_frag<T>(sO + c32 * kLD + col), bv[ks]);
          }
        }
        const bool msk = qt + BQ > N || k0 + BKV > Nk || (CAUSAL && qt < wave_kmin + 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ql = acc_row(r, hf);
          const int q = qt + ql;
          float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(S[r], c2, -sLse[ql]));
          if (msk && (q >= N || my_k >= Nk || (CAUSAL && my_k > q))) pv = 0.f;
          S[r] = pv;
          dP[r] = pv * (dP[r] - sDel[ql]);
        }
        if constexpr (X3) {  // each k-step's products in a fresh sum (x3_tile_sum)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const X3Frag bp = x3_split(acc_frag<float>(S, s)), bs = x3_split(acc_frag<float>(dP, s));
#pragma unroll
            for (int db = 0; db < NDB; ++db) {
              f32x16 t = f32x16{};
              mma_x3(t, x3_cols(sO3, PLANE, LDB, 16 * s + 4 * hf, db * 32, lane), bp);
              dV[db] += t;
              t = f32x16{};
              mma_x3(t, x3_cols(sQ3, PLANE, LDB, 16 * s + 4 * hf, db * 32, lane), bs);
              dK[db] += t;
            }
          }
        } else {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const Frag<T> bp = acc_frag<T>(S, s), bs = acc_frag<T>(dP, s);
#pragma unroll
            for (int db = 0; db < NDB; ++db) {
              mma(dV[db], col_frag<T>(sO, kLD, 16 * s + 4 * hf, db * 32, lane), bp);
              mma(dK[db], col_frag<T>(sQ, kLD, 16 * s + 4 * hf, db * 32, lane), bs);
            }
          }
        }
      }
      if (t + 1 < ntile) {
        pre_store((t + 1) & 1);
        if (t + 2 < ntile) pre_load(qt + 2 * BQ);
      }
      __syncthreads();
    }

    if (my_k < N) {
      T* dKg = (T*)p.dk + b * p.sdk[0] + hh * p.sdk[1] + (int64_t)my_k * p.sdk[2];
      T* dVg = (T*)p.dv + b * p.sdv[0] + hh * p.sdv[1] + (int64_t)my_k * p.sdv[2];
      const float sc = p.scale;
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int col = db * 32 + 8 * g + 4 * hf;
          if (col < d) {
            store4(dKg + col, dK[db][4 * g] * sc, dK[db][4 * g + 1] * sc, dK[db][4 * g + 2] * sc,
                   dK[db][4 * g + 3] * sc, true);
            store4(dVg + col, dV[db][4 * g], dV[db][4 * g + 1], dV[db][4 * g + 2], dV[db][4 * g + 3],
                   true);
          }
        }
    }
  }
}

// dQ: grid (nqb or ceil(nqb / 2) when PAIR, B*H); 4 waves x 32 queries; K/V tiles of 32
// keys streamed through the ring. X3 (fp32): K / V tiles as three bf16 planes each, the register
// Q / dO rows split per use, dS per tile, dQ's k-step sums fresh (as fa_bwd_dkv_ring).
template <typename T, int DT, bool CAUSAL, bool PAIR, bool X3 = false>
__global__ __launch_bounds__(256, 2) void fa_bwd_dq_ring(AttnArgs p) {
  // DT = 64, or 32 for d <= 32; rows padded by 16 B; NCK 16-B chunks per thread per 32-row tile
  constexpr int EPC = 16 / sizeof(T), kLD = DT + EPC, kCPR = DT / EPC;
  constexpr int NCK = (32 * kCPR + 255) / 256, KS = DT / 16, NDB = DT / 32;
  constexpr int BQ = 128, BK = 32;
  // K, V (elements of T); X3: K and V as three bf16 planes each ([32][DT + 8])
  constexpr int LDB = DT + 8, PLANE = BK * LDB;
  constexpr int SLOT = X3 ? 6 * PLANE * 2 / (int)sizeof(T) : 2 * BK * kLD;
  static_assert(!X3 || sizeof(T) == 4, "X3 splits fp32 operands");
  extern __shared__ __attribute__((aligned(16))) char ring_raw[];
  T* ring = (T*)ring_raw;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N, d = p.d;
  int ublk, bh;
  xcd_order(ublk, bh);
  const int b = bh / p.H, hh = bh % p.H;
  const int nqb = (N + BQ - 1) / BQ;
  const T* Qg = (const T*)p.q + b * p.sq[0] + hh * p.sq[1];
  const T* Kg = (const T*)p.k + b * p.sk[0] + hh * p.sk[1];
  const T* Vg = (const T*)p.v + b * p.sv[0] + hh * p.sv[1];
  const T* dOg = (const T*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const float c2 = p.scale_log2;

#pragma nounroll
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
    const int qblk = !PAIR ? ublk : pass == 0 ? ublk : nqb - 1 - ublk;
    if (PAIR && pass == 1) {
      if (qblk == ublk) break;  // odd nqb: the middle block runs alone
      __syncthreads();          // the first block's LDS reads are done
    }
    const int q0 = qblk * BQ;
    const int my_q = q0 + wave * 32 + c32;
    const int wave_qmax = q0 + wave * 32 + 31;
    Frag<T> bq[KS], bo[KS];
    float lse_q, del_q;
    {
      const int qr = min(my_q, N - 1);
      row_frags(bq, Qg + (int64_t)qr * p.sq[2], d, hf);
      row_frags(bo, dOg + (int64_t)qr * p.sdo[2], d, hf);
      lse_q = p.lse2[(int64_t)bh * N + qr];
      del_q = p.delta[(int64_t)bh * N + qr];
    }
    f32x16 dQ[NDB];
#pragma unroll
    for (int i = 0; i < NDB; ++i) dQ[i] = f32x16{};

    const int Nk = kv_keys(p, b);  // keys >= Nk are padding
    const int kend = CAUSAL ? min(Nk, q0 + BQ) : Nk;
    const int ntile = (kend + BK - 1) / BK;
    uint4 pk[NCK], pv[NCK];
    auto pre_load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < NCK; ++i) {
        const int ch = tid + 256 * i, r = ch / kCPR, cc = (ch % kCPR) * EPC, gr = k0 + r;
        pk[i] = pv[i] = make_uint4(0, 0, 0, 0);
        if (ch < 32 * kCPR && gr < N && cc < d) {
          pk[i] = *(const uint4*)(Kg + (int64_t)gr * p.sk[2] + cc);
          pv[i] = *(const uint4*)(Vg + (int64_t)gr * p.sv[2] + cc);
        }
      }
    };
    auto pre_store = [&](int s) __attribute__((always_inline)) {
      T* sK = ring + s * SLOT;
      T* sV = sK + BK * kLD;
#pragma unroll
      for (int i = 0; i < NCK; ++i) {
        const int ch = tid + 256 * i, r = ch / kCPR, cc = (ch % kCPR) * EPC;
        if (ch < 32 * kCPR) {
          if constexpr (X3) {
            bf16* k3 = (bf16*)sK + r * LDB + cc;
            x3_store4(k3, PLANE, pk[i]);
            x3_store4(k3 + 3 * PLANE, PLANE, pv[i]);
          } else {
            *(uint4*)(sK + r * kLD + cc) = pk[i];
            *(uint4*)(sV + r * kLD + cc) = pv[i];
          }
        }
      }
    };
    if (ntile > 0) {
      pre_load(0);
      pre_store(0);
      if (ntile > 1) pre_load(BK);
    }
    __syncthreads();

#pragma nounroll
    for (int t = 0; t < ntile; ++t) {
      const int k0 = t * BK;
      const T* sK = ring + (t & 1) * SLOT;
      const T* sV = sK + BK * kLD;
      const bf16* sK3 = (const bf16*)sK;  // X3: K planes, then V's
      const bf16* sV3 = sK3 + 3 * PLANE;
      if (!(CAUSAL && k0 > wave_qmax)) {
        // S and dP with the query on the lane: rows are keys k0 + acc_row(r, hf)
        f32x16 S = f32x16{}, dP = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int col = ks * 16 + 8 * hf;
          if constexpr (X3) {
            asm volatile("" : "+v"(bq[ks]), "+v"(bo[ks]));  // split per use (see fa_bwd_dkv_ring)
            mma_x3(S, x3_rows(sK3 + c32 * LDB + col, PLANE), x3_split(bq[ks]));
            mma_x3(dP, x3_rows(sV3 + c32 * LDB + col, PLANE), x3_split(bo[ks]));
          } else {
            mma(S, row_frag<T>(sK + c32 * kLD + col), bq[ks]);
            mma(dP, row_frag<T>(sV + c32 * kLD + col), bo[ks]);
          }
        }
        const bool msk = k0 + BK > Nk || (CAUSAL && k0 + BK - 1 > q0 + wave * 32);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + acc_row(r, hf);
          float pvv = __builtin_amdgcn_exp2f(__builtin_fmaf(S[r], c2, -lse_q));
          if (msk && (key >= Nk || (CAUSAL && key > my_q))) pvv = 0.f;
          dP[r] = pvv * (dP[r] - del_q);
        }
        if constexpr (X3) {  // the tile's products in a fresh sum (x3_tile_sum)
          const X3Frag bs0 = x3_split(acc_frag<float>(dP, 0)), bs1 = x3_split(acc_frag<float>(dP, 1));
#pragma unroll
          for (int db = 0; db < NDB; ++db) {
            f32x16 t = f32x16{};
            mma_x3(t, x3_cols(sK3, PLANE, LDB, 4 * hf, db * 32, lane), bs0);
            mma_x3(t, x3_cols(sK3, PLANE, LDB, 16 + 4 * hf, db * 32, lane), bs1);
            dQ[db] += t;
          }
        } else {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const Frag<T> bs = acc_frag<T>(dP, s);
#pragma unroll
            for (int db = 0; db < NDB; ++db)
              mma(dQ[db], col_frag<T>(sK, kLD, 16 * s + 4 * hf, db * 32, lane), bs);
          }
        }
      }
      if (t + 1 < ntile) {
        pre_store((t + 1) & 1);
        if (t + 2 < ntile) pre_load(k0 + 2 * BK);
      }
      __syncthreads();
    }

    if (my_q < N) {
      T* dQg = (T*)p.dq + b * p.sdq[0] + hh * p.sdq[1] + (int64_t)my_q * p.sdq[2];
      const float sc = p.scale;
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int col = db * 32 + 8 * g + 4 * hf;
          if (col < d)
            store4(dQg + col, dQ[db][4 * g] * sc, dQ[db][4 * g + 1] * sc, dQ[db][4 * g + 2] * sc,
                   dQ[db][4 * g + 3] * sc, true);
        }
    }
  }
}

// The fp32 backward with dQ in the dK/dV pass (fp32, 32 < d <= 64): 5 products per tile
// instead of the split's 7. The dK/dV half is fa_bwd_dkv_ring's (key on the lane, register-row
// K / V, Q / dO tiles of 32 queries through a two-slot ring) with 8 waves x 32 keys = 256 keys
// per workgroup, one workgroup per CU (two waves per SIMD); the dQ half needs the query on the
// lane, so each wave writes its dSᵀ values into an LDS image dS[query][key] (the transpose) and,
// after a barrier, wave w computes one 16 x 16 tile (query half w & 1, d quarter w >> 1) of
//     dQpart(tile) = dS(32 x 256) · K(256 x 64)
// on v_mfma_f32_16x16x4_f32 from that image and a Kᵀ image [d][key] staged once per block (the
// 256-key contraction in the permuted order key = 64 (lane >> 4) + s, so both operands are
// 16-B LDS reads), and stores it to the slab [head][key block][query][64]. fa_bwd_ring_dq_sum
// then sums each row's key blocks in block order: deterministic, no atomics (the reference
// accumulates dQ serially inside its single pass, src/flashattention_kernel.cu:226-235).
// LDS: ring 2 x 17.25 KiB + Kᵀ 65 KiB + dS 32.5 KiB = 132 KiB.
typedef __attribute__((ext_vector_type(4))) float f32x4;
constexpr int kFrBKV = 256, kFrTL = kFrBKV + 4;  // keys per workgroup; image row (floats)
constexpr int kFrSlot = 2 * 32 * 68 * 4 + 2 * 32 * 4;
constexpr int kFrSmem = 2 * kFrSlot + (64 + 32) * kFrTL * 4;
// X3: the Q and dO tiles as three bf16 planes each ([32][72]), then the row constants
constexpr int kFrLDB = 72, kFrPlane = 32 * kFrLDB;
constexpr int kFrSlotX3 = 6 * kFrPlane * 2 + 2 * 32 * 4;
constexpr int kFrSmemX3 = 2 * kFrSlotX3 + (64 + 32) * kFrTL * 4;

// PREP: the tile's row constants are formed here (lse2 = m·log2e + log2 l from the forward's
// (m, l); δ = rowsum(dO ∘ O) from the staged dO chunks and the O chunks loaded beside them, the
// 16 lanes of a row summed by xor shuffles: the prep kernel's arithmetic), no prep launch
// X3: the four key-on-the-lane products (S, dP, dVᵀ, dKᵀ) on the bf16 MFMA with every fp32
// operand in three bf16 pieces (fa_common.h mma_x3, fp32 accuracy): Q / dO tiles split once when
// written to the ring, K / V once per block, P and dS per tile; the dQ product stays on
// v_mfma_f32_16x16x4_f32 (its Kᵀ image as three planes would not fit the LDS)
template <bool CAUSAL, bool PAIR, bool PREP = true, bool X3 = true>
__global__ __launch_bounds__(512, 1) void fa_bwd_fused_ring(AttnArgs p, float* slab, int bh0) {
  using T = float;
  constexpr int DT = 64, EPC = 4, kLD = DT + EPC, kCPR = DT / EPC, KS = DT / 16, NDB = DT / 32;
  constexpr int BKV = kFrBKV, BQ = 32, SLOT = X3 ? kFrSlotX3 : kFrSlot, TL = kFrTL;
  constexpr int LDB = kFrLDB, PLANE = kFrPlane;
  extern __shared__ __attribute__((aligned(16))) char smem_fr[];
  char* ring = smem_fr;
  float* KT = (float*)(smem_fr + 2 * SLOT);  // [64 d][TL]: Kᵀ of the block's 256 keys
  float* dSi = KT + DT * TL;                 // [32 queries][TL]: the tile's dS
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N, d = p.d;
  int ublk, bhl;
  xcd_order(ublk, bhl);
  const int bh = bh0 + bhl;
  const int b = bh / p.H, hh = bh % p.H;
  const int nkb = (N + BKV - 1) / BKV;
  const T* Qg = (const T*)p.q + b * p.sq[0] + hh * p.sq[1];
  const T* Kg = (const T*)p.k + b * p.sk[0] + hh * p.sk[1];
  const T* Vg = (const T*)p.v + b * p.sv[0] + hh * p.sv[1];
  const T* dOg = (const T*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const T* Og = (const T*)p.o + b * p.so[0] + hh * p.so[1];
  const float* lse2 = p.lse2 + (int64_t)bh * N;
  const float* delta = p.delta + (int64_t)bh * N;
  const float c2 = p.scale_log2;
  // this wave's dQ tile: queries 16 qh .. + 15 of a 32-query tile, d columns 16 d4 .. + 15
  const int qh = wave & 1, d4 = wave >> 1;
  const int ia = (16 * qh + (lane & 15)) * TL + 64 * (lane >> 4);
  const int ib = (16 * d4 + (lane & 15)) * TL + 64 * (lane >> 4);

#pragma nounroll
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
    const int kblk = !PAIR ? ublk : pass == 0 ? nkb - 1 - ublk : ublk;
    if (PAIR && pass == 1) {
      if (kblk == nkb - 1 - ublk) break;  // odd nkb: the middle block runs alone
      __syncthreads();                     // the first block's LDS reads are done
    }
    const int k0 = kblk * BKV;
    const int my_k = k0 + wave * 32 + c32;
    const int wave_kmin = k0 + wave * 32;
    const int Nk = kv_keys(p, b);  // keys >= Nk are padding: zero gradients
    const int kval = min(N, Nk);
    Frag<T> bk[KS], bv[KS];
    {  // (X3: split per use; held split, the three pieces took 32 more VGPRs and spilled)
      const int kr = min(my_k, N - 1);
      row_frags(bk, Kg + (int64_t)kr * p.sk[2], d, hf);
      row_frags(bv, Vg + (int64_t)kr * p.sv[2], d, hf);
    }
    // Kᵀ image: key r fastest across the lanes (conflict-free column stores), zero past the
    // valid keys and past d
#pragma unroll
    for (int i = 0; i < (BKV * kCPR) / 512; ++i) {
      const int ch = tid + 512 * i, r = ch % BKV, cc = (ch / BKV) * EPC, gr = k0 + r;
      float4 v4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gr < kval && cc < d) v4 = *(const float4*)(Kg + (int64_t)gr * p.sk[2] + cc);
      KT[(cc + 0) * TL + r] = v4.x;
      KT[(cc + 1) * TL + r] = v4.y;
      KT[(cc + 2) * TL + r] = v4.z;
      KT[(cc + 3) * TL + r] = v4.w;
    }
    f32x16 dK[NDB], dV[NDB];
#pragma unroll
    for (int i = 0; i < NDB; ++i) { dK[i] = f32x16{}; dV[i] = f32x16{}; }

    const int qstart = CAUSAL ? k0 : 0;  // k0 is a multiple of BQ
    const int ntile = N > qstart && k0 < Nk ? (N - qstart + BQ - 1) / BQ : 0;
    uint4 pq, po, pa;
    float pl = 0.f, pd = 0.f;
    auto pre_load = [&](int qt) __attribute__((always_inline)) {
      const int r = tid / kCPR, cc = (tid % kCPR) * EPC, gr = qt + r;
      pq = po = pa = make_uint4(0, 0, 0, 0);
      if (gr < N && cc < d) {
        pq = *(const uint4*)(Qg + (int64_t)gr * p.sq[2] + cc);
        po = *(const uint4*)(dOg + (int64_t)gr * p.sdo[2] + cc);
        if (PREP) pa = *(const uint4*)(Og + (int64_t)gr * p.so[2] + cc);
      }
      if (tid < BQ) {
        const int q = qt + tid;
        if (PREP) {  // (m, l) here, lse2 at the store
          pl = q < N ? p.m[(int64_t)bh * N + q] : 0.f;
          pd = q < N ? p.l[(int64_t)bh * N + q] : 1.f;
        } else {
          pl = q < N ? lse2[q] : 0.f;
          pd = q < N ? delta[q] : 0.f;
        }
      }
    };
    auto pre_store = [&](int s) __attribute__((always_inline)) {
      T* sQ = (T*)(ring + s * SLOT);
      T* sO = sQ + BQ * kLD;
      const int r = tid / kCPR, cc = (tid % kCPR) * EPC;
      float* sRow;
      if constexpr (X3) {  // Q planes h, m, l then dO's: 8 B of each per 16-B chunk
        bf16* pl3 = (bf16*)(ring + s * SLOT);
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2) {
          const float4 f = __builtin_bit_cast(float4, t2 ? po : pq);
          unsigned h0, m0, l0, h1, m1, l1;
          x3_split2(f.x, f.y, h0, m0, l0);
          x3_split2(f.z, f.w, h1, m1, l1);
          bf16* q3 = pl3 + 3 * t2 * PLANE + r * LDB + cc;
          *(uint2*)(q3) = make_uint2(h0, h1);
          *(uint2*)(q3 + PLANE) = make_uint2(m0, m1);
          *(uint2*)(q3 + 2 * PLANE) = make_uint2(l0, l1);
        }
        sRow = (float*)(pl3 + 6 * PLANE);
      } else {
        *(uint4*)(sQ + r * kLD + cc) = pq;
        *(uint4*)(sO + r * kLD + cc) = po;
        sRow = (float*)(sO + BQ * kLD);
      }
      if (PREP) {
        const float4 x = __builtin_bit_cast(float4, pa), y = __builtin_bit_cast(float4, po);
        float a = 0.f;
        a += x.x * y.x;
        a += x.y * y.y;
        a += x.z * y.z;
        a += x.w * y.w;
#pragma unroll
        for (int off = 8; off > 0; off >>= 1) a += __shfl_xor(a, off);
        if ((tid & 15) == 0) sRow[BQ + r] = a;
        if (tid < BQ) sRow[tid] = pl * kLog2e + log2f(pd);
      } else if (tid < BQ) {
        sRow[tid] = pl;
        sRow[BQ + tid] = pd;
      }
    };
    if (ntile > 0) {
      pre_load(qstart);
      pre_store(0);
      if (ntile > 1) pre_load(qstart + BQ);
    }
    __syncthreads();
    float* dst_base = slab + ((int64_t)bhl * nkb + kblk) * N * DT;

    for (int t = 0; t < ntile; ++t) {
      const int qt = qstart + t * BQ;
      const T* sQ = (const T*)(ring + (t & 1) * SLOT);
      const T* sO = sQ + BQ * kLD;
      const bf16* sQ3 = (const bf16*)(ring + (t & 1) * SLOT);  // X3: Q planes, then dO's
      const bf16* sO3 = sQ3 + 3 * PLANE;
      const float* sLse = X3 ? (const float*)(sQ3 + 6 * PLANE) : (const float*)(sO + BQ * kLD);
      const float* sDel = sLse + BQ;
      if (!(CAUSAL && qt + BQ - 1 < wave_kmin)) {
        f32x16 S = f32x16{}, dP = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int col = ks * 16 + 8 * hf;
          if constexpr (X3) {
            const int o = c32 * LDB + col;
            X3Frag aq, ao;
            aq.h = *(const bf16x8*)(sQ3 + o);
            aq.m = *(const bf16x8*)(sQ3 + PLANE + o);
            aq.l = *(const bf16x8*)(sQ3 + 2 * PLANE + o);
            ao.h = *(const bf16x8*)(sO3 + o);
            ao.m = *(const bf16x8*)(sO3 + PLANE + o);
            ao.l = *(const bf16x8*)(sO3 + 2 * PLANE + o);
            // (an opaque use per tile keeps hipcc from hoisting the loop-invariant splits)
            asm volatile("" : "+v"(bk[ks]), "+v"(bv[ks]));
            mma_x3(S, aq, x3_split(bk[ks]));
            mma_x3(dP, ao, x3_split(bv[ks]));
          } else {
            mma(S, row_frag<T>(sQ + c32 * kLD + col), bk[ks]);
            mma(dP, row_frag<T>(sO + c32 * kLD + col), bv[ks]);
          }
        }
        const bool msk = qt + BQ > N || k0 + BKV > Nk || (CAUSAL && qt < wave_kmin + 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ql = acc_row(r, hf);
          const int q = qt + ql;
          float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(S[r], c2, -sLse[ql]));
          if (msk && (q >= N || my_k >= Nk || (CAUSAL && my_k > q))) pv = 0.f;
          S[r] = pv;
          dP[r] = pv * (dP[r] - sDel[ql]);
          dSi[ql * TL + wave * 32 + c32] = dP[r];
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if constexpr (X3) {
            const X3Frag bp = x3_split(acc_frag<float>(S, s)), bs = x3_split(acc_frag<float>(dP, s));
#pragma unroll
            for (int db = 0; db < NDB; ++db) {
              const int kq = 16 * s + 4 * hf;
              X3Frag ao, aq;
              ao.h = col_frag<bf16>(sO3, LDB, kq, db * 32, lane);
              ao.m = col_frag<bf16>(sO3 + PLANE, LDB, kq, db * 32, lane);
              ao.l = col_frag<bf16>(sO3 + 2 * PLANE, LDB, kq, db * 32, lane);
              mma_x3(dV[db], ao, bp);
              aq.h = col_frag<bf16>(sQ3, LDB, kq, db * 32, lane);
              aq.m = col_frag<bf16>(sQ3 + PLANE, LDB, kq, db * 32, lane);
              aq.l = col_frag<bf16>(sQ3 + 2 * PLANE, LDB, kq, db * 32, lane);
              mma_x3(dK[db], aq, bs);
            }
          } else {
            const Frag<T> bp = acc_frag<T>(S, s), bs = acc_frag<T>(dP, s);
#pragma unroll
            for (int db = 0; db < NDB; ++db) {
              mma(dV[db], col_frag<T>(sO, kLD, 16 * s + 4 * hf, db * 32, lane), bp);
              mma(dK[db], col_frag<T>(sQ, kLD, 16 * s + 4 * hf, db * 32, lane), bs);
            }
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) dSi[acc_row(r, hf) * TL + wave * 32 + c32] = 0.f;
      }
      __syncthreads();  // the tile's dS image is complete
      {
        f32x4 qa = f32x4{}, qb = f32x4{};
#pragma unroll
        for (int s4 = 0; s4 < 16; ++s4) {
          const float4 a4 = *(const float4*)(dSi + ia + 4 * s4);
          const float4 b4 = *(const float4*)(KT + ib + 4 * s4);
          qa = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, b4.x, qa, 0, 0, 0);
          qb = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, b4.y, qb, 0, 0, 0);
          qa = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, b4.z, qa, 0, 0, 0);
          qb = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, b4.w, qb, 0, 0, 0);
        }
        const int col = 16 * d4 + (lane & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = qt + 16 * qh + 4 * (lane >> 4) + j;
          if (q < N) dst_base[(int64_t)q * DT + col] = qa[j] + qb[j];
        }
      }
      if (t + 1 < ntile) {
        pre_store((t + 1) & 1);
        if (t + 2 < ntile) pre_load(qt + 2 * BQ);
      }
      __syncthreads();
    }

    if (my_k < N) {
      T* dKg = (T*)p.dk + b * p.sdk[0] + hh * p.sdk[1] + (int64_t)my_k * p.sdk[2];
      T* dVg = (T*)p.dv + b * p.sdv[0] + hh * p.sdv[1] + (int64_t)my_k * p.sdv[2];
      const float sc = p.scale;
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int col = db * 32 + 8 * g + 4 * hf;
          if (col < d) {
            store4(dKg + col, dK[db][4 * g] * sc, dK[db][4 * g + 1] * sc, dK[db][4 * g + 2] * sc,
                   dK[db][4 * g + 3] * sc, true);
            store4(dVg + col, dV[db][4 * g], dV[db][4 * g + 1], dV[db][4 * g + 2], dV[db][4 * g + 3],
                   true);
          }
        }
    }
  }
}

// dQ = scale · Σ_kb slab[head][kb][q][:] over the key blocks that wrote row q (kb below the valid
// keys' block count; causal: kb·256 <= q), in kb order. One thread per 16-B chunk of a row.
__global__ __launch_bounds__(256) void fa_bwd_ring_dq_sum(AttnArgs p, const float* slab, int bh0, int ng,
                                                          int causal) {
  const int N = p.N, nkb = (N + kFrBKV - 1) / kFrBKV;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)ng * N * 16) return;
  const int c = (int)(i & 15);
  const int64_t rq = i >> 4;
  const int bhl = (int)(rq / N), q = (int)(rq % N);
  if (4 * c >= p.d) return;
  const int bh = bh0 + bhl, b = bh / p.H, hh = bh % p.H;
  int kb1 = (min(N, kv_keys(p, b)) + kFrBKV - 1) / kFrBKV;
  if (causal) kb1 = min(kb1, q / kFrBKV + 1);
  const float* src = slab + ((int64_t)bhl * nkb * N + q) * 64 + 4 * c;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int kb = 0; kb < kb1; ++kb) {
    const float4 v = *(const float4*)(src + (int64_t)kb * N * 64);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  const float sc = p.scale;
  float* dst = (float*)p.dq + b * p.sdq[0] + hh * p.sdq[1] + (int64_t)q * p.sdq[2] + 4 * c;
  store4(dst, acc.x * sc, acc.y * sc, acc.z * sc, acc.w * sc, true);
}

// fp32 bytes of one head's dQ slab in the fused ring backward
int64_t ring_fused_head_slab(int64_t N) { return ((N + kFrBKV - 1) / kFrBKV) * N * 64 * 4; }
// the workspace region it asks for: the slab of one group of heads, at most 1 GiB per launch (0
// when one head's slab is larger: the split ring runs)
int64_t ring_fused_ws_bytes(int64_t B, int64_t H, int64_t N) {
  constexpr int64_t cap = (int64_t)1 << 30;
  const int64_t per = ring_fused_head_slab(N);
  return per > cap ? 0 : std::min<int64_t>(B * H, cap / per) * per;
}

// The fused fp32 backward after the prep kernel: heads in groups whose slab fits slab_bytes
// (the workspace's fused region), each group one pass and one ordered sum.
// prep: the kernel forms the row constants (PREP; the caller skipped the prep kernel), else
// the caller ran fa_bwd_prep.
hipError_t launch_bwd_ring_fused(const AttnArgs& a, bool causal, bool pair, int64_t slab_bytes, bool prep,
                                 hipStream_t st) {
  const int64_t per = ring_fused_head_slab(a.N), BH = (int64_t)a.B * a.H;
  const int64_t grp = std::min<int64_t>(BH, slab_bytes / per);
  if (grp < 1 || a.N < 1) return hipErrorInvalidValue;
  const int nkb = (a.N + kFrBKV - 1) / kFrBKV;
  bool x3 = true;
#ifdef MT_DIAGNOSTICS
  if (a.knob == 65) x3 = false;  // A/B: every product on the fp32 MFMA
#endif
  void (*kfn)(AttnArgs, float*, int) =
      x3 ? (prep ? (causal ? (pair ? fa_bwd_fused_ring<true, true> : fa_bwd_fused_ring<true, false>)
                           : fa_bwd_fused_ring<false, false>)
                 : (causal ? (pair ? fa_bwd_fused_ring<true, true, false> : fa_bwd_fused_ring<true, false, false>)
                           : fa_bwd_fused_ring<false, false, false>))
         : (prep ? (causal ? (pair ? fa_bwd_fused_ring<true, true, true, false> : fa_bwd_fused_ring<true, false, true, false>)
                           : fa_bwd_fused_ring<false, false, true, false>)
                 : (causal ? (pair ? fa_bwd_fused_ring<true, true, false, false> : fa_bwd_fused_ring<true, false, false, false>)
                           : fa_bwd_fused_ring<false, false, false, false>));
  const int smem = x3 ? kFrSmemX3 : kFrSmem;
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  if (e != hipSuccess) return e;
  for (int64_t bh0 = 0; bh0 < BH; bh0 += grp) {
    const int64_t ng = std::min<int64_t>(grp, BH - bh0);
    hipLaunchKernelGGL(kfn, dim3((unsigned)(pair ? (nkb + 1) / 2 : nkb), (unsigned)ng), dim3(512), smem, st, a,
                       (float*)a.slab, (int)bh0);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t nthr = ng * a.N * 16;
    hipLaunchKernelGGL(fa_bwd_ring_dq_sum, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, st, a,
                       (const float*)a.slab, (int)bh0, (int)ng, causal ? 1 : 0);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <typename T, int DT, bool CAUSAL, bool PAIR, bool X3 = false>
static hipError_t launch_bwd_ring_t(const AttnArgs& a, hipStream_t st) {
  constexpr int kLD = DT + 16 / (int)sizeof(T);
  constexpr size_t kTile = X3 ? 6 * 32 * (DT + 8) * 2 : 2 * 32 * kLD * sizeof(T);  // bytes per ring slot
  constexpr size_t kTileF = 2 * 32 * kLD * sizeof(T);
  const unsigned bhn = (unsigned)(a.B * a.H);
  bool x3kv = X3, x3q = X3;
#ifdef MT_DIAGNOSTICS
  if (a.knob == 66) x3q = false;   // A/B: X3 in the dK/dV pass only
  if (a.knob == 67) x3kv = false;  // A/B: X3 in the dQ pass only
#endif
  {
    const int nkb = (a.N + 127) / 128;
    const size_t smem = 2 * ((x3kv ? kTile : kTileF) + 2 * 32 * sizeof(float));
    auto kfn = x3kv ? fa_bwd_dkv_ring<T, DT, CAUSAL, PAIR, X3> : fa_bwd_dkv_ring<T, DT, CAUSAL, PAIR, false>;
    hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kfn, dim3(PAIR ? (nkb + 1) / 2 : nkb, bhn), dim3(256), smem, st, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  {
    const int nqb = (a.N + 127) / 128;
    const size_t smem = 2 * (x3q ? kTile : kTileF);
    auto kfn = x3q ? fa_bwd_dq_ring<T, DT, CAUSAL, PAIR, X3> : fa_bwd_dq_ring<T, DT, CAUSAL, PAIR, false>;
    hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kfn, dim3(PAIR ? (nqb + 1) / 2 : nqb, bhn), dim3(256), smem, st, a);
    return hipGetLastError();
  }
}

template <typename T, int DT, bool X3 = false>
static hipError_t launch_bwd_ring_d(const AttnArgs& a, bool causal, bool pair, hipStream_t st) {
  if (causal)
    return pair ? launch_bwd_ring_t<T, DT, true, true, X3>(a, st) : launch_bwd_ring_t<T, DT, true, false, X3>(a, st);
  return pair ? launch_bwd_ring_t<T, DT, false, true, X3>(a, st) : launch_bwd_ring_t<T, DT, false, false, X3>(a, st);
}

// 16-B rows, d <= 64 (fp32) or d < 64 (bf16, which the d = 64 MFMA backward does not take);
// the caller has run the prep kernel (lse2, delta). d <= 32: 32-column tiles, no zero-padded
// half (minitorch's MHA at config 5 has d = 32).
hipError_t launch_bwd_ring(const AttnArgs& a, bool bf16_io, bool causal, bool pair, hipStream_t st) {
  if (bf16_io)
    return a.d <= 32 ? launch_bwd_ring_d<bf16, 32>(a, causal, pair, st)
                     : launch_bwd_ring_d<bf16, 64>(a, causal, pair, st);
#ifdef MT_DIAGNOSTICS
  if (a.knob == 65)  // A/B: every product on the fp32 MFMA
    return a.d <= 32 ? launch_bwd_ring_d<float, 32>(a, causal, pair, st)
                     : launch_bwd_ring_d<float, 64>(a, causal, pair, st);
#endif
  // fp32: the four products on the bf16 MFMA in three pieces per operand (fa_common.h mma_x3)
  return a.d <= 32 ? launch_bwd_ring_d<float, 32, true>(a, causal, pair, st)
                   : launch_bwd_ring_d<float, 64, true>(a, causal, pair, st);
}

}  // namespace mt
