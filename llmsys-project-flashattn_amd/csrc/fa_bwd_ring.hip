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
template <typename T, int DT, bool CAUSAL, bool PAIR>
__global__ __launch_bounds__(256, 2) void fa_bwd_dkv_ring(AttnArgs p) {
  // DT = 64, or 32 for d <= 32; rows padded by 16 B; NCK 16-B chunks per thread per 32-row tile
  constexpr int EPC = 16 / sizeof(T), kLD = DT + EPC, kCPR = DT / EPC;
  constexpr int NCK = (32 * kCPR + 255) / 256, KS = DT / 16, NDB = DT / 32;
  constexpr int BKV = 128, BQ = 32;
  constexpr int SLOT = 2 * BQ * kLD * (int)sizeof(T) + 2 * BQ * 4;  // Q, dO, lse2, delta (bytes)
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
          *(uint4*)(sQ + r * kLD + cc) = pq[i];
          *(uint4*)(sO + r * kLD + cc) = po[i];
        }
      }
      if (tid < BQ) {
        float* sRow = (float*)(sO + BQ * kLD);
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

    for (int t = 0; t < ntile; ++t) {
      const int qt = qstart + t * BQ;
      const T* sQ = (const T*)(ring + (t & 1) * SLOT);
      const T* sO = sQ + BQ * kLD;
      const float* sLse = (const float*)(sO + BQ * kLD);
      const float* sDel = sLse + BQ;
      if (!(CAUSAL && qt + BQ - 1 < wave_kmin)) {
        // Sᵀ and dPᵀ: the lane's column is key my_k, rows are queries qt + acc_row(r, hf)
        f32x16 S = f32x16{}, dP = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int col = ks * 16 + 8 * hf;
          mma(S, row_frag<T>(sQ + c32 * kLD + col), bk[ks]);
          mma(dP, row_frag<T>(sO + c32 * kLD + col), bv[ks]);
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
// keys streamed through the ring.
template <typename T, int DT, bool CAUSAL, bool PAIR>
__global__ __launch_bounds__(256, 2) void fa_bwd_dq_ring(AttnArgs p) {
  // DT = 64, or 32 for d <= 32; rows padded by 16 B; NCK 16-B chunks per thread per 32-row tile
  constexpr int EPC = 16 / sizeof(T), kLD = DT + EPC, kCPR = DT / EPC;
  constexpr int NCK = (32 * kCPR + 255) / 256, KS = DT / 16, NDB = DT / 32;
  constexpr int BQ = 128, BK = 32;
  constexpr int SLOT = 2 * BK * kLD;  // K, V (elements)
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
          *(uint4*)(sK + r * kLD + cc) = pk[i];
          *(uint4*)(sV + r * kLD + cc) = pv[i];
        }
      }
    };
    if (ntile > 0) {
      pre_load(0);
      pre_store(0);
      if (ntile > 1) pre_load(BK);
    }
    __syncthreads();

    for (int t = 0; t < ntile; ++t) {
      const int k0 = t * BK;
      const T* sK = ring + (t & 1) * SLOT;
      const T* sV = sK + BK * kLD;
      if (!(CAUSAL && k0 > wave_qmax)) {
        // S and dP with the query on the lane: rows are keys k0 + acc_row(r, hf)
        f32x16 S = f32x16{}, dP = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int col = ks * 16 + 8 * hf;
          mma(S, row_frag<T>(sK + c32 * kLD + col), bq[ks]);
          mma(dP, row_frag<T>(sV + c32 * kLD + col), bo[ks]);
        }
        const bool msk = k0 + BK > Nk || (CAUSAL && k0 + BK - 1 > q0 + wave * 32);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + acc_row(r, hf);
          float pvv = __builtin_amdgcn_exp2f(__builtin_fmaf(S[r], c2, -lse_q));
          if (msk && (key >= Nk || (CAUSAL && key > my_q))) pvv = 0.f;
          dP[r] = pvv * (dP[r] - del_q);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const Frag<T> bs = acc_frag<T>(dP, s);
#pragma unroll
          for (int db = 0; db < NDB; ++db)
            mma(dQ[db], col_frag<T>(sK, kLD, 16 * s + 4 * hf, db * 32, lane), bs);
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

template <typename T, int DT, bool CAUSAL, bool PAIR>
static hipError_t launch_bwd_ring_t(const AttnArgs& a, hipStream_t st) {
  constexpr int kLD = DT + 16 / (int)sizeof(T);
  const unsigned bhn = (unsigned)(a.B * a.H);
  {
    const int nkb = (a.N + 127) / 128;
    const size_t smem = 2 * (2 * 32 * kLD * sizeof(T) + 2 * 32 * sizeof(float));
    auto kfn = fa_bwd_dkv_ring<T, DT, CAUSAL, PAIR>;
    hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kfn, dim3(PAIR ? (nkb + 1) / 2 : nkb, bhn), dim3(256), smem, st, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  {
    const int nqb = (a.N + 127) / 128;
    const size_t smem = 2 * 2 * 32 * kLD * sizeof(T);
    auto kfn = fa_bwd_dq_ring<T, DT, CAUSAL, PAIR>;
    hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kfn, dim3(PAIR ? (nqb + 1) / 2 : nqb, bhn), dim3(256), smem, st, a);
    return hipGetLastError();
  }
}

template <typename T, int DT>
static hipError_t launch_bwd_ring_d(const AttnArgs& a, bool causal, bool pair, hipStream_t st) {
  if (causal)
    return pair ? launch_bwd_ring_t<T, DT, true, true>(a, st) : launch_bwd_ring_t<T, DT, true, false>(a, st);
  return pair ? launch_bwd_ring_t<T, DT, false, true>(a, st) : launch_bwd_ring_t<T, DT, false, false>(a, st);
}

// 16-B rows, d <= 64 (fp32) or d < 64 (bf16, which the d = 64 MFMA backward does not take);
// the caller has run the prep kernel (lse2, delta). d <= 32: 32-column tiles, no zero-padded
// half (minitorch's MHA at config 5 has d = 32).
hipError_t launch_bwd_ring(const AttnArgs& a, bool bf16_io, bool causal, bool pair, hipStream_t st) {
  if (bf16_io)
    return a.d <= 32 ? launch_bwd_ring_d<bf16, 32>(a, causal, pair, st)
                     : launch_bwd_ring_d<bf16, 64>(a, causal, pair, st);
  return a.d <= 32 ? launch_bwd_ring_d<float, 32>(a, causal, pair, st)
                   : launch_bwd_ring_d<float, 64>(a, causal, pair, st);
}

}  // namespace mt
