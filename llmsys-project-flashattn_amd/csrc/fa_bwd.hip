// FlashAttention backward, generic tiled kernels (fp32 and bf16, any head dim).
//
// Replaces the reference backward_kernel / backward_kernel_causal
// (src/flashattention_kernel.cu:115-255, :547-690): given Q, K, V, O, dO and the
// forward's (m, l), produce dQ, dK, dV of O = softmax(QKᵀ/√d) V. The reference's
// dV term is wrong (:202/:637 use dO row t instead of y) and racy (:241/:676); this
// computes the exact gradient:
//     P = exp(s − m)/l,  dV = Pᵀ dO,  dP = dO Vᵀ,  δ = rowsum(dO ∘ O),
//     dS = P ∘ (dP − δ),  dQ = dS K/√d,  dK = dSᵀ Q/√d.
//
// MI355X design, three deterministic launches (no atomics, no HBM read-modify-write):
//  1. fa_bwd_prep : δ and lse2 = m·log2e + log2(l) per row (one wave per row).
//  2. fa_bwd_dkv  : "key on the lane" — a workgroup owns 128 keys (32 per wave) and
//                   sweeps all query tiles; S and dP come out of MFMA with the key on
//                   the lane, so they are directly the B operands of dVᵀ += dOᵀ·P and
//                   dKᵀ += Qᵀ·dS (dOᵀ/Qᵀ read with ds_read_b64_tr_b16).
//  3. fa_bwd_dq   : "query on the lane" — a workgroup owns 128 queries and sweeps the
//                   key tiles; dQᵀ += Kᵀ·dSᵀ.
// The dQ pass recomputes S and dP (7 MFMA products instead of 5) in exchange for
// no cross-workgroup reduction of dQ.
#include "fa_common.h"

namespace mt {

// ---------------------------------------------------------------------------
// 16 lanes per row, 16 rows per 256-thread workgroup and pass, kPrepPasses passes with every
// load issued first. VEC (16-B rows and strides): each lane reads 16-B chunks sub, sub + 16, ..
// of its row; else elements sub, sub + 16, ... (One wave per row, 4 rows per workgroup, had
// run the C2 fp32 prep at ≈2.2 TB/s: 32768 workgroups of 4-B loads.)
constexpr int kPrepPasses = 4;
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void fa_bwd_prep(AttnArgs p) {
  const int64_t rows = (int64_t)p.B * p.H * p.N;
  const int sub = threadIdx.x & 15;
  const int64_t row0 = (int64_t)blockIdx.x * 16 * kPrepPasses + (threadIdx.x >> 4);
  constexpr int EPC = 16 / sizeof(T);  // elements per 16-B chunk
  float acc[kPrepPasses];
#pragma unroll
  for (int u = 0; u < kPrepPasses; ++u) {
    acc[u] = 0.f;
    const int64_t row = row0 + 16 * u;
    if (row >= rows) continue;
    const int n = (int)(row % p.N);
    const int64_t bh = row / p.N;
    const int b = (int)(bh / p.H), hh = (int)(bh % p.H);
    const T* O = (const T*)p.o + b * p.so[0] + hh * p.so[1] + (int64_t)n * p.so[2];
    const T* dO = (const T*)p.dout + b * p.sdo[0] + hh * p.sdo[1] + (int64_t)n * p.sdo[2];
    if (VEC) {
      for (int c = sub * EPC; c < p.d; c += 16 * EPC) {
        const uint4 x = *(const uint4*)(O + c), y = *(const uint4*)(dO + c);
        const T* xo = (const T*)&x;
        const T* yo = (const T*)&y;
#pragma unroll
        for (int j = 0; j < EPC; ++j) acc[u] += to_f32(xo[j]) * to_f32(yo[j]);
      }
    } else {
      for (int c = sub; c < p.d; c += 16) acc[u] += to_f32(O[c]) * to_f32(dO[c]);
    }
  }
#pragma unroll
  for (int u = 0; u < kPrepPasses; ++u) {
    float a = acc[u];
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) a += __shfl_xor(a, off);
    const int64_t row = row0 + 16 * u;
    if (sub == 0 && row < rows) {
      p.delta[row] = a;
      p.lse2[row] = p.m[row] * kLog2e + log2f(p.l[row]);
    }
  }
}

// 16-B chunks of O and dO rows: d, the row strides and the bases on 16-B boundaries.
static bool prep_vec(const AttnArgs& a, int esize) {
  const int epc = 16 / esize;
  return a.d % epc == 0 && a.so[0] % epc == 0 && a.so[1] % epc == 0 && a.so[2] % epc == 0 &&
         a.sdo[0] % epc == 0 && a.sdo[1] % epc == 0 && a.sdo[2] % epc == 0 &&
         ((uintptr_t)a.o & 15) == 0 && ((uintptr_t)a.dout & 15) == 0;
}
template <typename T>
static hipError_t launch_prep(const AttnArgs& a, hipStream_t st) {
  const int64_t rows = (int64_t)a.B * a.H * a.N;
  const dim3 grid((unsigned)((rows + 16 * kPrepPasses - 1) / (16 * kPrepPasses)));
  if (prep_vec(a, sizeof(T))) hipLaunchKernelGGL((fa_bwd_prep<T, true>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((fa_bwd_prep<T, false>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// dK, dV: grid (ceil(N/128), B*H, ceil(d/DT)).
// PAIR (causal): a workgroup runs key blocks nkb - 1 - u (light) and then u (heavy) of one
// head in turn, so the grid is balanced (fa_bwd_bf16.hip, policy 107, same scheme).
template <typename T, int DT, int QB, bool VEC, bool CAUSAL, bool PAIR = false>
__global__ __launch_bounds__(256) void fa_bwd_dkv(AttnArgs p) {
  constexpr int BKV = 128, BQ = 32 * QB;
  constexpr int PAD = 16 / sizeof(T);
  constexpr int LD = DT + PAD;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* sK = (T*)smem;
  T* sV = sK + BKV * LD;
  T* sQ = sV + BKV * LD;
  T* sO = sQ + BQ * LD;  // dO tile
  float* sLse = (float*)(sO + BQ * LD);
  float* sDel = sLse + BQ;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N, d = p.d;
  int ublk, bh;
  xcd_order(ublk, bh);
  const int b = bh / p.H, hh = bh % p.H;
  const int nkb = (N + BKV - 1) / BKV;
#pragma nounroll
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
  const int kblk = !PAIR ? ublk : pass == 0 ? nkb - 1 - ublk : ublk;
  if (PAIR && pass == 1) {
    if (kblk == nkb - 1 - ublk) break;  // odd nkb: the middle block runs alone
    __syncthreads();                     // the first block's LDS reads are done
  }
  const int k0 = kblk * BKV;
  const int oc = blockIdx.z * DT;
  const T* Qg = (const T*)p.q + b * p.sq[0] + hh * p.sq[1];
  const T* Kg = (const T*)p.k + b * p.sk[0] + hh * p.sk[1];
  const T* Vg = (const T*)p.v + b * p.sv[0] + hh * p.sv[1];
  const T* dOg = (const T*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const float* lse2 = p.lse2 + (int64_t)bh * N;
  const float* delta = p.delta + (int64_t)bh * N;
  const int dpad = (d + 15) & ~15;
  const int nch = (dpad + DT - 1) / DT;
  const int my_k = k0 + wave * 32 + c32;  // this lane's key
  const int wave_kmin = k0 + wave * 32;
  const int Nk = kv_keys(p, b);  // keys >= Nk are padding: zero gradients

  f32x16 dK[DT / 32], dV[DT / 32];
#pragma unroll
  for (int i = 0; i < DT / 32; ++i) { dK[i] = f32x16{}; dV[i] = f32x16{}; }

  if (nch == 1) {
    stage_tile<T, BKV, DT, 256, VEC>(sK, LD, Kg, p.sk[2], k0, N, 0, d);
    stage_tile<T, BKV, DT, 256, VEC>(sV, LD, Vg, p.sv[2], k0, N, 0, d);
  }
  const int qstart = CAUSAL ? (k0 / BQ) * BQ : 0;
  // one d-chunk with 16-B rows: the Q / dO tile (and its row constants) of step qt + BQ is
  // loaded into registers while step qt computes (fa_fwd.hip, same scheme)
  const bool pref = VEC && nch == 1;
  constexpr int EPC = 16 / sizeof(T), CPR = DT / EPC, NCK = (BQ * CPR + 255) / 256;
  uint4 pq[NCK], po[NCK];
  float pl = 0.f, pd = 0.f;
  auto pre_load = [&](int qt) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NCK; ++i) {
      const int ch = tid + 256 * i, r = ch / CPR, cc = (ch % CPR) * EPC, gr = qt + r;
      pq[i] = po[i] = make_uint4(0, 0, 0, 0);
      if (ch < BQ * CPR && gr < N && cc < d) {
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
  auto pre_store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NCK; ++i) {
      const int ch = tid + 256 * i, r = ch / CPR, cc = (ch % CPR) * EPC;
      if (ch < BQ * CPR) {
        *(uint4*)(sQ + r * LD + cc) = pq[i];
        *(uint4*)(sO + r * LD + cc) = po[i];
      }
    }
    if (tid < BQ) {
      sLse[tid] = pl;
      sDel[tid] = pd;
    }
  };
  if (pref && qstart < N) pre_load(qstart);
  for (int qt = qstart; qt < N; qt += BQ) {
    const bool active = !(CAUSAL && qt + BQ - 1 < wave_kmin);
    f32x16 S[QB], dP[QB];
#pragma unroll
    for (int i = 0; i < QB; ++i) { S[i] = f32x16{}; dP[i] = f32x16{}; }
    for (int c = 0; c < nch; ++c) {
      __syncthreads();
      if (pref) {
        pre_store();
        if (qt + BQ < N) pre_load(qt + BQ);
      } else {
        if (nch > 1) {
          stage_tile<T, BKV, DT, 256, VEC>(sK, LD, Kg, p.sk[2], k0, N, c * DT, d);
          stage_tile<T, BKV, DT, 256, VEC>(sV, LD, Vg, p.sv[2], k0, N, c * DT, d);
        }
        stage_tile<T, BQ, DT, 256, VEC>(sQ, LD, Qg, p.sq[2], qt, N, c * DT, d);
        stage_tile<T, BQ, DT, 256, VEC>(sO, LD, dOg, p.sdo[2], qt, N, c * DT, d);
        if (c == 0 && tid < BQ) {
          const int q = qt + tid;
          sLse[tid] = q < N ? lse2[q] : 0.f;
          sDel[tid] = q < N ? delta[q] : 0.f;
        }
      }
      __syncthreads();
      const int ksteps = min(DT, dpad - c * DT) / 16;
      auto kstep = [&](int ks) __attribute__((always_inline)) {
        const int col = ks * 16 + 8 * hf;
        Frag<T> bk = row_frag<T>(sK + (wave * 32 + c32) * LD + col);
        Frag<T> bv = row_frag<T>(sV + (wave * 32 + c32) * LD + col);
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {
          Frag<T> aq = row_frag<T>(sQ + (qb * 32 + c32) * LD + col);
          Frag<T> ao = row_frag<T>(sO + (qb * 32 + c32) * LD + col);
          mma(S[qb], aq, bk);
          mma(dP[qb], ao, bv);
        }
      };
      if (active) {
        if (pref) {  // one zero-padded d-chunk: all DT / 16 k-steps, unrolled
#pragma unroll
          for (int ks = 0; ks < DT / 16; ++ks) kstep(ks);
        } else {
          for (int ks = 0; ks < ksteps; ++ks) kstep(ks);
        }
      }
    }
    // Row c32-lane holds S[q][my_k] for q = qt + qb*32 + acc_row(r, hf).
    if (active) {
      // p = exp2(c2·s − lse2): one fma into one v_exp_f32; masks only on tiles that reach
      // past N or below the wave's keys (causal)
      const float c2 = p.scale_log2;
      const bool msk = qt + BQ > N || k0 + BKV > Nk || (CAUSAL && qt < wave_kmin + 31);
#pragma unroll
      for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ql = qb * 32 + acc_row(r, hf);
          const int q = qt + ql;
          float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(S[qb][r], c2, -sLse[ql]));
          if (msk && (q >= N || my_k >= Nk || (CAUSAL && my_k > q))) pv = 0.f;
          S[qb][r] = pv;
          dP[qb][r] = pv * (dP[qb][r] - sDel[ql]);
        }
    }
    if (nch > 1 && oc != (nch - 1) * DT) {
      // The Q/dO tiles hold the last d-chunk; restage the output chunk.
      __syncthreads();
      stage_tile<T, BQ, DT, 256, VEC>(sQ, LD, Qg, p.sq[2], qt, N, oc, d);
      stage_tile<T, BQ, DT, 256, VEC>(sO, LD, dOg, p.sdo[2], qt, N, oc, d);
      __syncthreads();
    }
    if (active) {
#pragma unroll
      for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          Frag<T> bp = acc_frag<T>(S[qb], s);
          Frag<T> bs = acc_frag<T>(dP[qb], s);
#pragma unroll
          for (int db = 0; db < DT / 32; ++db) {
            Frag<T> ao = col_frag<T>(sO, LD, qb * 32 + 16 * s + 4 * hf, db * 32, lane);
            Frag<T> aq = col_frag<T>(sQ, LD, qb * 32 + 16 * s + 4 * hf, db * 32, lane);
            mma(dV[db], ao, bp);
            mma(dK[db], aq, bs);
          }
        }
    }
  }

  if (my_k < N) {
    T* dKg = (T*)p.dk + b * p.sdk[0] + hh * p.sdk[1] + (int64_t)my_k * p.sdk[2];
    T* dVg = (T*)p.dv + b * p.sdv[0] + hh * p.sdv[1] + (int64_t)my_k * p.sdv[2];
#pragma unroll
    for (int db = 0; db < DT / 32; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = oc + db * 32 + 8 * g + 4 * hf;
        const float ak[4] = {dK[db][4 * g] * p.scale, dK[db][4 * g + 1] * p.scale,
                             dK[db][4 * g + 2] * p.scale, dK[db][4 * g + 3] * p.scale};
        const float av[4] = {dV[db][4 * g], dV[db][4 * g + 1], dV[db][4 * g + 2], dV[db][4 * g + 3]};
        if (VEC && col + 3 < d) {
          store4(dKg + col, ak[0], ak[1], ak[2], ak[3], true);
          store4(dVg + col, av[0], av[1], av[2], av[3], true);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col + e < d) {
              dKg[col + e] = from_f32<T>(ak[e]);
              dVg[col + e] = from_f32<T>(av[e]);
            }
        }
      }
  }
  }  // pass
}

// ---------------------------------------------------------------------------
// dQ: grid (ceil(N/128), B*H, ceil(d/DT)).
// PAIR (causal): query blocks u (light) and then nqb - 1 - u (heavy) of one head in turn.
template <typename T, int DT, int KB, bool VEC, bool CAUSAL, bool PAIR = false>
__global__ __launch_bounds__(256) void fa_bwd_dq(AttnArgs p) {
  constexpr int BQ = 128, BK = 32 * KB;
  constexpr int PAD = 16 / sizeof(T);
  constexpr int LD = DT + PAD;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* sQ = (T*)smem;
  T* sO = sQ + BQ * LD;  // dO
  T* sK = sO + BQ * LD;
  T* sV = sK + BK * LD;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N, d = p.d;
  int ublk, bh;
  xcd_order(ublk, bh);
  const int b = bh / p.H, hh = bh % p.H;
  const int nqb = (N + BQ - 1) / BQ;
#pragma nounroll
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
  const int qblk = !PAIR ? ublk : pass == 0 ? ublk : nqb - 1 - ublk;
  if (PAIR && pass == 1) {
    if (qblk == ublk) break;  // odd nqb: the middle block runs alone
    __syncthreads();          // the first block's LDS reads are done
  }
  const int q0 = qblk * BQ;
  const int oc = blockIdx.z * DT;
  const T* Qg = (const T*)p.q + b * p.sq[0] + hh * p.sq[1];
  const T* Kg = (const T*)p.k + b * p.sk[0] + hh * p.sk[1];
  const T* Vg = (const T*)p.v + b * p.sv[0] + hh * p.sv[1];
  const T* dOg = (const T*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const int dpad = (d + 15) & ~15;
  const int nch = (dpad + DT - 1) / DT;
  const int my_q = q0 + wave * 32 + c32;
  const int wave_qmax = q0 + wave * 32 + 31;
  const float lse_q = my_q < N ? p.lse2[(int64_t)bh * N + my_q] : 0.f;
  const float del_q = my_q < N ? p.delta[(int64_t)bh * N + my_q] : 0.f;

  f32x16 dQ[DT / 32];
#pragma unroll
  for (int i = 0; i < DT / 32; ++i) dQ[i] = f32x16{};

  if (nch == 1) {
    stage_tile<T, BQ, DT, 256, VEC>(sQ, LD, Qg, p.sq[2], q0, N, 0, d);
    stage_tile<T, BQ, DT, 256, VEC>(sO, LD, dOg, p.sdo[2], q0, N, 0, d);
  }
  const int Nk = kv_keys(p, b);  // keys >= Nk are padding
  const int kend = CAUSAL ? min(Nk, q0 + BQ) : Nk;
  // one d-chunk with 16-B rows: the K / V tile of step k0 + BK is loaded into registers
  // while step k0 computes (fa_fwd.hip, same scheme)
  const bool pref = VEC && nch == 1;
  constexpr int EPC = 16 / sizeof(T), CPR = DT / EPC, NCK = (BK * CPR + 255) / 256;
  uint4 pk[NCK], pv[NCK];
  auto pre_load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NCK; ++i) {
      const int ch = tid + 256 * i, r = ch / CPR, cc = (ch % CPR) * EPC, gr = k0 + r;
      pk[i] = pv[i] = make_uint4(0, 0, 0, 0);
      if (ch < BK * CPR && gr < N && cc < d) {
        pk[i] = *(const uint4*)(Kg + (int64_t)gr * p.sk[2] + cc);
        pv[i] = *(const uint4*)(Vg + (int64_t)gr * p.sv[2] + cc);
      }
    }
  };
  auto pre_store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NCK; ++i) {
      const int ch = tid + 256 * i, r = ch / CPR, cc = (ch % CPR) * EPC;
      if (ch < BK * CPR) {
        *(uint4*)(sK + r * LD + cc) = pk[i];
        *(uint4*)(sV + r * LD + cc) = pv[i];
      }
    }
  };
  if (pref && kend > 0) pre_load(0);
  for (int k0 = 0; k0 < kend; k0 += BK) {
    const bool active = !(CAUSAL && k0 > wave_qmax);
    f32x16 S[KB], dP[KB];
#pragma unroll
    for (int i = 0; i < KB; ++i) { S[i] = f32x16{}; dP[i] = f32x16{}; }
    for (int c = 0; c < nch; ++c) {
      __syncthreads();
      if (pref) {
        pre_store();
        if (k0 + BK < kend) pre_load(k0 + BK);
      } else {
        if (nch > 1) {
          stage_tile<T, BQ, DT, 256, VEC>(sQ, LD, Qg, p.sq[2], q0, N, c * DT, d);
          stage_tile<T, BQ, DT, 256, VEC>(sO, LD, dOg, p.sdo[2], q0, N, c * DT, d);
        }
        stage_tile<T, BK, DT, 256, VEC>(sK, LD, Kg, p.sk[2], k0, N, c * DT, d);
        stage_tile<T, BK, DT, 256, VEC>(sV, LD, Vg, p.sv[2], k0, N, c * DT, d);
      }
      __syncthreads();
      const int ksteps = min(DT, dpad - c * DT) / 16;
      auto kstep = [&](int ks) __attribute__((always_inline)) {
        const int col = ks * 16 + 8 * hf;
        Frag<T> bq = row_frag<T>(sQ + (wave * 32 + c32) * LD + col);
        Frag<T> bo = row_frag<T>(sO + (wave * 32 + c32) * LD + col);
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
          Frag<T> ak = row_frag<T>(sK + (kb * 32 + c32) * LD + col);
          Frag<T> av = row_frag<T>(sV + (kb * 32 + c32) * LD + col);
          mma(S[kb], ak, bq);
          mma(dP[kb], av, bo);
        }
      };
      if (active) {
        if (pref) {  // one zero-padded d-chunk: all DT / 16 k-steps, unrolled
#pragma unroll
          for (int ks = 0; ks < DT / 16; ++ks) kstep(ks);
        } else {
          for (int ks = 0; ks < ksteps; ++ks) kstep(ks);
        }
      }
    }
    if (active) {
      const float c2 = p.scale_log2;
      const bool msk = k0 + BK > Nk || (CAUSAL && k0 + BK - 1 > q0 + wave * 32);
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + kb * 32 + acc_row(r, hf);
          float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(S[kb][r], c2, -lse_q));
          if (msk && (key >= Nk || (CAUSAL && key > my_q))) pv = 0.f;
          dP[kb][r] = pv * (dP[kb][r] - del_q);
        }
    }
    if (nch > 1 && oc != (nch - 1) * DT) {
      __syncthreads();
      stage_tile<T, BK, DT, 256, VEC>(sK, LD, Kg, p.sk[2], k0, N, oc, d);
      __syncthreads();
    }
    if (active) {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          Frag<T> bs = acc_frag<T>(dP[kb], s);
#pragma unroll
          for (int db = 0; db < DT / 32; ++db) {
            Frag<T> ak = col_frag<T>(sK, LD, kb * 32 + 16 * s + 4 * hf, db * 32, lane);
            mma(dQ[db], ak, bs);
          }
        }
    }
  }

  if (my_q < N) {
    T* dQg = (T*)p.dq + b * p.sdq[0] + hh * p.sdq[1] + (int64_t)my_q * p.sdq[2];
#pragma unroll
    for (int db = 0; db < DT / 32; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = oc + db * 32 + 8 * g + 4 * hf;
        const float a[4] = {dQ[db][4 * g] * p.scale, dQ[db][4 * g + 1] * p.scale,
                            dQ[db][4 * g + 2] * p.scale, dQ[db][4 * g + 3] * p.scale};
        if (VEC && col + 3 < d) {
          store4(dQg + col, a[0], a[1], a[2], a[3], true);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col + e < d) dQg[col + e] = from_f32<T>(a[e]);
        }
      }
  }
  }  // pass
}

// ---------------------------------------------------------------------------
template <typename T, int DT, int QB, int KB, bool VEC, bool CAUSAL, bool PAIR>
static hipError_t launch_bwd_t(const AttnArgs& a, hipStream_t st) {
  constexpr int LD = DT + 16 / sizeof(T);
  const int nz = (a.d + DT - 1) / DT;
  const int nblk = PAIR ? ((a.N + 127) / 128 + 1) / 2 : (a.N + 127) / 128;
  {
    const hipError_t e = launch_prep<T>(a, st);
    if (e != hipSuccess) return e;
  }
  {
    const size_t smem = sizeof(T) * (size_t)LD * (2 * 128 + 2 * 32 * QB) + 2 * sizeof(float) * 32 * QB;
    auto kfn = fa_bwd_dkv<T, DT, QB, VEC, CAUSAL, PAIR>;
    hipError_t e = hipFuncSetAttribute((const void*)kfn,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kfn, dim3(nblk, a.B * a.H, nz), dim3(256), smem, st, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  {
    const size_t smem = sizeof(T) * (size_t)LD * (2 * 128 + 2 * 32 * KB);
    auto kfn = fa_bwd_dq<T, DT, KB, VEC, CAUSAL, PAIR>;
    hipError_t e = hipFuncSetAttribute((const void*)kfn,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kfn, dim3(nblk, a.B * a.H, nz), dim3(256), smem, st, a);
    return hipGetLastError();
  }
}

template <typename T, int DT, int QB, int KB>
static hipError_t dispatch_bwd(const AttnArgs& a, bool vec, bool causal, bool pair, hipStream_t st) {
  if (causal && pair)
    return vec ? launch_bwd_t<T, DT, QB, KB, true, true, true>(a, st)
               : launch_bwd_t<T, DT, QB, KB, false, true, true>(a, st);
  if (vec)
    return causal ? launch_bwd_t<T, DT, QB, KB, true, true, false>(a, st)
                  : launch_bwd_t<T, DT, QB, KB, true, false, false>(a, st);
  return causal ? launch_bwd_t<T, DT, QB, KB, false, true, false>(a, st)
                : launch_bwd_t<T, DT, QB, KB, false, false, false>(a, st);
}

hipError_t launch_bwd_ring(const AttnArgs& a, bool bf16_io, bool causal, bool pair, hipStream_t st);
hipError_t launch_bwd_ring_fused(const AttnArgs& a, bool causal, bool pair, int64_t slab_bytes, bool prep,
                                 hipStream_t st);
int64_t ring_fused_head_slab(int64_t N);

// pair: 0 never, 1 always (causal), 2 when the paired grid keeps >= 2 workgroups per CU.
// ring: one d-chunk of 16-B rows (fp32 d <= 64, bf16 d < 64) runs the register-row kernels of
// fa_bwd_ring.hip. fused_slab: bytes of the workspace's fused region at a.slab (0: none); fp32
// with 32 < d <= 64 then runs dQ inside the dK/dV pass (fa_bwd_fused_ring) where its grid of
// 256-key blocks (light / heavy pairs when causal) fills a workgroup per CU.
hipError_t launch_bwd_generic(const AttnArgs& a, bool bf16_io, bool vec, bool causal,
                              hipStream_t st, int pair, bool ring, int64_t fused_slab) {
  const bool pr = pair == 1 || (pair == 2 && (int64_t)((a.N + 255) / 256) * a.B * a.H >= 512);
  if (ring && vec && (bf16_io ? a.d < 64 : a.d <= 64)) {
    const int64_t nkb = (a.N + 255) / 256;
    bool fpair = causal && nkb > 1;
    // the fused kernel's own row constants need 16-B O chunks; the paired causal X3 form keeps
    // the prep kernel (forming them in the pass spilled 47 VGPRs there: C2 causal 0.377 against
    // 0.360 ms, profiles/r6_ab_fp32_x3.txt)
    bool fprep = prep_vec(a, 4) && !(causal && fpair);
#ifdef MT_DIAGNOSTICS
    if (a.knob == 61) fpair = false;  // A/B: the causal fused ring backward unpaired
    if (a.knob == 62) fprep = false;  // A/B: the prep kernel ahead of the fused pass
#endif
    const bool fused = !bf16_io && a.d > 32 && a.slab && fused_slab >= ring_fused_head_slab(a.N) &&
                       (fpair ? (nkb + 1) / 2 : nkb) * a.B * a.H >= 256;
    if (!(fused && fprep)) {
      const hipError_t e = bf16_io ? launch_prep<bf16>(a, st) : launch_prep<float>(a, st);
      if (e != hipSuccess) return e;
    }
    if (fused) return launch_bwd_ring_fused(a, causal, fpair, fused_slab, fprep, st);
    return launch_bwd_ring(a, bf16_io, causal, pr, st);
  }
  if (bf16_io) {
    if (a.d <= 64) return dispatch_bwd<bf16, 64, 2, 2>(a, vec, causal, pr, st);
    return dispatch_bwd<bf16, 128, 1, 1>(a, vec, causal, pr, st);
  }
  // fp32 keeps 64-column chunks: a 128-column fp32 K+V pair would not fit the LDS.
  return dispatch_bwd<float, 64, 1, 1>(a, vec, causal, pr, st);
}

}  // namespace mt
