// dK/dV at one wave per SIMD (A/B policy 72), compiled on its own with
// -mllvm -amdgpu-mfma-vgpr-form: the S / dP products (builtins) then write VGPRs the softmax
// reads directly, while the dVᵀ / dKᵀ accumulators are pinned to AGPRs by inline asm.
#include "fa_bwd_bf16.h"

namespace mt {
using namespace bwdbf16;

// dVᵀ / dKᵀ accumulation into an AGPR tile. The operands are produced at least one MFMA gap
// earlier (packed P / dS one phase earlier, transposes by counted LDS waits), so the
// VALU-write-to-MFMA-read wait states hold without padding.
// Volatile, so the IR optimiser keeps it in its MFMA gap (sched_barrier fences only the
// machine scheduler; pure code may be moved across it before that).
__device__ __forceinline__ void mfma_acc(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// The same, padded on both sides (2 wait states after a VALU write of an operand, 21 for the
// result): for the drain after the loop, where hipcc may copy accumulators between AGPRs
// right after an asm MFMA it cannot see is still in flight.
__device__ __forceinline__ void mfma_acc_padded(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0\n\ts_nop 7\n\ts_nop 7\n\ts_nop 4"
               : "+a"(acc) : "v"(a), "v"(b));
}

// Pins a value to the program point: code that uses the result cannot be hoisted above it or
// computed in an earlier iteration (the optimiser otherwise moves a whole softmax out of its
// MFMA gaps, e.g. to the end of the previous iteration, where nothing overlaps it).
template <typename T>
__device__ __forceinline__ T pin(T x) {
  asm volatile("" : "+v"(x));
  return x;
}

// dK/dV, one wave per SIMD: workgroup = 4 waves = 256 keys, a wave owns 64 keys (two 32-key
// blocks kb), so every Q / dO operand fragment read from LDS feeds two MFMAs (half the LDS
// reads per MFMA of the 32-key forms), and the wave has the whole register file (512 VGPR +
// AGPR) to overlap its own work, with no partner wave on the SIMD.
// Tile t = 32 queries, staged by LDS-DMA two tiles ahead into a 3-slot ring (one barrier per
// tile). Iteration t runs 32 MFMA gaps in two phases:
//   A: dVᵀ/dKᵀ of (t, kb 0) ‖ S/dP of (t + 1, kb 0) ‖ softmax of (t, kb 1)
//   B: dVᵀ/dKᵀ of (t, kb 1) ‖ S/dP of (t + 1, kb 1) ‖ softmax of (t + 1, kb 0)
// (one score per lane per gap: one exponential per MFMA gap). A key block's scores are
// consumed in the phase before the one that overwrites them, so the loop carries one set of
// scores (t, kb 1) and one set of packed P / dS (t, kb 0), with no copies.
// Non-causal, N % 32 == 0 (every tile mask-free); the launcher sends other shapes elsewhere.
namespace {
constexpr int kQT = 32;
constexpr int kImgQ = kQT * D;                       // elements of one Q / dO image
constexpr int kBufQ = 4 * kImgQ * 2 + 2 * kQT * 4;   // bytes per ring slot: 4 images + 2 row vectors
constexpr int kW64Slot = kBufQ;  // 4 images of a 32-query tile + the two row-constant rows

struct W64Sc {
  f32x16 S, dP;  // one key block's scores (C-initialised, so p = exp2(c2·S), dS = p·dP)
};
struct W64P {
  bf16x8 pf[2], sf[2];  // packed P / dS of one key block, [16-query half s]
};

__device__ __forceinline__ bf16x8 w64_tr(const char* slot, int img, int s, int toff) {
  return tr_frag((const bf16*)slot + img * kImgQ, 16 * s, toff);
}

// C-init values of S and dP for a tile: rows acc_row(r, hf) of −lse2/c2 and −δ.
__device__ __forceinline__ void w64_init(const char* slot, int hf, f32x16& iS, f32x16& iD) {
  const float* nl = (const float*)((const bf16*)slot + 4 * kImgQ);
  const float* nd = nl + kQT;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 a = *(const float4*)(nl + 8 * g + 4 * hf);
    const float4 e = *(const float4*)(nd + 8 * g + 4 * hf);
    iS[4 * g] = a.x; iS[4 * g + 1] = a.y; iS[4 * g + 2] = a.z; iS[4 * g + 3] = a.w;
    iD[4 * g] = e.x; iD[4 * g + 1] = e.y; iD[4 * g + 2] = e.z; iD[4 * g + 3] = e.w;
  }
}

// p = exp2(c2·S'), dS = p·dP' of one key block, packed as the B operands.
__device__ __forceinline__ void w64_softmax(const W64Sc& x, float c2, W64P& o) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const float e = __builtin_amdgcn_exp2f(x.S[j] * c2);
    o.pf[j >> 3][j & 7] = (bf16)e;
    o.sf[j >> 3][j & 7] = (bf16)(e * x.dP[j]);
  }
}
}  // namespace

__global__ __launch_bounds__(256, 1) void fa_bwd_dkv_bf16_w64(AttnArgs p, int nkb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = logical / nkb, kblk = logical % nkb;
  const int b = bh / p.H, hh = bh % p.H;
  const int kw = kblk * 256 + wave * 64;  // first key of this wave

  bf16x8 kf[2][4], vf[2][4];
  int roff[4], toff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int kr = min(kw + 32 * j + c32, N - 1);
    const bf16* krow = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1] + (int64_t)kr * p.sk[2];
    const bf16* vrow = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1] + (int64_t)kr * p.sv[2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      kf[j][ks] = *(const bf16x8*)(krow + 16 * ks + 8 * hf);
      vf[j][ks] = *(const bf16x8*)(vrow + 16 * ks + 8 * hf);
    }
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) roff[ks] = k_swz<D>(c32, 2 * ks + hf);
  toff[0] = tr_off(lane, 0);
  toff[1] = tr_off(lane, 1);

  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Og = (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const int sqn = (int)p.sq[2], son = (int)p.sdo[2];
  const __amdgpu_buffer_rsrc_t rq = head_rsrc(Qg, N, sqn), ro = head_rsrc(Og, N, son);
  const float* nlse = p.lse2 + (int64_t)bh * N;
  const float* ndel = p.delta + (int64_t)bh * N;
  // DMA: wave w fills rows 8w .. 8w + 7 of each of the tile's four images
  const uint32_t lds0 = lds_base(smem) + __builtin_amdgcn_readfirstlane(wave) * 8 * D * 2;
  int gq0, gq1, go0, go1;
  {
    const int r = 8 * wave + (lane >> 3), pc = lane & 7;
    const int ck = pc ^ ((r >> 1) & 7), cv = pc ^ (((r >> 1) & 1) << 2);
    gq0 = (r * sqn + ck * 8) * 2;
    gq1 = (r * sqn + cv * 8) * 2;
    go0 = (r * son + ck * 8) * 2;
    go1 = (r * son + cv * 8) * 2;
  }
  const int ntile = N / kQT;
  float sv = 0.f;
  auto stage = [&](int t, int slot) __attribute__((always_inline)) {
    const uint32_t img = lds0 + slot * kW64Slot;
    const int oq = t * kQT * sqn * 2, oo = t * kQT * son * 2;
    dma_rows(img, rq, gq0 + oq);
    dma_rows(img + kImgQ * 2, rq, gq1 + oq);
    dma_rows(img + 2 * kImgQ * 2, ro, go0 + oo);
    dma_rows(img + 3 * kImgQ * 2, ro, go1 + oo);
    if (tid < 2 * kQT) {
      const int q = t * kQT + (tid & (kQT - 1));
      sv = tid < kQT ? nlse[q] : ndel[q];
    }
  };
  auto publish = [&](int slot) __attribute__((always_inline)) {
    if (tid < 2 * kQT) ((float*)((bf16*)(smem + slot * kW64Slot) + 4 * kImgQ))[tid] = sv;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  f32x16 dK[2][2], dV[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) { dK[i][j] = f32x16{}; dV[i][j] = f32x16{}; }
  const float c2 = p.scale_log2;

  stage(0, 0);
  publish(0);
  if (ntile > 1) {
    stage(1, 1);
    publish(1);
  }
  __syncthreads();

  W64Sc s0, s1;  // scores of key blocks 0 / 1
  W64P p0, p1;   // packed P / dS of key blocks 0 / 1
  {              // prologue: tile 0's scores, key block 0's softmax
    const bf16* Qr = (const bf16*)smem;
    const bf16* Or = Qr + 2 * kImgQ;
    f32x16 iS, iD;
    w64_init(smem, hf, iS, iD);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 qa = *(const bf16x8*)(Qr + roff[ks]), oa = *(const bf16x8*)(Or + roff[ks]);
      s0.S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[0][ks], ks ? s0.S : iS, 0, 0, 0);
      s0.dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(oa, vf[0][ks], ks ? s0.dP : iD, 0, 0, 0);
      s1.S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[1][ks], ks ? s1.S : iS, 0, 0, 0);
      s1.dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(oa, vf[1][ks], ks ? s1.dP : iD, 0, 0, 0);
    }
    w64_softmax(s0, c2, p0);
  }
  float e[16];  // exponentials of the phase's softmax (scores 12-15 finish in the next phase)
#pragma unroll
  for (int j = 12; j < 16; ++j) e[j] = __builtin_amdgcn_exp2f(s0.S[j] * c2);

  // tile 0's first two transposes (each iteration prefetches the next tile's at its end)
  bf16x8 ot[2][2], qt[2][2];  // transposes of tile t, [s][db]
  ot[0][0] = w64_tr(smem, 3, 0, toff[0]);
  qt[0][0] = w64_tr(smem, 1, 0, toff[0]);
  int sc = 0;  // byte offset of tile t's slot
  for (int t = 0; t + 1 < ntile; ++t) {
    const int sn = sc == 2 * kW64Slot ? 0 : sc + kW64Slot;  // tile t + 1's slot
    if (t + 2 < ntile) stage(t + 2, sn == 2 * kW64Slot ? 0 : sn / kW64Slot + 1);
    const char* SC = smem + sc;
    const char* SN = smem + sn;
    const bf16* Qrn = (const bf16*)SN;
    const float* nl = (const float*)(Qrn + 4 * kImgQ);
    const float* nd = nl + kQT;
    f32x16 iS, iD;
    bf16x8 qa[4], oa[4];  // rows of t + 1
#pragma unroll
    for (int g = 0; g < 32; ++g) {
      const int ph = g >> 4, j = g & 15;  // phase = key block of the products
      // LDS reads, each two or more gaps ahead of its first use (phase A; phase B reuses
      // them); the next tile's first two transposes at the end of phase B
      if (ph == 0) {
        if (j == 0) {
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const float4 a4 = *(const float4*)(nl + 8 * q4 + 4 * hf);
            iS[4 * q4] = a4.x; iS[4 * q4 + 1] = a4.y; iS[4 * q4 + 2] = a4.z; iS[4 * q4 + 3] = a4.w;
          }
        }
        if (j == 4) {
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const float4 a4 = *(const float4*)(nd + 8 * q4 + 4 * hf);
            iD[4 * q4] = a4.x; iD[4 * q4 + 1] = a4.y; iD[4 * q4 + 2] = a4.z; iD[4 * q4 + 3] = a4.w;
          }
        }
        if (j == 0) { qa[0] = *(const bf16x8*)(Qrn + roff[0]); ot[0][1] = w64_tr(SC, 3, 0, toff[1]); }
        if (j == 1) { qt[0][1] = w64_tr(SC, 1, 0, toff[1]); ot[1][0] = w64_tr(SC, 3, 1, toff[0]); }
        if (j == 2) { qt[1][0] = w64_tr(SC, 1, 1, toff[0]); ot[1][1] = w64_tr(SC, 3, 1, toff[1]); }
        if (j == 3) { qt[1][1] = w64_tr(SC, 1, 1, toff[1]); qa[1] = *(const bf16x8*)(Qrn + roff[1]); }
        if (j == 4) qa[2] = *(const bf16x8*)(Qrn + roff[2]);
        if (j == 5) { qa[3] = *(const bf16x8*)(Qrn + roff[3]); oa[0] = *(const bf16x8*)(Qrn + 2 * kImgQ + roff[0]); }
        if (j >= 6 && j <= 8) oa[j - 5] = *(const bf16x8*)(Qrn + 2 * kImgQ + roff[j - 5]);
      } else {
        if (j == 14) ot[0][0] = w64_tr(SN, 3, 0, toff[0]);
        if (j == 15) qt[0][0] = w64_tr(SN, 1, 0, toff[0]);
      }
      // phase A, gap j: V at 0 1 2 4 6 8 10 12, A at 3 5 7 9 (S chain) 11 13 14 15 (dP chain);
      // phase B (operands already in registers): A at 0 1 3 5 (S) 7 9 11 13 (dP), V at the
      // rest, so key block 1's chains end well before the loop's back edge
      const bool isv = ph == 0 ? (j < 3 || (j < 13 && !(j & 1))) : (j == 2 || (j >= 4 && !(j & 1)) || j == 15);
      const int vi = ph == 0 ? (j < 3 ? j : j / 2 + 1) : (j == 15 ? 7 : j / 2 - 1);
      const int ai = ph == 0 ? (j < 13 ? (j - 3) / 2 : j - 8) : (j < 2 ? j : (j - 1) / 2 + 1);
      W64P& pp = ph ? p1 : p0;
      W64Sc& nx = ph ? s1 : s0;  // receives (t + 1, ph)
      if (isv) {
        // (s, db, dV/dK) = (vi >> 2, (vi >> 1) & 1, vi & 1)
        const int s = vi >> 2, db = (vi >> 1) & 1;
        if (vi & 1) mfma_acc(dK[ph][db], qt[s][db], pp.sf[s]);
        else mfma_acc(dV[ph][db], ot[s][db], pp.pf[s]);
      } else {
        // the S chain first, then the dP chain, so the next phase's softmax finds S done
        const int ks = ai & 3;
        if (ai >= 4) nx.dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pin(oa[ks]), vf[ph][ks], ks ? nx.dP : iD, 0, 0, 0);
        else nx.S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pin(qa[ks]), kf[ph][ks], ks ? nx.S : iS, 0, 0, 0);
      }
      // softmax: phase A of (t, kb 1) from s1 into p1, phase B of (t + 1, kb 0) from s0 into
      // p0. Exponential of score j in gap j; its dS product and bf16 packs four gaps later
      // (the last four in gaps 0-3 of the next phase), so the dP chain that ended just
      // before the phase has landed.
      {
        W64Sc& src = ph ? s0 : s1;
        e[j] = __builtin_amdgcn_exp2f(src.S[j] * c2);
        const int v = j - 4;  // this phase's score whose products are due
        if (v >= 0 && (v & 1)) {
          W64P& dst = ph ? p0 : p1;
          dst.pf[v >> 3][(v & 7) - 1] = (bf16)e[v - 1];
          dst.pf[v >> 3][v & 7] = (bf16)e[v];
          dst.sf[v >> 3][(v & 7) - 1] = (bf16)(e[v - 1] * src.dP[v - 1]);
          dst.sf[v >> 3][v & 7] = (bf16)(e[v] * src.dP[v]);
          if ((v & 7) == 7) {  // a finished half: keep its packing in these gaps
            dst.pf[v >> 3] = pin(dst.pf[v >> 3]);
            dst.sf[v >> 3] = pin(dst.sf[v >> 3]);
          }
        }
        // the previous phase's scores 12-15 (phase A: those of iteration t - 1's phase B, or
        // of the prologue), whose exponentials e[12..15] are not overwritten before gap 12
        if (j < 4 && (j & 1)) {
          const int u = 12 + j;
          W64Sc& psrc = ph ? s1 : s0;
          W64P& pdst = ph ? p1 : p0;
          pdst.pf[1][(u & 7) - 1] = (bf16)e[u - 1];
          pdst.pf[1][u & 7] = (bf16)e[u];
          pdst.sf[1][(u & 7) - 1] = (bf16)(e[u - 1] * psrc.dP[u - 1]);
          pdst.sf[1][u & 7] = (bf16)(e[u] * psrc.dP[u]);
          if (u == 15) {
            pdst.pf[1] = pin(pdst.pf[1]);
            pdst.sf[1] = pin(pdst.sf[1]);
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t + 2 < ntile) publish(sn == 2 * kW64Slot ? 0 : sn / kW64Slot + 1);
    __syncthreads();
    sc = sn;
  }
  {  // last tile: key block 0's products, key block 1's softmax and products
    const char* SC = smem + sc;
#pragma unroll
    for (int u = 12; u < 16; ++u) {  // scores 12-15 of key block 0 (see the phase loop)
      p0.pf[1][u & 7] = (bf16)e[u];
      p0.sf[1][u & 7] = (bf16)(e[u] * s0.dP[u]);
    }
    w64_softmax(s1, c2, p1);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const W64P& pp = kb ? p1 : p0;
          mfma_acc_padded(dV[kb][db], w64_tr(SC, 3, s, toff[db]), pp.pf[s]);
          mfma_acc_padded(dK[kb][db], w64_tr(SC, 1, s, toff[db]), pp.sf[s]);
        }
  }

  // the last dVᵀ / dKᵀ MFMAs must retire before their AGPRs are read (hipcc does not pad
  // behind inline asm)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
               : "+a"(dK[0][0]), "+a"(dK[0][1]), "+a"(dK[1][0]), "+a"(dK[1][1]), "+a"(dV[0][0]),
                 "+a"(dV[0][1]), "+a"(dV[1][0]), "+a"(dV[1][1]));
  const float sc2 = p.scale;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = kw + 32 * j + c32;
    if (key < N) {
      bf16* dKg = (bf16*)p.dk + b * p.sdk[0] + hh * p.sdk[1] + (int64_t)key * p.sdk[2];
      bf16* dVg = (bf16*)p.dv + b * p.sdv[0] + hh * p.sdv[1] + (int64_t)key * p.sdv[2];
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int col = db * 32 + 8 * g + 4 * hf;
          store4(dKg + col, dK[j][db][4 * g] * sc2, dK[j][db][4 * g + 1] * sc2,
                 dK[j][db][4 * g + 2] * sc2, dK[j][db][4 * g + 3] * sc2, true);
          store4(dVg + col, dV[j][db][4 * g], dV[j][db][4 * g + 1], dV[j][db][4 * g + 2],
                 dV[j][db][4 * g + 3], true);
        }
    }
  }
}


hipError_t launch_dkv_w64(const AttnArgs& a, int nkb, unsigned nblk, size_t smem, hipStream_t st) {
  hipError_t e = hipFuncSetAttribute((const void*)fa_bwd_dkv_bf16_w64,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fa_bwd_dkv_bf16_w64, dim3(nblk), dim3(256), smem, st, a, nkb);
  return hipGetLastError();
}

}  // namespace mt
