// dQ of the bf16 d = 64 backward with an in-wave software pipeline (A/B policy 73).
//
// Same products as fa_bwd_dq_bf16 (fa_bwd_bf16.hip): a wave owns 32 queries (Q, dO rows as
// register-resident B operands), 8 waves = 256 queries per workgroup, two waves per SIMD, and
// the workgroup sweeps 64-key tiles (two 32-key blocks kb):
//     Sᵀ = K·Qᵀ, dPᵀ = V·dOᵀ − δ (C-init), p = exp2(c2·Sᵀ − lse2), dSᵀ = p·dPᵀ, dQᵀ += Kᵀ·dSᵀ.
// The plain kernel runs each tile's 16 S/dP products, then its 32 exponentials, then its 8 dQ
// products, so the softmax stands beside no MFMA of its own wave. Here iteration t runs 24
// MFMA gaps in two phases:
//   A: dQ of (t, kb 0) ‖ S/dP of (t + 1, kb 0) ‖ softmax of (t, kb 1)
//   B: dQ of (t, kb 1) ‖ S/dP of (t + 1, kb 1) ‖ softmax of (t + 1, kb 0)
// (16 exponentials over 12 gaps per phase). A key block's scores are consumed in the phase
// before the one that overwrites them, so one set of scores per key block is carried.
// K / Kᵀ / V images arrive by LDS-DMA two tiles ahead into a 3-slot ring, one barrier per
// tile. Operands and packed results are pinned to their gap (empty volatile asm): the IR
// optimiser otherwise moves pure code across sched_barrier, which fences only the machine
// scheduler. Non-causal, N % 64 == 0; the launcher sends other shapes to the plain kernel.
#include "fa_bwd_bf16.h"

namespace mt {
using namespace bwdbf16;

namespace {
constexpr int kKT = 64;
constexpr int kImgK = kKT * D;
constexpr int kBufK = 3 * kImgK * 2;  // K row image, K transpose image, V row image

template <typename T>
__device__ __forceinline__ T pin(T x) {
  asm volatile("" : "+v"(x));
  return x;
}

struct DqSc {
  f32x16 S, dP;  // one key block's Sᵀ and dPᵀ (query on the lane)
};
}  // namespace

__global__ __launch_bounds__(512, 2) void fa_bwd_dq_bf16_pipe(AttnArgs p, int nqb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = logical / nqb, qb = logical % nqb;
  const int b = bh / p.H, hh = bh % p.H;
  const int my_q = qb * 256 + wave * 32 + c32;

  bf16x8 qf[4], of[4];
  int roff[4], toff[2];
  float nlq, del;
  {
    const int qr = min(my_q, N - 1);
    const bf16* qrow = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1] + (int64_t)qr * p.sq[2];
    const bf16* orow = (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1] + (int64_t)qr * p.sdo[2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      qf[ks] = *(const bf16x8*)(qrow + 16 * ks + 8 * hf);
      of[ks] = *(const bf16x8*)(orow + 16 * ks + 8 * hf);
      roff[ks] = k_swz<D>(c32, 2 * ks + hf);
    }
    toff[0] = tr_off(lane, 0);
    toff[1] = tr_off(lane, 1);
    const int64_t row = (int64_t)bh * N + qr;
    nlq = p.lse2[row] * p.scale_log2;  // = −lse2
    del = -p.delta[row];
  }
  f32x16 dinit;
#pragma unroll
  for (int r = 0; r < 16; ++r) dinit[r] = -del;  // = −δ
  const float c2 = p.scale_log2;

  // DMA: wave w fills rows 8w .. 8w + 7 of each of the tile's three images
  const bf16* Kg = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1];
  const bf16* Vg = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1];
  const int skn = (int)p.sk[2], svn = (int)p.sv[2];
  const __amdgpu_buffer_rsrc_t rk = head_rsrc(Kg, N, skn), rv = head_rsrc(Vg, N, svn);
  const uint32_t lds0 = lds_base(smem) + __builtin_amdgcn_readfirstlane(wave) * 8 * D * 2;
  int gk0, gk1, gv0;
  {
    const int r = 8 * wave + (lane >> 3), pc = lane & 7;
    const int ck = pc ^ ((r >> 1) & 7), cv = pc ^ (((r >> 1) & 1) << 2);
    gk0 = (r * skn + ck * 8) * 2;
    gk1 = (r * skn + cv * 8) * 2;
    gv0 = (r * svn + ck * 8) * 2;
  }
  const int ntile = N / kKT;
  auto stage = [&](int t, int slot) __attribute__((always_inline)) {
    const uint32_t img = lds0 + slot * kBufK;
    const int ok = t * kKT * skn * 2, ov = t * kKT * svn * 2;
    dma_rows(img, rk, gk0 + ok);
    dma_rows(img + kImgK * 2, rk, gk1 + ok);
    dma_rows(img + 2 * kImgK * 2, rv, gv0 + ov);
  };

  f32x16 dQ[2] = {f32x16{}, f32x16{}};
  stage(0, 0);
  if (ntile > 1) stage(1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // Sᵀ / dPᵀ of one key block of the tile in `slot` (prologue / reference form)
  auto scores = [&](const char* slot, int kb, DqSc& x) __attribute__((always_inline)) {
    const bf16* Kr = (const bf16*)slot;
    const bf16* Vr = Kr + 2 * kImgK;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      x.S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(Kr + kb * 32 * D + roff[ks]), qf[ks],
                                                    ks ? x.S : f32x16{}, 0, 0, 0);
      x.dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(Vr + kb * 32 * D + roff[ks]), of[ks],
                                                     ks ? x.dP : dinit, 0, 0, 0);
    }
  };
  auto softmax = [&](const DqSc& x, bf16x8 (&ds)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      ds[r >> 3][r & 7] = (bf16)(__builtin_amdgcn_exp2f(__builtin_fmaf(x.S[r], c2, nlq)) * x.dP[r]);
  };
  auto ktr = [&](const char* slot, int kb, int s, int db) __attribute__((always_inline)) {
    return tr_frag((const bf16*)slot + kImgK, kb * 32 + 16 * s, toff[db]);
  };

  DqSc s0, s1;            // scores of key blocks 0 / 1
  bf16x8 d0[2], d1[2];    // packed dSᵀ of key blocks 0 / 1, [16-key half s]
  scores(smem, 0, s0);
  scores(smem, 1, s1);
  softmax(s0, d0);
  bf16x8 ka0 = ktr(smem, 0, 0, 0), ka1 = ktr(smem, 0, 0, 1);  // phase A's first two Kᵀ
  float e15 = __builtin_amdgcn_exp2f(__builtin_fmaf(s0.S[15], c2, nlq));  // see the phases

  int sc = 0;  // byte offset of tile t's slot
  for (int t = 0; t + 1 < ntile; ++t) {
    const int sn = sc == 2 * kBufK ? 0 : sc + kBufK;  // tile t + 1's slot
    if (t + 2 < ntile) stage(t + 2, sn == 2 * kBufK ? 0 : sn / kBufK + 1);
    const char* SC = smem + sc;
    const char* SN = smem + sn;
    const bf16* Krn = (const bf16*)SN;
    const bf16* Vrn = Krn + 2 * kImgK;
    bf16x8 kr[4], vr[4], kt[4];
    float e[16];
#pragma unroll
    for (int g = 0; g < 24; ++g) {
      const int ph = g / 12, j = g % 12;  // phase = key block of the products
      DqSc& nx = ph ? s1 : s0;            // receives (t + 1, ph)
      // LDS reads two or more gaps ahead: this phase's rows, the Kᵀ of V slots 2-3 here and
      // of the next phase's (or next iteration's) V slots 0-1
      if (j == 0) { kr[0] = *(const bf16x8*)(Krn + ph * 32 * D + roff[0]); kr[1] = *(const bf16x8*)(Krn + ph * 32 * D + roff[1]); }
      if (j == 1) { kr[2] = *(const bf16x8*)(Krn + ph * 32 * D + roff[2]); kr[3] = *(const bf16x8*)(Krn + ph * 32 * D + roff[3]); }
      if (j == 2) { kt[2] = ktr(SC, ph, 1, 0); kt[3] = ktr(SC, ph, 1, 1); }
      if (j == 3) { vr[0] = *(const bf16x8*)(Vrn + ph * 32 * D + roff[0]); vr[1] = *(const bf16x8*)(Vrn + ph * 32 * D + roff[1]); }
      if (j == 5) { vr[2] = *(const bf16x8*)(Vrn + ph * 32 * D + roff[2]); vr[3] = *(const bf16x8*)(Vrn + ph * 32 * D + roff[3]); }
      if (j == 9) {
        if (ph == 0) { kt[0] = ktr(SC, 1, 0, 0); kt[1] = ktr(SC, 1, 0, 1); }
        else { kt[0] = ktr(SN, 0, 0, 0); kt[1] = ktr(SN, 0, 0, 1); }
      }
      if (ph == 0 && j == 0) { kt[0] = ka0; kt[1] = ka1; }
      // gaps: 0 V0, 1 V1, 2 S0, 3 S1, 4 V2, 5 S2, 6 S3, 7 V3, 8-11 dP0-3
      const int vi = j == 0 ? 0 : j == 1 ? 1 : j == 4 ? 2 : j == 7 ? 3 : -1;
      if (vi >= 0) {
        const int s = vi >> 1, db = vi & 1;
        bf16x8 (&dd)[2] = ph ? d1 : d0;
        dQ[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pin(kt[vi]), pin(dd[s]), dQ[db], 0, 0, 0);
      } else {
        const int ai = j < 4 ? j - 2 : j < 7 ? j - 3 : j - 4;  // S0 S1 S2 S3 dP0 dP1 dP2 dP3
        const int ks = ai & 3;
        if (ai < 4) nx.S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pin(kr[ks]), qf[ks], ks ? nx.S : f32x16{}, 0, 0, 0);
        else nx.dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pin(vr[ks]), of[ks], ks ? nx.dP : dinit, 0, 0, 0);
      }
      // softmax: phase A of (t, kb 1) from s1 into d1, phase B of (t + 1, kb 0) from s0 into
      // d0. Score v's exponential in gap 3v/4, its dS and pack one gap later; score 15's
      // product opens the next phase (phase B's: the next iteration's phase A, via e15).
      {
        const DqSc& src = ph ? s0 : s1;
        bf16x8 (&dst)[2] = ph ? d0 : d1;
#pragma unroll
        for (int v = 0; v < 16; ++v)
          if ((3 * v) / 4 == j) e[v] = __builtin_amdgcn_exp2f(__builtin_fmaf(src.S[v], c2, nlq));
#pragma unroll
        for (int v = 0; v < 15; ++v)
          if ((3 * v) / 4 + 1 == j) dst[v >> 3][v & 7] = (bf16)(e[v] * src.dP[v]);
        if (j == 11) {  // keep the packing of scores 0-14 in this phase
          dst[0] = pin(dst[0]);
          dst[1] = pin(dst[1]);
        }
        if (j == 0) {  // score 15 of the previous phase
          const DqSc& psrc = ph ? s1 : s0;
          bf16x8 (&pdst)[2] = ph ? d1 : d0;
          pdst[1][7] = (bf16)(e15 * psrc.dP[15]);
          pdst[1] = pin(pdst[1]);
        }
        if (j == 11) e15 = e[15];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    ka0 = kt[0];
    ka1 = kt[1];
    if (t + 2 < ntile) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    sc = sn;
  }
  {  // last tile: score 15 of key block 0, key block 1's softmax, the eight dQ products
    const char* SC = smem + sc;
    d0[1][7] = (bf16)(e15 * s0.dP[15]);
    softmax(s1, d1);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int db = 0; db < 2; ++db)
          dQ[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ktr(SC, kb, s, db), kb ? d1[s] : d0[s], dQ[db], 0, 0, 0);
  }

  if (my_q < N) {
    bf16* dQg = (bf16*)p.dq + b * p.sdq[0] + hh * p.sdq[1] + (int64_t)my_q * p.sdq[2];
    const float sc2 = p.scale;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(dQg + db * 32 + 8 * g + 4 * hf, dQ[db][4 * g] * sc2, dQ[db][4 * g + 1] * sc2,
               dQ[db][4 * g + 2] * sc2, dQ[db][4 * g + 3] * sc2, true);
  }
}

hipError_t launch_dq_pipe(const AttnArgs& a, int nqb, unsigned nblk, hipStream_t st) {
  const size_t smem = 3 * (size_t)kBufK;
  hipError_t e = hipFuncSetAttribute((const void*)fa_bwd_dq_bf16_pipe,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fa_bwd_dq_bf16_pipe, dim3(nblk), dim3(512), smem, st, a, nqb);
  return hipGetLastError();
}

}  // namespace mt
