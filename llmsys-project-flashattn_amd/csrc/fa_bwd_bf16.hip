// FlashAttention backward, bf16 MFMA kernels for head dim 64 (BASELINE config 3).
//
// Same mathematics and the same deterministic three-launch split as the generic backward
// (fa_bwd.hip; reference backward_kernel, src/flashattention_kernel.cu:115-255, with the
// reference's dV term corrected):
//     P = exp(s − m)/l,  dV = Pᵀ dO,  dP = dO Vᵀ,  δ = rowsum(dO ∘ O),
//     dS = P ∘ (dP − δ),  dQ = dS K/√d,  dK = dSᵀ Q/√d,
// specialised for bf16 I/O at d = 64 the way the forward kernels are:
//  * prep   : 8 lanes per row; writes the row constants pre-negated and pre-scaled
//             (−lse2/c2 and −δ, c2 = log2e/√d) so they can seed MFMA accumulators.
//  * dkv    : a wave owns 32 keys (K, V rows as register-resident B operands) and sweeps
//             32-query tiles staged in LDS twice — a row image (ds_read_b128, A operand of
//             S = Q·Kᵀ and dP = dO·Vᵀ) and a transpose image (ds_read_b64_tr_b16, A operand
//             of dVᵀ += dOᵀ·P and dKᵀ += Qᵀ·dS). S and dP start from the row constants
//             (C-init), so p = exp2(c2·S') and dS = p·dP' need no subtraction; their
//             accumulators are directly the B operands of the next two products.
//  * dq     : a wave owns 32 queries (Q, dO rows in registers) and sweeps 64-key tiles
//             (K row + transpose images, V row image); Sᵀ, dPᵀ with the query on the lane,
//             dQᵀ += Kᵀ·dSᵀ.
// Staging uses buffer loads (rows past N read as zero) into a double-buffered LDS ring,
// one barrier per tile; masked tiles (ragged N, causal diagonal) are peeled from the bulk.
#include "fa_bwd_bf16.h"

namespace mt {

using namespace bwdbf16;

// ---------------------------------------------------------------------------------------
// prep: nlse = −(m·log2e + log2 l)/c2, ndel = −rowsum(dO ∘ O); 8 lanes per row, kPrepRows
// rows per lane group (all loads issued first: with one row per 32-row workgroup the
// C3 prep ran 16384 tiny workgroups at ≈2.2 TB/s).
constexpr int kPrepRows = 4;
// grid (ceil(N / (RPP kPrepRows)), B·H): the head from blockIdx.y, no 64-bit division per row
// (the 1-D form divided each row index by N and H). DH = 64 (8 lanes per row, RPP = 32 rows per
// pass) or 128 (16 lanes, 16 rows: the d = 128 backward, fa_bwd_d128.hip).
template <int DH = 64>
__global__ __launch_bounds__(256) void fa_bwd_prep_bf16(AttnArgs p) {
  constexpr int LPR = DH / 8, RPP = 256 / LPR;
  const int bh = blockIdx.y;
  const int b = bh / p.H, hh = bh % p.H;
  if (p.dq_cnt && blockIdx.x == 0) {  // the fused backward's arrival counters of this head
    const int nsa = (p.N + 63) / 64;
    for (int i = threadIdx.x; i < nsa; i += 256) p.dq_cnt[(int64_t)bh * nsa + i] = 0u;
  }
  const int n0 = blockIdx.x * RPP * kPrepRows + threadIdx.x / LPR;
  const int sub = threadIdx.x % LPR;
  const int64_t row0 = (int64_t)bh * p.N;
  const bf16* O = (const bf16*)p.o + b * p.so[0] + hh * p.so[1] + 8 * sub;
  const bf16* dO = (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1] + 8 * sub;
  bf16x8 o[kPrepRows], g[kPrepRows];
  float mm[kPrepRows], ll[kPrepRows];
#pragma unroll
  for (int u = 0; u < kPrepRows; ++u) {
    const int n = n0 + RPP * u;
    o[u] = bf16x8{};
    g[u] = bf16x8{};
    mm[u] = 0.f;
    ll[u] = 1.f;
    if (n < p.N) {
      o[u] = *(const bf16x8*)(O + (int64_t)n * p.so[2]);
      g[u] = *(const bf16x8*)(dO + (int64_t)n * p.sdo[2]);
      if (sub == 0) {
        mm[u] = p.m[row0 + n];
        ll[u] = p.l[row0 + n];
      }
    }
  }
#pragma unroll
  for (int u = 0; u < kPrepRows; ++u) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += (float)o[u][j] * (float)g[u][j];
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 4);
    if (LPR == 16) acc += __shfl_xor(acc, 8);
    const int n = n0 + RPP * u;
    if (n < p.N && sub == 0) {
      p.delta[row0 + n] = -acc;
      p.lse2[row0 + n] = -(mm[u] * kLog2e + log2f(ll[u])) / p.scale_log2;
    }
  }
}

// ---------------------------------------------------------------------------------------
// dK, dV. Workgroup = 4 waves = 128 keys; 32-query tiles.
namespace {
constexpr int kQT = 32;
constexpr int kImgQ = kQT * D;                       // elements of one Q / dO image
constexpr int kBufQ = 4 * kImgQ * 2 + 2 * kQT * 4;   // bytes per ring slot: 4 images + 2 row vectors

struct DkvCtx {
  bf16x8 kf[4], vf[4];  // B operands: K / V rows of this lane's key
  int roff[4];          // row-image offsets per k-step
  int toff[2];          // transpose-image offsets per d block
};

// ABL (diagnostic timing builds only, wrong results): bit 1 skips the softmax VALU (P = S,
// dS = dP' go straight to bf16).
template <bool CAUSAL, bool MASK, int ABL = 0>
__device__ __forceinline__ void dkv_tile(const char* slot, const DkvCtx& c, f32x16 (&dK)[2],
                                         f32x16 (&dV)[2], float c2, int qt, int N, int my_k, int hf) {
  const bf16* Qr = (const bf16*)slot;
  const bf16* Qt = Qr + kImgQ;
  const bf16* Or = Qr + 2 * kImgQ;
  const bf16* Ot = Qr + 3 * kImgQ;
  const float* nl = (const float*)(Qr + 4 * kImgQ);
  const float* nd = nl + kQT;
  f32x16 S, dP;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 a = *(const float4*)(nl + 8 * g + 4 * hf);
    const float4 e = *(const float4*)(nd + 8 * g + 4 * hf);
    S[4 * g] = a.x; S[4 * g + 1] = a.y; S[4 * g + 2] = a.z; S[4 * g + 3] = a.w;
    dP[4 * g] = e.x; dP[4 * g + 1] = e.y; dP[4 * g + 2] = e.z; dP[4 * g + 3] = e.w;
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(Qr + c.roff[ks]), c.kf[ks], S, 0, 0, 0);
    dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(Or + c.roff[ks]), c.vf[ks], dP, 0, 0, 0);
  }
  if (MASK) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = qt + acc_row(r, hf);
      if (q >= N || (CAUSAL && my_k > q)) S[r] = -INFINITY;
    }
  }
  if (!(ABL & 1)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pv = __builtin_amdgcn_exp2f(S[r] * c2);
      S[r] = pv;
      dP[r] = pv * dP[r];
    }
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const bf16x8 pf = to_bf16x8(S, s), sf = to_bf16x8(dP, s);
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      dV[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Ot, 16 * s, c.toff[db]), pf, dV[db], 0, 0, 0);
      dK[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Qt, 16 * s, c.toff[db]), sf, dK[db], 0, 0, 0);
    }
  }
}
// Software-pipelined bulk iteration of the dK/dV kernel (mask-free tiles t and t+1):
//   C-init S(t+1), dP(t+1) from the row constants of slot sn;
//   phase A: 8 x [Q/dO row read (2 ahead), S(t+1) or dP(t+1) MFMA, softmax of 2 scores of t]
//   phase B: 8 x [Qᵀ/dOᵀ transpose reads (2 ahead), dV(t) or dK(t) MFMA]
// so tile t's exponentials overlap tile t+1's score products inside one wave.
__device__ __forceinline__ void dkv_pipe(const char* slot_c, const char* slot_n, const DkvCtx& c,
                                         const f32x16& Sc, const f32x16& dPc, f32x16& Sn,
                                         f32x16& dPn, f32x16 (&dK)[2], f32x16 (&dV)[2], float c2,
                                         int hf) {
  const bf16* Qrn = (const bf16*)slot_n;
  const float* nln = (const float*)(Qrn + 4 * kImgQ);
  const float* ndn = nln + kQT;
  // per-lane operand bases: one add each, every read then takes an immediate offset
  const bf16* qr[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) qr[ks] = Qrn + c.roff[ks];
  const bf16* tq[2];
#pragma unroll
  for (int db = 0; db < 2; ++db) tq[db] = (const bf16*)slot_c + kImgQ + c.toff[db];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 a = *(const float4*)(nln + 8 * g + 4 * hf);
    const float4 e = *(const float4*)(ndn + 8 * g + 4 * hf);
    Sn[4 * g] = a.x; Sn[4 * g + 1] = a.y; Sn[4 * g + 2] = a.z; Sn[4 * g + 3] = a.w;
    dPn[4 * g] = e.x; dPn[4 * g + 1] = e.y; dPn[4 * g + 2] = e.z; dPn[4 * g + 3] = e.w;
  }
  bf16x8 af[8];
#define DKV_AREAD(I_) af[I_] = *(const bf16x8*)(qr[(I_) >> 1] + ((I_) & 1 ? 2 * kImgQ : 0));
  DKV_AREAD(0)
  DKV_AREAD(1)
  bf16x8 pf[2], sf[2];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i + 2 < 8) DKV_AREAD(i + 2)
    if (i & 1) dPn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], c.vf[i >> 1], dPn, 0, 0, 0);
    else Sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], c.kf[i >> 1], Sn, 0, 0, 0);
#pragma unroll
    for (int r = 2 * i; r < 2 * i + 2; ++r) {
      const float e = __builtin_amdgcn_exp2f(Sc[r] * c2);
      pf[r >> 3][r & 7] = (bf16)e;
      sf[r >> 3][r & 7] = (bf16)(e * dPc[r]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#undef DKV_AREAD
  bf16x8 bt[8];
  // MFMA n: 16-query step s = n/4, d block db = (n/2)%2, dV (even n) or dK (odd n)
#define DKV_BREAD(N_) bt[N_] = tr_frag(tq[((N_) >> 1) & 1] + (((N_) & 1) ? 0 : 2 * kImgQ), 16 * ((N_) >> 2), 0);
  DKV_BREAD(0)
  DKV_BREAD(1)
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    if (n + 2 < 8) DKV_BREAD(n + 2)
    const int s = n >> 2, db = (n >> 1) & 1;
    if (n & 1) dK[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bt[n], sf[s], dK[db], 0, 0, 0);
    else dV[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bt[n], pf[s], dV[db], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
#undef DKV_BREAD
}

// S(t), dP(t) for a mask-free tile (C-init + 8 MFMAs), the pipeline's entry.
__device__ __forceinline__ void dkv_scores(const char* slot, const DkvCtx& c, f32x16& S, f32x16& dP,
                                           int hf) {
  const bf16* Qr = (const bf16*)slot;
  const bf16* Or = Qr + 2 * kImgQ;
  const float* nl = (const float*)(Qr + 4 * kImgQ);
  const float* nd = nl + kQT;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 a = *(const float4*)(nl + 8 * g + 4 * hf);
    const float4 e = *(const float4*)(nd + 8 * g + 4 * hf);
    S[4 * g] = a.x; S[4 * g + 1] = a.y; S[4 * g + 2] = a.z; S[4 * g + 3] = a.w;
    dP[4 * g] = e.x; dP[4 * g + 1] = e.y; dP[4 * g + 2] = e.z; dP[4 * g + 3] = e.w;
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(Qr + c.roff[ks]), c.kf[ks], S, 0, 0, 0);
    dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(Or + c.roff[ks]), c.vf[ks], dP, 0, 0, 0);
  }
}

// softmax + dV/dK of a tile whose S, dP are already computed (the pipeline's exit).
__device__ __forceinline__ void dkv_finish(const char* slot, const DkvCtx& c, const f32x16& S,
                                           const f32x16& dP, f32x16 (&dK)[2], f32x16 (&dV)[2],
                                           float c2) {
  const bf16* Qt = (const bf16*)slot + kImgQ;
  const bf16* Ot = (const bf16*)slot + 3 * kImgQ;
  bf16x8 pf[2], sf[2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float e = __builtin_amdgcn_exp2f(S[r] * c2);
    pf[r >> 3][r & 7] = (bf16)e;
    sf[r >> 3][r & 7] = (bf16)(e * dP[r]);
  }
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      dV[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Ot, 16 * s, c.toff[db]), pf[s], dV[db], 0, 0, 0);
      dK[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Qt, 16 * s, c.toff[db]), sf[s], dK[db], 0, 0, 0);
    }
}
}  // namespace

// dK/dV with the software-pipelined bulk loop (3-slot LDS ring: an iteration reads the
// transposes of tile t and the rows of tile t+1 while tile t+2 is staged).
template <bool CAUSAL>
__global__ __launch_bounds__(256, 2) void fa_bwd_dkv_bf16_p(AttnArgs p, int nkb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = logical / nkb, kb = logical % nkb;
  const int b = bh / p.H, hh = bh % p.H;
  const int k0 = kb * 128;
  const int my_k = k0 + wave * 32 + c32;
  const int wk_lo = k0 + wave * 32;

  DkvCtx c;
  {
    const int kr = min(my_k, N - 1);
    const bf16* krow = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1] + (int64_t)kr * p.sk[2];
    const bf16* vrow = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1] + (int64_t)kr * p.sv[2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      c.kf[ks] = *(const bf16x8*)(krow + 16 * ks + 8 * hf);
      c.vf[ks] = *(const bf16x8*)(vrow + 16 * ks + 8 * hf);
      c.roff[ks] = k_swz<D>(c32, 2 * ks + hf);
    }
    c.toff[0] = tr_off(lane, 0);
    c.toff[1] = tr_off(lane, 1);
  }
  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Og = (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const int sqn = (int)p.sq[2], son = (int)p.sdo[2];
  const __amdgpu_buffer_rsrc_t rq = head_rsrc(Qg, N, sqn), ro = head_rsrc(Og, N, son);
  const int st_r = tid >> 3, st_c = tid & 7;
  const int goq = (st_r * sqn + st_c * 8) * 2, goo = (st_r * son + st_c * 8) * 2;
  const int srow = k_swz<D>(st_r, st_c), stri = v_swz<D>(st_r, st_c);
  const float* nlse = p.lse2 + (int64_t)bh * N;
  const float* ndel = p.delta + (int64_t)bh * N;

  const int qt0 = CAUSAL ? k0 : 0;
  const int ntile = N > qt0 ? (N - qt0 + kQT - 1) / kQT : 0;
  const int ndiag = CAUSAL ? min(ntile, 128 / kQT) : 0;
  const int nfull = max(ndiag, (N - qt0) / kQT);

  uint4 sq, so;
  float sv = 0.f;
#define DKV_LOAD(T_)                                                                     \
  {                                                                                      \
    const int qt_ = qt0 + (T_) * kQT;                                                    \
    sq = bload(rq, goq + qt_ * sqn * 2);                                                 \
    so = bload(ro, goo + qt_ * son * 2);                                                 \
    if (tid < 2 * kQT) {                                                                 \
      const int q_ = qt_ + (tid & (kQT - 1));                                            \
      sv = q_ < N ? (tid < kQT ? nlse[q_] : ndel[q_]) : 0.f;                             \
    }                                                                                    \
  }
#define DKV_STORE(T_)                                                                    \
  {                                                                                      \
    bf16* img = (bf16*)(smem + ((T_) % 3) * kBufQ);                                      \
    *(uint4*)(img + srow) = sq;                                                          \
    *(uint4*)(img + kImgQ + stri) = sq;                                                  \
    *(uint4*)(img + 2 * kImgQ + srow) = so;                                              \
    *(uint4*)(img + 3 * kImgQ + stri) = so;                                              \
    if (tid < 2 * kQT) ((float*)(img + 4 * kImgQ))[tid] = sv;                            \
  }
#define SLOT(T_) (smem + ((T_) % 3) * kBufQ)

  f32x16 dK[2], dV[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) { dK[i] = f32x16{}; dV[i] = f32x16{}; }
  const float c2 = p.scale_log2;

  // prologue: tiles 0 and 1 staged
  for (int i = 0; i < 2 && i < ntile; ++i) {
    DKV_LOAD(i)
    DKV_STORE(i)
  }
  __syncthreads();
  // general step: tile t from scratch (masks, per-wave causal skip); stages tile t+2
#define DKV_GEN(MASK_, T_)                                                               \
  {                                                                                      \
    const int t_ = (T_);                                                                 \
    const bool st_ = t_ + 2 < ntile;                                                     \
    if (st_) DKV_LOAD(t_ + 2)                                                            \
    const int qt_ = qt0 + t_ * kQT;                                                      \
    if (!(MASK_) || !CAUSAL || qt_ + kQT - 1 >= wk_lo)                                   \
      dkv_tile<CAUSAL, MASK_>(SLOT(t_), c, dK, dV, c2, qt_, N, my_k, hf);                \
    if (st_) DKV_STORE(t_ + 2)                                                           \
    __syncthreads();                                                                     \
  }
  int t = 0;
  for (; t < ndiag; ++t) DKV_GEN(true, t)
  if (nfull - t >= 2) {
    // pipelined bulk: S(t) computed ahead; iteration t also computes S(t+1)
    f32x16 SA, dPA, SB, dPB;
    dkv_scores(SLOT(t), c, SA, dPA, hf);
    // ring offsets rotate (current, next, write) without per-iteration modulo arithmetic
    int oc = (t % 3) * kBufQ, on = ((t + 1) % 3) * kBufQ, ow = ((t + 2) % 3) * kBufQ;
#define DKV_PIPE(T_, SC_, DPC_, SN_, DPN_)                                               \
  {                                                                                      \
    const int t_ = (T_);                                                                 \
    const bool st_ = t_ + 2 < ntile;                                                     \
    if (st_) DKV_LOAD(t_ + 2)                                                            \
    dkv_pipe(smem + oc, smem + on, c, SC_, DPC_, SN_, DPN_, dK, dV, c2, hf);             \
    if (st_) {                                                                           \
      bf16* img = (bf16*)(smem + ow);                                                    \
      *(uint4*)(img + srow) = sq;                                                        \
      *(uint4*)(img + kImgQ + stri) = sq;                                                \
      *(uint4*)(img + 2 * kImgQ + srow) = so;                                            \
      *(uint4*)(img + 3 * kImgQ + stri) = so;                                            \
      if (tid < 2 * kQT) ((float*)(img + 4 * kImgQ))[tid] = sv;                          \
    }                                                                                    \
    __syncthreads();                                                                     \
    const int o_ = oc;                                                                   \
    oc = on;                                                                             \
    on = ow;                                                                             \
    ow = o_;                                                                             \
  }
    for (; t + 2 < nfull; t += 2) {
      DKV_PIPE(t, SA, dPA, SB, dPB)
      DKV_PIPE(t + 1, SB, dPB, SA, dPA)
    }
    if (t + 1 < nfull) {
      DKV_PIPE(t, SA, dPA, SB, dPB)
      ++t;
      SA = SB;
      dPA = dPB;
    }
#undef DKV_PIPE
    // last bulk tile: S(t) in SA
    {
      const bool st_ = t + 2 < ntile;
      if (st_) DKV_LOAD(t + 2)
      dkv_finish(SLOT(t), c, SA, dPA, dK, dV, c2);
      if (st_) DKV_STORE(t + 2)
      __syncthreads();
      ++t;
    }
  }
  for (; t < ntile; ++t) {
    if (t < nfull) DKV_GEN(false, t) else DKV_GEN(true, t)
  }
#undef DKV_GEN
#undef DKV_LOAD
#undef DKV_STORE
#undef SLOT

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
}

// PAIR (causal): a workgroup owns key blocks nkb - 1 - u (light) and then u (heavy) of one
// head, so every workgroup walks about nkb + 1 query tiles and the grid has no tail of
// heavy blocks dispatched last (greedy list schedule of the head-ordered grid: ~10 %
// over the balanced bound at C3 causal).
template <bool CAUSAL, bool PAIR = false>
__global__ __launch_bounds__(256, 2) void fa_bwd_dkv_bf16(AttnArgs p, int nkb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int nslot = PAIR ? (nkb + 1) / 2 : nkb;
  const int bh = logical / nslot, u_ = logical % nslot;
  const int b = bh / p.H, hh = bh % p.H;
#pragma nounroll
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
  const int kb = PAIR ? (pass == 0 ? nkb - 1 - u_ : u_) : u_;
  if (PAIR && pass == 1) {
    if (kb == nkb - 1 - u_) break;  // odd nkb: the middle block has no partner
    __syncthreads();                 // the first block's last LDS reads are done
  }
  const int k0 = kb * 128;
  const int my_k = k0 + wave * 32 + c32;
  const int wk_lo = k0 + wave * 32;

  DkvCtx c;
  {
    const int kr = min(my_k, N - 1);
    const bf16* krow = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1] + (int64_t)kr * p.sk[2];
    const bf16* vrow = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1] + (int64_t)kr * p.sv[2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      c.kf[ks] = *(const bf16x8*)(krow + 16 * ks + 8 * hf);
      c.vf[ks] = *(const bf16x8*)(vrow + 16 * ks + 8 * hf);
      c.roff[ks] = k_swz<D>(c32, 2 * ks + hf);
    }
    c.toff[0] = tr_off(lane, 0);
    c.toff[1] = tr_off(lane, 1);
  }

  // Staging: thread -> (row, chunk) of the 32 x 64 Q and dO tiles; 64 threads move the
  // two row-constant vectors.
  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Og = (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const int sqn = (int)p.sq[2], son = (int)p.sdo[2];
  const __amdgpu_buffer_rsrc_t rq = head_rsrc(Qg, N, sqn), ro = head_rsrc(Og, N, son);
  const int st_r = tid >> 3, st_c = tid & 7;
  const int goq = (st_r * sqn + st_c * 8) * 2, goo = (st_r * son + st_c * 8) * 2;
  const int srow = k_swz<D>(st_r, st_c), stri = v_swz<D>(st_r, st_c);
  const float* nlse = p.lse2 + (int64_t)bh * N;
  const float* ndel = p.delta + (int64_t)bh * N;

  const int qt0 = CAUSAL ? k0 : 0;
  const int ntile = N > qt0 ? (N - qt0 + kQT - 1) / kQT : 0;
  // mask-free tiles: [ndiag, nfull)
  const int ndiag = CAUSAL ? min(ntile, 128 / kQT) : 0;
  const int nfull = max(ndiag, (N - qt0) / kQT);

  uint4 sq, so;
  float sv = 0.f;
#define DKV_LOAD(T_)                                                                     \
  {                                                                                      \
    const int qt_ = qt0 + (T_) * kQT;                                                    \
    sq = bload(rq, goq + qt_ * sqn * 2);                                                 \
    so = bload(ro, goo + qt_ * son * 2);                                                 \
    if (tid < 2 * kQT) {                                                                 \
      const int q_ = qt_ + (tid & (kQT - 1));                                            \
      sv = q_ < N ? (tid < kQT ? nlse[q_] : ndel[q_]) : 0.f;                             \
    }                                                                                    \
  }
#define DKV_STORE(SLOT_)                                                                 \
  {                                                                                      \
    bf16* img = (bf16*)(smem + (SLOT_) * kBufQ);                                         \
    *(uint4*)(img + srow) = sq;                                                          \
    *(uint4*)(img + kImgQ + stri) = sq;                                                  \
    *(uint4*)(img + 2 * kImgQ + srow) = so;                                              \
    *(uint4*)(img + 3 * kImgQ + stri) = so;                                              \
    if (tid < 2 * kQT) ((float*)(img + 4 * kImgQ))[tid] = sv;                            \
  }

  f32x16 dK[2], dV[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) { dK[i] = f32x16{}; dV[i] = f32x16{}; }
  const float c2 = p.scale_log2;

  if (ntile > 0) {
    DKV_LOAD(0)
    DKV_STORE(0)
  }
  __syncthreads();
#define DKV_STEP(MASK_, SLOT_, T_)                                                       \
  {                                                                                      \
    const int t_ = (T_);                                                                 \
    const bool more_ = t_ + 1 < ntile;                                                   \
    if (more_) DKV_LOAD(t_ + 1)                                                          \
    const int qt_ = qt0 + t_ * kQT;                                                      \
    if (!(MASK_) || !CAUSAL || qt_ + kQT - 1 >= wk_lo)                                   \
      dkv_tile<CAUSAL, MASK_>(smem + (SLOT_) * kBufQ, c, dK, dV, c2, qt_, N, my_k, hf);  \
    if (more_) DKV_STORE((SLOT_) ^ 1)                                                    \
    __syncthreads();                                                                     \
  }
  int t = 0;
  for (; t < ndiag; ++t) {
    if (t & 1) DKV_STEP(true, 1, t) else DKV_STEP(true, 0, t)
  }
  if ((t & 1) && t < nfull) {
    DKV_STEP(false, 1, t)
    ++t;
  }
  for (; t + 1 < nfull; t += 2) {
    DKV_STEP(false, 0, t)
    DKV_STEP(false, 1, t + 1)
  }
  for (; t < ntile; ++t) {
    if (t < nfull) {
      if (t & 1) DKV_STEP(false, 1, t) else DKV_STEP(false, 0, t)
    } else {
      if (t & 1) DKV_STEP(true, 1, t) else DKV_STEP(true, 0, t)
    }
  }
#undef DKV_STEP
#undef DKV_LOAD
#undef DKV_STORE

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
  }  // pass
}

// dK/dV with 64-query steps: each barrier-to-barrier step stages two 32-query sub-tiles
// (two ring sub-slots) and runs dkv_tile on both, halving the barriers and global-load
// round trips per MFMA against the 32-query kernel above (A/B variant).
// MINB = workgroups per CU the register budget targets: 2 (two waves per SIMD, 256 VGPRs,
// the compiler spills ~38 values into scratch inside the loop) or 1 (one wave per SIMD,
// 512 VGPR+AGPR, no spills, no second wave to overlap with).
// DMA: the Q / dO images arrive by LDS-DMA (dma_rows) instead of buffer loads into VGPRs
// plus ds_writes: no staging registers live across the step (policy 66, A/B variant).
// NW = waves per workgroup (32 keys each): 4, or 8 with DMA (256 keys per workgroup: every
// staged Q / dO step feeds twice the keys, halving the L2 -> LDS traffic per MFMA; each
// wave then stages one of the two 32-query sub-tiles).
// ABL (diagnostic timing builds only, wrong results): bit 1 no softmax VALU, bit 2 no
// staging after the first step, bit 4 no barrier per step.
// SUB = 32-query sub-tiles per barrier-to-barrier step: 2, or 4 in the 8-wave form (half the
// barriers and DMA waits per MFMA; 2 x 4 sub-slots of LDS, 133 KiB).
template <bool CAUSAL, int MINB = 2, bool DMA = false, int NW = 4, int ABL = 0, int SUB = 2>
__global__ __launch_bounds__(64 * NW, MINB) void fa_bwd_dkv_bf16_q64(AttnArgs p, int nkb) {
  static_assert(NW == 4 || (NW == 8 && DMA), "8-wave form: LDS-DMA staging only");
  static_assert(SUB == 2 || (SUB == 4 && NW == 8), "4 sub-tiles per step: 8-wave form only");
#ifndef MT_DIAGNOSTICS
  static_assert(ABL == 0, "wrong-result ablations exist only in the MT_DIAGNOSTICS build");
#endif
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = logical / nkb, kb = logical % nkb;
  const int b = bh / p.H, hh = bh % p.H;
  constexpr int kKB = 32 * NW;  // keys per workgroup
  const int k0 = kb * kKB;
  const int my_k = k0 + wave * 32 + c32;
  const int wk_lo = k0 + wave * 32;

  DkvCtx c;
  {
    const int kr = min(my_k, N - 1);
    const bf16* krow = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1] + (int64_t)kr * p.sk[2];
    const bf16* vrow = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1] + (int64_t)kr * p.sv[2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      c.kf[ks] = *(const bf16x8*)(krow + 16 * ks + 8 * hf);
      c.vf[ks] = *(const bf16x8*)(vrow + 16 * ks + 8 * hf);
      c.roff[ks] = k_swz<D>(c32, 2 * ks + hf);
    }
    c.toff[0] = tr_off(lane, 0);
    c.toff[1] = tr_off(lane, 1);
  }

  // Staging: thread -> (row, chunk) of each 32 x 64 sub-tile of Q and dO (one chunk per
  // sub-tile per tensor); 128 threads move the row constants of both sub-tiles.
  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Og = (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const int sqn = (int)p.sq[2], son = (int)p.sdo[2];
  const __amdgpu_buffer_rsrc_t rq = head_rsrc(Qg, N, sqn), ro = head_rsrc(Og, N, son);
  const int st_r = tid >> 3, st_c = tid & 7;
  const int goq = (st_r * sqn + st_c * 8) * 2, goo = (st_r * son + st_c * 8) * 2;
  const int srow = k_swz<D>(st_r, st_c), stri = v_swz<D>(st_r, st_c);
  const float* nlse = p.lse2 + (int64_t)bh * N;
  const float* ndel = p.delta + (int64_t)bh * N;
  // DMA: wave w fills rows 8w..8w+7 of each image; lane l -> row 8w + l/8, LDS chunk l%8,
  // which holds source chunk (l%8) ^ swz(row) (the swizzles are XOR, self-inverse)
  // this wave's rows 8w..8w+7 of every image (8 waves: rows 8(w%4).. of sub-tiles
  // G(w/4) .. G(w/4) + G - 1, G = SUB / 2), as a scalar LDS byte address; one set of per-lane
  // source offsets serves all G sub-tiles (the same rows, a wave-uniform query offset)
  constexpr int G = NW == 8 ? SUB / 2 : 1;
  int gdq[2] = {0, 0}, gdo[2] = {0, 0};
  const int wq = NW == 8 ? (wave & 3) : wave, wu = NW == 8 ? G * (wave >> 2) : 0;
  const uint32_t lds0 = lds_base(smem) + __builtin_amdgcn_readfirstlane(wq) * 8 * D * 2 +
                        __builtin_amdgcn_readfirstlane(wu) * kBufQ;
  if (DMA) {
    const int r = 8 * wq + (lane >> 3), pc = lane & 7;
    const int ck = pc ^ ((r >> 1) & 7), cv = pc ^ (((r >> 1) & 1) << 2);
    gdq[0] = (r * sqn + ck * 8) * 2;
    gdq[1] = (r * sqn + cv * 8) * 2;
    gdo[0] = (r * son + ck * 8) * 2;
    gdo[1] = (r * son + cv * 8) * 2;
  }

  constexpr int kStep = SUB * kQT;
  const int qt0 = CAUSAL ? k0 : 0;
  const int nstep = N > qt0 ? (N - qt0 + kStep - 1) / kStep : 0;

  uint4 sq[2], so[2];
  float sv = 0.f;
#define DKV2_LOAD(T_, SLOT_)                                                             \
  {                                                                                      \
    const int qs_ = qt0 + (T_) * kStep;                                                  \
    if (NW == 8) {                                                                       \
      _Pragma("unroll") for (int g = 0; g < G; ++g) {                                    \
        const uint32_t img_ = lds0 + (SUB * (SLOT_) + g) * kBufQ;                        \
        const int oq_ = (qs_ + (wu + g) * kQT) * sqn * 2, oo_ = (qs_ + (wu + g) * kQT) * son * 2; \
        dma_rows(img_, rq, gdq[0] + oq_);                                                \
        dma_rows(img_ + kImgQ * 2, rq, gdq[1] + oq_);                                    \
        dma_rows(img_ + 2 * kImgQ * 2, ro, gdo[0] + oo_);                                \
        dma_rows(img_ + 3 * kImgQ * 2, ro, gdo[1] + oo_);                                \
      }                                                                                  \
    } else _Pragma("unroll") for (int u = 0; u < 2; ++u) {                               \
      if (DMA) {                                                                         \
        const uint32_t img_ = lds0 + (2 * (SLOT_) + u) * kBufQ;                          \
        const int oq_ = (qs_ + u * kQT) * sqn * 2, oo_ = (qs_ + u * kQT) * son * 2;      \
        dma_rows(img_, rq, gdq[0] + oq_);                                                \
        dma_rows(img_ + kImgQ * 2, rq, gdq[1] + oq_);                                    \
        dma_rows(img_ + 2 * kImgQ * 2, ro, gdo[0] + oo_);                                \
        dma_rows(img_ + 3 * kImgQ * 2, ro, gdo[1] + oo_);                                \
      } else {                                                                           \
        sq[u] = bload(rq, goq + (qs_ + u * kQT) * sqn * 2);                              \
        so[u] = bload(ro, goo + (qs_ + u * kQT) * son * 2);                              \
      }                                                                                  \
    }                                                                                    \
    if (tid < SUB * 2 * kQT) {                                                           \
      const int q_ = qs_ + (tid >> 6) * kQT + (tid & (kQT - 1));                         \
      sv = q_ < N ? ((tid & kQT) == 0 ? nlse[q_] : ndel[q_]) : 0.f;                      \
    }                                                                                    \
  }
#define DKV2_STORE(SLOT_)                                                                \
  {                                                                                      \
    if (!DMA) {                                                                          \
      _Pragma("unroll") for (int u = 0; u < 2; ++u) {                                    \
        bf16* img = (bf16*)(smem + (2 * (SLOT_) + u) * kBufQ);                           \
        *(uint4*)(img + srow) = sq[u];                                                   \
        *(uint4*)(img + kImgQ + stri) = sq[u];                                           \
        *(uint4*)(img + 2 * kImgQ + srow) = so[u];                                       \
        *(uint4*)(img + 3 * kImgQ + stri) = so[u];                                       \
      }                                                                                  \
    }                                                                                    \
    if (tid < SUB * 2 * kQT)                                                             \
      ((float*)((bf16*)(smem + (SUB * (SLOT_) + (tid >> 6)) * kBufQ) + 4 * kImgQ))[tid & 63] = sv; \
    if (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                            \
  }

  f32x16 dK[2], dV[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) { dK[i] = f32x16{}; dV[i] = f32x16{}; }
  const float c2 = p.scale_log2;

  if (nstep > 0) {
    DKV2_LOAD(0, 0)
    DKV2_STORE(0)
  }
  __syncthreads();
  // steps: [0, nhead) causal diagonal (masked), [nhead, nfull) mask-free, [nfull, nstep)
  // ragged tail (masked)
  const int nhead = CAUSAL ? min(nstep, kKB / kStep) : 0;
  const int nfull = max(nhead, (N - qt0) / kStep);
#define DKV2_STEP(MASK_, SLOT_, T_)                                                      \
  {                                                                                      \
    const int t_ = (T_);                                                                 \
    const bool more_ = t_ + 1 < nstep && !(ABL & 2);                                     \
    if (more_) DKV2_LOAD(t_ + 1, (SLOT_) ^ 1)                                            \
    _Pragma("unroll") for (int u = 0; u < SUB; ++u) {                                    \
      const int qt_ = qt0 + t_ * kStep + u * kQT;                                        \
      if (!(MASK_) || (qt_ < N && (!CAUSAL || qt_ + kQT - 1 >= wk_lo)))                 \
        dkv_tile<CAUSAL, MASK_, ABL>(smem + (SUB * (SLOT_) + u) * kBufQ, c, dK, dV, c2, qt_, \
                                     N, my_k, hf);                                       \
      if (SUB > 2) __builtin_amdgcn_sched_barrier(0);                                    \
    }                                                                                    \
    if (more_) DKV2_STORE((SLOT_) ^ 1)                                                   \
    if (!(ABL & 4)) __syncthreads();                                                     \
  }
  int t = 0;
  for (; t < nhead; ++t) {
    if (t & 1) DKV2_STEP(true, 1, t) else DKV2_STEP(true, 0, t)
  }
  if ((t & 1) && t < nfull) {
    DKV2_STEP(false, 1, t)
    ++t;
  }
  for (; t + 1 < nfull; t += 2) {
    DKV2_STEP(false, 0, t)
    DKV2_STEP(false, 1, t + 1)
  }
  for (; t < nstep; ++t) {
    if (t < nfull) {
      if (t & 1) DKV2_STEP(false, 1, t) else DKV2_STEP(false, 0, t)
    } else {
      if (t & 1) DKV2_STEP(true, 1, t) else DKV2_STEP(true, 0, t)
    }
  }
#undef DKV2_STEP
#undef DKV2_LOAD
#undef DKV2_STORE

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
}

// dK/dV, 8 waves, with the two waves of each SIMD half a step apart (MI355X_MICROARCH.md,
// "Two waves per SIMD", item 9: partners running the same program with one barrier per
// block reach their MFMA bursts, their softmax VALU and their LDS reads together).
// Step t = 64 queries (sub-tiles u0, u1), staged by LDS-DMA two steps ahead into a 4-step
// ring (130 KiB, one workgroup per CU). Waves 0-3 (SIMD partners of waves 4-7) compute
// (t, u0) then (t, u1); waves 4-7 compute (t - 1, u1) then (t, u0), and (last, u1) after
// the loop, so the partner of a wave in its first sub-tile is in its second. Non-causal,
// N % 64 == 0 (every step mask-free); the launcher sends other shapes to the 64-query
// kernel.
#ifdef MT_DIAGNOSTICS  // an A/B form (policy 70): diagnostics build only
__global__ __launch_bounds__(512, 2) void fa_bwd_dkv_bf16_st(AttnArgs p, int nkb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int kStepB = 2 * kBufQ;  // bytes per ring step (2 sub-tiles)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = logical / nkb, kb = logical % nkb;
  const int b = bh / p.H, hh = bh % p.H;
  const int k0 = kb * 256;
  const int my_k = k0 + wave * 32 + c32;
  const bool late = __builtin_amdgcn_readfirstlane(wave) >= 4;

  DkvCtx c;
  {
    const int kr = min(my_k, N - 1);
    const bf16* krow = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1] + (int64_t)kr * p.sk[2];
    const bf16* vrow = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1] + (int64_t)kr * p.sv[2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      c.kf[ks] = *(const bf16x8*)(krow + 16 * ks + 8 * hf);
      c.vf[ks] = *(const bf16x8*)(vrow + 16 * ks + 8 * hf);
      c.roff[ks] = k_swz<D>(c32, 2 * ks + hf);
    }
    c.toff[0] = tr_off(lane, 0);
    c.toff[1] = tr_off(lane, 1);
  }
  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Og = (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1];
  const int sqn = (int)p.sq[2], son = (int)p.sdo[2];
  const __amdgpu_buffer_rsrc_t rq = head_rsrc(Qg, N, sqn), ro = head_rsrc(Og, N, son);
  const float* nlse = p.lse2 + (int64_t)bh * N;
  const float* ndel = p.delta + (int64_t)bh * N;
  // DMA: wave w stages rows 8(w%4) .. +7 of the four images of sub-tile w/4
  const int wq = wave & 3, wu = wave >> 2;
  const uint32_t lds0 = lds_base(smem) + __builtin_amdgcn_readfirstlane(wq) * 8 * D * 2 +
                        __builtin_amdgcn_readfirstlane(wu) * kBufQ;
  int gq0, gq1, go0, go1;
  {
    const int r = 8 * wq + (lane >> 3), pc = lane & 7;
    const int ck = pc ^ ((r >> 1) & 7), cv = pc ^ (((r >> 1) & 1) << 2);
    gq0 = (r * sqn + ck * 8) * 2 + wu * kQT * sqn * 2;
    gq1 = (r * sqn + cv * 8) * 2 + wu * kQT * sqn * 2;
    go0 = (r * son + ck * 8) * 2 + wu * kQT * son * 2;
    go1 = (r * son + cv * 8) * 2 + wu * kQT * son * 2;
  }
  const int nstep = N / 64;
  float sv = 0.f;
  auto stage = [&](int t, int slot) __attribute__((always_inline)) {
    const uint32_t img = lds0 + slot * kStepB;
    const int oq = t * 64 * sqn * 2, oo = t * 64 * son * 2;
    dma_rows(img, rq, gq0 + oq);
    dma_rows(img + kImgQ * 2, rq, gq1 + oq);
    dma_rows(img + 2 * kImgQ * 2, ro, go0 + oo);
    dma_rows(img + 3 * kImgQ * 2, ro, go1 + oo);
    if (tid < 4 * kQT) {
      const int q = t * 64 + (tid >> 6) * kQT + (tid & (kQT - 1));
      sv = (tid & kQT) == 0 ? nlse[q] : ndel[q];
    }
  };
  auto publish = [&](int slot) __attribute__((always_inline)) {
    if (tid < 4 * kQT)
      ((float*)((bf16*)(smem + slot * kStepB + (tid >> 6) * kBufQ) + 4 * kImgQ))[tid & 63] = sv;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  f32x16 dK[2], dV[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) { dK[i] = f32x16{}; dV[i] = f32x16{}; }
  const float c2 = p.scale_log2;

  // prologue: steps 0 and 1 staged
  stage(0, 0);
  publish(0);
  if (nstep > 1) {
    stage(1, 1);
    publish(1);
  }
  __syncthreads();
  // The same instruction stream for both halves, only the two sub-tile addresses differ
  // (a branch around the tiles would make the compiler copy the accumulators between
  // the two paths): early (t, u0), (t, u1); late (t - 1, u1), (t, u0). Step 0 is peeled
  // for the late half, which has no step -1.
  const uint32_t lateb = late ? 1u : 0u;
  for (int t = 0; t < nstep; ++t) {
    // 4-step ring: step t + 2 goes into the slot of step t - 2, which every wave finished
    // before the last barrier (waves 4-7 read step t - 2's sub-tile u1 during step t - 1)
    const bool more = t + 2 < nstep;
    if (more) stage(t + 2, (t + 2) & 3);
    const int cur = (t & 3) * kStepB, prv = ((t - 1) & 3) * kStepB;
    const int offA = lateb ? prv + kBufQ : cur, offB = lateb ? cur : cur + kBufQ;
    if (t > 0 || !late) dkv_tile<false, false>(smem + offA, c, dK, dV, c2, 0, N, my_k, hf);
    dkv_tile<false, false>(smem + offB, c, dK, dV, c2, 0, N, my_k, hf);
    if (more) publish((t + 2) & 3);
    __syncthreads();
  }
  if (late) dkv_tile<false, false>(smem + ((nstep - 1) & 3) * kStepB + kBufQ, c, dK, dV, c2, 0, N, my_k, hf);

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
}

#endif  // MT_DIAGNOSTICS

// ---------------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------------
// dQ. Workgroup = 4 waves = 128 queries; 64-key tiles.
namespace {
constexpr int kKT = 64;
constexpr int kImgK = kKT * D;
constexpr int kBufK = 3 * kImgK * 2;  // K row image, K transpose image, V row image

struct DqCtx {
  bf16x8 qf[4], of[4];  // B operands: Q / dO rows of this lane's query
  int roff[4];
  int toff[2];
};

template <bool CAUSAL, bool MASK>
// PF: the eight Kᵀ transpose fragments of the dQ products are read right after the S / dP
// products are issued (pinned there by a scheduling barrier), so they land during the
// softmax instead of in front of each dQ MFMA.
__device__ __forceinline__ void dq_tile(const char* slot, const DqCtx& c, f32x16 (&dQ)[2], float c2,
                                        float nlq, const f32x16& dinit, int k0, int N, int my_q, int hf,
                                        bool PF = false) {
  const bf16* Kr = (const bf16*)slot;
  const bf16* Kt = Kr + kImgK;
  const bf16* Vr = Kr + 2 * kImgK;
  f32x16 S[2], dP[2];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      S[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(Kr + kb * 32 * D + c.roff[ks]),
                                                      c.qf[ks], ks ? S[kb] : f32x16{}, 0, 0, 0);
      // dP chain starts from −δ (row constant as the initial accumulator): dP' = dP − δ
      dP[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(Vr + kb * 32 * D + c.roff[ks]),
                                                       c.of[ks], ks ? dP[kb] : dinit, 0, 0, 0);
    }
  bf16x8 kt[8];
  if (PF) {
#pragma unroll
    for (int i = 0; i < 8; ++i) kt[i] = tr_frag(Kt, (i >> 2) * 32 + 16 * ((i >> 1) & 1), c.toff[i & 1]);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (MASK) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = k0 + kb * 32 + acc_row(r, hf);
        if (key >= N || (CAUSAL && key > my_q)) S[kb][r] = -INFINITY;
      }
  }
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(S[kb][r], c2, nlq));
      dP[kb][r] = pv * dP[kb][r];
    }
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 sf = to_bf16x8(dP[kb], s);
#pragma unroll
      for (int db = 0; db < 2; ++db)
        dQ[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            PF ? kt[kb * 4 + s * 2 + db] : tr_frag(Kt, kb * 32 + 16 * s, c.toff[db]), sf, dQ[db], 0, 0, 0);
    }
}

}  // namespace

// NW = waves per workgroup (32 queries each): 4 or 8 (256 queries: every staged K / V tile
// feeds twice the queries).
// (Capping it at 3 waves per SIMD, 168 VGPRs, spills 42-70 values: not kept.)
// PAIR (causal): a workgroup owns query blocks u (light) and then nqb - 1 - u (heavy) of
// one head, as the paired dK/dV kernel does.
template <bool CAUSAL, int NW = 4, bool PF = false, bool PAIR = false>
__global__ __launch_bounds__(64 * NW, 2) void fa_bwd_dq_bf16(AttnArgs p, int nqb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int nslot = PAIR ? (nqb + 1) / 2 : nqb;
  const int bh = logical / nslot, u_ = logical % nslot;
  const int b = bh / p.H, hh = bh % p.H;
#pragma nounroll
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
  int qb = u_;
  if (PAIR) {
    qb = pass == 0 ? u_ : nqb - 1 - u_;
    if (pass == 1) {
      if (qb == u_) break;  // odd nqb: the middle block has no partner
      __syncthreads();      // the first block's last LDS reads are done
    }
  } else if (CAUSAL) {
    qb = nqb - 1 - qb;  // heaviest first
  }
  constexpr int kQB = 32 * NW;  // queries per workgroup
  constexpr int kRows = 8 / NW;  // 16-B staging chunks per thread per image (64 rows x 8)
  const int q0 = qb * kQB;
  const int my_q = q0 + wave * 32 + c32;
  const int wq_hi = q0 + wave * 32 + 31;

  DqCtx c;
  float nlq, del;
  {
    const int qr = min(my_q, N - 1);
    const bf16* qrow = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1] + (int64_t)qr * p.sq[2];
    const bf16* orow = (const bf16*)p.dout + b * p.sdo[0] + hh * p.sdo[1] + (int64_t)qr * p.sdo[2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      c.qf[ks] = *(const bf16x8*)(qrow + 16 * ks + 8 * hf);
      c.of[ks] = *(const bf16x8*)(orow + 16 * ks + 8 * hf);
      c.roff[ks] = k_swz<D>(c32, 2 * ks + hf);
    }
    c.toff[0] = tr_off(lane, 0);
    c.toff[1] = tr_off(lane, 1);
    const int64_t row = (int64_t)bh * N + qr;
    nlq = p.lse2[row] * p.scale_log2;  // = −lse2
    del = -p.delta[row];
  }

  const bf16* Kg = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1];
  const bf16* Vg = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1];
  const int skn = (int)p.sk[2], svn = (int)p.sv[2];
  const __amdgpu_buffer_rsrc_t rk = head_rsrc(Kg, N, skn), rv = head_rsrc(Vg, N, svn);
  int gk[kRows], gv[kRows], srow[kRows], stri[kRows];
#pragma unroll
  for (int i = 0; i < kRows; ++i) {
    const int r = (tid >> 3) + 8 * NW * i, cc = tid & 7;
    gk[i] = (r * skn + cc * 8) * 2;
    gv[i] = (r * svn + cc * 8) * 2;
    srow[i] = k_swz<D>(r, cc);
    stri[i] = v_swz<D>(r, cc);
  }

  const int kend = CAUSAL ? min(N, q0 + kQB) : N;
  const int ntile = (kend + kKT - 1) / kKT;
  const int nfull = CAUSAL ? min(N / kKT, q0 / kKT) : N / kKT;

  uint4 sk[kRows], svv[kRows];
#define DQ_LOAD(T_)                                                                      \
  {                                                                                      \
    const int k0_ = (T_) * kKT;                                                          \
    _Pragma("unroll") for (int i = 0; i < kRows; ++i) {                                  \
      sk[i] = bload(rk, gk[i] + k0_ * skn * 2);                                          \
      svv[i] = bload(rv, gv[i] + k0_ * svn * 2);                                         \
    }                                                                                    \
  }
#define DQ_STORE(SLOT_)                                                                  \
  {                                                                                      \
    bf16* img = (bf16*)(smem + (SLOT_) * kBufK);                                         \
    _Pragma("unroll") for (int i = 0; i < kRows; ++i) {                                  \
      *(uint4*)(img + srow[i]) = sk[i];                                                  \
      *(uint4*)(img + kImgK + stri[i]) = sk[i];                                          \
      *(uint4*)(img + 2 * kImgK + srow[i]) = svv[i];                                     \
    }                                                                                    \
  }

  f32x16 dQ[2] = {f32x16{}, f32x16{}};
  f32x16 dinit;
#pragma unroll
  for (int r = 0; r < 16; ++r) dinit[r] = -del;  // = −δ
  const float c2 = p.scale_log2;
  DQ_LOAD(0)
  DQ_STORE(0)
  __syncthreads();
#define DQ_STEP(MASK_, SLOT_, T_)                                                        \
  {                                                                                      \
    const int t_ = (T_);                                                                 \
    const bool more_ = t_ + 1 < ntile;                                                   \
    if (more_) DQ_LOAD(t_ + 1)                                                           \
    if (!(MASK_) || !CAUSAL || t_ * kKT <= wq_hi)                                        \
      dq_tile<CAUSAL, MASK_>(smem + (SLOT_) * kBufK, c, dQ, c2, nlq, dinit, t_ * kKT, N, \
                             my_q, hf, PF);                                              \
    if (more_) DQ_STORE((SLOT_) ^ 1)                                                     \
    __syncthreads();                                                                     \
  }
  int t = 0;
  for (; t + 1 < nfull; t += 2) {
    DQ_STEP(false, 0, t)
    DQ_STEP(false, 1, t + 1)
  }
  if (t < nfull) {
    DQ_STEP(false, 0, t)
    ++t;
  }
  for (; t < ntile; ++t) {
    if (t & 1) DQ_STEP(true, 1, t) else DQ_STEP(true, 0, t)
  }
#undef DQ_STEP
#undef DQ_LOAD
#undef DQ_STORE

  if (my_q < N) {
    bf16* dQg = (bf16*)p.dq + b * p.sdq[0] + hh * p.sdq[1] + (int64_t)my_q * p.sdq[2];
    const float sc = p.scale;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(dQg + db * 32 + 8 * g + 4 * hf, dQ[db][4 * g] * sc, dQ[db][4 * g + 1] * sc,
               dQ[db][4 * g + 2] * sc, dQ[db][4 * g + 3] * sc, true);
  }
  }  // pass
}

// ---------------------------------------------------------------------------------------
hipError_t launch_bwd_fused(const AttnArgs& a, bool causal, void* ws, hipStream_t st);

template <bool CAUSAL>
static hipError_t launch_bwd_bf16_t(const AttnArgs& a, int variant, hipStream_t st) {
  // (variant is adjusted below for shapes a form does not take)
  // 20: dQ folded into the dK/dV pass (fa_bwd_fused.hip: 5 products instead of 7); its
  // workspace (a.slab) starts with the arrival counters, which the prep kernel zeroes
  AttnArgs ap = a;
  ap.dq_cnt = variant == 20 ? (unsigned*)a.slab : nullptr;
  hipLaunchKernelGGL(fa_bwd_prep_bf16<64>, dim3((unsigned)((a.N + 32 * kPrepRows - 1) / (32 * kPrepRows)), (unsigned)(a.B * a.H)),
                     dim3(256), 0, st, ap);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (variant == 20) return launch_bwd_fused(a, CAUSAL, a.slab, st);
#ifndef MT_DIAGNOSTICS
  // product build: the split defaults 5 (non-causal), 18 / 0 (causal paired / not); the
  // other forms are A/B policies of the diagnostics build
  if (variant != 0 && variant != 5 && variant != 18) variant = CAUSAL ? 0 : 5;
#endif
  // variant -> (dK/dV form, dQ form). dK/dV: 0 32-query steps (128 keys), 1 software-
  // pipelined, 3 / 4 64-query steps (one wave per SIMD / LDS-DMA), 5 the 8-wave LDS-DMA form
  // (256 keys), 11 staggered SIMD partners. dQ: 4 (128 queries) or 8 waves (256), 8 with the
  // Kᵀ reads ahead (12). (Round 2's one-wave 64-key dK/dV (13, fa_bwd_w64.hip) and in-wave
  // pipelined dQ (14, fa_bwd_dq_pipe.hip) lost their A/Bs and were removed in round 5:
  // profiles/r2_ab_bwd_w64.txt)
  int dkv = variant, dq = variant >= 5 ? 8 : 4;
  if (variant == 12) dkv = 5;
  if (variant == 15) { dkv = 0; dq = 8; }   // causal A/B: 128-key dK/dV, 8-wave dQ
  if (variant == 16) { dkv = 4; dq = 8; }   // causal A/B: 4-wave LDS-DMA dK/dV, 8-wave dQ
  if (variant == 17) { dkv = 17; dq = 8; }  // 8-wave dK/dV with 128-query steps
  // causal: 18 = 0 with paired light/heavy blocks in both kernels, 19 = 18 with the 8-wave dQ
  const bool pair = CAUSAL && (variant == 18 || variant == 19);
  if (variant == 18) { dkv = 0; dq = 4; }
  if (variant == 19) { dkv = 0; dq = 8; }
  if (variant == 12) dq = 12;
  if (dkv == 11 && (CAUSAL || a.N % 64 != 0)) dkv = 5;  // staggered form: mask-free shapes
  {
    const int kkb = dkv >= 5 ? 256 : 128;  // keys per workgroup
    const int nthr = kkb * 2;
    const int nkb = (a.N + kkb - 1) / kkb;
    const int64_t nblk = (int64_t)(pair ? (nkb + 1) / 2 : nkb) * a.B * a.H;
    if (nblk > 0x7fffffff) return hipErrorInvalidValue;
    const size_t smem = (dkv == 11 || dkv == 17 ? 8 : dkv == 1 ? 3 : dkv >= 2 ? 4 : 2) * (size_t)kBufQ;
#ifndef MT_DIAGNOSTICS
    auto kfn = dkv == 5 ? fa_bwd_dkv_bf16_q64<CAUSAL, 2, true, 8>
               : pair   ? fa_bwd_dkv_bf16<CAUSAL, true>
                        : fa_bwd_dkv_bf16<CAUSAL>;
#else
    auto kfn = dkv == 1   ? fa_bwd_dkv_bf16_p<CAUSAL>
               : dkv == 3 ? fa_bwd_dkv_bf16_q64<CAUSAL, 1>
               : dkv == 4 ? fa_bwd_dkv_bf16_q64<CAUSAL, 2, true>
               : dkv == 5 ? fa_bwd_dkv_bf16_q64<CAUSAL, 2, true, 8>
               : dkv == 11 ? fa_bwd_dkv_bf16_st
               : dkv == 17 ? fa_bwd_dkv_bf16_q64<CAUSAL, 2, true, 8, 0, 4>
               : dkv == 6 ? fa_bwd_dkv_bf16_q64<CAUSAL, 2, true, 8, 1>
               : dkv == 7 ? fa_bwd_dkv_bf16_q64<CAUSAL, 2, true, 8, 2>
               : dkv == 8 ? fa_bwd_dkv_bf16_q64<CAUSAL, 2, true, 8, 6>
               : dkv == 9 ? fa_bwd_dkv_bf16_q64<CAUSAL, 2, true, 8, 7>
                          : pair ? fa_bwd_dkv_bf16<CAUSAL, true> : fa_bwd_dkv_bf16<CAUSAL>;
#endif
    {
      e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(kfn, dim3((unsigned)nblk), dim3(nthr), smem, st, a, nkb);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  {
    const int kqb = dq == 4 ? 128 : 256;  // queries per workgroup
    const int nqb = (a.N + kqb - 1) / kqb;
    const int64_t nblk = (int64_t)(pair ? (nqb + 1) / 2 : nqb) * a.B * a.H;
    const size_t smem = 2 * (size_t)kBufK;
#ifndef MT_DIAGNOSTICS
    auto kfn = pair ? fa_bwd_dq_bf16<CAUSAL, 4, false, true>
               : dq == 8 ? fa_bwd_dq_bf16<CAUSAL, 8> : fa_bwd_dq_bf16<CAUSAL>;
#else
    auto kfn = dq == 12 ? fa_bwd_dq_bf16<CAUSAL, 8, true>
               : pair ? (dq == 8 ? fa_bwd_dq_bf16<CAUSAL, 8, false, true> : fa_bwd_dq_bf16<CAUSAL, 4, false, true>)
               : dq == 8 ? fa_bwd_dq_bf16<CAUSAL, 8> : fa_bwd_dq_bf16<CAUSAL>;
#endif
    e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kfn, dim3((unsigned)nblk), dim3(kqb * 2), smem, st, a, nqb);
    return hipGetLastError();
  }
}

hipError_t launch_bwd_d128_passes(const AttnArgs& a, bool causal, hipStream_t st);

// the d = 128 prep as its own launch (the passes' forms that do not form the row constants)
hipError_t launch_prep_d128(const AttnArgs& a, hipStream_t st) {
  constexpr int rpp = 256 / 16;
  hipLaunchKernelGGL(fa_bwd_prep_bf16<128>, dim3((unsigned)((a.N + rpp * kPrepRows - 1) / (rpp * kPrepRows)), (unsigned)(a.B * a.H)),
                     dim3(256), 0, st, a);
  return hipGetLastError();
}

// bf16, d = 64 / 128, every per-head row offset of Q/K/V/dO (plus one tile past N) inside the
// 31-bit buffer range; otherwise the caller falls back to the generic kernels. d = 128: the
// split form on the 16x16x32 MFMA (fa_bwd_d128.hip; no key padding).
hipError_t launch_bwd_bf16(const AttnArgs& a, bool causal, int variant, hipStream_t st, bool* handled) {
  *handled = false;
  if (a.d == 128 && !a.kv_len) {
    const int64_t lim = (int64_t)1 << 31;
    for (const int64_t s : {a.sq[2], a.sk[2], a.sv[2], a.sdo[2]})
      if (((int64_t)a.N + 64) * s * 2 >= lim) return hipSuccess;
    if ((int64_t)a.B * a.H > 65535 || (int64_t)a.B * a.H * a.N * 4 >= lim) return hipSuccess;
    *handled = true;
    return launch_bwd_d128_passes(a, causal, st);
  }
  if (a.d != 64) return hipSuccess;
  const int64_t lim = (int64_t)1 << 31;
  for (const int64_t s : {a.sq[2], a.sk[2], a.sv[2], a.sdo[2]})
    if (((int64_t)a.N + 64) * s * 2 >= lim) return hipSuccess;
  if ((int64_t)a.B * a.H > 65535) return hipSuccess;  // the prep kernel's grid.y
  *handled = true;
  return causal ? launch_bwd_bf16_t<true>(a, variant, st) : launch_bwd_bf16_t<false>(a, variant, st);
}

}  // namespace mt
