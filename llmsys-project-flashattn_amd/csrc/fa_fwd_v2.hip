// FlashAttention forward, bf16 MFMA kernel v2 (head dims 64 and 128).
//
// Same contract and data flow as fa_fwd_bf16_fast (fa_fwd_fast.hip): Sᵀ = K·Qᵀ with the
// query on the lane, in-register online softmax, Oᵀ = Vᵀ·Pᵀ, register-staged K/V tiles
// double-buffered in XOR-swizzled LDS, one barrier per tile. What v2 changes is the
// per-tile instruction stream, which at d = 64 is VALU-issue bound (the two MFMA
// products of a 64-key tile are only 16 x 32 cycles per wave):
//  * masked tiles are peeled: the ragged last tile and the causal diagonal tiles run a
//    separate instantiation of the tile body; the bulk of the loop carries no compare /
//    select code at all;
//  * the loop is unrolled by the LDS double-buffer parity, and every LDS operand address
//    is a per-lane base computed once plus a compile-time immediate;
//  * K/V staging uses buffer loads (32-bit per-lane offset, hardware range check: keys
//    past N read as zero, no clamping);
//  * the O rescale of the deferred-max softmax can sit behind a wave-uniform branch
//    (RESC 0) and run only when some row's max grows by more than kThr log2 units;
//  * the scale-and-shift stays in scalar v_fma_f32 (the TU is built with
//    -fno-slp-vectorize: packed f32 ops beside MFMAs cost more than two scalar ones).
#include "fa_fwd_bf16.h"

namespace mt {

namespace {

using namespace fwdbf16;
constexpr int kBK = 64;
constexpr float kThr = 8.0f;       // log2 units: deferred-rescale threshold

struct Stage2 {
  uint4 k[4], v[4];
};

template <int D, int NW>
struct V2 {
  static constexpr int kThreads = 64 * NW;
  static constexpr int kBQ = 32 * NW;
  static constexpr int CPR = D / 8;
  static constexpr int LPT = kBK * CPR / kThreads;  // 16-B chunks per thread per tile
  static constexpr int RSTEP = kThreads / CPR;
  static constexpr int KSTEPS = D / 16;
  static constexpr int DB = D / 32;
  static constexpr int TILE = kBK * D;  // elements per K (or V) tile
};

// One K/V tile of the forward for one wave. MASK: apply key < N and causal masks.
// RESC selects how the deferred-max rescale of O / L is expressed: 0 = behind a
// wave-uniform branch (runs only when some row's max grew by more than kThr log2 units),
// 1 = an unconditional multiply by alpha (alpha = 1 unless a row grew).
template <int D, int NW, bool CAUSAL, bool MASK, int RESC, int BUF>
__device__ __forceinline__ void v2_tile(const bf16* __restrict__ smem, const int (&koff)[D / 16],
                                        const int (&voff)[D / 32], const bf16x8 (&qf)[D / 16],
                                        f32x16 (&O)[D / 32], f32x16& L, float& m_run, float c2,
                                        int k0, int N, int my_q, int hf, const bf16x8& ones) {
  using C = V2<D, NW>;
  const bf16* sk = smem + BUF * C::TILE;
  const bf16* sv = smem + 2 * C::TILE + BUF * C::TILE;
  f32x16 S[2];
#pragma unroll
  for (int ks = 0; ks < C::KSTEPS; ++ks)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const bf16x8 a = *(const bf16x8*)(sk + kb * 32 * D + koff[ks]);
      S[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], ks ? S[kb] : f32x16{}, 0, 0, 0);
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
  const float tmax = row_max32(S[0], S[1]);
  const bool grow = (tmax - m_run) * c2 > kThr;
  if (RESC == 0) {
    if (__builtin_amdgcn_ballot_w64(grow)) {
      const float m_new = fmaxf(m_run, tmax);
      const float alpha = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m_run - m_new) * c2);
      m_run = m_new;
#pragma unroll
      for (int i = 0; i < C::DB; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) O[i][r] *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) L[r] *= alpha;
    }
  } else {
    float alpha = 1.f;
    if (__builtin_amdgcn_ballot_w64(grow)) {
      const float m_new = fmaxf(m_run, tmax);
      alpha = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m_run - m_new) * c2);
      m_run = m_new;
    }
#pragma unroll
    for (int i = 0; i < C::DB; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) O[i][r] *= alpha;
#pragma unroll
    for (int r = 0; r < 16; ++r) L[r] *= alpha;
  }
  const float nmc = -(m_run * c2);
  bf16x8 pf[4];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        pf[2 * kb + s][j] = (bf16)__builtin_amdgcn_exp2f(__builtin_fmaf(S[kb][8 * s + j], c2, nmc));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef __attribute__((ext_vector_type(8))) short s16x8;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int db = 0; db < C::DB; ++db) {
        const bf16* a1 = sv + (kb * 32 + 16 * s) * D + voff[db];
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1 + 8 * D));
        const s16x8 av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        O[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av),
                                                        pf[2 * kb + s], O[db], 0, 0, 0);
      }
      L = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[2 * kb + s], L, 0, 0, 0);
    }
}

template <int D, int NW>
__device__ __forceinline__ void v2_load(Stage2& st, __amdgpu_buffer_rsrc_t rk, __amdgpu_buffer_rsrc_t rv,
                                        const int (&kgo)[4], const int (&vgo)[4], int kstep_k,
                                        int kstep_v) {
#pragma unroll
  for (int i = 0; i < V2<D, NW>::LPT; ++i) {
    st.k[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rk, kgo[i] + kstep_k, 0, 0));
    st.v[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rv, vgo[i] + kstep_v, 0, 0));
  }
}

template <int D, int NW, int BUF>
__device__ __forceinline__ void v2_store(bf16* smem, const Stage2& st, const int (&kso)[4],
                                         const int (&vso)[4]) {
  using C = V2<D, NW>;
#pragma unroll
  for (int i = 0; i < C::LPT; ++i) {
    *(uint4*)(smem + BUF * C::TILE + kso[i]) = st.k[i];
    *(uint4*)(smem + 2 * C::TILE + BUF * C::TILE + vso[i]) = st.v[i];
  }
}

}  // namespace

template <int D, bool CAUSAL, int NW, int RESC>
__global__ __launch_bounds__(64 * NW, 2) void fa_fwd_bf16_v2(AttnArgs p, int nqb) {
  using C = V2<D, NW>;
  static_assert(C::LPT >= 1 && C::LPT <= 4, "staging layout");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* smem = (bf16*)smem_raw;  // K[2][TILE], V[2][TILE]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int N = p.N;

  // XCD-aware bijective block remap (see fa_fwd_fast.hip).
  const int nblk = gridDim.x;
  const int hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3;
  const int qd = nblk >> 3, rm = nblk & 7;
  const int logical = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + slot;
  const int bh = logical / nqb;
  int qb = logical % nqb;
  if (CAUSAL) qb = nqb - 1 - qb;  // heaviest first
  const int b = bh / p.H, hh = bh % p.H;
  const int q0 = qb * C::kBQ;

  const bf16* Qg = (const bf16*)p.q + b * p.sq[0] + hh * p.sq[1];
  const bf16* Kg = (const bf16*)p.k + b * p.sk[0] + hh * p.sk[1];
  const bf16* Vg = (const bf16*)p.v + b * p.sv[0] + hh * p.sv[1];
  const int skn = (int)p.sk[2], svn = (int)p.sv[2];
  // Buffer descriptors over this head's K / V rows (keys >= N read back as zero).
  const __amdgpu_buffer_rsrc_t rk =
      __builtin_amdgcn_make_buffer_rsrc((void*)Kg, (short)0, ((N - 1) * skn + D) * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv =
      __builtin_amdgcn_make_buffer_rsrc((void*)Vg, (short)0, ((N - 1) * svn + D) * 2, 0x00020000);

  const int my_q = q0 + wave * 32 + c32;
  const int wq_hi = q0 + wave * 32 + 31;

  bf16x8 qf[C::KSTEPS];
  {
    const int qr = min(my_q, N - 1);
    const bf16* qrow = Qg + (int64_t)qr * p.sq[2];
#pragma unroll
    for (int ks = 0; ks < C::KSTEPS; ++ks) qf[ks] = *(const bf16x8*)(qrow + ks * 16 + 8 * hf);
  }

  // Per-lane LDS operand offsets (elements, without tile buffer / kb / s terms).
  int koff[C::KSTEPS], voff[C::DB];
#pragma unroll
  for (int ks = 0; ks < C::KSTEPS; ++ks) koff[ks] = k_swz<D>(c32, 2 * ks + hf);
  {
    const int i16 = lane & 15, g = (lane >> 4) & 1;
#pragma unroll
    for (int db = 0; db < C::DB; ++db) {
      const int col = db * 32 + 16 * g + 4 * (i16 & 3);
      voff[db] = v_swz<D>(4 * hf + (i16 >> 2), col >> 3) + (col & 7);
    }
  }
  // Staging: this thread's chunk(s) of a tile.
  const int st_r = tid / C::CPR, st_c = tid % C::CPR;
  int kgo[4], vgo[4], kso[4], vso[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = st_r + i * C::RSTEP;
    kgo[i] = (r * skn + st_c * 8) * 2;
    vgo[i] = (r * svn + st_c * 8) * 2;
    kso[i] = k_swz<D>(r, st_c);
    vso[i] = v_swz<D>(r, st_c);
  }
  const int ktile_b = kBK * skn * 2, vtile_b = kBK * svn * 2;

  f32x16 O[C::DB];
#pragma unroll
  for (int i = 0; i < C::DB; ++i) O[i] = f32x16{};
  f32x16 L = f32x16{};
  float m_run = -INFINITY;
  const float c2 = p.scale_log2;
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;

  const int kend = CAUSAL ? min(N, q0 + C::kBQ) : N;
  const int ntiles = (kend + kBK - 1) / kBK;
  // tiles [0, nfull) need no mask for any query of the workgroup
  const int nfull = CAUSAL ? min(N / kBK, q0 / kBK) : N / kBK;

  Stage2 st;
  v2_load<D, NW>(st, rk, rv, kgo, vgo, 0, 0);
  v2_store<D, NW, 0>(smem, st, kso, vso);
  __syncthreads();

  // Step t: stage tile t+1 (global -> registers), compute tile t, write the staged tile
  // to the other LDS buffer, one barrier. Unrolled by the buffer parity so every LDS
  // address is a per-lane base plus an immediate.
#define V2_STEP(MASK_, BUF_, T_)                                                              \
  {                                                                                           \
    const int t_ = (T_);                                                                      \
    const bool more_ = t_ + 1 < ntiles;                                                       \
    if (more_) v2_load<D, NW>(st, rk, rv, kgo, vgo, (t_ + 1) * ktile_b, (t_ + 1) * vtile_b);  \
    if (!(MASK_) || !CAUSAL || t_ * kBK <= wq_hi)                                             \
      v2_tile<D, NW, CAUSAL, MASK_, RESC, BUF_>(smem, koff, voff, qf, O, L, m_run, c2,        \
                                                t_ * kBK, N, my_q, hf, ones);                 \
    if (more_) v2_store<D, NW, (BUF_) ^ 1>(smem, st, kso, vso);                               \
    __syncthreads();                                                                          \
  }

  int t = 0;
  for (; t + 1 < nfull; t += 2) {
    V2_STEP(false, 0, t)
    V2_STEP(false, 1, t + 1)
  }
  if (t < nfull) {
    V2_STEP(false, 0, t)
    ++t;
  }
  for (; t < ntiles; ++t) {
    if (t & 1) V2_STEP(true, 1, t) else V2_STEP(true, 0, t)
  }
#undef V2_STEP

  const float l_tot = L[0];
  const float inv_l = 1.f / l_tot;
  if (my_q < N) {
    bf16* Og = (bf16*)p.out + b * p.so[0] + hh * p.so[1] + (int64_t)my_q * p.so[2];
#pragma unroll
    for (int db = 0; db < C::DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(Og + db * 32 + 8 * g + 4 * hf, O[db][4 * g] * inv_l, O[db][4 * g + 1] * inv_l,
               O[db][4 * g + 2] * inv_l, O[db][4 * g + 3] * inv_l, true);
    if (hf == 0) {
      const int64_t row = (int64_t)bh * N + my_q;
      if (p.m) p.m[row] = m_run * p.scale;
      if (p.l) p.l[row] = l_tot;
    }
  }
}

template <int D, bool CAUSAL, int NW, int RESC>
static hipError_t launch_v2_t(const AttnArgs& a, hipStream_t st) {
  const size_t smem = 4 * (size_t)kBK * D * sizeof(bf16);
  auto kfn = fa_fwd_bf16_v2<D, CAUSAL, NW, RESC>;
  hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)smem);
  if (e != hipSuccess) return e;
  const int nqb = (a.N + 32 * NW - 1) / (32 * NW);
  const int64_t nblk = (int64_t)nqb * a.B * a.H;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kfn, dim3((unsigned)nblk), dim3(64 * NW), smem, st, a, nqb);
  return hipGetLastError();
}

// v2 applies when d is 64 or 128 and every per-head K/V byte offset (including the
// up-to-63 keys read past N by the last tile) fits the 31-bit buffer offset.
hipError_t launch_fwd_v2(const AttnArgs& a, bool causal, int nw, int resc, hipStream_t st,
                         bool* handled) {
  *handled = false;
  const int d = a.d;
  if (d != 64) return hipSuccess;  // d = 128 needs > 256 registers in this form: fast kernel
  const int64_t lim = (int64_t)1 << 31;
  if (((int64_t)a.N + kBK) * a.sk[2] * 2 >= lim || ((int64_t)a.N + kBK) * a.sv[2] * 2 >= lim)
    return hipSuccess;
  *handled = true;
#define V2_DISPATCH(NW_, R_) \
  return causal ? launch_v2_t<64, true, NW_, R_>(a, st) : launch_v2_t<64, false, NW_, R_>(a, st);
  if (nw == 8) V2_DISPATCH(8, 0)
  if (resc == 1) V2_DISPATCH(4, 1)
  V2_DISPATCH(4, 0)
#undef V2_DISPATCH
}

}  // namespace mt
