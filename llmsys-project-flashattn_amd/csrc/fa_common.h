// Shared CDNA4 (gfx950) primitives for the FlashAttention kernels.
//
// Every attention product in this library is expressed on one MFMA shape, the
// 32x32 output tile with a 16-deep k step:
//   bf16 : one  v_mfma_f32_32x32x16_bf16
//   fp32 : eight v_mfma_f32_32x32x2_f32  (exact fp32 fma chain, no xf32 on gfx950)
// In both cases lane l (c = l&31, h = l>>5) supplies 8 elements of row c of A
// and column c of B, for the k indices {8h .. 8h+7} of the step ("Frag<T>"),
// and receives the C/D tile with column c on the lane and rows
//   row(r, h) = (r&3) + 8*(r>>2) + 4*h ,   r = 0..15            (f32x16 "Acc").
// An accumulator is reused as the B operand of the next product by taking
// registers 8s..8s+7 as k-step s; element j of lane half h then stands for
// k = 16s + 8(j>>2) + 4h + (j&3), so the A operand of that product must be
// gathered with the same k order (col_frag below).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mt {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) float f32x8;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __bf16 bf16;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

template <typename T> struct FragT;
template <> struct FragT<bf16> { typedef bf16x8 type; };
template <> struct FragT<float> { typedef f32x8 type; };
template <typename T> using Frag = typename FragT<T>::type;

__device__ __forceinline__ void mma(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
}
__device__ __forceinline__ void mma(f32x16& acc, const f32x8& a, const f32x8& b) {
#pragma unroll
  for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
}

__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// 8 contiguous elements of one LDS row (row fragment). p must be 16-B aligned.
__device__ __forceinline__ bf16x8 row_frag(const bf16* p, bf16x8*) { return *(const bf16x8*)p; }
__device__ __forceinline__ f32x8 row_frag(const float* p, f32x8*) {
  f32x8 r;
  float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w; r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
  return r;
}
template <typename T> __device__ __forceinline__ Frag<T> row_frag(const T* p) {
  return row_frag(p, (Frag<T>*)nullptr);
}

// Column ("transposed") fragment of an LDS tile with row stride ld (elements):
// element j = tile[(k0 + 8(j>>2) + (j&3)) * ld + col], where the caller passes
// k0 = base + 16s + 4h and col = cbase + (lane&31). bf16 uses the gfx950
// ds_read_b64_tr_b16 transpose read (two per fragment); EXEC must be full.
__device__ __forceinline__ bf16x8 col_frag(const bf16* tile, int ld, int k0, int cbase, int lane,
                                           bf16x8*) {
  const int i = lane & 15, g = (lane >> 4) & 1;
  const bf16* a = tile + (k0 + (i >> 2)) * ld + cbase + 16 * g + 4 * (i & 3);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 8 * ld));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}
__device__ __forceinline__ f32x8 col_frag(const float* tile, int ld, int k0, int cbase, int lane,
                                          f32x8*) {
  const float* a = tile + k0 * ld + cbase + (lane & 31);
  f32x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[(8 * (j >> 2) + (j & 3)) * ld];
  return r;
}
template <typename T>
__device__ __forceinline__ Frag<T> col_frag(const T* tile, int ld, int k0, int cbase, int lane) {
  return col_frag(tile, ld, k0, cbase, lane, (Frag<T>*)nullptr);
}

// Accumulator registers 8s..8s+7 as a B-operand fragment.
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s, bf16x8*) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)a[8 * s + j];
  return r;
}
__device__ __forceinline__ f32x8 acc_frag(const f32x16& a, int s, f32x8*) {
  f32x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[8 * s + j];
  return r;
}
template <typename T> __device__ __forceinline__ Frag<T> acc_frag(const f32x16& a, int s) {
  return acc_frag(a, s, (Frag<T>*)nullptr);
}

// ---- fp32 products on the bf16 MFMA ("x3": three bf16 pieces per fp32 value) --------------
// x = x1 + x2 + x3 exactly for normal fp32 x: x1 = x truncated to its top 16 bits (a bf16),
// r1 = x − x1 (exact, ≤ 16 significant bits), x2 = r1 truncated, r2 = r1 − x2 (exact, ≤ 8
// significant bits, so x3 = r2's top 16 bits is r2). A product a·b then takes the six bf16
// MFMA terms a1b1 + a1b2 + a2b1 + a1b3 + a3b1 + a2b2 (each bf16·bf16 product is exact in
// fp32); the three dropped terms are below 2^-23·|a·b| together, the order of one fp32
// rounding. Six bf16 MFMAs of a 32x32x16 step take 6 x 32 cycles against 8 x 64 for the
// eight v_mfma_f32_32x32x2_f32 of the same step: 2.67x the fp32 MFMA rate at fp32 accuracy.
struct X3Frag { bf16x8 h, m, l; };
__device__ __forceinline__ void x3_split2(float x, float y, unsigned& h, unsigned& m, unsigned& l) {
  const unsigned ux = __float_as_uint(x), uy = __float_as_uint(y);
  const float rx = x - __uint_as_float(ux & 0xffff0000u), ry = y - __uint_as_float(uy & 0xffff0000u);
  const unsigned vx = __float_as_uint(rx), vy = __float_as_uint(ry);
  const float sx = rx - __uint_as_float(vx & 0xffff0000u), sy = ry - __uint_as_float(vy & 0xffff0000u);
  // (y's top half << 16) | x's top half, one v_perm_b32 each
  h = __builtin_amdgcn_perm(uy, ux, 0x07060302u);
  m = __builtin_amdgcn_perm(vy, vx, 0x07060302u);
  l = __builtin_amdgcn_perm(__float_as_uint(sy), __float_as_uint(sx), 0x07060302u);
}
__device__ __forceinline__ X3Frag x3_split(const f32x8& a) {
  unsigned h[4], m[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) x3_split2(a[2 * i], a[2 * i + 1], h[i], m[i], l[i]);
  X3Frag r;
  r.h = __builtin_bit_cast(bf16x8, h);
  r.m = __builtin_bit_cast(bf16x8, m);
  r.l = __builtin_bit_cast(bf16x8, l);
  return r;
}
// acc += a·b over one 16-deep k step, fp32-accurate, on six bf16 32x32x16 MFMAs (largest
// terms last, so the small ones accumulate first)
__device__ __forceinline__ void mma_x3(f32x16& acc, const X3Frag& a, const X3Frag& b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, acc, 0, 0, 0);
}
// x3_tile_sum: the bf16 MFMA's accumulation rounds toward -inf and loses more than an fp32
// rounding when a small product meets a large running sum (measured, round 6: a dV row summed
// over 32 tiles in one register sum drifted by about -7e-8 of its mean magnitude and erred 4x
// the fp32-MFMA form on the MHA test's inputs; scripts/probe_x3_ring2.py). A kernel that
// accumulates X3 products across tiles therefore takes each tile's products in a fresh
// accumulator and adds it to the running sum with a VALU fp32 add (round to nearest).
// LDS tiles held as three bf16 planes `plane` elements apart (h, m, l): a 16-B chunk of four
// fp32 values goes in as 8 B per plane; fragments come out as row_frag / col_frag of each plane
__device__ __forceinline__ void x3_store4(bf16* dst, int plane, const uint4& v) {
  const float4 f = __builtin_bit_cast(float4, v);
  unsigned h0, m0, l0, h1, m1, l1;
  x3_split2(f.x, f.y, h0, m0, l0);
  x3_split2(f.z, f.w, h1, m1, l1);
  *(uint2*)(dst) = make_uint2(h0, h1);
  *(uint2*)(dst + plane) = make_uint2(m0, m1);
  *(uint2*)(dst + 2 * plane) = make_uint2(l0, l1);
}
__device__ __forceinline__ X3Frag x3_rows(const bf16* p, int plane) {
  X3Frag f;
  f.h = *(const bf16x8*)p;
  f.m = *(const bf16x8*)(p + plane);
  f.l = *(const bf16x8*)(p + 2 * plane);
  return f;
}
__device__ __forceinline__ X3Frag x3_cols(const bf16* tile, int plane, int ld, int k0, int cbase, int lane) {
  X3Frag f;
  f.h = col_frag(tile, ld, k0, cbase, lane, (bf16x8*)nullptr);
  f.m = col_frag(tile + plane, ld, k0, cbase, lane, (bf16x8*)nullptr);
  f.l = col_frag(tile + 2 * plane, ld, k0, cbase, lane, (bf16x8*)nullptr);
  return f;
}

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// Store 4 consecutive fp32 accumulator values (one row group) as T.
__device__ __forceinline__ void store4(float* p, float a, float b, float c, float d, bool vec) {
  if (vec) {
    *(float4*)p = make_float4(a, b, c, d);
  } else {
    p[0] = a; p[1] = b; p[2] = c; p[3] = d;
  }
}
__device__ __forceinline__ void store4(bf16* p, float a, float b, float c, float d, bool vec) {
  if (vec) {
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    bf16x4 v = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
    *(bf16x4*)p = v;
  } else {
    p[0] = (bf16)a; p[1] = (bf16)b; p[2] = (bf16)c; p[3] = (bf16)d;
  }
}

// Cooperative global -> LDS staging of a ROWS x COLS tile (COLS a multiple of
// 16 B worth of T). Row r of the tile is global row row0 + r (stride gstride
// elements), columns col0 .. col0+COLS-1; rows >= nrows or columns >= ncols are
// zero-filled. VEC: every 16-B chunk is either fully inside ncols and aligned
// (host-checked), so it is moved with one 16-B load.
template <typename T, int ROWS, int COLS, int NTHREADS, bool VEC>
__device__ __forceinline__ void stage_tile(T* lds, int ld, const T* g, int64_t gstride, int row0,
                                           int nrows, int col0, int ncols) {
  constexpr int EPC = 16 / sizeof(T);          // elements per 16-B chunk
  constexpr int CPR = COLS / EPC;              // chunks per row
  constexpr int NCH = ROWS * CPR;
  for (int c = threadIdx.x; c < NCH; c += NTHREADS) {
    const int r = c / CPR, cc = (c % CPR) * EPC;
    const int gr = row0 + r, gc = col0 + cc;
    T* dst = lds + r * ld + cc;
    if (VEC) {
      uint4 val = make_uint4(0, 0, 0, 0);
      if (gr < nrows && gc < ncols) val = *(const uint4*)(g + (int64_t)gr * gstride + gc);
      *(uint4*)dst = val;
    } else {
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        T val = from_f32<T>(0.f);
        if (gr < nrows && gc + e < ncols) val = g[(int64_t)gr * gstride + gc + e];
        dst[e] = val;
      }
    }
  }
}

// XCD-aware block order for (blocks per head, B·H) grids: the grid's (x, y) is flattened
// and dealt out so that the blocks of one (b,h) run on one XCD and share its L2 (the
// hardware hands consecutive workgroups to the 8 XCDs in turn).
__device__ __forceinline__ void xcd_order(int& blk, int& bh) {
  const int nx = gridDim.x, nblk = gridDim.x * gridDim.y;
  const int hw = blockIdx.y * nx + blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3, qd = nblk >> 3, rm = nblk & 7;
  const int logical = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + slot;
  blk = logical % nx;
  bh = logical / nx;
}

// xcd_order for causal grids that cannot pair blocks: when each XCD's chunk holds whole heads,
// it takes the heaviest block of each of its heads first, then the next heaviest, ... (a
// longest-first list schedule; "heavy" = the highest block index, as in a causal forward).
__device__ __forceinline__ void xcd_order_heavy_first(int& blk, int& bh) {
  const int nx = gridDim.x, nblk = gridDim.x * gridDim.y;
  const int hw = blockIdx.y * nx + blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3, qd = nblk >> 3, rm = nblk & 7;
  const int start = xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd;
  const int len = xcd < rm ? qd + 1 : qd;
  if (start % nx == 0 && len % nx == 0) {
    const int nh = len / nx;
    blk = nx - 1 - slot / nh;
    bh = start / nx + slot % nh;
  } else {
    blk = (start + slot) % nx;
    bh = (start + slot) / nx;
  }
}

// Parameters shared by the forward / backward launches (all strides in elements;
// the head dimension d is always unit-stride).
struct AttnArgs {
  const void* q; const void* k; const void* v; const void* o; const void* dout;
  void* out;   // O (fwd)
  void* dq; void* dk; void* dv;
  float* m; float* l;              // fwd outputs / bwd inputs, [B*H*N]
  float* lse2; float* delta;       // bwd workspace, [B*H*N]
  void* slab;                      // bwd workspace: dQ partials of the fused bf16 backward
  unsigned* dq_cnt;                // bwd workspace: its per-(head, query step) arrival counters
  const int* kv_len;               // [B] valid keys per batch row (keys >= kv_len masked), or null
  int o_f32;                       // bf16 forward: O is fp32 (MT_BF16_F32OUT), else O has the input type
  int knob;                        // A/B schedule knob (diagnostics build: env MT_KNOB; product: 0)
  unsigned long long* dbg;         // diagnostics build: in-kernel stamp sums (never an output)
  int64_t sq[3], sk[3], sv[3], so[3], sdo[3], sdq[3], sdk[3], sdv[3];  // (b, h, n)
  int B, H, N, d;
  float scale;       // 1/sqrt(d)
  float scale_log2;  // log2(e)/sqrt(d)
};

// Keys of batch row b that attend: all N, or the first kv_len[b] (clamped to [0, N]) when a
// key-padding length vector is given (mt_flash_attn_*_varlen).
__device__ __forceinline__ int kv_keys(const AttnArgs& p, int b) {
  return p.kv_len ? max(0, min(p.N, p.kv_len[b])) : p.N;
}

// Row q of O in the bf16 forward kernels: bf16, or fp32 when the caller asked for an fp32
// output (o_f32; the caller guarantees 16-B aligned rows and columns in multiples of 4).
struct ORow {
  void* p;
  int f32;
};
__device__ __forceinline__ ORow o_row(const AttnArgs& a, int b, int hh, int64_t q) {
  const int64_t e = b * a.so[0] + hh * a.so[1] + q * a.so[2];
  return ORow{a.o_f32 ? (void*)((float*)a.out + e) : (void*)((bf16*)a.out + e), a.o_f32};
}
__device__ __forceinline__ void store4(const ORow& o, int col, float x, float y, float z, float w) {
  if (o.f32) store4((float*)o.p + col, x, y, z, w, true);
  else store4((bf16*)o.p + col, x, y, z, w, true);
}

// A device buffer per (pool, device, stream), grown on demand and never freed while the process
// runs: an outgrown buffer is retired, because a captured hipGraph (minitorch/graphs.py) keeps
// the address it was captured with. Its users on one stream share it in that stream's order;
// two streams never share one. Returns nullptr when it would have to grow inside a stream
// capture (the caller then takes a path without it). Pools: kScratchReduce (column-reduction
// partials, split-K GEMM partials; combine.hip), kScratchPad (zero-padded head-dim copies;
// capi_flash.hip). Defined in combine.hip.
enum { kScratchReduce = 0, kScratchPad = 1 };
void* stream_scratch(int pool, size_t bytes, hipStream_t st);

}  // namespace mt
