// Helpers shared by the bf16 d = 64 backward kernels (fa_bwd_bf16.hip, fa_bwd_fused.hip):
// transpose fragments, XCD-aware block order, buffer resources and the LDS-DMA row copy.
#pragma once
#include "fa_fwd_bf16.h"

namespace mt {
namespace bwdbf16 {

using namespace fwdbf16;
constexpr int D = 64;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

// A operand Xᵀ (rows = d block db, k = rows row0..row0+15 of X in the 8(j>>2)+4h+(j&3)
// order of an accumulator reused as B) from a transpose-swizzled image of X [rows][64].
__device__ __forceinline__ bf16x8 tr_frag(const bf16* img, int row0, int voff) {
  const bf16* a1 = img + row0 * D + voff;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1 + 8 * D));
  const s16x8 av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, av);
}

__device__ __forceinline__ int tr_off(int lane, int db) {
  const int hf = lane >> 5, i16 = lane & 15, g = (lane >> 4) & 1;
  const int col = db * 32 + 16 * g + 4 * (i16 & 3);
  return v_swz<D>(4 * hf + (i16 >> 2), col >> 3) + (col & 7);
}

__device__ __forceinline__ bf16x8 to_bf16x8(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)a[8 * s + j];
  return r;
}

__device__ __forceinline__ int xcd_remap(int hw, int nblk) {
  const int xcd = hw & 7, slot = hw >> 3;
  const int qd = nblk >> 3, rm = nblk & 7;
  return (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + slot;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t head_rsrc(const bf16* base, int N, int stride) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, ((N - 1) * stride + D) * 2, 0x00020000);
}

__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// LDS-DMA: one wave instruction moves 64 x 16 B from per-lane buffer offsets (go) to 1 KiB
// of LDS at byte address lds (wave-uniform, an SGPR) in lane order (8 rows of a [rows][64]
// bf16 image); the image swizzle is applied on the per-lane source. Issued from inline asm
// so hipcc's waitcnt pass does not put a vmcnt(0) in front of the next LDS read (fa_fwd_v5.hip
// dma5, VAR bit 524288); the caller waits vmcnt(0) before the barrier that publishes the
// slot. M0 is saved/restored. The LDS address is a 32-bit scalar (the workgroup's LDS base
// read once, plus constants): a generic pointer here costs a 64-bit VGPR pair per
// destination, a readfirstlane pair and a null check per instruction, and spills.
__device__ __forceinline__ void dma_rows(uint32_t lds, __amdgpu_buffer_rsrc_t rs, int go) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(go), "s"(lds), "s"(rs)
      : "memory");
}

// The same for 64 x 4 B: lane l's dword lands at lds + 4 l (row constants).
__device__ __forceinline__ void dma_dwords(uint32_t lds, __amdgpu_buffer_rsrc_t rs, int go) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "buffer_load_dword %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(go), "s"(lds), "s"(rs)
      : "memory");
}

// The workgroup's dynamic-LDS base as a wave-uniform 32-bit byte address.
__device__ __forceinline__ uint32_t lds_base(const void* smem) {
  return __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem);
}

}  // namespace bwdbf16

}  // namespace mt
