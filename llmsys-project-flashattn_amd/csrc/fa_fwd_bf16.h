// Helpers shared by the bf16 MFMA kernels (fa_fwd_v4/v5/d128.hip, fa_bwd_bf16.hip):
// the XOR swizzles of the K / V LDS images and the wave's per-query row max.
#pragma once
#include "fa_common.h"

namespace mt {
namespace fwdbf16 {

// K image, read by ds_read_b128 (16 lanes = 16 different rows, same chunk):
//   D=64  (128-B rows, 2 per 256-B bank row): chunk c of row r at c ^ ((r >> 1) & 7)
//   D=128 (256-B rows):                        chunk c of row r at c ^ (r & 15)
// V image, read by ds_read_b64_tr_b16 (a half-wave reads 4 consecutive rows x 64 B):
//   D=64 : chunk c of row r at c ^ (((r >> 1) & 1) << 2)
//   D=128: chunk c of row r at c ^ ((r & 3) << 2)
// Both depend only on the low row bits a lane owns, so an operand address is a per-lane
// base plus a compile-time immediate for the 16-/32-row block offsets.
template <int D>
__device__ __forceinline__ int k_swz(int r, int c) {
  if (D == 64) return r * D + (c ^ ((r >> 1) & 7)) * 8;
  return r * D + (c ^ (r & 15)) * 8;
}
template <int D>
__device__ __forceinline__ int v_swz(int r, int c) {
  if (D == 64) return r * D + (c ^ (((r >> 1) & 1) << 2)) * 8;
  return r * D + (c ^ ((r & 3) << 2)) * 8;
}

// Max over a lane's 32 scores of a 64-key tile (both 32-key blocks), then across the two
// lane halves holding the same query.
__device__ __forceinline__ float row_max32(const f32x16& a, const f32x16& b) {
  float m0 = fmaxf(fmaxf(a[0], a[1]), a[2]);
  float m1 = fmaxf(fmaxf(b[0], b[1]), b[2]);
#pragma unroll
  for (int r = 3; r < 15; r += 2) {
    m0 = fmaxf(fmaxf(m0, a[r]), a[r + 1]);
    m1 = fmaxf(fmaxf(m1, b[r]), b[r + 1]);
  }
  float m = fmaxf(fmaxf(m0, m1), fmaxf(a[15], b[15]));
  auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
}


}  // namespace fwdbf16
}  // namespace mt
