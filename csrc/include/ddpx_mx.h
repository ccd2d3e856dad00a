// ddpx — OCP MX-FP8 helpers shared by the quantisers (gemm_mx8.hip) and the optimizer streams that emit the
// fp8 weight copy next to the bf16 one (ddpx_wgrad_sgd.h, optim_elementwise.hip).
//
// An MX block is 32 consecutive elements of a row sharing one E8M0 exponent e (value = code * 2^e):
// e = exponent of amax / maxv (frexp), clamped to [-127, 127]; codes are round-to-nearest-even fp8 of
// clamp(x * 2^-e, +-maxv).  The optimizer streams hold 4 consecutive elements per lane, so a block is
// 8 neighbouring lanes and its amax is three DPP steps (quad xor 1, quad xor 2, half-row mirror).
#pragma once

#include "ddpx_common.h"

namespace ddpx {
namespace mx {

constexpr float kMaxE4M3 = 448.f;
constexpr float kMaxE5M2 = 57344.f;

template <bool HI>
__device__ __forceinline__ unsigned cvt_pk(float a, float b, unsigned old, bool e5m2) {
  if (e5m2) return (unsigned)__builtin_amdgcn_cvt_pk_bf8_f32(a, b, (int)old, HI);
  return (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(a, b, (int)old, HI);
}

// E8M0 exponent e such that amax * 2^-e <= maxv (e = ceil-ish(log2(amax / maxv))), clamped.
__device__ __forceinline__ int block_exp(float amax, float maxv) {
  if (!(amax > 0.f)) return -127;
  int ex;
  (void)frexpf(amax / maxv, &ex);  // amax/maxv = m * 2^ex, m in [0.5, 1)
  return ex < -127 ? -127 : (ex > 127 ? 127 : ex);
}

// 4 values -> one dword of 4 fp8 codes (scale 2^-e already folded into inv).
__device__ __forceinline__ unsigned quant4(float x0, float x1, float x2, float x3, float inv, float maxv, bool e5m2) {
  const unsigned r = cvt_pk<false>(fminf(fmaxf(x0 * inv, -maxv), maxv), fminf(fmaxf(x1 * inv, -maxv), maxv), 0u, e5m2);
  return cvt_pk<true>(fminf(fmaxf(x2 * inv, -maxv), maxv), fminf(fmaxf(x3 * inv, -maxv), maxv), r, e5m2);
}

// Max over the 8 aligned lanes (l & ~7 .. l | 7) that hold one MX block.  Every lane of the wave must be
// active (DPP reads the neighbours' registers).
__device__ __forceinline__ float group8_max(float v) {
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false)));
  return v;
}

// The e4m3 MX code of this lane's 4 elements of an 8-lane block, from fp32 values rounded to bf16 first
// (the bf16 compute copy is what the separate quantiser reads, so both paths produce the same bytes).
// Returns the packed codes; *e_out = the block's E8M0 byte (same on all 8 lanes).
__device__ __forceinline__ unsigned e4m3_group8(f32x4 po, unsigned* e_out) {
  const float v0 = bf2f(f2bf(po[0])), v1 = bf2f(f2bf(po[1])), v2 = bf2f(f2bf(po[2])), v3 = bf2f(f2bf(po[3]));
  const float amax = group8_max(fmaxf(fmaxf(fabsf(v0), fabsf(v1)), fmaxf(fabsf(v2), fabsf(v3))));
  const int e = block_exp(amax, kMaxE4M3);
  *e_out = (unsigned)(e + 127);
  return quant4(v0, v1, v2, v3, ldexpf(1.f, -e), kMaxE4M3, false);
}

}  // namespace mx
}  // namespace ddpx
