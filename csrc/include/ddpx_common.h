// ddpx — MI355X (gfx950 / CDNA4) native kernels: shared device helpers.
//
// Everything here is written for CDNA4 directly: 64-lane wavefronts, MFMA
// fragments, LDS (160 KiB/CU), 8 XCDs with private L2s.  No CUDA shims.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define DDPX_API extern "C" __attribute__((visibility("default")))

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef short short8v __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define LDS_AS __attribute__((address_space(3)))

namespace ddpx {

constexpr int kWave = 64;
constexpr int kNumXcd = 8;

// bf16 <-> f32 (round-to-nearest-even; NaN kept NaN by the hardware cvt).
__device__ __forceinline__ float bf2f(unsigned short v) {
  return __uint_as_float(((unsigned)v) << 16);
}
__device__ __forceinline__ unsigned short f2bf(float f) {
  __bf16 b = (__bf16)f;  // hipcc emits v_cvt_pk_bf16_f32 on gfx950
  return __builtin_bit_cast(unsigned short, b);
}
__device__ __forceinline__ unsigned pack_bf2(float lo, float hi) {
  return (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
}

// Bijective XCD-aware remap of a 1-D workgroup id (cdna_hip_programming §5 T1):
// workgroups dealt round-robin over the 8 XCDs are renumbered so that each XCD
// receives one contiguous range of logical tiles (neighbouring tiles share
// operand panels through that XCD's L2).  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & (kNumXcd - 1);
  const int q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Fused SGD (torch.optim.SGD semantics, dampening 0, momentum buffer zero-initialised so the
// first step equals torch's clone(d)).  Used by epilogues that update parameters in place
// instead of materialising gradients (single-process training: optimizer fused into backward).
struct SgdArgs {
  float* p;               // fp32 master
  float* buf;             // momentum buffer (may be null when mom == 0)
  unsigned short* shadow; // bf16 compute copy (may be null)
  const float* lr;        // device scalar
  float mom, wd;
  // MX-FP8 (e4m3) copy of the updated weights, written next to the bf16 one by the optimizer streams
  // that support it (ddpx_mx.h): codes at the element offset, E8M0 scales at element offset / 32.
  unsigned char* q8 = nullptr;
  unsigned char* s8 = nullptr;
  // the transposed MX-FP8 copy W^T [N][M] with 32-blocks along M (the data gradient's B operand): codes at
  // n * M + m, scales at n * (M / 32) + m / 32 (ddpx_wgrad_sgd.h, 8 stream waves)
  unsigned char* q8t = nullptr;
  unsigned char* s8t = nullptr;
};

// sgd_apply with the parameter and momentum already loaded (pv, mv: prefetched by the caller well before the
// gradient is known, so the update costs no load round trip at the end of a reduction).  Same fma sequence.
__device__ __forceinline__ float sgd_apply_pre(const SgdArgs& s, size_t i, float g, float lr, float pv, float mv) {
  float d = fmaf(s.wd, pv, g);
  if (s.mom != 0.f) {
    d = fmaf(s.mom, mv, d);
    __builtin_nontemporal_store(d, s.buf + i);
  }
  const float p = fmaf(-lr, d, pv);
  __builtin_nontemporal_store(p, s.p + i);
  if (s.shadow) s.shadow[i] = f2bf(p);
  return p;
}

// Master and momentum are read-once / write-once streams: non-temporal, so the update leaves no
// dirty L2 / MALL lines for the next forward's GEMMs to write back (profiles/r1_sgdnt).
// Returns the updated parameter (for epilogues that also write it in a derived layout).
__device__ __forceinline__ float sgd_apply(const SgdArgs& s, size_t i, float g, float lr) {
  float p = __builtin_nontemporal_load(s.p + i);
  float d = fmaf(s.wd, p, g);
  if (s.mom != 0.f) {
    d = fmaf(s.mom, __builtin_nontemporal_load(s.buf + i), d);
    __builtin_nontemporal_store(d, s.buf + i);
  }
  p = fmaf(-lr, d, p);
  __builtin_nontemporal_store(p, s.p + i);
  if (s.shadow) s.shadow[i] = f2bf(p);
  return p;
}

}  // namespace ddpx
