// ddpx — inverted Dropout(p) forward on bf16 with a Philox4x32-10 counter-based generator.
//
// Reference layer: nn.Dropout(0.1) inside DeepNN's classifier (/root/reference/singlegpu.py:36;
// SURVEY §2.2 N18).  Semantics: training mode keeps each element with probability 1-p and scales
// kept elements by 1/(1-p); eval mode is the identity (the host skips the launch).
//
// MI355X design:
//   * the generator state (seed, offset) lives in DEVICE memory, so the launch is HIP-graph
//     capturable and every replay draws a fresh mask: the last workgroup to finish advances
//     `offset` (completion counter + fence), after every workgroup has read it;
//   * no mask is stored: the backward of Dropout∘ReLU is "h > 0" on the dropped output h
//     (kept AND positive), applied by the classifier head's backward kernel with dh_scale = 1/(1-p);
//   * one thread = 8 consecutive bf16 (one 16-B load/store) = two Philox blocks of 4 x u32.
#include "ddpx_common.h"

namespace ddpx {
namespace rng {

struct u32x4s { unsigned x, y, z, w; };

__device__ __forceinline__ u32x4s philox4x32_10(u32x4s c, unsigned k0, unsigned k1) {
  constexpr unsigned M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned lo0 = M0 * c.x, hi0 = __umulhi(M0, c.x);
    const unsigned lo1 = M1 * c.z, hi1 = __umulhi(M1, c.z);
    c = u32x4s{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

__device__ __forceinline__ float u01(unsigned r) { return (float)(r >> 8) * (1.0f / 16777216.0f); }

__global__ void __launch_bounds__(256)
dropout_fwd_kernel(const unsigned short* __restrict__ x, unsigned short* __restrict__ out, int64_t n8, float p,
                   float scale, int64_t* __restrict__ state, unsigned* __restrict__ done) {
  const uint64_t seed = (uint64_t)state[0];
  const uint64_t offset = (uint64_t)state[1];
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < n8) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(x + t * 8);
    const unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
    const u32x4s r0 = philox4x32_10(u32x4s{(unsigned)t, (unsigned)(t >> 32), (unsigned)offset, 0u}, k0, k1);
    const u32x4s r1 = philox4x32_10(u32x4s{(unsigned)t, (unsigned)(t >> 32), (unsigned)offset, 1u}, k0, k1);
    const unsigned rr[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = __uint_as_float(v[j] << 16), b = __uint_as_float(v[j] & 0xffff0000u);
      const float ka = u01(rr[2 * j]) >= p ? scale : 0.f;
      const float kb = u01(rr[2 * j + 1]) >= p ? scale : 0.f;
      o[j] = pack_bf2(a * ka, b * kb);
    }
    *reinterpret_cast<u32x4*>(out + t * 8) = o;
  }
  // last workgroup out advances the offset (every workgroup has read it before arriving here)
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned prev = atomicAdd(done, 1u);
    if (prev == gridDim.x - 1) {
      state[1] = (int64_t)(offset + 1);
      *done = 0u;
      __threadfence();
    }
  }
}

// fp32 variant (the reference's precision): one thread = 4 consecutive floats = one Philox block (counter word
// 3 = 2 keeps its stream apart from the bf16 kernel's two blocks per thread).
__global__ void __launch_bounds__(256)
dropout_fwd_f32_kernel(const float* __restrict__ x, float* __restrict__ out, int64_t n4, float p, float scale,
                       int64_t* __restrict__ state, unsigned* __restrict__ done) {
  const uint64_t seed = (uint64_t)state[0];
  const uint64_t offset = (uint64_t)state[1];
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < n4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + t * 4);
    const u32x4s r = philox4x32_10(u32x4s{(unsigned)t, (unsigned)(t >> 32), (unsigned)offset, 2u}, (unsigned)seed,
                                   (unsigned)(seed >> 32));
    const unsigned rr[4] = {r.x, r.y, r.z, r.w};
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = v[j] * (u01(rr[j]) >= p ? scale : 0.f);
    *reinterpret_cast<f32x4*>(out + t * 4) = o;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned prev = atomicAdd(done, 1u);
    if (prev == gridDim.x - 1) {
      state[1] = (int64_t)(offset + 1);
      *done = 0u;
      __threadfence();
    }
  }
}

}  // namespace rng
}  // namespace ddpx

using namespace ddpx;

// out = dropout(x) for n bf16 elements (n % 8 == 0, 16-B aligned).  state: int64 [seed, offset] on the
// device (offset advanced by one per launch); done: u32 scratch counter, zero before the first launch.
DDPX_API int ddpx_dropout_fwd(const void* x, void* out, int64_t n, float p, int64_t* state, unsigned* done,
                              hipStream_t s) {
  if (n % 8 || p < 0.f || p >= 1.f) return -1;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) & 15) return -3;
  const int64_t n8 = n / 8;
  const int64_t blocks = (n8 + 255) / 256;
  if (blocks < 1 || blocks > 0x7fffffff) return -4;
  hipLaunchKernelGGL(rng::dropout_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const unsigned short*)x,
                     (unsigned short*)out, n8, p, 1.f / (1.f - p), state, done);
  return (int)hipGetLastError();
}

// fp32 inverted dropout, n % 4 == 0 (same device-resident generator state protocol as ddpx_dropout_fwd).
DDPX_API int ddpx_dropout_fwd_f32(const void* x, void* out, int64_t n, float p, int64_t* state, unsigned* done,
                                  hipStream_t s) {
  if (n % 4 || p < 0.f || p >= 1.f) return -1;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) & 15) return -3;
  const int64_t n4 = n / 4;
  const int64_t blocks = (n4 + 255) / 256;
  if (blocks < 1 || blocks > 0x7fffffff) return -4;
  hipLaunchKernelGGL(rng::dropout_fwd_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const float*)x,
                     (float*)out, n4, p, 1.f / (1.f - p), state, done);
  return (int)hipGetLastError();
}
