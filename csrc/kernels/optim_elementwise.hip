// ddpx — memory-bound kernels: fused flat-buffer SGD, casts, column sums.
//
// All parameters of a model live in ONE flat fp32 buffer (ddpx.optim.flat),
// with a parallel momentum buffer, a parallel gradient buffer (the DDP bucket
// storage) and a parallel bf16 "compute shadow" that the MFMA GEMMs read.
// One SGD launch therefore replaces torch's foreach SGD (4 multi-tensor
// passes over 26 tensors, /root/reference/singlegpu.py:136-141 →
// torch/optim/sgd.py `_multi_tensor_sgd`): every element is read once and
// p, momentum and the bf16 shadow are written once.  16-B vector accesses,
// grid-stride, sized for 256 CUs.
#include "ddpx_common.h"
#include "ddpx_mx.h"

namespace ddpx {

static inline int grid_for(int64_t n_vec, int block = 256, int max_blocks = 256 * 8) {
  int64_t b = (n_vec + block - 1) / block;
  if (b > max_blocks) b = max_blocks;
  if (b < 1) b = 1;
  return (int)b;
}

// torch.optim.SGD semantics (dampening=0):
//   d = g*gscale + wd*p ; buf = first ? d : mom*buf + d ; d = nesterov ? d + mom*buf : buf
//   p -= lr * d
template <bool GBF16>
__global__ void __launch_bounds__(256)
sgd_flat_kernel(float* __restrict__ p, float* __restrict__ buf, const void* __restrict__ g,
                unsigned short* __restrict__ shadow, int64_t n, const float* __restrict__ lr_ptr,
                float lr_host, float mom, float wd, float gscale, int nesterov, int first,
                unsigned char* __restrict__ q8, unsigned char* __restrict__ s8) {
  const float lr = lr_ptr ? *lr_ptr : lr_host;
  const int64_t nv = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // read-once / write-once streams (master, momentum, gradient): non-temporal, so the optimizer does
  // not leave hundreds of MB of dirty lines in L2 / MALL for the next forward's GEMMs to write back
  auto load_g = [&](int64_t i) -> f32x4 {
    f32x4 gv;
    if constexpr (GBF16) {
      u32x2 raw = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(g) + i);
      gv[0] = __uint_as_float(raw[0] << 16);
      gv[1] = __uint_as_float(raw[0] & 0xffff0000u);
      gv[2] = __uint_as_float(raw[1] << 16);
      gv[3] = __uint_as_float(raw[1] & 0xffff0000u);
    } else {
      gv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g) + i);
    }
    return gv;
  };
  auto update = [&](int64_t i, f32x4 pv, f32x4 gv, f32x4 b) {
    // same fma sequence as sgd_apply() (fused-backward epilogues): bitwise-identical updates
    f32x4 po, bo;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float d = fmaf(wd, pv[q], gv[q] * gscale);
      if (mom != 0.f) {
        const float bb = first ? d : fmaf(mom, b[q], d);
        bo[q] = bb;
        d = nesterov ? fmaf(mom, bb, d) : bb;
      }
      po[q] = fmaf(-lr, d, pv[q]);
    }
    if (mom != 0.f) __builtin_nontemporal_store(bo, reinterpret_cast<f32x4*>(buf) + i);
    __builtin_nontemporal_store(po, reinterpret_cast<f32x4*>(p) + i);
    if (shadow) {
      u32x2 sh = {pack_bf2(po[0], po[1]), pack_bf2(po[2], po[3])};
      reinterpret_cast<u32x2*>(shadow)[i] = sh;
    }
    if (q8) {  // MX-FP8 copy: vectors 8k..8k+7 (8 neighbouring lanes, all active: n % 32 == 0) = block k
      unsigned e8;
      const unsigned q = mx::e4m3_group8(po, &e8);
      reinterpret_cast<unsigned*>(q8)[i] = q;
      if ((i & 7) == 0) s8[i >> 3] = (unsigned char)e8;
    }
  };
  // two vectors per thread per iteration, all six loads issued before either update: twice the
  // bytes in flight per wave of the one-vector loop
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += 2 * stride) {
    const int64_t j = i + stride;
    const bool two = j < nv;
    const f32x4 p0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p) + i);
    const f32x4 g0 = load_g(i);
    const f32x4 b0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(buf) + i);
    f32x4 p1 = p0, g1 = g0, b1 = b0;
    if (two) {
      p1 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p) + j);
      g1 = load_g(j);
      b1 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(buf) + j);
    }
    update(i, p0, g0, b0);
    if (two) update(j, p1, g1, b1);
  }
  // scalar tail (n not a multiple of 4)
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t j = (nv << 2) + threadIdx.x;
    float gv = GBF16 ? bf2f(reinterpret_cast<const unsigned short*>(g)[j])
                     : reinterpret_cast<const float*>(g)[j];
    float d = fmaf(wd, p[j], gv * gscale);
    if (mom != 0.f) {
      const float b = first ? d : fmaf(mom, buf[j], d);
      buf[j] = b;
      d = nesterov ? fmaf(mom, b, d) : b;
    }
    p[j] = fmaf(-lr, d, p[j]);
    if (shadow) shadow[j] = f2bf(p[j]);
  }
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, unsigned short* __restrict__ y,
                                     int64_t n) {
  const int64_t nv = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    u32x2 s = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
    reinterpret_cast<u32x2*>(y)[i] = s;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t j = (nv << 2) + threadIdx.x;
    y[j] = f2bf(x[j]);
  }
}

// out[n] (=|+=) scale * sum_m X[m][n] for a bf16 [M][N] matrix (bias gradient).
// One workgroup per 128 columns; each lane owns two adjacent columns (4-B
// loads, 256 B per wave-row); the 4 waves split the rows and meet in LDS.
__global__ void __launch_bounds__(256)
colsum_bf16_kernel(const unsigned short* __restrict__ X, float* __restrict__ out, int M, int N,
                   int ldx, float scale, int accumulate) {
  __shared__ float red[4][128];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x * 128 + lane * 2;
  float s0 = 0.f, s1 = 0.f;
  if (n + 1 < N) {
    for (int m = w; m < M; m += 4) {
      const unsigned v = *reinterpret_cast<const unsigned*>(X + (size_t)m * ldx + n);
      s0 += __uint_as_float(v << 16);
      s1 += __uint_as_float(v & 0xffff0000u);
    }
  } else if (n < N) {
    for (int m = w; m < M; m += 4) s0 += bf2f(X[(size_t)m * ldx + n]);
  }
  red[w][lane * 2] = s0;
  red[w][lane * 2 + 1] = s1;
  __syncthreads();
  if (threadIdx.x < 128) {
    const int c = blockIdx.x * 128 + threadIdx.x;
    if (c < N) {
      float t = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
      t *= scale;
      out[c] = accumulate ? out[c] + t : t;
    }
  }
}

// Elementwise scale (used for gradient averaging when the collective sums).
__global__ void scale_f32_kernel(float* __restrict__ x, int64_t n, float s) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] *= s;
}

}  // namespace ddpx

using namespace ddpx;

DDPX_API int ddpx_sgd_flat(float* p, float* buf, const void* g, int g_bf16, void* shadow, int64_t n,
                           const float* lr_dev, float lr_host, float momentum, float weight_decay,
                           float grad_scale, int nesterov, int first, void* q8, void* s8, hipStream_t s) {
  if (n <= 0) return 0;
  if (q8 && (n % 32 || !s8 || (reinterpret_cast<uintptr_t>(q8) & 3))) return -1;
  if ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(buf)) & 15) return -1;
  if (reinterpret_cast<uintptr_t>(g) & (g_bf16 ? 7 : 15)) return -1;
  if (reinterpret_cast<uintptr_t>(shadow) & 7) return -1;
  const int grid = grid_for((n >> 2) + 1);
  if (g_bf16)
    hipLaunchKernelGGL(sgd_flat_kernel<true>, dim3(grid), dim3(256), 0, s, p, buf, g,
                       (unsigned short*)shadow, n, lr_dev, lr_host, momentum, weight_decay, grad_scale,
                       nesterov, first, (unsigned char*)q8, (unsigned char*)s8);
  else
    hipLaunchKernelGGL(sgd_flat_kernel<false>, dim3(grid), dim3(256), 0, s, p, buf, g,
                       (unsigned short*)shadow, n, lr_dev, lr_host, momentum, weight_decay, grad_scale,
                       nesterov, first, (unsigned char*)q8, (unsigned char*)s8);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_cast_f32_bf16(const float* x, void* y, int64_t n, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for((n >> 2) + 1)), dim3(256), 0, s, x,
                     (unsigned short*)y, n);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_colsum_bf16(const void* X, float* out, int M, int N, int ldx, float scale,
                              int accumulate, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if ((ldx & 1) || (reinterpret_cast<uintptr_t>(X) & 3)) return -1;
  hipLaunchKernelGGL(colsum_bf16_kernel, dim3((N + 127) / 128), dim3(256), 0, s,
                     (const unsigned short*)X, out, M, N, ldx, scale, accumulate);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_scale_f32(float* x, int64_t n, float scale, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(scale_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, n, scale);
  return (int)hipGetLastError();
}

// Device-side LR schedule: lr = table[min(step, n-1)], step += 1 — one thread, captured inside the
// training-step HIP graph, so a replayed step needs no host write of the learning rate.
__global__ void lr_advance_kernel(const float* __restrict__ table, int n, int* __restrict__ counter,
                                  float* __restrict__ lr) {
  const int k = *counter;
  *lr = table[k < n ? k : n - 1];
  *counter = k + 1;
}

DDPX_API int ddpx_lr_advance(const float* table, int n, int* counter, float* lr, hipStream_t s) {
  if (n <= 0) return -1;
  hipLaunchKernelGGL(lr_advance_kernel, dim3(1), dim3(1), 0, s, table, n, counter, lr);
  return (int)hipGetLastError();
}

