// ddpx — GPU-resident data pipeline: gather + RandomCrop(32, padding=4) +
// RandomHorizontalFlip + ToTensor in one kernel.
//
// Replaces the reference's per-sample CPU PIL transforms and the blocking
// pinned H2D copy of every batch (/root/reference/singlegpu.py:155-159 train
// transform, :114-115 `source.to(gpu_id)`).  The uint8
// dataset ([N][3][32][32], 150 MiB for CIFAR-10 train) stays resident in HBM
// (and mostly in the 256 MiB Infinity Cache); each step gathers the sampler's
// indices, applies a per-sample crop offset and flip drawn from a counter-based
// hash, scales by 1/255 (no mean/std, as in the reference) and writes the batch
// in the layout the model consumes.
#include "ddpx_common.h"

namespace ddpx {

enum OutLayout : int { OUT_NCHW_F32 = 0, OUT_NCHW_BF16 = 1, OUT_NHWC_BF16 = 2, OUT_NHWC_F32 = 3, OUT_NHWC8_BF16 = 4,
                       OUT_NHWC4_F32 = 5 };

// x mod m for a small m (the crop range 2 * pad + 1) with 32-bit operations only: x = hi * 2^32 + lo, so
// x mod m = ((hi mod m) * (2^32 mod m) + lo mod m) mod m — exactly the 64-bit remainder the CPU twin takes.
__device__ __forceinline__ unsigned mod64(uint64_t x, int m) {
  const unsigned um = (unsigned)m;
  const unsigned p32 = (0xFFFFFFFFu % um + 1u) % um;
  const unsigned hi = (unsigned)(x >> 32) % um, lo = (unsigned)x % um;
  return (hi * p32 + lo) % um;  // < m * m + m: no overflow for the small m used here (m < 65536)
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// NCHW / flat layouts: one thread per (sample, channel, row, 8-pixel group);
// each thread gathers its 8 source bytes (L2/Infinity-Cache hits) and writes
// 8 contiguous outputs with one 16-B (bf16) or two 16-B (fp32) stores.
// NHWC layouts: one thread per (sample, row, pixel), C channels each.
// Per-sample crop offsets and flip, from the counter-based hash (the CPU twin draws the same).
__device__ __forceinline__ void sample_params(uint64_t seed, int b, int pad, int train, int& dy, int& dx, int& flip) {
  dy = pad;
  dx = pad;
  flip = 0;
  if (train) {
    const uint64_t r = splitmix64(seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(b + 1)));
    dy = (int)mod64(r, 2 * pad + 1);
    dx = (int)mod64(r >> 16, 2 * pad + 1);
    flip = (int)((r >> 40) & 1);
  }
}

// prm (optional, LDS): [dy, dx, flip] of samples b0, b0 + 1, ... drawn once per workgroup (the hash and its
// 64-bit remainders cost more VALU than the rest of a thread's work, and up to 384 threads share a sample)
__device__ __forceinline__ void augment_body(const uint8_t* __restrict__ images, const int64_t* __restrict__ labels,
                                             const int64_t* __restrict__ idx, int B, int C, int H, int W, int pad,
                                             uint64_t seed, int train, int layout, void* __restrict__ out,
                                             int64_t* __restrict__ tgt_out, const int* prm = nullptr, int b0 = 0) {
  const bool nhwc = (layout == OUT_NHWC_BF16 || layout == OUT_NHWC_F32 || layout == OUT_NHWC8_BF16 ||
                     layout == OUT_NHWC4_F32);
  const int G = W / 8;  // 8-pixel groups per row (W % 8 == 0 checked on the host)
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = nhwc ? B * H * W : B * C * H * G;
  if (t >= total) return;
  int b, c = 0, y, xg = 0, xo = 0;
  if (nhwc) {
    xo = t % W;
    y = (t / W) % H;
    b = t / (W * H);
  } else {
    xg = t % G;
    y = (t / G) % H;
    c = (t / (G * H)) % C;
    b = t / (G * H * C);
  }
  const int64_t src = idx ? idx[b] : b;
  int dy, dx, flip;
  if (prm) {
    dy = prm[(b - b0) * 3];
    dx = prm[(b - b0) * 3 + 1];
    flip = prm[(b - b0) * 3 + 2];
  } else {
    sample_params(seed, b, pad, train, dy, dx, flip);
  }
  if (tgt_out && y == 0 && c == 0 && xg == 0 && xo == 0) tgt_out[b] = labels[src];
  const int sy = y + dy - pad;
  const bool row_ok = (sy >= 0) && (sy < H);
  const float inv = 1.f / 255.f;
  const uint8_t* img = images + (size_t)src * C * H * W;
  if (!nhwc) {
    const uint8_t* row = img + (size_t)c * H * W + (size_t)(row_ok ? sy : 0) * W;
    float v[8];
    if (W == 32 && (((uintptr_t)row) & 15) == 0) {
      // CIFAR rows: the whole 32-B source row in two 16-B loads (2 address operations per lane instead of 8
      // byte loads), bytes picked in registers
      const u32x4 lo = *reinterpret_cast<const u32x4*>(row), hi = *reinterpret_cast<const u32x4*>(row + 16);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ox = xg * 8 + j;
        const int x = flip ? (W - 1 - ox) : ox;
        const int sx = x + dx - pad;
        const int d = (sx >> 2) & 7;
        const unsigned w = d < 4 ? (d < 2 ? (d == 0 ? lo[0] : lo[1]) : (d == 2 ? lo[2] : lo[3]))
                                 : (d < 6 ? (d == 4 ? hi[0] : hi[1]) : (d == 6 ? hi[2] : hi[3]));
        const unsigned byte = (w >> (8 * (sx & 3))) & 0xFFu;
        v[j] = (row_ok && sx >= 0 && sx < W) ? (float)byte * inv : 0.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ox = xg * 8 + j;                 // output column
        const int x = flip ? (W - 1 - ox) : ox;    // column of the cropped image
        const int sx = x + dx - pad;
        v[j] = (row_ok && sx >= 0 && sx < W) ? (float)row[sx] * inv : 0.f;
      }
    }
    const size_t o = (((size_t)b * C + c) * H + y) * W + xg * 8;
    if (layout == OUT_NCHW_BF16) {
      u32x4 pk = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7])};
      *reinterpret_cast<u32x4*>(reinterpret_cast<unsigned short*>(out) + o) = pk;
    } else {
      f32x4* d = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(out) + o);
      d[0] = (f32x4){v[0], v[1], v[2], v[3]};
      d[1] = (f32x4){v[4], v[5], v[6], v[7]};
    }
  } else {
    const int x = flip ? (W - 1 - xo) : xo;
    const int sx = x + dx - pad;
    const bool ok = row_ok && sx >= 0 && sx < W;
    if (layout == OUT_NHWC8_BF16) {
      // NHWC with the channels zero-padded to 8 (16-B pixels: the conv0 implicit-GEMM input)
      float v[8];
#pragma unroll
      for (int cc = 0; cc < 8; ++cc)
        v[cc] = (ok && cc < C) ? (float)img[(size_t)cc * H * W + sy * W + sx] * inv : 0.f;
      u32x4 pk = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7])};
      *reinterpret_cast<u32x4*>(reinterpret_cast<unsigned short*>(out) + (((size_t)b * H + y) * W + xo) * 8) = pk;
      return;
    }
    if (layout == OUT_NHWC4_F32) {
      // NHWC fp32 with the channels zero-padded to 4 (16-B pixels: the fp32 conv0 implicit-GEMM input)
      f32x4 v;
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) v[cc] = (ok && cc < C) ? (float)img[(size_t)cc * H * W + sy * W + sx] * inv : 0.f;
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(out) + (((size_t)b * H + y) * W + xo) * 4) = v;
      return;
    }
    const size_t o = (((size_t)b * H + y) * W + xo) * C;
    for (int cc = 0; cc < C; ++cc) {
      const float v = ok ? (float)img[(size_t)cc * H * W + sy * W + sx] * inv : 0.f;
      if (layout == OUT_NHWC_BF16) reinterpret_cast<unsigned short*>(out)[o + cc] = f2bf(v);
      else reinterpret_cast<float*>(out)[o + cc] = v;
    }
  }
}

// cursor (optional): device-side step counter k (read only).  The batch is rows [k % nbatch * B, +B) of
// the epoch's index permutation `idx` and the augmentation seed is seed + k (DeviceLoader.batch_seed(k)),
// so a captured training step draws a new batch on every replay with no host work.  The counter is
// advanced by its owner (the training step's LR-table kernel); advancing it here would need a
// completion counter every workgroup hits with an atomic — measured 26 vs 6.6 us for 768 workgroups.
__global__ void __launch_bounds__(256)
augment_kernel(const uint8_t* __restrict__ images, const int64_t* __restrict__ labels,
               const int64_t* __restrict__ idx, int B, int C, int H, int W, int pad, uint64_t seed,
               int train, int layout, void* __restrict__ out, int64_t* __restrict__ tgt_out,
               const int* __restrict__ cursor, int nbatch) {
  if (cursor) {
    const int k = *cursor;
    idx += (size_t)(k % nbatch) * B;
    seed += (uint64_t)k;
  }
  constexpr int kMaxSamples = 8;
  __shared__ int prm[kMaxSamples * 3];
  const bool nhwc = (layout == OUT_NHWC_BF16 || layout == OUT_NHWC_F32 || layout == OUT_NHWC8_BF16 ||
                     layout == OUT_NHWC4_F32);
  const int per = nhwc ? H * W : C * H * (W / 8);  // threads per sample
  const int total = B * per;
  const int t0 = blockIdx.x * blockDim.x;
  const int t1 = min(total, t0 + (int)blockDim.x) - 1;
  const int b0 = t0 / per, nb = t1 >= t0 ? t1 / per - b0 + 1 : 0;
  if (nb > kMaxSamples) {  // tiny images: every thread draws its own sample's parameters
    augment_body(images, labels, idx, B, C, H, W, pad, seed, train, layout, out, tgt_out);
    return;
  }
  if ((int)threadIdx.x < nb) {
    int dy, dx, flip;
    sample_params(seed, b0 + (int)threadIdx.x, pad, train, dy, dx, flip);
    prm[threadIdx.x * 3] = dy;
    prm[threadIdx.x * 3 + 1] = dx;
    prm[threadIdx.x * 3 + 2] = flip;
  }
  __syncthreads();
  augment_body(images, labels, idx, B, C, H, W, pad, seed, train, layout, out, tgt_out, prm, b0);
}

}  // namespace ddpx

using namespace ddpx;

DDPX_API int ddpx_augment(const void* images, const int64_t* labels, const int64_t* idx, int B, int C, int H,
                          int W, int pad, uint64_t seed, int train, int layout, void* out, int64_t* tgt_out,
                          hipStream_t s) {
  if (B <= 0) return 0;
  if (W % 8) return -1;
  if (pad < 0 || pad > 4096) return -4;  // mod64's 32-bit arithmetic assumes a small crop range
  const bool nhwc = (layout == OUT_NHWC_BF16 || layout == OUT_NHWC_F32 || layout == OUT_NHWC8_BF16 ||
                     layout == OUT_NHWC4_F32);
  if ((layout == OUT_NHWC8_BF16 && C > 8) || (layout == OUT_NHWC4_F32 && C > 4)) return -2;
  const int n = nhwc ? B * H * W : B * C * H * (W / 8);
  hipLaunchKernelGGL(augment_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const uint8_t*)images, labels,
                     idx, B, C, H, W, pad, seed, train, layout, out, tgt_out, (const int*)nullptr, 1);
  return (int)hipGetLastError();
}

// Batch k = *cursor of a device-resident epoch permutation (idx_all: nbatch x B indices), seed + k.
// The cursor is read, not advanced.  Graph-capturable.
DDPX_API int ddpx_augment_cursor(const void* images, const int64_t* labels, const int64_t* idx_all, int nbatch,
                                 int B, int C, int H, int W, int pad, uint64_t seed, int train, int layout, void* out,
                                 int64_t* tgt_out, const int* cursor, hipStream_t s) {
  if (B <= 0 || nbatch <= 0 || !cursor) return -3;
  if (W % 8) return -1;
  if (pad < 0 || pad > 4096) return -4;  // mod64's 32-bit arithmetic assumes a small crop range
  const bool nhwc = (layout == OUT_NHWC_BF16 || layout == OUT_NHWC_F32 || layout == OUT_NHWC8_BF16 ||
                     layout == OUT_NHWC4_F32);
  if ((layout == OUT_NHWC8_BF16 && C > 8) || (layout == OUT_NHWC4_F32 && C > 4)) return -2;
  const int n = nhwc ? B * H * W : B * C * H * (W / 8);
  hipLaunchKernelGGL(augment_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const uint8_t*)images, labels,
                     idx_all, B, C, H, W, pad, seed, train, layout, out, tgt_out, cursor, nbatch);
  return (int)hipGetLastError();
}
