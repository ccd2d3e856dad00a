// ddpx — BatchNorm2d (training/eval) + ReLU + MaxPool2d(2) on NHWC bf16, fused.
//
// Reference layers (/root/reference/singlegpu.py:64-70, per conv block):
//   nn.BatchNorm2d(x) -> nn.ReLU(True) [-> nn.MaxPool2d(2)]
// (SURVEY §2.2 N8/N9/N10).  Semantics kept exactly: batch statistics over
// N*H*W with the biased variance for normalisation, running_mean/var updated
// with momentum 0.1 using the UNBIASED variance, num_batches_tracked += 1,
// eps 1e-5, eval mode uses the running statistics; max-pool backward routes
// the gradient to the FIRST maximum of each 2x2 window in scan order (torch's
// max_pool2d_with_indices tie rule).
//
// Data flow (MI355X-first):
//   * the conv forward GEMM epilogue already produced per-tile (mean, M2) of
//     its bf16 output y; bn_finalize merges them (Chan et al.) per channel —
//     numerically robust, no E[y^2]-E[y]^2 cancellation over 524288 pixels;
//   * bn_apply reads y once and writes relu(a*y+b) (pooled when a pool
//     follows) — 8 channels per thread, 16-B accesses;
//   * backward never stores indices or masks: the ReLU mask and the pool
//     argmax are recomputed from y, a, b.  Pass 1 reduces sum(g) and
//     sum(g*xhat) per channel (per-block partials, fixed-order merge); pass 2
//     writes dy = a*(g - mean(g) - xhat*mean(g*xhat)) in bf16 for the conv
//     dgrad/wgrad GEMMs.
#include <cstdlib>

#include "ddpx_common.h"

namespace ddpx {
namespace bn {

// ---------------------------------------------------------------- finalize
// stats[t][0][c] = tile mean, stats[t][1][c] = tile M2; tile t covers rows [t*BM, min(M,(t+1)*BM)).
// 64 threads (one wave) per channel: each lane merges a strided subset of tiles,
// then a fixed-shape butterfly merges the lanes.
__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
  if (nb <= 0.f) return;  // (a trailing epilogue part wholly past M: min(BM, M - t*BM) < 0)
  if (n == 0.f) { n = nb; mean = meanb; m2 = m2b; return; }
  const float nn = n + nb;
  const float d = meanb - mean;
  mean += d * (nb / nn);
  m2 += m2b + d * d * (n * nb / nn);
  n = nn;
}

// One 256-thread workgroup per channel: every thread merges a strided subset of the tiles (at most
// T/256, loads issued ahead of the merges), a fixed-shape butterfly merges each wave, and thread 0
// merges the 4 wave results in wave order — deterministic, and enough workgroups (C of them) to keep
// the per-tile load latency off a serial chain (VGG's 32x32 layers have T = 2048 tiles).
__device__ __forceinline__ void wave_chan_merge(float& n, float& mu, float& m2, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float nb = __shfl_xor(n, o, 64), mb = __shfl_xor(mu, o, 64), qb = __shfl_xor(m2, o, 64);
    // lower lane merges the upper lane's state; the upper lane computes the same merge in the same order
    if ((lane & o) == 0) chan_merge(n, mu, m2, nb, mb, qb);
    else {
      float n2 = nb, mu2 = mb, q2 = qb;
      chan_merge(n2, mu2, q2, n, mu, m2);
      n = n2; mu = mu2; m2 = q2;
    }
  }
}

__global__ void __launch_bounds__(256)
finalize_kernel(const float* __restrict__ stats, int T, int BM, int M, int C, const float* __restrict__ gamma,
                const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar,
                int64_t* __restrict__ nbt, float momentum, float eps, int training, float* __restrict__ a_out,
                float* __restrict__ b_out, float* __restrict__ mean_out, float* __restrict__ rstd_out,
                float* __restrict__ merged_out) {
  __shared__ float wres[4][3];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = blockIdx.x;
  float mean, var;
  if (training) {
    float n = 0.f, mu = 0.f, m2 = 0.f;
    int t = tid;
    for (; t + 3 * 256 < T; t += 4 * 256) {  // 4 tiles' loads in flight per thread
      float tm[4], tq[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        tm[u] = stats[((size_t)(t + u * 256) * 2) * C + c];
        tq[u] = stats[((size_t)(t + u * 256) * 2 + 1) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) chan_merge(n, mu, m2, (float)min(BM, M - (t + u * 256) * BM), tm[u], tq[u]);
    }
    for (; t < T; t += 256)
      chan_merge(n, mu, m2, (float)min(BM, M - t * BM), stats[((size_t)t * 2) * C + c],
                 stats[((size_t)t * 2 + 1) * C + c]);
    wave_chan_merge(n, mu, m2, lane);
    if (lane == 0) { wres[w][0] = n; wres[w][1] = mu; wres[w][2] = m2; }
    __syncthreads();
    if (tid != 0) return;
    n = wres[0][0]; mu = wres[0][1]; m2 = wres[0][2];
    for (int q = 1; q < 4; ++q) chan_merge(n, mu, m2, wres[q][0], wres[q][1], wres[q][2]);
    if (merged_out) {  // SyncBN: this rank's (mean, M2) in the tile-stats layout [2][C]; merged across ranks next
      merged_out[c] = mu;
      merged_out[C + c] = m2;
      return;
    }
    mean = mu;
    var = m2 / (float)M;  // biased, for normalisation
    const float unbiased = M > 1 ? m2 / (float)(M - 1) : m2;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * unbiased;
    if (c == 0 && nbt) nbt[0] += 1;
  } else {
    if (tid != 0) return;
    mean = rmean[c];
    var = rvar[c];
  }
  const float rstd = rsqrtf(var + eps);
  const float a = gamma[c] * rstd;
  a_out[c] = a;
  b_out[c] = beta[c] - mean * a;
  mean_out[c] = mean;
  rstd_out[c] = rstd;
}

// ---------------------------------------------------------------- two-level, channel-coalesced merges
// The per-channel kernels above read one channel of a [T][2][C] partial array per wave: every lane touches a
// different row, so a 64-channel line is fetched by up to 64 waves (VGG's 32x32 layers: T = 2048, 22 us for a
// 1 MB merge).  Here a lane is a channel (a wave reads 256 contiguous bytes of one tile row), the tiles are split
// over S workgroups per 64-channel group, and the LAST workgroup of a group to finish (agent-scope ticket)
// merges the S partials in split order: deterministic, and the hand-off is MI355X_MICROARCH "Valid forms" row 1
// (sc1 stores drained by vmcnt(0) before the ticket, sc1 loads after it).  Tickets reset by their last arriver.
// up to 32 splits (every split takes one ticket on the same address: 128 splits measured no faster), a lane's
// tiles loaded 16 at a time (profiles/r5_conv/NOTES.md)
constexpr int kMergeMaxC = 1024, kFinMaxS = 32, kBwdMaxS = 32;
// Which merges use the two-level kernels: 0 both, 1 neither (the per-channel kernels above), 2 the backward sums
// only (default).  Split, the forward statistics merge measured no faster (86.8 vs 87 us per VGG step) and the
// backward one 83 -> 61 us; both match fp64 like the per-channel ones (tests/test_gpu_vgg.py).  A changed
// summation order moves any single deterministic bf16 VGG trajectory (0.53 -> 0.71 tail loss on one seed,
// profiles/r3_bn), but over an ensemble of seeds at the reference's batch size the three orders end in the same
// place as torch fp32 (profiles/r4_parity: mean last-20 loss fp32 0.415, per-channel 0.320, split 0.329, backward
// split 0.430), which is what tests/test_gpu_parity.py now checks.  DDPX_BN_MERGE=split|legacy|bwd, or
// ddpx_bn_set_merge(mode) (mode < 0: back to the environment / default).
static int g_merge_mode = -1;
static inline int merge_mode() {
  if (g_merge_mode < 0) {
    const char* e = getenv("DDPX_BN_MERGE");
    g_merge_mode = !e ? 2 : (e[0] == 's' ? 0 : (e[0] == 'l' ? 1 : 2));
  }
  return g_merge_mode;
}
// forward statistics: the default mode still splits the merge when the tile count is large (T > 4096: the
// per-channel kernel's strided loads took 25.5 us at T = 8192, profiles/r5_conv/NOTES.md; the conv epilogue now
// writes one statistics row per row tile, so VGG's largest is conv1's 4096)
static inline bool merge_legacy(int T = 0) { return merge_mode() == 1 || (merge_mode() == 2 && T <= 4096); }
static inline bool merge_legacy_bwd() { return merge_mode() == 1; }    // backward sums
__device__ int g_merge_tickets[2][kMergeMaxC / 64];
__device__ float g_fin_scratch[kFinMaxS * 3 * kMergeMaxC];
__device__ float g_bwd_scratch[kBwdMaxS * 2 * kMergeMaxC];

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* base, unsigned bytes, unsigned off_bytes) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000);
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off_bytes, 0, 16));
}
// lane 0 of wave 0 takes the ticket after every wave's sc1 stores drained (vmcnt(0) + barrier)
__device__ __forceinline__ bool take_last(int* ticket, int S, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) *flag = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
  __syncthreads();
  return *flag != 0;
}

static inline int fin_splits(int T) {
  int S = (T + 63) / 64;  // <= 16 tiles per lane
  return S < 1 ? 1 : (S > kFinMaxS ? kFinMaxS : S);
}
static inline int bwd_splits(int B) {
  int S = (B + 31) / 32;
  return S < 1 ? 1 : (S > kBwdMaxS ? kBwdMaxS : S);
}

// Training statistics: tiles t = 4 s + w (+ 4 S j) merged per lane, waves merged in order, then the split
// partials in split order by the last workgroup, which also runs finalize_kernel's epilogue.
__global__ void __launch_bounds__(256)
finalize_split_kernel(const float* __restrict__ stats, int T, int BM, int M, int C, int S,
                      const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ rmean,
                      float* __restrict__ rvar, int64_t* __restrict__ nbt, float momentum, float eps,
                      float* __restrict__ a_out, float* __restrict__ b_out, float* __restrict__ mean_out,
                      float* __restrict__ rstd_out, float* __restrict__ merged_out) {
  __shared__ float wres[4][3][64];
  __shared__ int flag;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cg = blockIdx.x, sp = blockIdx.y;
  const int c = cg * 64 + lane;
  const bool cok = c < C;
  const int cc = cok ? c : 0;
  float n = 0.f, mu = 0.f, m2 = 0.f;
  const int step = 4 * S;
  int t = 4 * sp + w;
  for (; t + 15 * step < T; t += 16 * step) {  // 16 tiles' loads in flight per lane
    float tm[16], tq[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      tm[u] = stats[((size_t)(t + u * step) * 2) * C + cc];
      tq[u] = stats[((size_t)(t + u * step) * 2 + 1) * C + cc];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) chan_merge(n, mu, m2, (float)min(BM, M - (t + u * step) * BM), tm[u], tq[u]);
  }
  for (; t + 3 * step < T; t += 4 * step) {
    float tm[4], tq[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      tm[u] = stats[((size_t)(t + u * step) * 2) * C + cc];
      tq[u] = stats[((size_t)(t + u * step) * 2 + 1) * C + cc];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) chan_merge(n, mu, m2, (float)min(BM, M - (t + u * step) * BM), tm[u], tq[u]);
  }
  for (; t < T; t += step)
    chan_merge(n, mu, m2, (float)min(BM, M - t * BM), stats[((size_t)t * 2) * C + cc], stats[((size_t)t * 2 + 1) * C + cc]);
  wres[w][0][lane] = n;
  wres[w][1][lane] = mu;
  wres[w][2][lane] = m2;
  __syncthreads();
  float* part = g_fin_scratch;
  if (w == 0) {
    for (int q = 1; q < 4; ++q) chan_merge(n, mu, m2, wres[q][0][lane], wres[q][1][lane], wres[q][2][lane]);
    if (cok) {
      st_sc1(part + ((size_t)sp * 3 + 0) * C + c, n);
      st_sc1(part + ((size_t)sp * 3 + 1) * C + c, mu);
      st_sc1(part + ((size_t)sp * 3 + 2) * C + c, m2);
    }
  }
  if (!take_last(&g_merge_tickets[0][cg], S, &flag)) return;
  if (threadIdx.x == 0) __hip_atomic_store(&g_merge_tickets[0][cg], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // all 4 waves: wave w merges partials w, w + 4, ... with every load issued first (one round trip), then the
  // waves' states merge in wave order through LDS (a fixed tree: deterministic)
  {
    const unsigned bytes = (unsigned)((size_t)S * 3 * C * 4);
    constexpr int PC = 8;  // partials per chunk, all loads of a chunk in flight together
    n = mu = m2 = 0.f;
    for (int u0 = 0; 4 * u0 < S; u0 += PC) {
      float v[PC][3];
#pragma unroll
      for (int u = 0; u < PC; ++u)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int sp2 = w + 4 * (u0 + u);
          v[u][k] = (cok && sp2 < S) ? ld_sc1(part, bytes, (unsigned)((((size_t)sp2 * 3 + k) * C + c) * 4)) : 0.f;
        }
#pragma unroll
      for (int u = 0; u < PC; ++u) chan_merge(n, mu, m2, v[u][0], v[u][1], v[u][2]);
    }
    __syncthreads();  // wres reuse
    wres[w][0][lane] = n;
    wres[w][1][lane] = mu;
    wres[w][2][lane] = m2;
    __syncthreads();
  }
  if (w != 0 || !cok) return;
  n = wres[0][0][lane];
  mu = wres[0][1][lane];
  m2 = wres[0][2][lane];
  for (int q = 1; q < 4; ++q) chan_merge(n, mu, m2, wres[q][0][lane], wres[q][1][lane], wres[q][2][lane]);
  if (merged_out) {
    merged_out[c] = mu;
    merged_out[C + c] = m2;
    return;
  }
  const float var = m2 / (float)M;
  const float unbiased = M > 1 ? m2 / (float)(M - 1) : m2;
  rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
  rvar[c] = (1.f - momentum) * rvar[c] + momentum * unbiased;
  if (c == 0 && nbt) nbt[0] += 1;
  const float rstd = rsqrtf(var + eps);
  const float a = gamma[c] * rstd;
  a_out[c] = a;
  b_out[c] = beta[c] - mu * a;
  mean_out[c] = mu;
  rstd_out[c] = rstd;
}

// Backward sums: part[B][2][C] (sum gz, sum gz*xhat per reduce block) -> c1 = sum/M, c2, and dgamma / dbeta
// stored or applied (bwd_finalize_kernel's epilogue), blocks split over S workgroups per channel group.
__global__ void __launch_bounds__(256)
bwd_finalize_split_kernel(const float* __restrict__ part, int B, int C, int M, int S, float* __restrict__ c1,
                          float* __restrict__ c2, void* __restrict__ dgamma, void* __restrict__ dbeta, int out_bf16,
                          int accumulate, SgdArgs sg, SgdArgs sb) {
  __shared__ float wres[4][2][64];
  __shared__ int flag;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cg = blockIdx.x, sp = blockIdx.y;
  const int c = cg * 64 + lane;
  const bool cok = c < C;
  const int cc = cok ? c : 0;
  float s1 = 0.f, s2 = 0.f;
  const int step = 4 * S;
  int k = 4 * sp + w;
  for (; k + 15 * step < B; k += 16 * step) {  // 16 partials' loads in flight per lane
    float a[16], q[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      a[u] = part[((size_t)(k + u * step) * 2) * C + cc];
      q[u] = part[((size_t)(k + u * step) * 2 + 1) * C + cc];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) { s1 += a[u]; s2 += q[u]; }
  }
  for (; k + 3 * step < B; k += 4 * step) {
    float a[4], q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = part[((size_t)(k + u * step) * 2) * C + cc];
      q[u] = part[((size_t)(k + u * step) * 2 + 1) * C + cc];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) { s1 += a[u]; s2 += q[u]; }
  }
  for (; k < B; k += step) {
    s1 += part[((size_t)k * 2) * C + cc];
    s2 += part[((size_t)k * 2 + 1) * C + cc];
  }
  wres[w][0][lane] = s1;
  wres[w][1][lane] = s2;
  __syncthreads();
  float* sc = g_bwd_scratch;
  if (w == 0) {
    s1 = ((wres[0][0][lane] + wres[1][0][lane]) + wres[2][0][lane]) + wres[3][0][lane];
    s2 = ((wres[0][1][lane] + wres[1][1][lane]) + wres[2][1][lane]) + wres[3][1][lane];
    if (cok) {
      st_sc1(sc + ((size_t)sp * 2) * C + c, s1);
      st_sc1(sc + ((size_t)sp * 2 + 1) * C + c, s2);
    }
  }
  if (!take_last(&g_merge_tickets[1][cg], S, &flag)) return;
  if (threadIdx.x == 0) __hip_atomic_store(&g_merge_tickets[1][cg], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  {
    const unsigned bytes = (unsigned)((size_t)S * 2 * C * 4);
    constexpr int PC = 8;
    s1 = s2 = 0.f;
    for (int u0 = 0; 4 * u0 < S; u0 += PC) {
      float v[PC][2];
#pragma unroll
      for (int u = 0; u < PC; ++u)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int sp2 = w + 4 * (u0 + u);
          v[u][j] = (cok && sp2 < S) ? ld_sc1(sc, bytes, (unsigned)((((size_t)sp2 * 2 + j) * C + c) * 4)) : 0.f;
        }
#pragma unroll
      for (int u = 0; u < PC; ++u) { s1 += v[u][0]; s2 += v[u][1]; }
    }
    __syncthreads();
    wres[w][0][lane] = s1;
    wres[w][1][lane] = s2;
    __syncthreads();
  }
  if (w != 0 || !cok) return;
  s1 = ((wres[0][0][lane] + wres[1][0][lane]) + wres[2][0][lane]) + wres[3][0][lane];
  s2 = ((wres[0][1][lane] + wres[1][1][lane]) + wres[2][1][lane]) + wres[3][1][lane];
  c1[c] = s1 / (float)M;
  c2[c] = s2 / (float)M;
  auto put = [&](const SgdArgs& sgd, void* out, float v) {
    if (sgd.p) {
      sgd_apply(sgd, c, v, *sgd.lr);
    } else if (out_bf16) {
      unsigned short* d = reinterpret_cast<unsigned short*>(out) + c;
      *d = f2bf(accumulate ? v + bf2f(*d) : v);
    } else if (out) {
      float* d = reinterpret_cast<float*>(out) + c;
      *d = accumulate ? v + *d : v;
    }
  };
  put(sg, dgamma, s2);
  put(sb, dbeta, s1);
}

// ---------------------------------------------------------------- apply
__device__ __forceinline__ void unpack8(const u32x4 v, float (&f)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(v[j] << 16);
    f[2 * j + 1] = __uint_as_float(v[j] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8(const float (&f)[8]) {
  return (u32x4){pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7])};
}

// out = relu(a*y + b), optionally 2x2 max-pooled.  One thread per (output pixel, 8-channel group).
__global__ void __launch_bounds__(256)
apply_kernel(const unsigned short* __restrict__ y, const float* __restrict__ a, const float* __restrict__ b, int N,
             int H, int W, int C, int relu, int pool, unsigned short* __restrict__ out) {
  const int G = C / 8;
  const int Ho = pool ? H / 2 : H, Wo = pool ? W / 2 : W;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= N * Ho * Wo * G) return;
  const int g = t % G;
  const int pix = t / G;
  const int wo = pix % Wo, ho = (pix / Wo) % Ho, n = pix / (Wo * Ho);
  float av[8], bv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    av[j] = a[g * 8 + j];
    bv[j] = b[g * 8 + j];
  }
  float r[8];
  if (!pool) {
    float f[8];
    unpack8(*reinterpret_cast<const u32x4*>(y + (size_t)pix * C + g * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      r[j] = fmaf(av[j], f[j], bv[j]);
      if (relu) r[j] = fmaxf(r[j], 0.f);
    }
  } else {
    u32x4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int hh = 2 * ho + (q >> 1), ww = 2 * wo + (q & 1);
      v[q] = *reinterpret_cast<const u32x4*>(y + (((size_t)n * H + hh) * W + ww) * C + g * 8);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = -INFINITY;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float f[8];
      unpack8(v[q], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float z = fmaf(av[j], f[j], bv[j]);
        if (relu) z = fmaxf(z, 0.f);
        r[j] = fmaxf(r[j], z);
      }
    }
  }
  *reinterpret_cast<u32x4*>(out + (size_t)pix * C + g * 8) = pack8(r);
}

// ---------------------------------------------------------------- backward
// gz for the 8 channels of pre-pool pixel (n, h, w): routes the pooled gradient to the
// first max of the 2x2 window (recomputed from y) and applies the ReLU mask.
__device__ __forceinline__ void grad_z(const unsigned short* __restrict__ gout, const unsigned short* __restrict__ y,
                                       const float (&av)[8], const float (&bv)[8], int n, int h, int w, int H, int W,
                                       int C, int g, int pool, int relu, const float (&yself)[8], float (&gz)[8]) {
  float zs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    zs[j] = fmaf(av[j], yself[j], bv[j]);
  }
  if (!pool) {
    float gg[8];
    unpack8(*reinterpret_cast<const u32x4*>(gout + (((size_t)n * H + h) * W + w) * C + g * 8), gg);
#pragma unroll
    for (int j = 0; j < 8; ++j) gz[j] = (!relu || zs[j] > 0.f) ? gg[j] : 0.f;
    return;
  }
  const int ho = h >> 1, wo = w >> 1, Ho = H >> 1, Wo = W >> 1;
  const int me = ((h & 1) << 1) | (w & 1);
  float gg[8];
  unpack8(*reinterpret_cast<const u32x4*>(gout + (((size_t)n * Ho + ho) * Wo + wo) * C + g * 8), gg);
  u32x4 v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int hh = 2 * ho + (q >> 1), ww = 2 * wo + (q & 1);
    v[q] = *reinterpret_cast<const u32x4*>(y + (((size_t)n * H + hh) * W + ww) * C + g * 8);
  }
  float best[8];
  int arg[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float f[8];
    unpack8(v[q], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float z = fmaf(av[j], f[j], bv[j]);
      if (relu) z = fmaxf(z, 0.f);
      if (z > best[j]) { best[j] = z; arg[j] = q; }  // strict: first max wins
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) gz[j] = (arg[j] == me && (!relu || zs[j] > 0.f)) ? gg[j] : 0.f;
}

// Pooled layers, one thread per (2x2 window, 8-channel group): the window's 4 y vectors and the pooled
// gradient are read once (not once per pre-pool pixel) and the routed, ReLU-masked gradient gz of all
// four pixels comes out together (same first-max tie rule and mask as grad_z).
__device__ __forceinline__ void grad_window(const unsigned short* __restrict__ gout,
                                            const unsigned short* __restrict__ y, const float (&av)[8],
                                            const float (&bv)[8], int n, int ho, int wo, int H, int W, int C, int g,
                                            int relu, float (&f)[4][8], float (&gz)[4][8]) {
  const int Ho = H >> 1, Wo = W >> 1;
  float gg[8];
  unpack8(*reinterpret_cast<const u32x4*>(gout + (((size_t)n * Ho + ho) * Wo + wo) * C + g * 8), gg);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int hh = 2 * ho + (q >> 1), ww = 2 * wo + (q & 1);
    unpack8(*reinterpret_cast<const u32x4*>(y + (((size_t)n * H + hh) * W + ww) * C + g * 8), f[q]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float best = -INFINITY;
    int arg = 0;
    float zs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      zs[q] = fmaf(av[j], f[q][j], bv[j]);
      const float z = relu ? fmaxf(zs[q], 0.f) : zs[q];
      if (z > best) { best = z; arg = q; }  // strict: first max wins
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) gz[q][j] = (arg == q && (!relu || zs[q] > 0.f)) ? gg[j] : 0.f;
  }
}

// Pass 1: part[blk][0][c] = sum gz, part[blk][1][c] = sum gz * xhat over this block's pixels.
// Block = 256 threads = (C/8 channel groups) x (256/(C/8) pixel lanes); grid-strided over pixels.
__global__ void __launch_bounds__(256)
bwd_reduce_kernel(const unsigned short* __restrict__ gout, const unsigned short* __restrict__ y,
                  const float* __restrict__ a, const float* __restrict__ b, const float* __restrict__ mean,
                  const float* __restrict__ rstd, int N, int H, int W, int C, int pool, int relu,
                  float* __restrict__ part, unsigned short* __restrict__ dyw) {
  // dyw (bias + activation only, no normalisation): the routed, masked gradient gz IS dy and does not depend on
  // the sums, so this pass also writes it and bwd_apply_kernel's second read of gout and y goes away
  __shared__ float red[2][256 * 8];
  const int G = C / 8;
  const int lanes = 256 / G;  // pixel lanes per block (G <= 64 => >= 4)
  const int g = threadIdx.x % G, pl = threadIdx.x / G;
  const int P = N * H * W;
  float av[8], bv[8], mu[8], rs[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    av[j] = a[g * 8 + j]; bv[j] = b[g * 8 + j]; mu[j] = mean[g * 8 + j]; rs[j] = rstd[g * 8 + j];
    s1[j] = 0.f; s2[j] = 0.f;
  }
  if (pool) {
    const int Ho = H >> 1, Wo = W >> 1, PP = N * Ho * Wo;
    for (int pp = blockIdx.x * lanes + pl; pp < PP; pp += gridDim.x * lanes) {
      const int wo = pp % Wo, ho = (pp / Wo) % Ho, n = pp / (Wo * Ho);
      float f[4][8], gz[4][8];
      grad_window(gout, y, av, bv, n, ho, wo, H, W, C, g, relu, f, gz);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s1[j] += gz[q][j];
          s2[j] = fmaf(gz[q][j], (f[q][j] - mu[j]) * rs[j], s2[j]);
        }
      if (dyw) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int hh = 2 * ho + (q >> 1), ww = 2 * wo + (q & 1);
          *reinterpret_cast<u32x4*>(dyw + (((size_t)n * H + hh) * W + ww) * C + g * 8) = pack8(gz[q]);
        }
      }
    }
  } else {
    for (int pix = blockIdx.x * lanes + pl; pix < P; pix += gridDim.x * lanes) {
      const int w = pix % W, h = (pix / W) % H, n = pix / (W * H);
      float f[8], gz[8];
      unpack8(*reinterpret_cast<const u32x4*>(y + (size_t)pix * C + g * 8), f);
      grad_z(gout, y, av, bv, n, h, w, H, W, C, g, pool, relu, f, gz);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += gz[j];
        s2[j] = fmaf(gz[j], (f[j] - mu[j]) * rs[j], s2[j]);
      }
      if (dyw) *reinterpret_cast<u32x4*>(dyw + (size_t)pix * C + g * 8) = pack8(gz);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][threadIdx.x * 8 + j] = s1[j];
    red[1][threadIdx.x * 8 + j] = s2[j];
  }
  __syncthreads();
  // channel c = g*8 + j: sum over the pixel lanes pl (threads t = pl*G + g)
  for (int i = threadIdx.x; i < 2 * C; i += 256) {
    const int which = i / C, c = i % C, gg = c / 8, j = c % 8;
    float s = 0.f;
    for (int q = 0; q < lanes; ++q) s += red[which][(q * G + gg) * 8 + j];
    part[((size_t)blockIdx.x * 2 + which) * C + c] = s;
  }
}

// Fixed-order merge of the pass-1 partials: dbeta = sum gz, dgamma = sum gz*xhat; also the
// pass-2 coefficients c1 = dbeta/M, c2 = dgamma/M.  Gradients stored or applied (fused SGD).
__global__ void __launch_bounds__(256)
bwd_finalize_kernel(const float* __restrict__ part, int B, int C, int M, float* __restrict__ c1,
                    float* __restrict__ c2, void* __restrict__ dgamma, void* __restrict__ dbeta, int out_bf16,
                    int accumulate, SgdArgs sg, SgdArgs sb) {
  // one wave (64 lanes) per channel: strided partial sums with 4 loads in flight, then a fixed
  // butterfly (deterministic)
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
    int k = lane;
    for (; k + 3 * 64 < B; k += 4 * 64) {
      float a[4], q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = part[((size_t)(k + u * 64) * 2) * C + c];
        q[u] = part[((size_t)(k + u * 64) * 2 + 1) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { s1 += a[u]; s2 += q[u]; }
    }
    for (; k < B; k += 64) {
      s1 += part[((size_t)k * 2) * C + c];
      s2 += part[((size_t)k * 2 + 1) * C + c];
    }
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (c >= C || lane != 0) return;
  c1[c] = s1 / (float)M;
  c2[c] = s2 / (float)M;
  auto put = [&](const SgdArgs& sgd, void* out, float v) {
    if (sgd.p) {
      sgd_apply(sgd, c, v, *sgd.lr);
    } else if (out_bf16) {
      unsigned short* d = reinterpret_cast<unsigned short*>(out) + c;
      *d = f2bf(accumulate ? v + bf2f(*d) : v);
    } else if (out) {
      float* d = reinterpret_cast<float*>(out) + c;
      *d = accumulate ? v + *d : v;
    }
  };
  put(sg, dgamma, s2);
  put(sb, dbeta, s1);
}

// Pass 2: dy = a * (gz - c1 - xhat * c2)   (bf16 [P][C]);  norm == 0: dy = gz (conv bias + ReLU only)
__global__ void __launch_bounds__(256)
bwd_apply_kernel(const unsigned short* __restrict__ gout, const unsigned short* __restrict__ y,
                 const float* __restrict__ a, const float* __restrict__ b, const float* __restrict__ mean,
                 const float* __restrict__ rstd, const float* __restrict__ c1, const float* __restrict__ c2, int N,
                 int H, int W, int C, int pool, int relu, int norm, unsigned short* __restrict__ dy) {
  const int G = C / 8;
  const int t = blockIdx.x * 256 + threadIdx.x;
  float av[8], bv[8];
  if (pool) {  // one thread per (2x2 window, channel group): writes the window's 4 dy vectors
    const int Ho = H >> 1, Wo = W >> 1;
    if (t >= N * Ho * Wo * G) return;
    const int g = t % G, pp = t / G;
    const int wo = pp % Wo, ho = (pp / Wo) % Ho, n = pp / (Wo * Ho);
    // per-channel coefficients in registers once per window (not re-loaded for each of the 4 pixels)
    float mu[8], rs[8], k1[8], k2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      av[j] = a[g * 8 + j];
      bv[j] = b[g * 8 + j];
      mu[j] = mean[g * 8 + j];
      rs[j] = rstd[g * 8 + j];
      k1[j] = c1[g * 8 + j];
      k2[j] = c2[g * 8 + j];
    }
    float f[4][8], gz[4][8];
    grad_window(gout, y, av, bv, n, ho, wo, H, W, C, g, relu, f, gz);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float out[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (f[q][j] - mu[j]) * rs[j];
        out[j] = norm ? av[j] * (gz[q][j] - k1[j] - xh * k2[j]) : gz[q][j];
      }
      const int hh = 2 * ho + (q >> 1), ww = 2 * wo + (q & 1);
      *reinterpret_cast<u32x4*>(dy + (((size_t)n * H + hh) * W + ww) * C + g * 8) = pack8(out);
    }
    return;
  }
  const int P = N * H * W;
  if (t >= P * G) return;
  const int g = t % G, pix = t / G;
  const int w = pix % W, h = (pix / W) % H, n = pix / (W * H);
  float f[8], gz[8], out[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { av[j] = a[g * 8 + j]; bv[j] = b[g * 8 + j]; }
  unpack8(*reinterpret_cast<const u32x4*>(y + (size_t)pix * C + g * 8), f);
  grad_z(gout, y, av, bv, n, h, w, H, W, C, g, pool, relu, f, gz);
  if (norm) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = g * 8 + j;
      const float xh = (f[j] - mean[c]) * rstd[c];
      out[j] = av[j] * (gz[j] - c1[c] - xh * c2[c]);
    }
  } else {  // bias + activation only (conv with bias, no BN): dy = routed, masked gradient
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = gz[j];
  }
  *reinterpret_cast<u32x4*>(dy + (size_t)pix * C + g * 8) = pack8(out);
}

// [N][S][C] -> [N][C] mean over S pixels (global average pool) and its backward.
__global__ void __launch_bounds__(256) avgpool_kernel(const unsigned short* __restrict__ x, int N, int S, int C,
                                                      unsigned short* __restrict__ out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= N * C) return;
  const int c = t % C, n = t / C;
  float s = 0.f;
  for (int i = 0; i < S; ++i) s += bf2f(x[((size_t)n * S + i) * C + c]);
  out[t] = f2bf(s / (float)S);
}

__global__ void __launch_bounds__(256) avgpool_bwd_kernel(const unsigned short* __restrict__ g, int N, int S, int C,
                                                          unsigned short* __restrict__ gx) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= N * S * C) return;
  const int c = t % C, n = t / (S * C);
  gx[t] = f2bf(bf2f(g[(size_t)n * C + c]) / (float)S);
}

}  // namespace bn
}  // namespace ddpx

using namespace ddpx;

DDPX_API void ddpx_bn_set_merge(int mode) { bn::g_merge_mode = mode < 0 || mode > 2 ? -1 : mode; }

DDPX_API int ddpx_bn_finalize(const float* stats, int T, int BM, int M, int C, const float* gamma, const float* beta,
                              float* rmean, float* rvar, int64_t* nbt, float momentum, float eps, int training,
                              float* a, float* b, float* mean, float* rstd, hipStream_t s) {
  if (training && C <= bn::kMergeMaxC && !bn::merge_legacy(T)) {
    const int S = bn::fin_splits(T);
    hipLaunchKernelGGL(bn::finalize_split_kernel, dim3((C + 63) / 64, S), dim3(256), 0, s, stats, T, BM, M, C, S,
                       gamma, beta, rmean, rvar, nbt, momentum, eps, a, b, mean, rstd, (float*)nullptr);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bn::finalize_kernel, dim3(C), dim3(256), 0, s, stats, T, BM, M, C, gamma, beta, rmean,
                     rvar, nbt, momentum, eps, training, a, b, mean, rstd, (float*)nullptr);
  return (int)hipGetLastError();
}

// SyncBatchNorm, forward: this rank's per-channel (mean, M2) over its M rows, merged from the conv
// epilogue's tile statistics, written as ONE tile [2][C].  The ranks' tiles are all-gathered into
// [ws][2][C] and ddpx_bn_finalize(gathered, T = ws, BM = M, M = ws * M) merges them in rank order — the
// same Chan merge on every rank, so every rank normalises with bitwise-identical statistics.
DDPX_API int ddpx_bn_local_stats(const float* stats, int T, int BM, int M, int C, float* out, hipStream_t s) {
  if (C <= bn::kMergeMaxC && !bn::merge_legacy(T)) {
    const int S = bn::fin_splits(T);
    hipLaunchKernelGGL(bn::finalize_split_kernel, dim3((C + 63) / 64, S), dim3(256), 0, s, stats, T, BM, M, C, S,
                       (const float*)nullptr, (const float*)nullptr, (float*)nullptr, (float*)nullptr,
                       (int64_t*)nullptr, 0.f, 0.f, (float*)nullptr, (float*)nullptr, (float*)nullptr,
                       (float*)nullptr, out);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bn::finalize_kernel, dim3(C), dim3(256), 0, s, stats, T, BM, M, C, (const float*)nullptr,
                     (const float*)nullptr, (float*)nullptr, (float*)nullptr, (int64_t*)nullptr, 0.f, 0.f, 1,
                     (float*)nullptr, (float*)nullptr, (float*)nullptr, (float*)nullptr, out);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_bn_apply(const void* y, const float* a, const float* b, int N, int H, int W, int C, int relu,
                           int pool, void* out, hipStream_t s) {
  if (C % 8 || (pool && (H % 2 || W % 2))) return -1;
  const int n = N * (pool ? H / 2 : H) * (pool ? W / 2 : W) * (C / 8);
  hipLaunchKernelGGL(bn::apply_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const unsigned short*)y, a, b, N, H,
                     W, C, relu, pool, (unsigned short*)out);
  return (int)hipGetLastError();
}

namespace {
hipError_t launch_bwd_finalize(const float* part, int B, int C, int M, float* c1, float* c2, void* dgamma, void* dbeta,
                               int out_bf16, int accumulate, SgdArgs sg, SgdArgs sb, hipStream_t s) {
  if (C <= bn::kMergeMaxC && !bn::merge_legacy_bwd()) {
    const int S = bn::bwd_splits(B);
    hipLaunchKernelGGL(bn::bwd_finalize_split_kernel, dim3((C + 63) / 64, S), dim3(256), 0, s, part, B, C, M, S, c1,
                       c2, dgamma, dbeta, out_bf16, accumulate, sg, sb);
  } else {
    hipLaunchKernelGGL(bn::bwd_finalize_kernel, dim3((C + 3) / 4), dim3(256), 0, s, part, B, C, M, c1, c2, dgamma,
                       dbeta, out_bf16, accumulate, sg, sb);
  }
  return hipGetLastError();
}
}  // namespace

DDPX_API int ddpx_bn_bwd_blocks(int N, int H, int W, int C) {
  const int lanes = 256 / (C / 8);
  const int P = N * H * W;
  int blocks = (P + lanes * 16 - 1) / (lanes * 16);  // >= 16 pixels per lane
  if (blocks > 1024) blocks = 1024;
  return blocks < 1 ? 1 : blocks;
}

DDPX_API int ddpx_bn_bwd(const void* gout, const void* y, const float* a, const float* b, const float* mean,
                         const float* rstd, int N, int H, int W, int C, int pool, int relu, float* part, float* c1,
                         float* c2, void* dgamma, void* dbeta, int out_bf16, int accumulate, void* dy, float* sg_p,
                         float* sg_buf, float* sb_p, float* sb_buf, const float* lr, float mom, float wd,
                         hipStream_t s) {
  if (C % 8 || C > 512 || (pool && (H % 2 || W % 2))) return -1;
  const int B = ddpx_bn_bwd_blocks(N, H, W, C);
  hipLaunchKernelGGL(bn::bwd_reduce_kernel, dim3(B), dim3(256), 0, s, (const unsigned short*)gout,
                     (const unsigned short*)y, a, b, mean, rstd, N, H, W, C, pool, relu, part, nullptr);
  launch_bwd_finalize(part, B, C, N * H * W, c1, c2, dgamma, dbeta, out_bf16, accumulate,
                      SgdArgs{sg_p, sg_buf, nullptr, lr, mom, wd}, SgdArgs{sb_p, sb_buf, nullptr, lr, mom, wd}, s);
  const int n = (pool ? N * (H / 2) * (W / 2) : N * H * W) * (C / 8);
  hipLaunchKernelGGL(bn::bwd_apply_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const unsigned short*)gout,
                     (const unsigned short*)y, a, b, mean, rstd, c1, c2, N, H, W, C, pool, relu, 1,
                     (unsigned short*)dy);
  return (int)hipGetLastError();
}

// Backward of  out = [maxpool2](relu(y + bias))  — a 3x3 conv WITH bias followed by ReLU (and pool),
// no BatchNorm: the reference's DeepNN blocks (/root/reference/singlegpu.py:21-31).  BatchNorm's pass 1 with
// a = 1, b = bias, mean = 0, rstd = 1 yields dbias = sum gz (fixed-order, deterministic) and, as dy = gz needs no
// sums, writes dy for the conv dgrad / wgrad GEMMs in the same pass (no second read of gout and y).
// SyncBatchNorm, backward in two halves around an all-reduce of sums[2][C] = (sum dy, sum dy*xhat):
// ddpx_bn_bwd_sums stores this rank's sums and the LOCAL dgamma / dbeta (DDP averages those, as torch's
// SyncBatchNorm does); after the all-reduce and a 1/M_global scale, ddpx_bn_bwd_apply forms dy.
DDPX_API int ddpx_bn_bwd_sums(const void* gout, const void* y, const float* a, const float* b, const float* mean,
                              const float* rstd, int N, int H, int W, int C, int pool, int relu, float* part,
                              float* sums, void* dgamma, void* dbeta, int out_bf16, int accumulate, hipStream_t s) {
  if (C % 8 || C > 512 || (pool && (H % 2 || W % 2))) return -1;
  const int B = ddpx_bn_bwd_blocks(N, H, W, C);
  hipLaunchKernelGGL(bn::bwd_reduce_kernel, dim3(B), dim3(256), 0, s, (const unsigned short*)gout,
                     (const unsigned short*)y, a, b, mean, rstd, N, H, W, C, pool, relu, part, nullptr);
  launch_bwd_finalize(part, B, C, 1, sums, sums + C, dgamma, dbeta, out_bf16, accumulate,
                      SgdArgs{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f},
                      SgdArgs{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f}, s);
  return (int)hipGetLastError();
}

// The second half of ddpx_bn_bwd when the pass-1 partials part[B][2][C] were produced elsewhere (the conv data
// gradient's EPI_BNBWD_BF16 epilogue): merge them (c1, c2, dgamma / dbeta or their fused SGD), then dy.
DDPX_API int ddpx_bn_bwd_tail(const void* gout, const void* y, const float* a, const float* b, const float* mean,
                              const float* rstd, int N, int H, int W, int C, int pool, int relu, const float* part,
                              int B, float* c1, float* c2, void* dgamma, void* dbeta, int out_bf16, int accumulate,
                              void* dy, float* sg_p, float* sg_buf, float* sb_p, float* sb_buf, const float* lr,
                              float mom, float wd, hipStream_t s) {
  if (C % 8 || C > 512 || B < 1 || (pool && (H % 2 || W % 2))) return -1;
  launch_bwd_finalize(part, B, C, N * H * W, c1, c2, dgamma, dbeta, out_bf16, accumulate,
                      SgdArgs{sg_p, sg_buf, nullptr, lr, mom, wd}, SgdArgs{sb_p, sb_buf, nullptr, lr, mom, wd}, s);
  const int n = (pool ? N * (H / 2) * (W / 2) : N * H * W) * (C / 8);
  hipLaunchKernelGGL(bn::bwd_apply_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const unsigned short*)gout,
                     (const unsigned short*)y, a, b, mean, rstd, c1, c2, N, H, W, C, pool, relu, 1,
                     (unsigned short*)dy);
  return (int)hipGetLastError();
}

// SyncBatchNorm with the pass-1 partials from the data-gradient epilogue: sums[2][C] (M = 1) and the local
// dgamma / dbeta, as ddpx_bn_bwd_sums without its reduce pass.
DDPX_API int ddpx_bn_bwd_sums_from_part(const float* part, int B, int C, float* sums, void* dgamma, void* dbeta,
                                        int out_bf16, int accumulate, hipStream_t s) {
  if (C % 8 || C > 512 || B < 1) return -1;
  launch_bwd_finalize(part, B, C, 1, sums, sums + C, dgamma, dbeta, out_bf16, accumulate,
                      SgdArgs{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f},
                      SgdArgs{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f}, s);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_bn_bwd_apply(const void* gout, const void* y, const float* a, const float* b, const float* mean,
                               const float* rstd, const float* c1, const float* c2, int N, int H, int W, int C,
                               int pool, int relu, void* dy, hipStream_t s) {
  if (C % 8 || C > 512 || (pool && (H % 2 || W % 2))) return -1;
  const int n = (pool ? N * (H / 2) * (W / 2) : N * H * W) * (C / 8);
  hipLaunchKernelGGL(bn::bwd_apply_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const unsigned short*)gout,
                     (const unsigned short*)y, a, b, mean, rstd, c1, c2, N, H, W, C, pool, relu, 1,
                     (unsigned short*)dy);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_bias_act_bwd_sgd(const void* gout, const void* y, const float* bias, const float* ones,
                                   const float* zeros, int N, int H, int W, int C, int pool, int relu, float* part,
                                   float* c1, float* c2, void* dbias, int out_bf16, int accumulate, void* dy,
                                   float* sb_p, float* sb_buf, void* sb_shadow, const float* lr, float mom, float wd,
                                   hipStream_t s) {
  // sb_p (optional): the bias gradient is applied as its fused SGD update in the merge (no gradient stored)
  if (C % 8 || C > 512 || (pool && (H % 2 || W % 2)) || (sb_p && !lr) || (!sb_p && !dbias)) return -1;
  const int B = ddpx_bn_bwd_blocks(N, H, W, C);
  hipLaunchKernelGGL(bn::bwd_reduce_kernel, dim3(B), dim3(256), 0, s, (const unsigned short*)gout,
                     (const unsigned short*)y, ones, bias, zeros, ones, N, H, W, C, pool, relu, part, (unsigned short*)dy);
  launch_bwd_finalize(part, B, C, N * H * W, c1, c2, nullptr, dbias, out_bf16, accumulate,
                      SgdArgs{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f},
                      SgdArgs{sb_p, sb_buf, (unsigned short*)sb_shadow, lr, mom, wd}, s);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_bias_act_bwd(const void* gout, const void* y, const float* bias, const float* ones,
                               const float* zeros, int N, int H, int W, int C, int pool, int relu, float* part,
                               float* c1, float* c2, void* dbias, int out_bf16, int accumulate, void* dy,
                               hipStream_t s) {
  if (C % 8 || C > 512 || (pool && (H % 2 || W % 2))) return -1;
  const int B = ddpx_bn_bwd_blocks(N, H, W, C);
  hipLaunchKernelGGL(bn::bwd_reduce_kernel, dim3(B), dim3(256), 0, s, (const unsigned short*)gout,
                     (const unsigned short*)y, ones, bias, zeros, ones, N, H, W, C, pool, relu, part, (unsigned short*)dy);
  launch_bwd_finalize(part, B, C, N * H * W, c1, c2, nullptr, dbias, out_bf16, accumulate,
                      SgdArgs{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f},
                      SgdArgs{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f}, s);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_avgpool(const void* x, int N, int S, int C, void* out, hipStream_t s) {
  const int n = N * C;
  hipLaunchKernelGGL(bn::avgpool_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const unsigned short*)x, N, S, C,
                     (unsigned short*)out);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_avgpool_bwd(const void* g, int N, int S, int C, void* gx, hipStream_t s) {
  const int n = N * S * C;
  hipLaunchKernelGGL(bn::avgpool_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const unsigned short*)g, N, S,
                     C, (unsigned short*)gx);
  return (int)hipGetLastError();
}
