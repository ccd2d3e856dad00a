// ddpx — the reference's fp32 recipe on MI355X (``--dtype fp32``; /root/reference/singlegpu.py:134 trains
// VGG in fp32 and reports "fp32 model has accuracy", :248-249).
//
// Every operation of the VGG / MLP training step in exact fp32, on CDNA4 directly:
//
//   * one GEMM core for Linear fwd / dgrad / wgrad and the 3x3 convolutions as implicit GEMMs (NHWC, the
//     im2col never materialised): v_mfma_f32_16x16x4_f32 — f32 in, f32 accumulate, bitwise an fmaf chain,
//     64 FLOP/clk/SIMD = the f32 vector peak (157 TF; gfx950 has no xf32).  256-thread workgroups of
//     2x2 waves, 128x128 / 128x64 / 64x64 tiles, BK = 16, register-staged global loads of tile t+1 issued
//     before the MFMAs of tile t, double-buffered LDS (one barrier per K step), rows padded by 20 floats
//     (conflict-free fragment reads and transposing stores on the 64-bank LDS), XCD-aware tile order;
//   * weight gradients of the convolutions split over K (= N*H*W) into fixed-order partial slabs reduced
//     (and permuted to torch's [Co][Ci][3][3]) by one pass — deterministic, no float atomics;
//   * BatchNorm2d training statistics as per-chunk (mean, M2) merged by Chan's formula in the finalize
//     (running stats: momentum, unbiased variance; num_batches_tracked on device), apply + ReLU +
//     MaxPool2d(2) fused in one pass, backward with the pool routing (first maximum of each window, as
//     torch) and the ReLU mask recomputed from the saved pre-BN activation;
//   * global average pool, and the 10-class head: logits + softmax cross-entropy + dlogits, with
//     dW / db / dfeature (+ ReLU mask for the MLP) in the backward.
#include <cstdlib>

#include "ddpx_common.h"

namespace ddpx {
namespace f32k {

enum Mode { DENSE_KC = 0, DENSE_OC = 1, IM2COL_KC = 2, IM2COL_OC = 3 };

// A logical operand X(o, k): o = row of A / column of B ("outer"), k = reduction index.
//   DENSE_KC : p[o * ld + k]           (contiguous along k; K % 4 == 0)
//   DENSE_OC : p[k * ld + o]           (contiguous along o; O % 4 == 0)
//   IM2COL_KC: o = pixel m, k = (r*3+s)*C + c -> x[n][h+sgn(r-1)][w+sgn(s-1)][c]   (forward / data gradient A)
//   IM2COL_OC: o = (r*3+s)*C + c, k = pixel m  (same element)                         (weight gradient B)
// Out-of-range rows / k / padding taps read as 0.  C, H, W are powers of two (log2 given).
struct Operand {
  const float* p;
  int ld, O;
  int lc, lh, lw, sgn;
};

__device__ __forceinline__ f32x4 im2col4(const Operand& X, int m, int k) {
  const int n = m >> (X.lh + X.lw);
  const int h = (m >> X.lw) & ((1 << X.lh) - 1);
  const int w = m & ((1 << X.lw) - 1);
  const int rs = k >> X.lc;
  const int c = k & ((1 << X.lc) - 1);
  const int r = (rs * 11) >> 5;  // rs / 3 for rs < 9
  const int s = rs - 3 * r;
  const int ih = h + X.sgn * (r - 1), iw = w + X.sgn * (s - 1);
  if (rs >= 9 || ih < 0 || iw < 0 || ih >= (1 << X.lh) || iw >= (1 << X.lw)) return (f32x4){0.f, 0.f, 0.f, 0.f};
  const size_t off = ((((size_t)n << X.lh | ih) << X.lw | iw) << X.lc) | c;
  return *reinterpret_cast<const f32x4*>(X.p + off);
}

template <int MODE>
__device__ __forceinline__ f32x4 load4(const Operand& X, int o, int k, int kend) {
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  if (o >= X.O || k >= kend) return zero;
  if constexpr (MODE == DENSE_KC) return *reinterpret_cast<const f32x4*>(X.p + (size_t)o * X.ld + k);
  if constexpr (MODE == DENSE_OC) return *reinterpret_cast<const f32x4*>(X.p + (size_t)k * X.ld + o);
  if constexpr (MODE == IM2COL_KC) return im2col4(X, o, k);
  return im2col4(X, k, o);
}

constexpr int BK = 16, PAD = 20, NT = 256;  // Stage<KC> maps 4 float4 per row: BK is 16

template <int MODE, int BO>
struct Stage {
  static constexpr int NV = BO * BK / 4 / NT;  // float4 per thread per tile
  static constexpr bool KC = (MODE == DENSE_KC || MODE == IM2COL_KC);
  f32x4 r[NV];
  __device__ __forceinline__ void load(const Operand& X, int o0, int kt, int kend, int tid) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = tid + NT * v;
      if constexpr (KC) r[v] = load4<MODE>(X, o0 + (idx >> 2), kt + (idx & 3) * 4, kend);
      else r[v] = load4<MODE>(X, o0 + (idx % (BO / 4)) * 4, kt + idx / (BO / 4), kend);
    }
  }
  __device__ __forceinline__ void store(float (*S)[BO + PAD], int tid) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = tid + NT * v;
      if constexpr (KC) {
        const int o = idx >> 2, kq = (idx & 3) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) S[kq + e][o] = r[v][e];
      } else {
        *reinterpret_cast<f32x4*>(&S[idx / (BO / 4)][(idx % (BO / 4)) * 4]) = r[v];
      }
    }
  }
};

enum Flags { F_RELU = 1, F_ACCUM = 2, F_SPLIT = 4, F_VEC = 8 };  // F_VEC: LDS-DMA core's 16-B store epilogue

// C[m][n] (+)= sum_k A(m,k) B(k,n)  [+ bias[n]] [relu] [* (mask[m][n] > 0)]; F_SPLIT: the K range of
// blockIdx's split z goes to the raw slab C + z * split_stride.
template <int BM, int BN, int AM, int BMD, bool PLAIN>
__global__ void __launch_bounds__(NT)
gemm_f32_kernel(const Operand A, const Operand B, int M, int N, int K, int kchunk, float* __restrict__ C, int ldc,
                long split_stride, const float* __restrict__ bias, const float* __restrict__ mask, int flags,
                int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) float As[2][BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][BN + PAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int per = tiles_m * tiles_n;
  const int z = bid / per, t2 = bid - z * per;
  // consecutive ids (one XCD's range) walk down M inside one column panel of B: the B panel stays in L2
  const int tm = t2 % tiles_m, tn = t2 / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int k0 = z * kchunk, k1 = min(K, k0 + kchunk);
  const int nk = (k1 - k0 + BK - 1) / BK;

  constexpr int FM = BM / 32, FN = BN / 32;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  Stage<AM, BM> sa;
  Stage<BMD, BN> sb;
  if (nk > 0) {
    sa.load(A, m0, k0, k1, tid);
    sb.load(B, n0, k0, k1, tid);
    sa.store(As[0], tid);
    sb.store(Bs[0], tid);
  }
  __syncthreads();
  const int lr = lane >> 4, lc = lane & 15;
  for (int it = 0; it < nk; ++it) {
    const int cur = it & 1;
    const bool more = it + 1 < nk;
    if (more) {
      sa.load(A, m0, k0 + (it + 1) * BK, k1, tid);
      sb.load(B, n0, k0 + (it + 1) * BK, k1, tid);
    }
    // blocked summation (PLAIN = false): each K step's 16 products go into a fresh accumulator that is then
    // added to the running sum — the rounding chain is K/16 long instead of K (4x smaller error at K = 4608,
    // where a plain MFMA chain left the conv7 output 4e-6 from fp64).  PLAIN: one MFMA chain over K, the
    // summation order of the fp32 library kernels (held to their error vs fp64: tests/test_gpu_f32.py).
    f32x4 part[FM][FN];
    if constexpr (PLAIN) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) part[i][j] = acc[i][j];
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      float a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = As[cur][kk + lr][wm * (BM / 2) + i * 16 + lc];
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = Bs[cur][kk + lr][wn * (BN / 2) + j * 16 + lc];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          part[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(
              a[i], b[j], (PLAIN || kk) ? part[i][j] : (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if constexpr (PLAIN) acc[i][j] = part[i][j];
        else acc[i][j] += part[i][j];
      }
    if (more) {
      sa.store(As[cur ^ 1], tid);
      sb.store(Bs[cur ^ 1], tid);
    }
    __syncthreads();
  }

  float* out = (flags & F_SPLIT) ? C + (size_t)z * split_stride : C;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * (BM / 2) + i * 16 + lr * 4 + e;
        const int col = n0 + wn * (BN / 2) + j * 16 + lc;
        if (row >= M || col >= N) continue;
        float v = acc[i][j][e];
        const size_t o = (size_t)row * ldc + col;
        if (!(flags & F_SPLIT)) {
          if (bias) v += bias[col];
          if (flags & F_ACCUM) v += out[o];
          if (flags & F_RELU) v = fmaxf(v, 0.f);
          if (mask && !(mask[o] > 0.f)) v = 0.f;
        }
        out[o] = v;
      }
}

// ------------------------------------------------------------------ LDS-DMA ring variant
// Same tiles, fragments, MFMA sequence and summation order as gemm_f32_kernel (bitwise-identical results), but the
// operand tiles go global -> LDS by `buffer_load_dword ... lds` (LDS-DMA: no staging VGPRs, no ds_write pass, no
// per-element transposing stores) into an S-stage ring with S-1 K-steps in flight, one raw s_barrier per K-step
// and counted vmcnt waits — the register-staged kernel above exposed a whole K-step of global-load latency per
// barrier with only 2 waves per SIMD (244 VGPRs) to hide it.
// LDS images (16-B chunks = 4 floats, lane-linear DMA writes, bank swizzles applied to the SOURCE chunk):
//   KC operand  [rows][16 k]   row = 64 B, chunk c at c ^ ((row >> 2) & 3)        (conflict-free b32 fragment reads)
//   OC operand  [16 k][rows]   row = 4*rows B, chunk c at c ^ (4 * (k & 3))        (rows >= 64)
constexpr unsigned kOOB32 = 0x80000000u;

template <int MODE>
__device__ __forceinline__ unsigned f32_chunk_off(const Operand& X, int o, int k, int kend) {
  if (o >= X.O || k >= kend) return kOOB32;
  if constexpr (MODE == DENSE_KC) return (unsigned)(((size_t)o * X.ld + k) * 4);
  if constexpr (MODE == DENSE_OC) return (unsigned)(((size_t)k * X.ld + o) * 4);
  const int m = MODE == IM2COL_KC ? o : k, q = MODE == IM2COL_KC ? k : o;
  const int n = m >> (X.lh + X.lw);
  const int h = (m >> X.lw) & ((1 << X.lh) - 1);
  const int w = m & ((1 << X.lw) - 1);
  const int rs = q >> X.lc;
  const int c = q & ((1 << X.lc) - 1);
  const int r = (rs * 11) >> 5;
  const int s2 = rs - 3 * r;
  const int ih = h + X.sgn * (r - 1), iw = w + X.sgn * (s2 - 1);
  if (rs >= 9 || ih < 0 || iw < 0 || ih >= (1 << X.lh) || iw >= (1 << X.lw)) return kOOB32;
  return (unsigned)((((((size_t)n << X.lh | ih) << X.lw | iw) << X.lc) | c) * 4);
}

// Stage one operand tile (ROWS x 16 k) of K-step k0 into an LDS slot: ROWS*64/1024 wave-instructions over 4 waves.
template <int MODE, int ROWS>
__device__ __forceinline__ void f32_stage(__amdgpu_buffer_rsrc_t rs, char* slot, const Operand& X, int o0, int k0,
                                          int kend, int wave, int lane) {
  constexpr bool KC = (MODE == DENSE_KC || MODE == IM2COL_KC);
  constexpr int NI = ROWS * 64 / 1024 / 4;  // instructions per wave
  static_assert(NI * 4 * 1024 == ROWS * 64, "tile must split over 4 waves");
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int inst = j * 4 + wave;
    const int pc = inst * 64 + lane;  // LDS chunk position
    unsigned off;
    if constexpr (KC) {
      const int row = pc >> 2, cpos = pc & 3;
      const int kc = cpos ^ ((row >> 2) & 3);
      off = f32_chunk_off<MODE>(X, o0 + row, k0 + 4 * kc, kend);
    } else {
      constexpr int CPR = ROWS / 4;  // chunks per k-row
      const int krow = pc / CPR, cpos = pc % CPR;
      const int oc = cpos ^ (4 * (krow & 3));
      off = f32_chunk_off<MODE>(X, o0 + 4 * oc, k0 + krow, kend);
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)(slot + inst * 1024), 16, off, 0, 0, 0);
  }
}

template <int MODE, int ROWS>
__device__ __forceinline__ float f32_frag(const char* img, int r, int k) {
  constexpr bool KC = (MODE == DENSE_KC || MODE == IM2COL_KC);
  int byte;
  if constexpr (KC) byte = r * 64 + ((((k >> 2) ^ ((r >> 2) & 3)) << 4) | ((k & 3) << 2));
  else byte = k * (ROWS * 4) + ((((r >> 2) ^ (4 * (k & 3)))) << 4) + ((r & 3) << 2);
  return *reinterpret_cast<const float*>(img + byte);
}

// KB (blocked summation only): K-steps of 16 per fresh block accumulator.  1 = the register-staged kernel's order
// (bitwise equal); 2 = 32-k blocks, half the block adds (DDPX_F32_BLOCK=2).
template <int BM, int BN, int AM, int BMD, bool PLAIN, int STAGES, int KB = 1>
__global__ void __launch_bounds__(NT)
gemm_f32_dma_kernel(const Operand A, const Operand B, int M, int N, int K, int kchunk, float* __restrict__ C,
                    int ldc, long split_stride, const float* __restrict__ bias, const float* __restrict__ mask,
                    int flags, int tiles_m, int tiles_n, unsigned a_bytes, unsigned b_bytes,
                    float* __restrict__ stats, SgdArgs sgd) {
  constexpr int A_SUB = BM * 64, B_SUB = BN * 64, SLOT = A_SUB + B_SUB;
  constexpr int LW = (BM + BN) * 64 / 1024 / 4;  // DMA instructions per wave per stage
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int per = tiles_m * tiles_n;
  const int z = bid / per, t2 = bid - z * per;
  const int tm = t2 % tiles_m, tn = t2 / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int k0 = z * kchunk, k1 = min(K, k0 + kchunk);
  const int nk = (k1 - k0 + BK - 1) / BK;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A.p, 0, a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B.p, 0, b_bytes, 0x00020000);

  constexpr int FM = BM / 32, FN = BN / 32;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t) {
    char* slot = smem + (t % STAGES) * SLOT;
    f32_stage<AM, BM>(ra, slot, A, m0, k0 + t * BK, k1, wave, lane);
    f32_stage<BMD, BN>(rb, slot + A_SUB, B, n0, k0 + t * BK, k1, wave, lane);
  };
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s);
  const int lr = lane >> 4, lc = lane & 15;
  constexpr int KBE = PLAIN ? 1 : KB;
  for (int it0 = 0; it0 < nk; it0 += KBE) {
    f32x4 part[FM][FN];
    if constexpr (PLAIN) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) part[i][j] = acc[i][j];
    }
#pragma unroll
    for (int u = 0; u < KBE; ++u) {
      const int it = it0 + u;
      if (KBE > 1 && it >= nk) break;
      const int ahead = min(STAGES - 2, nk - 1 - it);  // younger stages allowed in flight
      if (STAGES >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LW) : "memory");
      else if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (it + STAGES - 1 < nk) issue(it + STAGES - 1);
      const char* sa = smem + (it % STAGES) * SLOT;
      const char* sb = sa + A_SUB;
      // every fragment of the K-step read up front (one LDS-latency exposure per K-step; reading them kk by kk
      // into reused registers made hipcc wait lgkmcnt(0) every 8 MFMAs)
      float a[BK / 4][FM], b[BK / 4][FN];
#pragma unroll
      for (int q = 0; q < BK / 4; ++q) {
#pragma unroll
        for (int i = 0; i < FM; ++i) a[q][i] = f32_frag<AM, BM>(sa, wm * (BM / 2) + i * 16 + lc, 4 * q + lr);
#pragma unroll
        for (int j = 0; j < FN; ++j) b[q][j] = f32_frag<BMD, BN>(sb, wn * (BN / 2) + j * 16 + lc, 4 * q + lr);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep every read issued before the first MFMA (counted lgkmcnt waits)
#pragma unroll
      for (int q = 0; q < BK / 4; ++q)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            part[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                a[q][i], b[q][j], (PLAIN || u || q) ? part[i][j] : (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if constexpr (PLAIN) acc[i][j] = part[i][j];
        else acc[i][j] += part[i][j];
      }
  }

  if (stats) {
    // BatchNorm training statistics of this output tile, straight from the accumulators (the conv forward's raw
    // output): per column, the tile mean and M2 over its valid rows -> stats[tile_m][0 / 1][col] (the chunk
    // statistics bn_finalize merges with Chan's formula; chunk = BM rows).  Fixed reduction order: the 4 lanes
    // sharing a column (xor 16, 32), then the two row-halves of the tile in order.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done with the LDS ring: reuse it
    float* red = reinterpret_cast<float*>(smem);  // [4][BN]: sums of the 2 row halves, then their M2
    const int rows_t = min(BM, M - m0);
    float mean[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (m0 + wm * (BM / 2) + i * 16 + lr * 4 + e < M) sm += acc[i][j][e];
      sm += __shfl_xor(sm, 16, 64);
      sm += __shfl_xor(sm, 32, 64);
      if (lr == 0) red[wm * BN + wn * (BN / 2) + j * 16 + lc] = sm;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wn * (BN / 2) + j * 16 + lc;
      mean[j] = (red[col] + red[BN + col]) / (float)rows_t;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (m0 + wm * (BM / 2) + i * 16 + lr * 4 + e < M) {
            const float d = acc[i][j][e] - mean[j];
            q = fmaf(d, d, q);
          }
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (lr == 0) red[(2 + wm) * BN + col] = q;
    }
    __syncthreads();
    if (wm == 0 && lr == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * (BN / 2) + j * 16 + lc;
        if (n0 + col < N) {
          stats[(size_t)tm * 2 * N + n0 + col] = mean[j];
          stats[(size_t)tm * 2 * N + N + n0 + col] = red[2 * BN + col] + red[3 * BN + col];
        }
      }
    }
  }
  float* out = (flags & F_SPLIT) ? C + (size_t)z * split_stride : C;
  if (sgd.p && !(flags & F_SPLIT)) {
    // fused optimizer (single-process weight gradients): the tile's gradient updates the parameter it belongs to
    // right here, with sgd_apply's fma sequence (bitwise the flat SGD's); the gradient is never stored.  The
    // accumulators are staged through the (now idle) LDS ring in row parts so every thread streams 16-B vectors
    // of the master / momentum rows (per-element 4-B accesses ran the update at a fraction of the HBM rate).
    constexpr int TLD = BN + 4;
    constexpr int EH = (BM * TLD * 4 <= STAGES * SLOT) ? 1 : 2;
    constexpr int BMH = BM / EH;
    static_assert(BMH * TLD * 4 <= STAGES * SLOT, "SGD epilogue staging does not fit the ring");
    constexpr int Q = BN / 4, RSTEP = NT / Q, NV = BMH / RSTEP, CH = NV < 4 ? NV : 4;
    float* T = reinterpret_cast<float*>(smem);
    const float slr = *sgd.lr;
    const bool has_mom = sgd.mom != 0.f;
    const int cq = tid % Q, r0 = tid / Q;
    const int col = n0 + 4 * cq;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int h = 0; h < EH; ++h) {
      __syncthreads();  // the ring (h = 0) / the previous part's reads (h = 1) are done
      if (wm == h || EH == 1) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = (EH == 1 ? wm * (BM / 2) : 0) + i * 16 + lr * 4 + e;
              T[r * TLD + wn * (BN / 2) + j * 16 + lc] = acc[i][j][e];
            }
      }
      __syncthreads();
      const int mh = m0 + h * BMH;
#pragma unroll
      for (int i0 = 0; i0 < NV; i0 += CH) {
        f32x4 pv[CH], bv[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int row = mh + r0 + (i0 + i) * RSTEP;
          pv[i] = bv[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
          if (row >= M || col >= N) continue;
          const size_t o = (size_t)row * ldc + col;
          pv[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(sgd.p + o));
          if (has_mom) bv[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(sgd.buf + o));
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int r = r0 + (i0 + i) * RSTEP;
          const int row = mh + r;
          if (row >= M || col >= N) continue;
          const size_t o = (size_t)row * ldc + col;
          const f32x4 g = *reinterpret_cast<const f32x4*>(T + r * TLD + 4 * cq);
          f32x4 po, bo;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float d = fmaf(sgd.wd, pv[i][q], g[q]);
            if (has_mom) d = fmaf(sgd.mom, bv[i][q], d);
            bo[q] = d;
            po[q] = fmaf(-slr, d, pv[i][q]);
          }
          __builtin_nontemporal_store(po, reinterpret_cast<f32x4*>(sgd.p + o));
          if (has_mom) __builtin_nontemporal_store(bo, reinterpret_cast<f32x4*>(sgd.buf + o));
          if (sgd.shadow)
            *reinterpret_cast<u32x2*>(sgd.shadow + o) = (u32x2){pack_bf2(po[0], po[1]), pack_bf2(po[2], po[3])};
        }
      }
    }
    return;
  }
  if (flags & F_VEC) {
    // Output tile staged through the idle LDS ring in row parts, then stored as 16-B row vectors (a 128-wide tile
    // row is 512 contiguous bytes).  The fragment-order stores below write 4-B lanes in 64-B row pieces: DeepNN's
    // first conv (K = 36, 256 MB of output) ran 171 us, store-bound, on them (profiles/r6_deepnn).  Same values,
    // same epilogue order (bias, accumulate, ReLU, mask) — bitwise the scalar form.
    constexpr int TLD = BN + 4;
    constexpr int EH = (BM * TLD * 4 <= STAGES * SLOT) ? 1 : 2;
    constexpr int BMH = BM / EH;
    static_assert(BMH * TLD * 4 <= STAGES * SLOT, "epilogue staging does not fit the ring");
    constexpr int Q = BN / 4, RSTEP = NT / Q, NV = BMH / RSTEP;
    float* T = reinterpret_cast<float*>(smem);
    const int cq = tid % Q, r0 = tid / Q;
    const int col = n0 + 4 * cq;
    const bool epi = !(flags & F_SPLIT);
    f32x4 bv = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (epi && bias && col < N) bv = *reinterpret_cast<const f32x4*>(bias + col);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int h = 0; h < EH; ++h) {
      __syncthreads();  // the ring / the statistics scratch (h = 0), the previous part's reads (h = 1) are done
      if (wm == h || EH == 1) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = (EH == 1 ? wm * (BM / 2) : 0) + i * 16 + lr * 4 + e;
              T[r * TLD + wn * (BN / 2) + j * 16 + lc] = acc[i][j][e];
            }
      }
      __syncthreads();
      const int mh = m0 + h * BMH;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int r = r0 + i * RSTEP;
        const int row = mh + r;
        if (row >= M || col >= N) continue;
        const size_t o = (size_t)row * ldc + col;
        f32x4 v = *reinterpret_cast<const f32x4*>(T + r * TLD + 4 * cq);
        if (epi) {
          const f32x4 prev = (flags & F_ACCUM) ? *reinterpret_cast<const f32x4*>(out + o) : bv;
          const f32x4 mk = mask ? *reinterpret_cast<const f32x4*>(mask + o) : (f32x4){1.f, 1.f, 1.f, 1.f};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float x = v[q];
            if (bias) x += bv[q];
            if (flags & F_ACCUM) x += prev[q];
            if (flags & F_RELU) x = fmaxf(x, 0.f);
            if (!(mk[q] > 0.f)) x = 0.f;
            v[q] = x;
          }
        }
        *reinterpret_cast<f32x4*>(out + o) = v;
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * (BM / 2) + i * 16 + lr * 4 + e;
        const int col = n0 + wn * (BN / 2) + j * 16 + lc;
        if (row >= M || col >= N) continue;
        float v = acc[i][j][e];
        const size_t o = (size_t)row * ldc + col;
        if (!(flags & F_SPLIT)) {
          if (bias) v += bias[col];
          if (flags & F_ACCUM) v += out[o];
          if (flags & F_RELU) v = fmaxf(v, 0.f);
          if (mask && !(mask[o] > 0.f)) v = 0.f;
        }
        out[o] = v;
      }
}

// Summation order of the f32 core (DDPX_F32_SUM=plain|blocked|auto, default auto).  The bar is the stock fp32
// libraries' own error vs fp64 on the same inputs (tests/test_gpu_f32.py::test_error_no_worse_than_stock,
// MI355X: profiles/r3_f32): the plain chain matches hipBLASLt on the MLP's fc1 (1.15e-6 vs 1.15e-6 rel-L2)
// and is 1.15-1.3x MIOpen's error on VGG's conv7 / conv4, where a few max-pool routing flips then move the
// gradients below them 4x further than torch's own fp32 run does; the blocked form is 2-4x MORE accurate
// than the libraries.  auto: plain for dense GEMMs (Linear layers: 1.056 vs 1.150 ms per toy-MLP step),
// blocked for the im2col convolution GEMMs.
static int f32_sum_mode() {  // 0 auto, 1 plain, 2 blocked
  static const int v = [] {
    const char* e = getenv("DDPX_F32_SUM");
    return !e ? 0 : e[0] == 'p' ? 1 : e[0] == 'b' ? 2 : 0;
  }();
  return v;
}

// 3-slot ring for im2col GEMMs with K <= 48 (DDPX_F32_SMALLK=0 disables; A/B).  Same summation: bitwise equal.
static bool f32_small_k_ring() {
  static const bool v = [] {
    const char* e = getenv("DDPX_F32_SMALLK");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Operand staging: DDPX_F32_STAGING=dma (LDS-DMA ring, default) | reg (register-staged, double-buffered LDS).
static int g_f32_staging = -1;  // -1: from the environment; ddpx_f32_set_staging() overrides (tests, A/B)
static bool f32_dma() {
  if (g_f32_staging < 0) {
    const char* e = getenv("DDPX_F32_STAGING");
    g_f32_staging = (e && e[0] == 'r') ? 0 : 1;
  }
  return g_f32_staging == 1;
}
constexpr int kF32Stages = 4;
// Output stores of the LDS-DMA core: 16-B row vectors staged through LDS (default) or the fragment-order 4-B
// stores (DDPX_F32_EPI=scalar; A/B).  Bitwise the same results.
static bool f32_vec_epi() {
  static const bool v = [] {
    const char* e = getenv("DDPX_F32_EPI");
    return !(e && e[0] == 's');
  }();
  return v;
}
// Summation block of the LDS-DMA core's blocked mode, in 16-k K-steps (DDPX_F32_BLOCK=1|2|4, default 4): a fresh
// block accumulator per 64 k, added to the running sum.  Measured on MI355X (profiles/r4_f32): the rounding
// error of a length-K dot product is smallest near blocks of sqrt(K) (~64 at VGG's K = 2304-4608: conv7 / conv4
// outputs 0.26x MIOpen's own error vs fp64, against 0.42x / 0.37x with 16-k blocks), and the adds of fewer
// blocks cost less (VGG fp32 step 19.07 ms vs 21.35 ms with 16-k blocks).  1 = the register-staged kernel's
// exact summation order (bitwise equal to it).
static int g_f32_block = -1;
static int f32_block() {
  if (g_f32_block < 0) {
    const char* e = getenv("DDPX_F32_BLOCK");
    g_f32_block = (e && e[0] == '1') ? 1 : (e && e[0] == '2') ? 2 : (e && e[0] == '8') ? 8 : 4;
  }
  return g_f32_block;
}

template <int BM, int BN, int AM, int BMD>
static void launch(const Operand& A, const Operand& B, int M, int N, int K, int splits, float* C, int ldc,
                   long split_stride, const float* bias, const float* mask, int flags, hipStream_t s,
                   unsigned a_bytes, unsigned b_bytes, float* stats = nullptr, SgdArgs sgd = SgdArgs{}) {
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + BK - 1) / BK * BK;
  const int nwg = tm * tn * splits;
  const int mode = f32_sum_mode();
  const bool conv = AM == IM2COL_KC || BMD == IM2COL_OC;
  const bool plain = mode == 1 || (mode == 0 && !conv);
  if (f32_dma() && a_bytes && b_bytes) {
    const auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (f32_vec_epi() && N % 4 == 0 && ldc % 4 == 0 && split_stride % 4 == 0 && al16(C) && al16(bias) && al16(mask))
      flags |= F_VEC;
    if constexpr (AM == IM2COL_KC) {
      // the image's first convolution (K = 36: 3 K-steps): a 3-slot ring holds the whole K range, and the smaller
      // LDS footprint (48 KB at 128x128, not 64) fits 3 workgroups per CU instead of 2
      if (!plain && kchunk <= 3 * BK && f32_block() == 4 && f32_small_k_ring()) {
        hipLaunchKernelGGL((gemm_f32_dma_kernel<BM, BN, AM, BMD, false, 3, 4>), dim3(nwg), dim3(NT), 0, s, A, B, M, N,
                           K, kchunk, C, ldc, split_stride, bias, mask, flags, tm, tn, a_bytes, b_bytes, stats, sgd);
        return;
      }
    }
    if (plain)
      hipLaunchKernelGGL((gemm_f32_dma_kernel<BM, BN, AM, BMD, true, kF32Stages>), dim3(nwg), dim3(NT), 0, s, A, B, M,
                         N, K, kchunk, C, ldc, split_stride, bias, mask, flags, tm, tn, a_bytes, b_bytes, stats, sgd);
    else if (f32_block() == 2)
      hipLaunchKernelGGL((gemm_f32_dma_kernel<BM, BN, AM, BMD, false, kF32Stages, 2>), dim3(nwg), dim3(NT), 0, s, A,
                         B, M, N, K, kchunk, C, ldc, split_stride, bias, mask, flags, tm, tn, a_bytes, b_bytes, stats, sgd);
    else if (f32_block() == 4)
      hipLaunchKernelGGL((gemm_f32_dma_kernel<BM, BN, AM, BMD, false, kF32Stages, 4>), dim3(nwg), dim3(NT), 0, s, A,
                         B, M, N, K, kchunk, C, ldc, split_stride, bias, mask, flags, tm, tn, a_bytes, b_bytes, stats, sgd);
    else if (f32_block() == 8)
      hipLaunchKernelGGL((gemm_f32_dma_kernel<BM, BN, AM, BMD, false, kF32Stages, 8>), dim3(nwg), dim3(NT), 0, s, A,
                         B, M, N, K, kchunk, C, ldc, split_stride, bias, mask, flags, tm, tn, a_bytes, b_bytes, stats, sgd);
    else
      hipLaunchKernelGGL((gemm_f32_dma_kernel<BM, BN, AM, BMD, false, kF32Stages>), dim3(nwg), dim3(NT), 0, s, A, B,
                         M, N, K, kchunk, C, ldc, split_stride, bias, mask, flags, tm, tn, a_bytes, b_bytes, stats, sgd);
    return;
  }
  if (plain)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, AM, BMD, true>), dim3(nwg), dim3(NT), 0, s, A, B, M, N, K, kchunk, C,
                       ldc, split_stride, bias, mask, flags, tm, tn);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, AM, BMD, false>), dim3(nwg), dim3(NT), 0, s, A, B, M, N, K, kchunk, C,
                       ldc, split_stride, bias, mask, flags, tm, tn);
}

template <int AM, int BMD>
static void dispatch_tile(int tile, const Operand& A, const Operand& B, int M, int N, int K, int splits, float* C,
                          int ldc, long ss, const float* bias, const float* mask, int flags, hipStream_t s,
                          unsigned ab, unsigned bb, float* stats = nullptr, SgdArgs sgd = SgdArgs{}) {
  switch (tile) {
    case 0: launch<128, 128, AM, BMD>(A, B, M, N, K, splits, C, ldc, ss, bias, mask, flags, s, ab, bb, stats, sgd); break;
    case 1: launch<128, 64, AM, BMD>(A, B, M, N, K, splits, C, ldc, ss, bias, mask, flags, s, ab, bb, stats, sgd); break;
    case 3: launch<64, 128, AM, BMD>(A, B, M, N, K, splits, C, ldc, ss, bias, mask, flags, s, ab, bb, stats, sgd); break;
    default: launch<64, 64, AM, BMD>(A, B, M, N, K, splits, C, ldc, ss, bias, mask, flags, s, ab, bb, stats, sgd); break;
  }
}

// Bytes an operand spans (the LDS-DMA buffer resource's bound; 0 = too large for 32-bit offsets: register path)
static unsigned operand_bytes(int mode, int ld, int O, int K, int C, int npix) {
  size_t n;
  if (mode == DENSE_KC) n = ((size_t)(O - 1) * ld + K) * 4;
  else if (mode == DENSE_OC) n = ((size_t)(K - 1) * ld + O) * 4;
  else n = (size_t)npix * C * 4;
  return n >= 0x80000000ull ? 0u : (unsigned)n;
}

// ------------------------------------------------------------------ conv helpers
// Forward / data-gradient GEMM weights from torch's [Co][Ci][3][3] fp32 master:
//   wf[(r*3+s)*Cp + ci][co]  (Cp >= Ci zero-padded input channels)     — B of the forward
//   wd[(r*3+s)*Co + co][ci]  (only when wd != null)                     — B of the data gradient
__global__ void __launch_bounds__(256) wprep_kernel(const float* __restrict__ w, int Co, int Ci, int Cp,
                                                     float* __restrict__ wf, float* __restrict__ wd) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // over 9 * Cp * Co
  if (i >= 9 * Cp * Co) return;
  const int co = i % Co, k = i / Co, ci = k % Cp, rs = k / Cp;
  const float v = ci < Ci ? w[((size_t)co * Ci + ci) * 9 + rs] : 0.f;
  wf[i] = v;
  if (wd && ci < Ci) wd[((size_t)rs * Co + co) * Ci + ci] = v;
}

// grad[co][ci][r][s] (+)= sum_z part[z][co][(r*3+s)*Cp + ci]   (fixed order over z)
// Threads walk the slab layout (ci fastest: coalesced reads of every slab, 8 slabs' loads in flight) and scatter
// into torch's [Co][Ci][3][3] order; the sum over z runs in the same order as before (bitwise unchanged).
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ part, int S, int Co, int Ci,
                                                            int Cp, float* __restrict__ grad, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // over Co * 9 * Ci, slab order
  if (i >= Co * Ci * 9) return;
  const int ci = i % Ci, rs = (i / Ci) % 9, co = i / (9 * Ci);
  const size_t stride = (size_t)Co * 9 * Cp;
  const float* p = part + (size_t)co * 9 * Cp + rs * Cp + ci;
  float acc = 0.f;
  int z = 0;
  // 32 slabs' loads in flight: the first conv (3 input channels: 14 workgroups, 512 slabs) was latency-bound at
  // 8 (28 us in the DeepNN fp32 step); same adds in the same order
  for (; z + 32 <= S; z += 32) {
    float v[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) v[u] = p[(size_t)(z + u) * stride];
#pragma unroll
    for (int u = 0; u < 32; ++u) acc += v[u];
  }
  for (; z + 8 <= S; z += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(size_t)(z + u) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; z < S; ++z) acc += p[(size_t)z * stride];
  const size_t o = ((size_t)co * Ci + ci) * 9 + rs;
  grad[o] = accumulate ? grad[o] + acc : acc;
}

// out[i] (+)= sum_z part[z][i]
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ part, int S, long n,
                                                             float* __restrict__ out, int accumulate) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float acc = 0.f;
  for (int z = 0; z < S; ++z) acc += part[z * n + i];
  out[i] = accumulate ? out[i] + acc : acc;
}

// Split-K finish of a [M][N] fp32 GEMM with its epilogue: out = relu?(sum_z part[z] + bias[n]) * (mask > 0)?,
// 16-B vectors (N % 4 == 0), slabs summed in split order.
__global__ void __launch_bounds__(256) splitk_epi_kernel(const float* __restrict__ part, int S, int M, int N,
                                                          float* __restrict__ out, const float* __restrict__ bias,
                                                          const float* __restrict__ mask, int relu) {
  const long nv = (long)M * N / 4;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= nv) return;
  const long n4 = (long)M * N / 4;
  f32x4 acc = reinterpret_cast<const f32x4*>(part)[i];
  for (int z = 1; z < S; ++z) {
    const f32x4 v = reinterpret_cast<const f32x4*>(part)[z * n4 + i];
    acc += v;
  }
  const int col = (int)((i * 4) % N);
  f32x4 mk = {1.f, 1.f, 1.f, 1.f};
  if (mask) mk = reinterpret_cast<const f32x4*>(mask)[i];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float v = acc[q];
    if (bias) v += bias[col + q];
    if (relu) v = fmaxf(v, 0.f);
    if (mask && !(mk[q] > 0.f)) v = 0.f;
    acc[q] = v;
  }
  reinterpret_cast<f32x4*>(out)[i] = acc;
}

// ------------------------------------------------------------------ BatchNorm (NHWC [P][C], fp32)
// Threads: channel c = tid % C, row group g = tid / C (G = blockDim / C groups).  blockDim = max(256, C).
__device__ __forceinline__ float block_group_sum(float v, float* red, int C, int G, int tid) {
  red[tid] = v;
  __syncthreads();
  float s = 0.f;
  if (tid < C)
    for (int g = 0; g < G; ++g) s += red[g * C + tid];
  __syncthreads();
  return s;  // valid on tid < C
}

// part[t][0][c] = mean of chunk t, part[t][1][c] = M2 of chunk t (two passes over the L2-resident chunk)
__global__ void __launch_bounds__(512) bn_stats_kernel(const float* __restrict__ y, int P, int C, int R,
                                                        float* __restrict__ part) {
  __shared__ float red[512];
  __shared__ float bc[512];
  const int tid = threadIdx.x, c = tid % C, G = blockDim.x / C, g = tid / C;
  const int r0 = blockIdx.x * R, r1 = min(P, r0 + R);
  float s = 0.f;
  for (int r = r0 + g; r < r1; r += G) s += y[(size_t)r * C + c];
  s = block_group_sum(s, red, C, G, tid);
  if (tid < C) bc[tid] = s / (float)(r1 - r0);
  __syncthreads();
  const float mu = bc[c];
  float q = 0.f;
  for (int r = r0 + g; r < r1; r += G) {
    const float d = y[(size_t)r * C + c] - mu;
    q = fmaf(d, d, q);
  }
  q = block_group_sum(q, red, C, G, tid);
  if (tid < C) {
    part[(size_t)blockIdx.x * 2 * C + c] = mu;
    part[(size_t)blockIdx.x * 2 * C + C + c] = q;
  }
}

// Chan merge of the chunk statistics + running-stat update + affine coefficients a = gamma*rstd, b = beta.
// The normalisation is applied as a*(y - mean) + beta, not a*y + (beta - a*mean): the folded form cancels
// two terms of size |mean|/std and loses that many bits per layer.  Eval: running statistics.
// 1024 threads = 64 channels x 16 chunk groups per workgroup; fp64 merge, fixed order (deterministic).
__global__ void __launch_bounds__(1024) bn_finalize_kernel(const float* __restrict__ part, int T, int R, int P, int C,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            float* __restrict__ rmean, float* __restrict__ rvar,
                                                            int64_t* __restrict__ nbt, float momentum, float eps,
                                                            int training, float* __restrict__ a,
                                                            float* __restrict__ b, float* __restrict__ mean_out,
                                                            float* __restrict__ rstd_out) {
  __shared__ double red[16][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const bool ok = c < C;
  if (blockIdx.x == 0 && threadIdx.x == 0 && training && nbt) *nbt += 1;
  float mu = 0.f, var = 0.f;
  if (training) {
    double sm = 0.0;
    if (ok) {  // 8 chunks' loads in flight, summed in the same chunk order as one at a time
      int t = g;
      for (; t + 7 * 16 < T; t += 8 * 16) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(t + 16 * u) * 2 * C + c];
#pragma unroll
        for (int u = 0; u < 8; ++u) sm += (double)min(R, P - (t + 16 * u) * R) * v[u];
      }
      for (; t < T; t += 16) sm += (double)min(R, P - t * R) * part[(size_t)t * 2 * C + c];
    }
    red[g][cl] = sm;
    __syncthreads();
    double m = 0.0;
    for (int k = 0; k < 16; ++k) m += red[k][cl];
    m /= P;
    __syncthreads();
    double m2 = 0.0;
    if (ok) {
      int t = g;
      for (; t + 7 * 16 < T; t += 8 * 16) {
        float mv[8], qv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          mv[u] = part[(size_t)(t + 16 * u) * 2 * C + c];
          qv[u] = part[(size_t)(t + 16 * u) * 2 * C + C + c];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const double d = mv[u] - m;
          m2 += qv[u] + (double)min(R, P - (t + 16 * u) * R) * d * d;
        }
      }
      for (; t < T; t += 16) {
        const double d = part[(size_t)t * 2 * C + c] - m;
        m2 += part[(size_t)t * 2 * C + C + c] + (double)min(R, P - t * R) * d * d;
      }
    }
    red[g][cl] = m2;
    __syncthreads();
    m2 = 0.0;
    for (int k = 0; k < 16; ++k) m2 += red[k][cl];
    if (g != 0 || !ok) return;
    mu = (float)m;
    var = (float)(m2 / P);
    const float unb = P > 1 ? (float)(m2 / (P - 1)) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
  } else {
    if (g != 0 || !ok) return;
    mu = rmean[c];
    var = rvar[c];
  }
  const float rs = 1.f / sqrtf(var + eps);
  a[c] = gamma[c] * rs;
  b[c] = beta[c];
  mean_out[c] = mu;
  rstd_out[c] = rs;
}

// The same merge split over chunk ranges, for few channels and many chunks (VGG conv0 / conv1: C = 64 / 128,
// T = 2048 / 4096, one or two workgroups of the kernel above: 78 / 52 us).  Three launches: (1) per split the
// fp64 sum of n * mean; (2) the mean from all splits' sums (split order), then per split the fp64 M2 sum;
// (3) the M2 of all splits (split order) and the outputs.  Deterministic; within a split the same 16-group
// interleave as bn_finalize_kernel.  The per-split partials live in a caller-allocated fp64 workspace
// ws[2][kFinSplitMax][C] (stream-ordered by the caller's allocator: two merges in flight on different streams
// cannot overwrite each other's partials).
constexpr int kFinSplitMax = 32, kFinSplitMaxC = 1024;

// sum_{k < S} v[k * C + c] in k order, 8 loads in flight (the fp64 adds stay in order: deterministic)
__device__ __forceinline__ double fin_split_sum(const double* v, int S, int C, int c) {
  double r = 0.0;
  int k = 0;
  for (; k + 8 <= S; k += 8) {
    double t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = v[(size_t)(k + u) * C + c];
#pragma unroll
    for (int u = 0; u < 8; ++u) r += t[u];
  }
  for (; k < S; ++k) r += v[(size_t)k * C + c];
  return r;
}

__device__ __forceinline__ double fin_group_tree(double v, double (*red)[64], int g, int cl) {
  red[g][cl] = v;
  __syncthreads();
  double r = 0.0;
  for (int k = 0; k < 16; ++k) r += red[k][cl];
  return r;
}

__global__ void __launch_bounds__(1024) bn_fin_sum_kernel(const float* __restrict__ part, int T, int Ts, int R,
                                                           int P, int C, double* __restrict__ fin_s1) {
  __shared__ double red[16][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, sp = blockIdx.y;
  const int t0 = sp * Ts, t1 = min(T, t0 + Ts);
  double sm = 0.0;
  if (c < C) {
    int t = t0 + g;
    for (; t + 7 * 16 < t1; t += 8 * 16) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(t + 16 * u) * 2 * C + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) sm += (double)min(R, P - (t + 16 * u) * R) * v[u];
    }
    for (; t < t1; t += 16) sm += (double)min(R, P - t * R) * part[(size_t)t * 2 * C + c];
  }
  sm = fin_group_tree(sm, red, g, cl);
  if (g == 0 && c < C) fin_s1[(size_t)sp * C + c] = sm;
}

__global__ void __launch_bounds__(1024) bn_fin_m2_kernel(const float* __restrict__ part, int T, int Ts, int S, int R,
                                                          int P, int C, const double* __restrict__ fin_s1,
                                                          double* __restrict__ fin_s2) {
  __shared__ double red[16][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, sp = blockIdx.y;
  const int t0 = sp * Ts, t1 = min(T, t0 + Ts);
  double m2 = 0.0;
  if (c < C) {
    const double m = fin_split_sum(fin_s1, S, C, c) / P;
    int t = t0 + g;
    for (; t + 7 * 16 < t1; t += 8 * 16) {
      float mv[8], qv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        mv[u] = part[(size_t)(t + 16 * u) * 2 * C + c];
        qv[u] = part[(size_t)(t + 16 * u) * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const double d = mv[u] - m;
        m2 += qv[u] + (double)min(R, P - (t + 16 * u) * R) * d * d;
      }
    }
    for (; t < t1; t += 16) {
      const double d = part[(size_t)t * 2 * C + c] - m;
      m2 += part[(size_t)t * 2 * C + C + c] + (double)min(R, P - t * R) * d * d;
    }
  }
  m2 = fin_group_tree(m2, red, g, cl);
  if (g == 0 && c < C) fin_s2[(size_t)sp * C + c] = m2;
}

__global__ void __launch_bounds__(64) bn_fin_out_kernel(int S, int P, int C, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float* __restrict__ rmean,
                                                         float* __restrict__ rvar, int64_t* __restrict__ nbt,
                                                         float momentum, float eps, float* __restrict__ a,
                                                         float* __restrict__ b, float* __restrict__ mean_out,
                                                         float* __restrict__ rstd_out,
                                                         const double* __restrict__ fin_s1,
                                                         const double* __restrict__ fin_s2) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
  if (c >= C) return;
  const double m = fin_split_sum(fin_s1, S, C, c) / P;
  const double m2 = fin_split_sum(fin_s2, S, C, c);
  const float mu = (float)m, var = (float)(m2 / P);
  const float unb = P > 1 ? (float)(m2 / (P - 1)) : var;
  rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
  rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
  const float rs = 1.f / sqrtf(var + eps);
  a[c] = gamma[c] * rs;
  b[c] = beta[c];
  mean_out[c] = mu;
  rstd_out[c] = rs;
}

// out = [maxpool2](relu(a*(y - mean) + b)), 4 channels per thread
__global__ void __launch_bounds__(256) bn_apply_kernel(const float* __restrict__ y, const float* __restrict__ a,
                                                        const float* __restrict__ b, const float* __restrict__ mean,
                                                        int N, int H, int W, int C, int relu, int pool,
                                                        float* __restrict__ out) {
  const int Ho = pool ? H / 2 : H, Wo = pool ? W / 2 : W, C4 = C / 4;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * Ho * Wo * C4) return;
  const int c = (int)(i % C4) * 4;
  const long pix = i / C4;
  const int wo = (int)(pix % Wo), ho = (int)((pix / Wo) % Ho), n = (int)(pix / ((long)Wo * Ho));
  const f32x4 av = *reinterpret_cast<const f32x4*>(a + c), bv = *reinterpret_cast<const f32x4*>(b + c);
  const f32x4 mv = *reinterpret_cast<const f32x4*>(mean + c);
  f32x4 r;
  if (!pool) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(y + (size_t)pix * C + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float z = fmaf(av[e], v[e] - mv[e], bv[e]);
      r[e] = relu ? fmaxf(z, 0.f) : z;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = -INFINITY;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const size_t p = ((size_t)n * H + 2 * ho + dy) * W + 2 * wo + dx;
        const f32x4 v = *reinterpret_cast<const f32x4*>(y + p * C + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float z = fmaf(av[e], v[e] - mv[e], bv[e]);
          if (relu) z = fmaxf(z, 0.f);
          r[e] = fmaxf(r[e], z);
        }
      }
  }
  *reinterpret_cast<f32x4*>(out + (size_t)i * 4) = r;
}

// Gradient at pre-BN pixel (n,h,w,c) of the block output's gradient g: ReLU mask and the 2x2 max-pool routing
// (the FIRST maximum of the window in row-major order gets the gradient, as torch's max_pool2d backward).
__device__ __forceinline__ float routed_grad(const float* __restrict__ g, const float* __restrict__ y, float av,
                                             float bv, float mu, int n, int h, int w, int H, int W, int C, int c,
                                             int pool, float z) {
  if (!(z > 0.f)) return 0.f;  // ReLU(z) == 0: no gradient (torch threshold_backward)
  if (!pool) return g[(((size_t)n * H + h) * W + w) * C + c];
  const int h0 = h & ~1, w0 = w & ~1;
  int first = -1;
  float best = -INFINITY;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const size_t p = ((size_t)n * H + h0 + (q >> 1)) * W + w0 + (q & 1);
    const float zz = fmaxf(fmaf(av, y[p * C + c] - mu, bv), 0.f);
    if (zz > best) { best = zz; first = q; }
  }
  if (first != ((h - h0) << 1 | (w - w0))) return 0.f;
  return g[(((size_t)n * (H / 2) + (h >> 1)) * (W / 2) + (w >> 1)) * C + c];
}

// part[t][0][c] = sum gz, part[t][1][c] = sum gz * xhat over pixel chunk t
__global__ void __launch_bounds__(512) bn_bwd_sums_kernel(const float* __restrict__ g, const float* __restrict__ y,
                                                           const float* __restrict__ a, const float* __restrict__ b,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, int N, int H, int W, int C,
                                                           int pool, int R, float* __restrict__ part) {
  __shared__ float red[512];
  const int tid = threadIdx.x, c = tid % C, G = blockDim.x / C, gi = tid / C;
  const int P = N * H * W;
  const int r0 = blockIdx.x * R, r1 = min(P, r0 + R);
  const float av = a[c], bv = b[c], mu = mean[c], rs = rstd[c];
  float s1 = 0.f, s2 = 0.f;
  for (int r = r0 + gi; r < r1; r += G) {
    const int w = r % W, h = (r / W) % H, n = r / (W * H);
    const float yv = y[(size_t)r * C + c];
    const float gz = routed_grad(g, y, av, bv, mu, n, h, w, H, W, C, c, pool, fmaf(av, yv - mu, bv));
    s1 += gz;
    s2 = fmaf(gz, (yv - mu) * rs, s2);
  }
  s1 = block_group_sum(s1, red, C, G, tid);
  s2 = block_group_sum(s2, red, C, G, tid);
  if (tid < C) {
    part[(size_t)blockIdx.x * 2 * C + c] = s1;
    part[(size_t)blockIdx.x * 2 * C + C + c] = s2;
  }
}

// c1 = sum gz / P, c2 = sum gz*xhat / P;  dgamma (+)= sum gz*xhat, dbeta (+)= sum gz
// (64 channels x 16 chunk groups per workgroup, fp64, fixed order)
__global__ void __launch_bounds__(1024) bn_bwd_finalize_kernel(const float* __restrict__ part, int T, int P, int C,
                                                                float* __restrict__ c1, float* __restrict__ c2,
                                                                float* __restrict__ dgamma,
                                                                float* __restrict__ dbeta, int accumulate) {
  __shared__ double red[2][16][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {  // 8 chunks' loads in flight, same summation order
    int t = g;
    for (; t + 7 * 16 < T; t += 8 * 16) {
      float v1[8], v2[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v1[u] = part[(size_t)(t + 16 * u) * 2 * C + c];
        v2[u] = part[(size_t)(t + 16 * u) * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s1 += v1[u];
        s2 += v2[u];
      }
    }
    for (; t < T; t += 16) {
      s1 += part[(size_t)t * 2 * C + c];
      s2 += part[(size_t)t * 2 * C + C + c];
    }
  }
  red[0][g][cl] = s1;
  red[1][g][cl] = s2;
  __syncthreads();
  if (g != 0 || c >= C) return;
  s1 = s2 = 0.0;
  for (int k = 0; k < 16; ++k) {
    s1 += red[0][k][cl];
    s2 += red[1][k][cl];
  }
  c1[c] = (float)(s1 / P);
  c2[c] = (float)(s2 / P);
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)s2 : (float)s2;
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)s1 : (float)s1;
}

// The same sums split over chunk ranges for few channel groups and many chunks (BN0's 64 channels x 2048 chunks
// took 29 us in one workgroup): per split, the 16-group interleave and tree of bn_bwd_finalize_kernel into the
// split scratch; then the splits in order (bn_bwd_fin_out_kernel).  Deterministic.
__global__ void __launch_bounds__(1024) bn_bwd_fin_sum_kernel(const float* __restrict__ part, int T, int Ts, int C,
                                                               double* __restrict__ fin_s1,
                                                               double* __restrict__ fin_s2) {
  __shared__ double red[2][16][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, sp = blockIdx.y;
  const int t0 = sp * Ts, t1 = min(T, t0 + Ts);
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    int t = t0 + g;
    for (; t + 7 * 16 < t1; t += 8 * 16) {
      float v1[8], v2[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v1[u] = part[(size_t)(t + 16 * u) * 2 * C + c];
        v2[u] = part[(size_t)(t + 16 * u) * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s1 += v1[u];
        s2 += v2[u];
      }
    }
    for (; t < t1; t += 16) {
      s1 += part[(size_t)t * 2 * C + c];
      s2 += part[(size_t)t * 2 * C + C + c];
    }
  }
  red[0][g][cl] = s1;
  red[1][g][cl] = s2;
  __syncthreads();
  if (g != 0 || c >= C) return;
  s1 = s2 = 0.0;
  for (int k = 0; k < 16; ++k) {
    s1 += red[0][k][cl];
    s2 += red[1][k][cl];
  }
  fin_s1[(size_t)sp * C + c] = s1;
  fin_s2[(size_t)sp * C + c] = s2;
}

__global__ void __launch_bounds__(64) bn_bwd_fin_out_kernel(int S, int P, int C, float* __restrict__ c1,
                                                             float* __restrict__ c2, float* __restrict__ dgamma,
                                                             float* __restrict__ dbeta, int accumulate,
                                                             const double* __restrict__ fin_s1,
                                                             const double* __restrict__ fin_s2) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= C) return;
  const double s1 = fin_split_sum(fin_s1, S, C, c), s2 = fin_split_sum(fin_s2, S, C, c);
  c1[c] = (float)(s1 / P);
  c2[c] = (float)(s2 / P);
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)s2 : (float)s2;
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)s1 : (float)s1;
}

// dy = a * (gz - c1 - xhat * c2)
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const float* __restrict__ g, const float* __restrict__ y,
                                                            const float* __restrict__ a, const float* __restrict__ b,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const float* __restrict__ c1, const float* __restrict__ c2,
                                                            int N, int H, int W, int C, int pool,
                                                            float* __restrict__ dy) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * H * W * C) return;
  const int c = (int)(i % C);
  const long r = i / C;
  const int w = (int)(r % W), h = (int)((r / W) % H), n = (int)(r / ((long)W * H));
  const float av = a[c], bv = b[c], mu = mean[c], yv = y[i];
  const float gz = routed_grad(g, y, av, bv, mu, n, h, w, H, W, C, c, pool, fmaf(av, yv - mu, bv));
  const float xh = (yv - mu) * rstd[c];
  dy[i] = av * (gz - c1[c] - xh * c2[c]);
}

// Vectorised BatchNorm(+ReLU+MaxPool) backward: a thread owns 4 channels of one "unit" — a 2x2 pool window (its 4
// pre-pool pixels and its pooled gradient are read once, 16-B accesses) or, without a pool, one pixel.  The
// per-element kernels above re-read the whole window for every pixel (4x the loads) and moved 4 B per access.
// Same routing (first maximum in row-major window order) and ReLU mask as routed_grad.
struct Win4 {
  f32x4 gz[4], xh[4];
};

__device__ __forceinline__ Win4 window_grads(const float* __restrict__ g, const float* __restrict__ y, f32x4 av,
                                             f32x4 bv, f32x4 mu, f32x4 rs, size_t pix0, int W, size_t gpix, int C,
                                             int c, int pool) {
  Win4 o;
  const int nq = pool ? 4 : 1;
  f32x4 yv[4], pre[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q < nq) {
      const size_t pp = pix0 + (size_t)(q >> 1) * W + (q & 1);
      yv[q] = *reinterpret_cast<const f32x4*>(y + pp * C + c);
    } else {
      yv[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  }
  const f32x4 gv = *reinterpret_cast<const f32x4*>(g + gpix * C + c);
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      pre[q][e] = fmaf(av[e], yv[q][e] - mu[e], bv[e]);
      o.xh[q][e] = (yv[q][e] - mu[e]) * rs[e];
    }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    int first = 0;
    if (pool) {
      float best = -INFINITY;
      first = -1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float zz = fmaxf(pre[q][e], 0.f);
        if (zz > best) { best = zz; first = q; }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) o.gz[q][e] = (q < nq && q == first && pre[q][e] > 0.f) ? gv[e] : 0.f;
  }
  return o;
}

// unit u of the tensor -> its first pre-pool pixel and its gradient pixel
__device__ __forceinline__ void unit_pixels(long u, int H, int W, int pool, size_t& pix0, size_t& gpix) {
  if (!pool) {
    pix0 = gpix = (size_t)u;
    return;
  }
  const int Wo = W / 2, Ho = H / 2;
  const int wo = (int)(u % Wo);
  const long r = u / Wo;
  const int ho = (int)(r % Ho);
  const long n = r / Ho;
  pix0 = ((size_t)n * H + 2 * ho) * W + 2 * wo;
  gpix = (size_t)u;
}

// part[t][0][c] = sum gz, part[t][1][c] = sum gz * xhat over the units of chunk t (R pre-pool pixels, a multiple
// of 2W when pooled: whole window rows).  256 threads = (C/4 channel quads) x G unit groups, fixed order.
__global__ void __launch_bounds__(256) bn_bwd_sums4_kernel(const float* __restrict__ g, const float* __restrict__ y,
                                                            const float* __restrict__ a, const float* __restrict__ b,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, int N, int H, int W, int C,
                                                            int pool, int R, float* __restrict__ part,
                                                            float* __restrict__ dyw) {
  // dyw (bias + activation only: a = 1, mean = 0, rstd = 1, c1 = c2 = 0): dy = gz needs no sums, so this pass writes
  // it too and bn_bwd_apply4_kernel's second read of g and y goes away (DeepNN fp32's pooled blocks)
  __shared__ f32x4 red[2][256];
  const int tid = threadIdx.x, C4 = C / 4, cq = tid % C4, gi = tid / C4, G = 256 / C4;
  const int c = 4 * cq;
  const long P = (long)N * H * W;
  const long r0 = (long)blockIdx.x * R, r1 = min(P, r0 + (long)R);
  const long u0 = pool ? r0 / 4 : r0, u1 = pool ? r1 / 4 : r1;  // windows: 4 pixels each, chunks window-aligned
  const f32x4 av = *reinterpret_cast<const f32x4*>(a + c), bv = *reinterpret_cast<const f32x4*>(b + c);
  const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + c), rs = *reinterpret_cast<const f32x4*>(rstd + c);
  f32x4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
  for (long u = u0 + gi; u < u1; u += G) {
    size_t pix0, gpix;
    unit_pixels(u, H, W, pool, pix0, gpix);
    const Win4 w = window_grads(g, y, av, bv, mu, rs, pix0, W, gpix, C, c, pool);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s1[e] += w.gz[q][e];
        s2[e] = fmaf(w.gz[q][e], w.xh[q][e], s2[e]);
      }
    if (dyw) {
      const int nq = pool ? 4 : 1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q >= nq) break;
        const size_t pp = pix0 + (size_t)(q >> 1) * W + (q & 1);
        *reinterpret_cast<f32x4*>(dyw + pp * C + c) = (f32x4){w.gz[q][0], w.gz[q][1], w.gz[q][2], w.gz[q][3]};
      }
    }
  }
  red[0][tid] = s1;
  red[1][tid] = s2;
  __syncthreads();
  if (gi == 0) {
    f32x4 t1 = {0.f, 0.f, 0.f, 0.f}, t2 = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < G; ++k) {
      t1 += red[0][k * C4 + cq];
      t2 += red[1][k * C4 + cq];
    }
    *reinterpret_cast<f32x4*>(part + (size_t)blockIdx.x * 2 * C + c) = t1;
    *reinterpret_cast<f32x4*>(part + (size_t)blockIdx.x * 2 * C + C + c) = t2;
  }
}

// dy = a * (gz - c1 - xhat * c2) for every pixel of one unit (window or pixel), 4 channels, 16-B stores.
__global__ void __launch_bounds__(256) bn_bwd_apply4_kernel(const float* __restrict__ g, const float* __restrict__ y,
                                                             const float* __restrict__ a, const float* __restrict__ b,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ c1, const float* __restrict__ c2,
                                                             int N, int H, int W, int C, int pool,
                                                             float* __restrict__ dy) {
  const int C4 = C / 4;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long units = pool ? (long)N * (H / 2) * (W / 2) : (long)N * H * W;
  if (i >= units * C4) return;
  const int c = (int)(i % C4) * 4;
  const long u = i / C4;
  size_t pix0, gpix;
  unit_pixels(u, H, W, pool, pix0, gpix);
  const f32x4 av = *reinterpret_cast<const f32x4*>(a + c), bv = *reinterpret_cast<const f32x4*>(b + c);
  const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + c), rs = *reinterpret_cast<const f32x4*>(rstd + c);
  const f32x4 k1 = *reinterpret_cast<const f32x4*>(c1 + c), k2 = *reinterpret_cast<const f32x4*>(c2 + c);
  const Win4 w = window_grads(g, y, av, bv, mu, rs, pix0, W, gpix, C, c, pool);
  const int nq = pool ? 4 : 1;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q >= nq) break;
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = av[e] * (w.gz[q][e] - k1[e] - w.xh[q][e] * k2[e]);
    const size_t pp = pix0 + (size_t)(q >> 1) * W + (q & 1);
    *reinterpret_cast<f32x4*>(dy + pp * C + c) = o;
  }
}

// ------------------------------------------------------------------ pooling / head
__global__ void __launch_bounds__(256) avgpool_kernel(const float* __restrict__ x, int N, int S, int C,
                                                       float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i % C;
  float s = 0.f;
  for (int k = 0; k < S; ++k) s += x[((size_t)n * S + k) * C + c];
  out[i] = s / (float)S;
}

__global__ void __launch_bounds__(256) avgpool_bwd_kernel(const float* __restrict__ g, int N, int S, int C,
                                                           float* __restrict__ dx) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * S * C) return;
  const int c = (int)(i % C);
  const long n = i / ((long)S * C);
  dx[i] = g[n * C + c] / (float)S;
}

// logits[m][j] = h[m] . w[j] + bias[j]: one wave per row, lanes stride K with 16-B loads and keep all NC (<= 16)
// class sums, then one wave reduction per class (the head is far below MFMA size; h is read once).
constexpr int kMaxNC = 16;
__global__ void __launch_bounds__(256) head_logits_kernel(const float* __restrict__ h, const float* __restrict__ w,
                                                           const float* __restrict__ bias, int M, int K, int NC,
                                                           float* __restrict__ logits) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  float acc[kMaxNC];
#pragma unroll
  for (int j = 0; j < kMaxNC; ++j) acc[j] = 0.f;
  const f32x4* hp = reinterpret_cast<const f32x4*>(h + (size_t)m * K);
  for (int k4 = lane; k4 < K / 4; k4 += 64) {
    const f32x4 x = hp[k4];
#pragma unroll
    for (int j = 0; j < kMaxNC; ++j) {
      if (j >= NC) break;
      const f32x4 y = reinterpret_cast<const f32x4*>(w + (size_t)j * K)[k4];
      acc[j] = fmaf(x[0], y[0], fmaf(x[1], y[1], fmaf(x[2], y[2], fmaf(x[3], y[3], acc[j]))));
    }
  }
#pragma unroll
  for (int j = 0; j < kMaxNC; ++j) {
    if (j >= NC) break;
    const float v = wave_sum(acc[j]);
    if (lane == 0) logits[(size_t)m * NC + j] = v + bias[j];
  }
}

// The reference's 10-class head: one workgroup per row, the row's K / 4 vectors split over 256 threads with
// every load issued before the FMAs, then a wave + workgroup reduction in fixed order.  (One wave per row
// walking 16 dependent K-steps ran 63 us at M = 512, K = 4096: profiles/r3_models.)
template <int NC>
__global__ void __launch_bounds__(256) head_logits_row_kernel(const float* __restrict__ h, const float* __restrict__ w,
                                                              const float* __restrict__ bias, int K,
                                                              float* __restrict__ logits) {
  __shared__ float red[4][NC];
  const int m = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int K4 = K / 4;
  float acc[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) acc[j] = 0.f;
  const f32x4* hp = reinterpret_cast<const f32x4*>(h + (size_t)m * K);
  for (int k0 = tid; k0 < K4; k0 += 4 * 256) {
    f32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = k0 + u * 256 < K4 ? hp[k0 + u * 256] : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const f32x4* wp = reinterpret_cast<const f32x4*>(w + (size_t)j * K);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4 y = k0 + u * 256 < K4 ? wp[k0 + u * 256] : (f32x4){0.f, 0.f, 0.f, 0.f};
        acc[j] = fmaf(x[u][0], y[0], fmaf(x[u][1], y[1], fmaf(x[u][2], y[2], fmaf(x[u][3], y[3], acc[j]))));
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const float v = wave_sum(acc[j]);
    if (lane == 0) red[wv][j] = v;
  }
  __syncthreads();
  if (tid < NC) logits[(size_t)m * NC + tid] = ((red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid])) + bias[tid];
}

// One workgroup: per-row log-softmax, loss = mean_m (lse - logit[target]), dl = (softmax - onehot) / M.
__global__ void __launch_bounds__(1024) xent_kernel(const float* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                     int M, int NC, float* __restrict__ loss,
                                                     float* __restrict__ dl) {
  __shared__ float red[1024];
  const int tid = threadIdx.x;
  float acc = 0.f;
  for (int m = tid; m < M; m += 1024) {
    const float* l = logits + (size_t)m * NC;
    float mx = -INFINITY;
    for (int j = 0; j < NC; ++j) mx = fmaxf(mx, l[j]);
    float se = 0.f;
    for (int j = 0; j < NC; ++j) se += expf(l[j] - mx);
    const float lse = mx + logf(se);
    const int t = (int)tgt[m];
    acc += lse - l[t];
    if (dl)
      for (int j = 0; j < NC; ++j) dl[(size_t)m * NC + j] = (expf(l[j] - lse) - (j == t ? 1.f : 0.f)) / (float)M;
  }
  red[tid] = acc;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0 && loss) *loss = red[0] / (float)M;
}

// dW[j][k] (+)= go * sum_m dl[m][j] h[m][k];  db[j] (+)= go * sum_m dl[m][j]
// Workgroups of 64 columns k x 16 row groups (h read once, coalesced; all NC classes per thread), fixed-order
// LDS reduction over the row groups; the last workgroup also sums db (one wave per class).
constexpr int kHeadDlLds = 8192;  // floats of dlogits staged in LDS (M * NC; 512 x 10 at the reference's batch)
__global__ void __launch_bounds__(1024) head_wgrad_kernel(const float* __restrict__ dl, const float* __restrict__ go,
                                                           const float* __restrict__ h, int M, int K, int NC,
                                                           float* __restrict__ dW, float* __restrict__ db,
                                                           int accumulate) {
  __shared__ float red[16][kMaxNC][64];
  const float s = go ? *go : 1.f;
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  if (blockIdx.x == gridDim.x - 1) {  // bias gradient
    if (g < NC && db) {
      float acc = 0.f;
      for (int m = cl; m < M; m += 64) acc += dl[(size_t)m * NC + g];
      acc = wave_sum(acc) * s;
      if (cl == 0) db[g] = accumulate ? db[g] + acc : acc;
    }
    return;
  }
  const int k = blockIdx.x * 64 + cl;
  float acc[kMaxNC];
#pragma unroll
  for (int j = 0; j < kMaxNC; ++j) acc[j] = 0.f;
  // dlogits staged in LDS once per workgroup (every wave reads every row of it: broadcast LDS reads instead of
  // 10 global loads per row per lane)
  __shared__ float dls[kHeadDlLds];
  auto rows = [&](const auto* dsrc) {
    // 8 rows' loads in flight per thread (a dependent load per row was latency bound: 35 us at M = 512)
    int m = g;
    for (; m + 7 * 16 < M; m += 8 * 16) {
      float hv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) hv[u] = h[(size_t)(m + u * 16) * K + k];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < kMaxNC; ++j) {
          if (j >= NC) break;
          acc[j] = fmaf(dsrc[(size_t)(m + u * 16) * NC + j], hv[u], acc[j]);
        }
    }
    for (; m < M; m += 16) {
      const float hv = h[(size_t)m * K + k];
#pragma unroll
      for (int j = 0; j < kMaxNC; ++j) {
        if (j >= NC) break;
        acc[j] = fmaf(dsrc[(size_t)m * NC + j], hv, acc[j]);
      }
    }
  };
  if (M * NC <= kHeadDlLds) {
    for (int i = threadIdx.x; i < M * NC; i += 1024) dls[i] = dl[i];
    __syncthreads();
    if (k < K) rows(dls);
  } else if (k < K) {
    rows(dl);
  }
#pragma unroll
  for (int j = 0; j < kMaxNC; ++j) red[g][j][cl] = acc[j];
  __syncthreads();
  if (g < NC && k < K) {
    float t = 0.f;
    for (int q = 0; q < 16; ++q) t += red[q][g][cl];
    t *= s;
    const size_t o = (size_t)g * K + k;
    dW[o] = accumulate ? dW[o] + t : t;
  }
}

// dh[m][k] = go * dh_scale * sum_j dl[m][j] w[j][k]   [* (h[m][k] > 0)]
// (dh_scale = 1/(1-p) when h is the output of an inverted Dropout(p) after a ReLU: h > 0 is then exactly "kept
// and positive", so the dropout + ReLU backward costs nothing extra; 1 otherwise)
__global__ void __launch_bounds__(256) head_dgrad_kernel(const float* __restrict__ dl, const float* __restrict__ go,
                                                          const float* __restrict__ w, const float* __restrict__ h,
                                                          int M, int K, int NC, int relu_mask, float dh_scale,
                                                          float* __restrict__ dh) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)M * K) return;
  const int m = (int)(i / K), k = (int)(i % K);
  float acc = 0.f;
  for (int j = 0; j < NC; ++j) acc = fmaf(dl[(size_t)m * NC + j], w[(size_t)j * K + k], acc);
  acc *= (go ? *go : 1.f) * dh_scale;
  if (relu_mask && !(h[i] > 0.f)) acc = 0.f;
  dh[i] = acc;
}

// Same as head_dgrad_kernel with 4 consecutive columns per thread (16-B loads / stores of w, h, dh); the sum over
// the classes runs in the same order, so the result is bitwise that of the scalar kernel.
__global__ void __launch_bounds__(256) head_dgrad4_kernel(const float* __restrict__ dl, const float* __restrict__ go,
                                                           const float* __restrict__ w, const float* __restrict__ h,
                                                           int M, int K, int NC, int relu_mask, float dh_scale,
                                                           float* __restrict__ dh) {
  const long i4 = (long)blockIdx.x * 256 + threadIdx.x;
  const int K4 = K / 4;
  if (i4 >= (long)M * K4) return;
  const int m = (int)(i4 / K4), k4 = (int)(i4 % K4);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < NC; ++j) {
    const float d = dl[(size_t)m * NC + j];
    const f32x4 wv = reinterpret_cast<const f32x4*>(w + (size_t)j * K)[k4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = fmaf(d, wv[q], acc[q]);
  }
  const float g = (go ? *go : 1.f) * dh_scale;
  const f32x4 hv = reinterpret_cast<const f32x4*>(h + (size_t)m * K)[k4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    acc[q] *= g;
    if (relu_mask && !(hv[q] > 0.f)) acc[q] = 0.f;
  }
  reinterpret_cast<f32x4*>(dh + (size_t)m * K)[k4] = acc;
}

// out[n] (+)= sum_m x[m][n]: workgroups of 64 columns x 16 row groups, fixed-order LDS reduction
// part[t][0][c] = sum of x[r][c] over chunk t's R rows, part[t][1][c] = 0 (the [T][2][C] layout
// ddpx_f32_bn_bwd_finalize merges in fixed order): the bias gradient of a conv + ReLU block whose data gradient
// was masked by the producing GEMM.  C / 4 lanes per row (16-B loads), 256 / (C / 4) rows in parallel, their
// partial sums combined in row-lane order (deterministic).
__global__ void __launch_bounds__(256) colsum_part_kernel(const float* __restrict__ x, int P, int C, int R,
                                                          float* __restrict__ part) {
  __shared__ f32x4 red[256];
  const int Q = C / 4, RP = 256 / Q;
  const int q = threadIdx.x % Q, rl = threadIdx.x / Q;
  const int r0 = blockIdx.x * R, r1 = min(P, r0 + R);
  f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (rl < RP) {
    int r = r0 + rl;
    for (; r + 3 * RP < r1; r += 4 * RP) {
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f32x4*>(x + (size_t)(r + u * RP) * C + 4 * q);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc += v[u];
    }
    for (; r < r1; r += RP) acc += *reinterpret_cast<const f32x4*>(x + (size_t)r * C + 4 * q);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x < Q) {
    f32x4 t = red[threadIdx.x];
    for (int j = 1; j < RP; ++j) t += red[j * Q + threadIdx.x];
    *reinterpret_cast<f32x4*>(part + (size_t)blockIdx.x * 2 * C + 4 * threadIdx.x) = t;
    *reinterpret_cast<f32x4*>(part + (size_t)blockIdx.x * 2 * C + C + 4 * threadIdx.x) = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
}

__global__ void __launch_bounds__(1024) colsum_kernel(const float* __restrict__ x, int M, int N,
                                                       float* __restrict__ out, int accumulate) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + cl;
  float acc = 0.f;
  if (n < N) {
    // 8 rows' loads in flight, summed in the same row order as one at a time (bitwise unchanged)
    int m = g;
    for (; m + 7 * 16 < M; m += 8 * 16) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = x[(size_t)(m + u * 16) * N + n];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; m < M; m += 16) acc += x[(size_t)m * N + n];
  }
  red[g][cl] = acc;
  __syncthreads();
  if (g == 0 && n < N) {
    float t = 0.f;
    for (int q = 0; q < 16; ++q) t += red[q][cl];
    out[n] = accumulate ? out[n] + t : t;
  }
}

// torch.flatten(x, 1) of an NCHW activation held as NHWC: out[n][c * S + s] = x[n][s][c] (backward = 0), or the
// inverse for its gradient: out[n][s][c] = x[n][c * S + s] (backward = 1).  One thread per element, the NHWC
// side read / written contiguously.
__global__ void __launch_bounds__(256) nchw_flatten_kernel(const float* __restrict__ x, int N, int S, int C,
                                                            int backward, float* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;  // NHWC index
  if (i >= (long)N * S * C) return;
  const int c = (int)(i % C);
  const long r = i / C;
  const int sp = (int)(r % S);
  const long n = r / S;
  const size_t f = (size_t)n * S * C + (size_t)c * S + sp;
  if (backward) out[i] = x[f];
  else out[f] = x[i];
}

// bf16 version for the native DeepNN's classifier input (2048 = 32 channels x 8 x 8 features per image): one
// workgroup per image stages the image's S x C values in LDS, so both the NHWC side and the (C, H, W) side are
// read / written contiguously (2-byte elements).  S * C <= kFlatLds.
constexpr int kFlatLds = 16384;
__global__ void __launch_bounds__(256) nchw_flatten_bf16_kernel(const unsigned short* __restrict__ x, int S, int C,
                                                                 int backward, unsigned short* __restrict__ out) {
  __shared__ unsigned short img[kFlatLds];
  const int SC = S * C;
  const size_t base = (size_t)blockIdx.x * SC;
  for (int i = threadIdx.x; i < SC; i += 256) img[i] = x[base + i];
  __syncthreads();
  for (int j = threadIdx.x; j < SC; j += 256) {
    if (backward) {  // out NHWC j = s * C + c  <-  x (C, S) order c * S + s
      const int sp = j / C, c = j - sp * C;
      out[base + j] = img[c * S + sp];
    } else {         // out (C, S) order j = c * S + s  <-  x NHWC s * C + c
      const int c = j / S, sp = j - c * S;
      out[base + j] = img[sp * C + c];
    }
  }
}

// 0 = 128x128, 1 = 128x64, 2 = 64x64, 3 = 64x128.  Thin operands get the tile that does not compute padding:
// M <= 64 (the weight gradients of 64-channel layers: M = Co) takes 64-row tiles.
static int auto_tile(int M, int N, int splits) {
  if (M <= 64) return N <= 64 ? 2 : 3;
  const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128) * splits;
  return N <= 64 ? 1 : (t128 >= 512 ? 0 : 2);
}

static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return (1 << l) == v ? l : -1;
}

}  // namespace f32k
}  // namespace ddpx

using namespace ddpx;
using namespace ddpx::f32k;

static inline unsigned nblk(long n, int b = 256) { return (unsigned)((n + b - 1) / b); }

// C (+)= A B on the f32 MFMA core.  amode/bmode: Mode; conv geometry (C, H, W of the NHWC tensor an
// IM2COL operand reads, and the tap sign) applies to whichever operand is IM2COL.  splits > 1: raw partial
// slabs C + z*split_stride (no epilogue).  tile: 0 = 128x128, 1 = 128x64, 2 = 64x64, 3 = 64x128, -1 = auto.
DDPX_API int ddpx_f32_gemm(int amode, const float* a, int lda, int bmode, const float* b, int ldb, int M, int N, int K,
                           int gc, int gh, int gw, int sgn, int splits, float* c, int ldc, int64_t split_stride,
                           const float* bias, const float* mask, int flags, int tile, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  const bool kc = amode == DENSE_KC || amode == IM2COL_KC || bmode == DENSE_KC;
  if ((kc && K % 4) || splits < 1) return -1;  // k-contiguous operands load 4 consecutive k
  const bool im = amode >= IM2COL_KC || bmode >= IM2COL_KC;
  int lc = 0, lh = 0, lw = 0;
  if (im) {
    lc = ilog2(gc), lh = ilog2(gh), lw = ilog2(gw);
    if (lc < 2 || lh < 0 || lw < 0) return -2;  // channels: power of two >= 4 (16-B taps)
    if ((amode == IM2COL_KC && K != 9 * gc) || (bmode == IM2COL_OC && N != 9 * gc)) return -2;
  }
  if ((amode == DENSE_OC && M % 4) || (bmode == DENSE_OC && N % 4) || (bmode == IM2COL_OC && N % 4)) return -3;
  if ((amode == DENSE_KC && lda % 4) || (bmode == DENSE_KC && ldb % 4) || (amode == DENSE_OC && lda % 4) ||
      (bmode == DENSE_OC && ldb % 4))
    return -4;
  if (splits > 1) flags |= F_SPLIT;
  Operand A{a, lda, M, lc, lh, lw, sgn}, B{b, ldb, N, lc, lh, lw, sgn};
  const unsigned ab = operand_bytes(amode, lda, M, K, gc, M), bb = operand_bytes(bmode, ldb, N, K, gc, K);
  if (tile < 0) {
    tile = auto_tile(M, N, splits);
    // first convolution (K <= 48, 3-slot ring): 128x64 tiles, 105 vs 128 us at 3 -> 128 channels, batch 512
    // (benchmarks/f32_first_conv_probe.py, profiles/r6_f32epi)
    if (amode == IM2COL_KC && K <= 3 * BK && splits == 1 && tile == 0) tile = 1;
  }
  const int key = amode * 4 + bmode;
  switch (key) {
    case DENSE_KC * 4 + DENSE_KC:
      dispatch_tile<DENSE_KC, DENSE_KC>(tile, A, B, M, N, K, splits, c, ldc, split_stride, bias, mask, flags, s, ab,
                                          bb);
      break;
    case DENSE_KC * 4 + DENSE_OC:
      dispatch_tile<DENSE_KC, DENSE_OC>(tile, A, B, M, N, K, splits, c, ldc, split_stride, bias, mask, flags, s, ab,
                                          bb);
      break;
    case DENSE_OC * 4 + DENSE_OC:
      dispatch_tile<DENSE_OC, DENSE_OC>(tile, A, B, M, N, K, splits, c, ldc, split_stride, bias, mask, flags, s, ab,
                                          bb);
      break;
    case IM2COL_KC * 4 + DENSE_OC:
      dispatch_tile<IM2COL_KC, DENSE_OC>(tile, A, B, M, N, K, splits, c, ldc, split_stride, bias, mask, flags, s, ab,
                                          bb);
      break;
    case DENSE_OC * 4 + IM2COL_OC:
      dispatch_tile<DENSE_OC, IM2COL_OC>(tile, A, B, M, N, K, splits, c, ldc, split_stride, bias, mask, flags, s, ab,
                                          bb);
      break;
    default:
      return -5;
  }
  return (int)hipGetLastError();
}

// Weight gradient dW [N][K] = dy^T x (dy [M][N], x [M][K], both DENSE_OC) applied straight to the parameter by an
// SGD epilogue (single process, SGD(fused_backward)): no gradient stored.  LDS-DMA core only (-6 otherwise).
DDPX_API int ddpx_f32_wgrad_sgd(const float* dy, int ldy, const float* x, int ldx, int M, int N, int K, int tile,
                                float* sgd_p, float* sgd_buf, void* sgd_shadow, const float* lr, float mom, float wd,
                                hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (!f32_dma()) return -6;
  if (!sgd_p || !lr || (mom != 0.f && !sgd_buf)) return -1;
  if (N % 4 || K % 4 || ldy % 4 || ldx % 4) return -3;
  // output [N rows][K cols]: A = dy^T (rows = N, reduction = M), B = x (cols = K)
  Operand A{dy, ldy, N, 0, 0, 0, 1}, B{x, ldx, K, 0, 0, 0, 1};
  const unsigned ab = operand_bytes(DENSE_OC, ldy, N, M, 0, 0), bb = operand_bytes(DENSE_OC, ldx, K, M, 0, 0);
  if (!ab || !bb) return -4;
  if (tile < 0) tile = auto_tile(N, K, 1);
  dispatch_tile<DENSE_OC, DENSE_OC>(tile, A, B, N, K, M, 1, sgd_p, K, 0, nullptr, nullptr, 0, s, ab, bb, nullptr,
                                    SgdArgs{sgd_p, sgd_buf, (unsigned short*)sgd_shadow, lr, mom, wd});
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_splitk_reduce(const float* part, int S, int64_t n, float* out, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(nblk(n)), dim3(256), 0, s, part, S, (long)n, out, accumulate);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_splitk_epi(const float* part, int S, int M, int N, float* out, const float* bias,
                                 const float* mask, int relu, hipStream_t s) {
  if (N % 4 || S < 1) return -1;
  const long nv = (long)M * N / 4;
  hipLaunchKernelGGL(splitk_epi_kernel, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, part, S, M, N, out, bias,
                     mask, relu);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_conv_wprep(const float* w, int Co, int Ci, int Cp, float* wf, float* wd, hipStream_t s) {
  if (Cp < Ci || (wd && Cp != Ci)) return -1;
  hipLaunchKernelGGL(wprep_kernel, dim3(nblk((long)9 * Cp * Co)), dim3(256), 0, s, w, Co, Ci, Cp, wf, wd);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_conv_wgrad_reduce(const float* part, int S, int Co, int Ci, int Cp, float* grad, int accumulate,
                                        hipStream_t s) {
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(nblk((long)Co * Ci * 9)), dim3(256), 0, s, part, S, Co, Ci, Cp, grad,
                     accumulate);
  return (int)hipGetLastError();
}

static int bn_threads(int C) { return C >= 256 ? C : 256; }

DDPX_API int ddpx_f32_bn_stats(const float* y, int P, int C, int R, float* part, hipStream_t s) {
  if (C > 512 || (256 % C && C % 256)) return -1;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(nblk(P, R)), dim3(bn_threads(C)), 0, s, y, P, C, R, part);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_bn_finalize(const float* part, int T, int R, int P, int C, const float* gamma, const float* beta,
                                  float* rmean, float* rvar, int64_t* nbt, float momentum, float eps, int training,
                                  float* a, float* b, float* mean, float* rstd, double* ws, hipStream_t s) {
  // few channel groups and many chunks: the split merge (DDPX_F32_BN_SPLIT=0 keeps the one-kernel merge)
  static const bool split_ok = [] {
    const char* e = getenv("DDPX_F32_BN_SPLIT");
    return !(e && e[0] == '0');
  }();
  if (split_ok && ws && training && C <= kFinSplitMaxC && T >= 1024 && nblk(C, 64) < 8) {
    const int S = min(kFinSplitMax, (T + 127) / 128);
    const int Ts = (T + S - 1) / S;
    const int Sr = (T + Ts - 1) / Ts;  // splits with a chunk range
    double* s1 = ws;
    double* s2 = ws + (size_t)kFinSplitMax * C;
    hipLaunchKernelGGL(bn_fin_sum_kernel, dim3(nblk(C, 64), Sr), dim3(1024), 0, s, part, T, Ts, R, P, C, s1);
    hipLaunchKernelGGL(bn_fin_m2_kernel, dim3(nblk(C, 64), Sr), dim3(1024), 0, s, part, T, Ts, Sr, R, P, C, s1, s2);
    hipLaunchKernelGGL(bn_fin_out_kernel, dim3(nblk(C, 64)), dim3(64), 0, s, Sr, P, C, gamma, beta, rmean, rvar, nbt,
                       momentum, eps, a, b, mean, rstd, s1, s2);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(nblk(C, 64)), dim3(1024), 0, s, part, T, R, P, C, gamma, beta, rmean, rvar,
                     nbt, momentum, eps, training, a, b, mean, rstd);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_bn_apply(const float* y, const float* a, const float* b, const float* mean, int N, int H, int W,
                               int C, int relu, int pool, float* out, hipStream_t s) {
  if (C % 4 || (pool && (H % 2 || W % 2))) return -1;
  const long n = (long)N * (pool ? H / 2 : H) * (pool ? W / 2 : W) * (C / 4);
  hipLaunchKernelGGL(bn_apply_kernel, dim3(nblk(n)), dim3(256), 0, s, y, a, b, mean, N, H, W, C, relu, pool, out);
  return (int)hipGetLastError();
}

// The vectorised backward kernels need 4-channel quads that split a 256-thread block evenly and (pooled) chunks
// of whole window rows; DDPX_F32_BN_VEC=0 keeps the per-element kernels (A/B checks).
static bool bn_vec_ok(int C, int W, int pool, int R) {
  static const bool on = [] {
    const char* e = getenv("DDPX_F32_BN_VEC");
    return !(e && e[0] == '0');
  }();
  return on && C % 4 == 0 && C / 4 <= 256 && 256 % (C / 4) == 0 && (!pool || R % (2 * W) == 0);
}

DDPX_API int ddpx_f32_bn_bwd_sums(const float* g, const float* y, const float* a, const float* b, const float* mean,
                                  const float* rstd, int N, int H, int W, int C, int pool, int R, float* part,
                                  hipStream_t s) {
  if (pool && (H % 2 || W % 2)) return -1;
  if (bn_vec_ok(C, W, pool, R)) {
    hipLaunchKernelGGL(bn_bwd_sums4_kernel, dim3(nblk((long)N * H * W, R)), dim3(256), 0, s, g, y, a, b, mean, rstd,
                       N, H, W, C, pool, R, part, (float*)nullptr);
    return (int)hipGetLastError();
  }
  if (C > 512 || (256 % C && C % 256)) return -1;
  hipLaunchKernelGGL(bn_bwd_sums_kernel, dim3(nblk((long)N * H * W, R)), dim3(bn_threads(C)), 0, s, g, y, a, b, mean,
                     rstd, N, H, W, C, pool, R, part);
  return (int)hipGetLastError();
}

// Bias + activation backward (a = 1, b = 0, mean = 0, rstd = 1): the sums pass also writes dy = gz.  Returns 1
// when it did (the caller skips ddpx_f32_bn_bwd_apply), 0 when only the sums were written (no 4-channel path).
DDPX_API int ddpx_f32_bias_act_bwd_sums(const float* g, const float* y, const float* one, const float* zero, int N,
                                        int H, int W, int C, int pool, int R, float* part, float* dy, hipStream_t s) {
  if (pool && (H % 2 || W % 2)) return -1;
  if (bn_vec_ok(C, W, pool, R)) {
    hipLaunchKernelGGL(bn_bwd_sums4_kernel, dim3(nblk((long)N * H * W, R)), dim3(256), 0, s, g, y, one, zero, zero,
                       one, N, H, W, C, pool, R, part, dy);
    const int e = (int)hipGetLastError();
    return e ? -e : 1;
  }
  const int e = ddpx_f32_bn_bwd_sums(g, y, one, zero, zero, one, N, H, W, C, pool, R, part, s);
  return e ? (e < 0 ? e : -e) : 0;
}

DDPX_API int ddpx_f32_bn_bwd_finalize(const float* part, int T, int P, int C, float* c1, float* c2, float* dgamma,
                                      float* dbeta, int accumulate, double* ws, hipStream_t s) {
  static const bool split_ok = [] {
    const char* e = getenv("DDPX_F32_BN_SPLIT");
    return !(e && e[0] == '0');
  }();
  if (split_ok && ws && C <= kFinSplitMaxC && T >= 1024 && nblk(C, 64) < 8) {
    const int S = min(kFinSplitMax, (T + 127) / 128);
    const int Ts = (T + S - 1) / S;
    const int Sr = (T + Ts - 1) / Ts;
    double* s1 = ws;
    double* s2 = ws + (size_t)kFinSplitMax * C;
    hipLaunchKernelGGL(bn_bwd_fin_sum_kernel, dim3(nblk(C, 64), Sr), dim3(1024), 0, s, part, T, Ts, C, s1, s2);
    hipLaunchKernelGGL(bn_bwd_fin_out_kernel, dim3(nblk(C, 64)), dim3(64), 0, s, Sr, P, C, c1, c2, dgamma, dbeta,
                       accumulate, s1, s2);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(nblk(C, 64)), dim3(1024), 0, s, part, T, P, C, c1, c2, dgamma, dbeta,
                     accumulate);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_bn_bwd_apply(const float* g, const float* y, const float* a, const float* b, const float* mean,
                                   const float* rstd, const float* c1, const float* c2, int N, int H, int W, int C,
                                   int pool, float* dy, hipStream_t s) {
  if (bn_vec_ok(C, W, pool, pool ? 2 * W : 1)) {
    const long units = pool ? (long)N * (H / 2) * (W / 2) : (long)N * H * W;
    hipLaunchKernelGGL(bn_bwd_apply4_kernel, dim3(nblk(units * (C / 4))), dim3(256), 0, s, g, y, a, b, mean, rstd, c1,
                       c2, N, H, W, C, pool, dy);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(nblk((long)N * H * W * C)), dim3(256), 0, s, g, y, a, b, mean, rstd,
                     c1, c2, N, H, W, C, pool, dy);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_avgpool(const float* x, int N, int S, int C, float* out, int backward, hipStream_t s) {
  if (backward)
    hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(nblk((long)N * S * C)), dim3(256), 0, s, x, N, S, C, out);
  else
    hipLaunchKernelGGL(avgpool_kernel, dim3(nblk((long)N * C)), dim3(256), 0, s, x, N, S, C, out);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_head_fwd(const float* h, const float* w, const float* bias, const int64_t* tgt, int M, int K,
                               int NC, float* logits, float* loss, float* dl, hipStream_t s) {
  if (K % 4) return -1;
  if (NC > kMaxNC) return -2;
  if (NC == 10 && K % 4 == 0)
    hipLaunchKernelGGL(head_logits_row_kernel<10>, dim3(M), dim3(256), 0, s, h, w, bias, K, logits);
  else
    hipLaunchKernelGGL(head_logits_kernel, dim3(nblk(M, 4)), dim3(256), 0, s, h, w, bias, M, K, NC, logits);
  if (tgt) hipLaunchKernelGGL(xent_kernel, dim3(1), dim3(1024), 0, s, logits, tgt, M, NC, loss, dl);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_head_bwd(const float* dl, const float* go, const float* h, const float* w, int M, int K, int NC,
                               float* dW, float* db, int accumulate, float* dh, int relu_mask, float dh_scale,
                               hipStream_t s) {
  if (NC > kMaxNC) return -2;
  if (dW) hipLaunchKernelGGL(head_wgrad_kernel, dim3(nblk(K, 64) + 1), dim3(1024), 0, s, dl, go, h, M, K, NC, dW, db,
                             accumulate);
  if (dh && K % 4 == 0 && !(((uintptr_t)w | (uintptr_t)h | (uintptr_t)dh) & 15))
    hipLaunchKernelGGL(head_dgrad4_kernel, dim3(nblk((long)M * (K / 4))), dim3(256), 0, s, dl, go, w, h, M, K, NC,
                       relu_mask, dh_scale, dh);
  else if (dh)
    hipLaunchKernelGGL(head_dgrad_kernel, dim3(nblk((long)M * K)), dim3(256), 0, s, dl, go, w, h, M, K, NC,
                       relu_mask, dh_scale, dh);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_colsum_part(const float* x, int P, int C, int R, float* part, hipStream_t s) {
  if (C % 4 || C > 1024 || R < 1 || ((uintptr_t)x & 15) || ((uintptr_t)part & 15)) return -1;
  hipLaunchKernelGGL(colsum_part_kernel, dim3((P + R - 1) / R), dim3(256), 0, s, x, P, C, R, part);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_colsum(const float* x, int M, int N, float* out, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(colsum_kernel, dim3(nblk(N, 64)), dim3(1024), 0, s, x, M, N, out, accumulate);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_f32_nchw_flatten(const float* x, int N, int S, int C, int backward, float* out, hipStream_t s) {
  hipLaunchKernelGGL(nchw_flatten_kernel, dim3(nblk((long)N * S * C)), dim3(256), 0, s, x, N, S, C, backward, out);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_bf16_nchw_flatten(const void* x, int N, int S, int C, int backward, void* out, hipStream_t s) {
  if (S * C > kFlatLds || N <= 0) return -1;
  hipLaunchKernelGGL(nchw_flatten_bf16_kernel, dim3(N), dim3(256), 0, s, (const unsigned short*)x, S, C, backward,
                     (unsigned short*)out);
  return (int)hipGetLastError();
}

// Summation block (1, 2 or 4 K-steps of 16) of the LDS-DMA core; returns the previous setting.
DDPX_API int ddpx_f32_set_block(int kb) {
  const int prev = f32_block();
  g_f32_block = (kb == 1 || kb == 2 || kb == 8) ? kb : 4;
  return prev;
}

// 1 = LDS-DMA ring GEMM core, 0 = register-staged; returns the previous setting.
DDPX_API int ddpx_f32_set_staging(int dma) {
  const int prev = f32_dma() ? 1 : 0;
  g_f32_staging = dma ? 1 : 0;
  return prev;
}

// Forward 3x3 convolution y [N*H*W][Co] = conv(x NHWC [N][H][W][C], wf) on the LDS-DMA core with the BatchNorm
// tile statistics emitted by its epilogue: stats[tiles_m][2][Co] (tile mean, M2).  Returns the tile's row count
// (the chunk size bn_finalize needs), or a negative code when the fused path does not apply (register-staged
// core selected, or an operand beyond 32-bit offsets): the caller then runs the separate statistics pass.
DDPX_API int ddpx_f32_conv_fwd_stats(const float* x, const float* wf, float* y, int N, int H, int W, int C, int Co,
                                     float* stats, hipStream_t s) {
  if (!f32_dma()) return -10;
  const int lc = ilog2(C), lh = ilog2(H), lw = ilog2(W);
  if (lc < 2 || lh < 0 || lw < 0 || Co % 4) return -2;
  const int M = N * H * W, K = 9 * C;
  Operand A{x, 0, M, lc, lh, lw, 1}, B{wf, Co, Co, lc, lh, lw, 1};
  const unsigned ab = operand_bytes(IM2COL_KC, 0, M, K, C, M), bb = operand_bytes(DENSE_OC, Co, Co, K, C, K);
  if (!ab || !bb) return -11;
  const int tile = auto_tile(M, Co, 1);
  dispatch_tile<IM2COL_KC, DENSE_OC>(tile, A, B, M, Co, K, 1, y, Co, 0, nullptr, nullptr, 0, s, ab, bb, stats);
  const int err = (int)hipGetLastError();
  return err ? -err : ((tile == 2 || tile == 3) ? 64 : 128);
}
