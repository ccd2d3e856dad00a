// ddpx — pipelined bf16 MFMA GEMM for gfx950: LDS-DMA multi-stage ring.
//
// Same contract and operand layouts as gemm_bf16.hip (see there), re-built
// for the regime the MLP shapes live in (M = 512 rows against N, K = 3-16 K):
// a 64x128 / 128x128 tile gives only 256 / 128 workgroups, one per CU, so the
// kernel is bound by how many bytes each CU keeps in flight, not by MFMA.
//
//  * Operand tiles go HBM/L2 -> LDS by `buffer_load_dwordx4 ... lds` (LDS-DMA,
//    cdna_hip_programming §5 "Async global->LDS"): no VGPR staging, no
//    ds_write, 1 KiB per wave-instruction.
//  * STAGES-deep ring of LDS slots; STAGES-1 K-tiles are in flight while one
//    is consumed.  Each iteration: counted `s_waitcnt vmcnt(N)` for the oldest
//    stage -> raw `s_barrier` (never __syncthreads, whose fence would drain the
//    DMA queue, §5 "Pipelining across barriers") -> issue the next stage into
//    the slot freed one iteration ago -> ds_read + MFMA on the landed slot.
//  * LDS images are lane-linear (DMA writes base + lane*16), so the bank
//    swizzles of gemm_bf16.hip are applied to the per-lane SOURCE address and
//    undone on the read (rule 21): same images, same fragment readers.
//  * Buffer-resource bounds checking returns zeros for out-of-range lanes
//    (voffset forced past num_records), which handles ragged M/N/K tails with
//    no branches in the load path.
//  * XCD-aware workgroup remap (T1) as in v1.
//  * Epilogues: bias (+ReLU) -> bf16, fp32 (+accumulate) for gradients
//    written straight into DDP buckets, bf16 (+accumulate), ReLU-mask
//    backward, and an optional per-tile column sum of the stored output (the
//    bias gradient of the layer below) written as [tiles_m][N] partials.
#include <cstdlib>

#include "ddpx_pipe.h"

namespace ddpx {
namespace pipe {

// out[n] (=|+=) sum_t partial[t][n]   (fixed order: deterministic)
__global__ void __launch_bounds__(256) reduce_partials_kernel(const float* __restrict__ part, int T, int N,
                                                              float* __restrict__ out, int out_bf16, int accumulate,
                                                              SgdArgs sgd) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int t = 0; t < T; ++t) s += part[(size_t)t * N + n];
  if (sgd.p) {
    sgd_apply(sgd, n, s, *sgd.lr);
  } else if (out_bf16) {
    unsigned short* o = reinterpret_cast<unsigned short*>(out);
    if (accumulate) s += bf2f(o[n]);
    o[n] = f2bf(s);
  } else {
    out[n] = accumulate ? out[n] + s : s;
  }
}

// Split-K finish: out = epi( sum_s part[s] ) in fixed split order (deterministic), plus per-4-row-block
// column sums of the stored values (colsum [ceil(M/4)][N], the fused bias gradient of dgrad).
// Block = 64 column quads x 4 rows; one f32x4 per thread per slab: a pure stream with >2k blocks.
template <int E>
__global__ void __launch_bounds__(256) splitk_finish_kernel(Params p, const float* __restrict__ part, int S) {
  const int cq = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int n = blockIdx.x * 256 + cq * 4;
  const int m = blockIdx.y * 4 + ty;
  const size_t slab = (size_t)p.M * p.N;
  float st[4] = {0.f, 0.f, 0.f, 0.f};
  if (n < p.N && m < p.M) {
    f32x4 v[8];
    const int S8 = S < 8 ? S : 8;
#pragma unroll
    for (int sp = 0; sp < 8; ++sp)
      if (sp < S8) v[sp] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(part + sp * slab + (size_t)m * p.N + n));
    f32x4 acc = v[0];
#pragma unroll
    for (int sp = 1; sp < 8; ++sp)
      if (sp < S8) { acc[0] += v[sp][0]; acc[1] += v[sp][1]; acc[2] += v[sp][2]; acc[3] += v[sp][3]; }
    for (int sp = 8; sp < S; ++sp) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(part + sp * slab + (size_t)m * p.N + n);
      acc[0] += w[0]; acc[1] += w[1]; acc[2] += w[2]; acc[3] += w[3];
    }
    const size_t off = (size_t)m * p.ldc + n;
    float cin[4] = {0.f, 0.f, 0.f, 0.f};
    unsigned short av[4] = {0, 0, 0, 0};
    if constexpr (E == EPI_F32) {
      if (p.accumulate) for (int q = 0; q < 4; ++q) cin[q] = reinterpret_cast<const float*>(p.C)[off + q];
    } else if constexpr (E == EPI_BF16) {
      if (p.accumulate) for (int q = 0; q < 4; ++q) cin[q] = bf2f(reinterpret_cast<const unsigned short*>(p.C)[off + q]);
    } else if constexpr (E == EPI_RELUMASK_BF16) {
      const u32x2 a = *reinterpret_cast<const u32x2*>(p.aux + (size_t)m * p.ldaux + n);
      av[0] = a[0] & 0xffffu; av[1] = a[0] >> 16; av[2] = a[1] & 0xffffu; av[3] = a[1] >> 16;
    }
    for (int q = 0; q < 4; ++q) {
      float po, bo;
      st[q] = epi_one<E>(p, p.C, off + q, n + q, acc[q], 0.f, cin[q], av[q], 0.f, 0.f, &po, &bo);
    }
    if constexpr (E == EPI_F32 || E == EPI_BIAS_F32) {
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.C) + off) = (f32x4){st[0], st[1], st[2], st[3]};
    } else {
      *reinterpret_cast<u32x2*>(reinterpret_cast<unsigned short*>(p.C) + off) =
          (u32x2){pack_bf2(st[0], st[1]), pack_bf2(st[2], st[3])};
    }
  }
  if (!p.colsum) return;
  __shared__ float red[4][256];
  for (int q = 0; q < 4; ++q) red[ty][cq * 4 + q] = st[q];
  __syncthreads();
  const int t = threadIdx.x;
  if (blockIdx.x * 256 + t < p.N)
    p.colsum[(size_t)blockIdx.y * p.N + blockIdx.x * 256 + t] = red[0][t] + red[1][t] + red[2][t] + red[3][t];
}

// Split-K plan for the M = 512-row products (forward, dgrad): 256x128 tiles on 8 waves (2x the
// arithmetic intensity of 128x128: the 64x64-tile kernel is bound by L2->LDS operand traffic, not
// MFMA), K split so that ~256 workgroups fill the CUs.  Returns splits (1 = no split-K).
static int splitk_plan(int M, int N, int K, bool ak, bool bk) {
  if (!ak || M > 2048 || K < 1024) return 1;  // wgrad-shaped / large-M / short-K: regular tiles
  const int tiles = ((M + 255) / 256) * ((N + 127) / 128);
  if (tiles >= 192) return 1;
  int s = (256 + tiles - 1) / tiles;
  const int kb = K / 64;
  while (s > 1 && kb / s < 8) --s;  // keep >= 8 K-steps per split
  return s < 1 ? 1 : s;
}

// Default tile per operand-layout class, from the MI355X sweep of the MLP shapes
// (benchmarks/mlp_gemm_bench.py, benchmarks/sgd_bw.py; profiles/r1_gemm2): the M=512-row products
// want 64x64 tiles with 128-wide K stages (fwd 27.1 vs 29.1 us, dgrad 36.5 vs 45.1 us at H=4096),
// the K=512 weight-gradient products 64x128/3 stages.
static int pick(int M, int N, int K, bool ak, bool bk) {
  auto tiles = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  if (!ak && !bk) return tiles(64, 128) >= 512 ? 5 : 7;      // wgrad-shaped (reduction over batch)
  if (tiles(128, 128) >= 512 && K >= 2048) return 0;         // wide layers: 128x128 halves L2 traffic
  return 12;  // M=512-row forward / dgrad: 64x64, BK=128 (one barrier per 128 of K), 2 WG/CU
}

}  // namespace pipe
}  // namespace ddpx

using namespace ddpx;

// Number of row tiles (M direction) the kernel will use for cfg (for sizing colsum partials).
DDPX_API int ddpx_gemm_pipe_tiles_m(int M, int N, int K, int a_kcontig, int b_kcontig, int tile_cfg) {
  const int cfg = tile_cfg >= 0 ? tile_cfg : pipe::pick(M, N, K, a_kcontig, b_kcontig);
  int bm, bn;
  pipe::tile_of(cfg, &bm, &bn);
  return (M + bm - 1) / bm;
}

DDPX_API int ddpx_gemm_pipe(const void* A, const void* B, void* C, const float* bias, const void* aux, float* colsum,
                            int M, int N, int K, int lda, int ldb, int ldc, int ldaux, int a_kcontig, int b_kcontig,
                            int epi, int accumulate, float alpha, int tile_cfg, float* sgd_p, float* sgd_buf,
                            void* sgd_shadow, const float* sgd_lr, float sgd_mom, float sgd_wd, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (a_kcontig ? (K % 8 || lda % 8) : (M % 8 || lda % 8)) return -1;
  if (b_kcontig ? (K % 8 || ldb % 8) : (N % 8 || ldb % 8)) return -2;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -3;
  const size_t a_bytes = (size_t)(a_kcontig ? (size_t)(M - 1) * lda + K : (size_t)(K - 1) * lda + M) * 2;
  const size_t b_bytes = (size_t)(b_kcontig ? (size_t)(N - 1) * ldb + K : (size_t)(K - 1) * ldb + N) * 2;
  if (a_bytes >= 0x80000000ull || b_bytes >= 0x80000000ull) return -4;  // 32-bit buffer offsets
  pipe::Params p{(const unsigned short*)A, (const unsigned short*)B, C, bias, (const unsigned short*)aux, colsum,
                 M, N, K, lda, ldb, ldc, ldaux, epi, accumulate, alpha, (unsigned)a_bytes, (unsigned)b_bytes,
                 SgdArgs{sgd_p, sgd_buf, (unsigned short*)sgd_shadow, sgd_lr, sgd_mom, sgd_wd},
                 pipe::make_geom(0, 0, 0, 0), 0, 0};
  if (epi == pipe::EPI_SGD && (!sgd_p || !sgd_lr || (sgd_mom != 0.f && !sgd_buf))) return -5;
  static const int sgd_plain = [] {
    const char* e = getenv("DDPX_SGD_PLAIN");
    return e && e[0] == '1' ? 1 : 0;
  }();
  p.sgd_plain = sgd_plain;
  int cfg = tile_cfg >= 0 ? tile_cfg : pipe::pick(M, N, K, a_kcontig, b_kcontig);
  // Weight gradients stored to a buffer (DDP path: bf16 / fp32 gradient output, no fused optimizer):
  // the 256x256 8-wave tile moves a quarter of the 64x128 tile's L2->LDS operand bytes and is faster
  // once it fills half the chip (MI355X, K = 512: 35.4 vs 46.1 us on 4096x4096, 30.9 vs 38.6 us on
  // 4096x3072, fp32 out; benchmarks/wgrad_probe.py, profiles/r1_wgrad).  The fused-SGD epilogue keeps
  // 64x128 (its HBM stream wants two resident workgroups per CU: 78.9 vs 72.8 us).
  if (tile_cfg < 0 && !a_kcontig && !b_kcontig && epi != pipe::EPI_SGD && !colsum &&
      ((M + 255) / 256) * ((N + 255) / 256) >= 128)
    cfg = 13;
  // Master/momentum LDS prefetch for the fused-SGD tiles: opt-in (DDPX_SGD_PREFETCH=1).  Measured
  // slower on MI355X (toy fc1 64x128: 112 vs 77 us; profiles/r1_epi): the 64 KiB side buffer halves
  // occupancy and the prefetch lands on the critical path of short (K = 512) main loops.
  static const int sgd_pf = [] {
    const char* e = getenv("DDPX_SGD_PREFETCH");
    return e && e[0] == '1' ? 1 : 0;
  }();
  if (epi == pipe::EPI_SGD && sgd_pf && !a_kcontig && !b_kcontig && (ldc & 3) == 0 &&
      (size_t)M * ldc * 4 < 0x80000000ull && (cfg == 3 || cfg == 5 || cfg == 7 || cfg == 12)) {
    return (int)pipe::dispatch_sgd_prefetch<false, false>(p, cfg, stream);
  }
  hipError_t e;
  if (a_kcontig && b_kcontig) e = pipe::dispatch<true, true, pipe::MODE_PLAIN, pipe::MODE_PLAIN>(p, cfg, 1, stream);
  else if (a_kcontig) e = pipe::dispatch<true, false, pipe::MODE_PLAIN, pipe::MODE_PLAIN>(p, cfg, 1, stream);
  else if (b_kcontig) e = pipe::dispatch<false, true, pipe::MODE_PLAIN, pipe::MODE_PLAIN>(p, cfg, 1, stream);
  else e = pipe::dispatch<false, false, pipe::MODE_PLAIN, pipe::MODE_PLAIN>(p, cfg, 1, stream);
  return (int)e;
}

// Split-K plan query: splits (>1 means ddpx_gemm_pipe_splitk applies), scratch floats, colsum rows.
DDPX_API int ddpx_gemm_splitk_plan(int M, int N, int K, int a_kcontig, int b_kcontig, long long* scratch_floats,
                                   int* colsum_rows) {
  const int s = pipe::splitk_plan(M, N, K, a_kcontig, b_kcontig);
  *scratch_floats = s > 1 ? (long long)s * M * N : 0;
  *colsum_rows = (M + 3) / 4;
  return s;
}

// C = epi(A.B) via split-K on the 8-wave 256x128 tile: fp32 partial slabs in `scratch`, then a
// fixed-order reduction kernel that applies the epilogue (and per-64-row column sums).
DDPX_API int ddpx_gemm_pipe_splitk(const void* A, const void* B, void* C, const float* bias, const void* aux,
                                   float* colsum, int M, int N, int K, int lda, int ldb, int ldc, int ldaux,
                                   int a_kcontig, int b_kcontig, int epi, int accumulate, float alpha, int splits,
                                   float* scratch, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (splits < 1 || !scratch) return -7;
  if (!a_kcontig || (K % 8) || (lda % 8)) return -1;
  if (b_kcontig ? (K % 8 || ldb % 8) : (N % 8 || ldb % 8)) return -2;
  if (N % 4 || ldc % 4) return -8;
  if (epi == pipe::EPI_SGD || epi == pipe::EPI_BNSTAT_BF16) return -6;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -3;
  const size_t a_bytes = ((size_t)(M - 1) * lda + K) * 2;
  const size_t b_bytes = (size_t)(b_kcontig ? (size_t)(N - 1) * ldb + K : (size_t)(K - 1) * ldb + N) * 2;
  if (a_bytes >= 0x80000000ull || b_bytes >= 0x80000000ull) return -4;
  int klen = (K + splits - 1) / splits;
  klen = (klen + 63) / 64 * 64;
  const int S = (K + klen - 1) / klen;
  pipe::Params pp{(const unsigned short*)A, (const unsigned short*)B, scratch, nullptr, nullptr, nullptr,
                  M, N, K, lda, ldb, N, 0, pipe::EPI_F32, 0, 1.f, (unsigned)a_bytes, (unsigned)b_bytes,
                  SgdArgs{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f}, pipe::make_geom(0, 0, 0, 0), klen,
                  (long long)M * N};
  hipError_t e = b_kcontig
                     ? pipe::dispatch<true, true, pipe::MODE_PLAIN, pipe::MODE_PLAIN>(pp, 8, S, stream)
                     : pipe::dispatch<true, false, pipe::MODE_PLAIN, pipe::MODE_PLAIN>(pp, 8, S, stream);
  if (e != hipSuccess) return (int)e;
  pipe::Params fp{(const unsigned short*)A, (const unsigned short*)B, C, bias, (const unsigned short*)aux, colsum,
                  M, N, K, lda, ldb, ldc, ldaux, epi, accumulate, alpha, 0u, 0u,
                  SgdArgs{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f}, pipe::make_geom(0, 0, 0, 0), 0, 0};
  const dim3 grid((N + 255) / 256, (M + 3) / 4);
  switch (epi) {
    case pipe::EPI_F32: hipLaunchKernelGGL(pipe::splitk_finish_kernel<pipe::EPI_F32>, grid, dim3(256), 0, stream, fp, scratch, S); break;
    case pipe::EPI_BF16: hipLaunchKernelGGL(pipe::splitk_finish_kernel<pipe::EPI_BF16>, grid, dim3(256), 0, stream, fp, scratch, S); break;
    case pipe::EPI_BIAS_BF16: hipLaunchKernelGGL(pipe::splitk_finish_kernel<pipe::EPI_BIAS_BF16>, grid, dim3(256), 0, stream, fp, scratch, S); break;
    case pipe::EPI_BIAS_RELU_BF16: hipLaunchKernelGGL(pipe::splitk_finish_kernel<pipe::EPI_BIAS_RELU_BF16>, grid, dim3(256), 0, stream, fp, scratch, S); break;
    case pipe::EPI_BIAS_F32: hipLaunchKernelGGL(pipe::splitk_finish_kernel<pipe::EPI_BIAS_F32>, grid, dim3(256), 0, stream, fp, scratch, S); break;
    case pipe::EPI_RELUMASK_BF16: hipLaunchKernelGGL(pipe::splitk_finish_kernel<pipe::EPI_RELUMASK_BF16>, grid, dim3(256), 0, stream, fp, scratch, S); break;
    default: return -6;
  }
  return (int)hipGetLastError();
}

DDPX_API int ddpx_reduce_partials(const float* part, int T, int N, void* out, int out_bf16, int accumulate,
                                  float* sgd_p, float* sgd_buf, void* sgd_shadow, const float* sgd_lr, float sgd_mom,
                                  float sgd_wd, hipStream_t s) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(pipe::reduce_partials_kernel, dim3((N + 255) / 256), dim3(256), 0, s, part, T, N, (float*)out,
                     out_bf16, accumulate, SgdArgs{sgd_p, sgd_buf, (unsigned short*)sgd_shadow, sgd_lr, sgd_mom, sgd_wd});
  return (int)hipGetLastError();
}
