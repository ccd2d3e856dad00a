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

// Default tile per operand-layout class, from the MI355X sweep of the MLP shapes
// (benchmarks/gemm_sweep.py; profiles/): M=512-row products want many small
// tiles (64x64, 2-3 WG/CU), the K=512 weight-gradient products 64x128/3 stages.
static int pick(int M, int N, int K, bool ak, bool bk) {
  auto tiles = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  if (!ak && !bk) return tiles(64, 128) >= 512 ? 5 : 7;      // wgrad-shaped (reduction over batch)
  if (ak && !bk) return 3;                                   // dgrad-shaped
  if (tiles(128, 128) >= 1024 && K >= 2048) return 0;        // big forward GEMMs
  return 7;                                                  // forward, small M
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
                 pipe::ConvGeom{0, 0, 0, 0}, 0, 0};
  if (epi == pipe::EPI_SGD && (!sgd_p || !sgd_lr || (sgd_mom != 0.f && !sgd_buf))) return -5;
  const int cfg = tile_cfg >= 0 ? tile_cfg : pipe::pick(M, N, K, a_kcontig, b_kcontig);
  hipError_t e;
  if (a_kcontig && b_kcontig) e = pipe::dispatch<true, true, pipe::MODE_PLAIN, pipe::MODE_PLAIN>(p, cfg, 1, stream);
  else if (a_kcontig) e = pipe::dispatch<true, false, pipe::MODE_PLAIN, pipe::MODE_PLAIN>(p, cfg, 1, stream);
  else if (b_kcontig) e = pipe::dispatch<false, true, pipe::MODE_PLAIN, pipe::MODE_PLAIN>(p, cfg, 1, stream);
  else e = pipe::dispatch<false, false, pipe::MODE_PLAIN, pipe::MODE_PLAIN>(p, cfg, 1, stream);
  return (int)e;
}

DDPX_API int ddpx_reduce_partials(const float* part, int T, int N, void* out, int out_bf16, int accumulate,
                                  float* sgd_p, float* sgd_buf, void* sgd_shadow, const float* sgd_lr, float sgd_mom,
                                  float sgd_wd, hipStream_t s) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(pipe::reduce_partials_kernel, dim3((N + 255) / 256), dim3(256), 0, s, part, T, N, (float*)out,
                     out_bf16, accumulate, SgdArgs{sgd_p, sgd_buf, (unsigned short*)sgd_shadow, sgd_lr, sgd_mom, sgd_wd});
  return (int)hipGetLastError();
}
