// ddpx — weight gradient + SGD in one warp-specialised persistent kernel (gfx950).
//
//   W -= lr * sgd_direction( dY^T X )          dY [K=batch][M=out] bf16, X [K][N=in] bf16, W fp32 [M][N]
//
// The single-process optimizer fused into backward (SGD(fused_backward=True)) streams 18 B per weight
// (master + momentum in, master + momentum + bf16 shadow out) right where the weight gradient is born,
// so the gradient never round-trips through HBM.  In the tile-per-workgroup GEMM that stream ran AFTER
// each tile's MFMA main loop: both halves serialised and the fused kernels (toy MLP fc1 / fc0: 97 / 78 us,
// profiles/r2_head) were no faster than a stored fp32 gradient plus one flat SGD pass.
//
// Here every workgroup (one per CU, 8 waves) owns a list of 64x128 tiles and splits its waves by role:
//   * waves 0-3 (math): the LDS-DMA ring + v_mfma_f32_16x16x32_bf16 main loop of tile i (the pipe core of
//     ddpx_pipe.h), then its fp32 accumulators into one of two LDS tile buffers;
//   * waves 4-7 (stream): the optimizer update of tile i-1 from the other buffer — master / momentum loads
//     for tile i issued one iteration ahead, non-temporal, and the update spread over the K-steps —
//     so a CU's HBM stream runs while its matrix cores work on the next tile.
// Both roles execute exactly nk + 1 s_barriers per iteration (nk K-steps of 64, then the buffer hand-off)
// for nt + 1 iterations (one drain iteration), so the barrier sequence matches by construction.
// The update arithmetic is sgd_apply's fma sequence: bitwise equal to the stored-gradient + flat-SGD path.
#pragma once

#include <cstdlib>

#include "ddpx_pipe.h"

namespace ddpx {
namespace wsgd {

constexpr int BM = 64, BN = 128;
constexpr int A_SUB = BM * 64 * 2, B_SUB = BN * 64 * 2, SLOT = A_SUB + B_SUB;
constexpr int VPT = BM * BN / 4 / 256;  // f32x4 vectors per stream thread per tile (8)
// STAGES-deep LDS-DMA ring for the math waves + two fp32 tile buffers (math -> stream hand-off).
//   3 stages: row stride BN + 4 (conflict-free accumulator stores), 138 KiB;
//   4 stages: one more 24 KiB stage in flight (the math side's K-steps are L2->LDS latency bound with
//             only 4 DMA-issuing waves), which fits the 160 KiB LDS only with unpadded rows (4-way
//             conflicts on the once-per-tile accumulator store).
template <int STAGES>
struct Cfg {
  static constexpr int ALD = STAGES >= 4 ? BN : BN + 4;
  static constexpr int ACC_BYTES = BM * ALD * 4;
  static constexpr int LDS_BYTES = STAGES * SLOT + 2 * ACC_BYTES;
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

// Two GEMMs may share one launch (p0's tiles, then p1's: the toy MLP's fc1 and fc0 weight gradients are
// independent once fc1's data gradient ran): one fill and one drain iteration instead of two, one launch
// boundary fewer.  Single GEMM: p1 = p0 and nt1 = 0.  Both must have the same K, lr, momentum, wd, alpha.
template <int STAGES>
__global__ void __launch_bounds__(512) wgrad_sgd_ws_kernel(pipe::Params p0, pipe::Params p1, int nt1, int spread) {
  constexpr int ALD = Cfg<STAGES>::ALD, ACC_BYTES = Cfg<STAGES>::ACC_BYTES, LDS_BYTES = Cfg<STAGES>::LDS_BYTES;
  constexpr int FM = 2, FN = 4;                  // math wave tile 32 x 64
  constexpr int LPW = (BM + BN) / (8 * 4);       // LDS-DMA instructions per math wave per stage
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  float* const accb = reinterpret_cast<float*>(smem + STAGES * SLOT);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m0 = p0.M / BM, tiles_m1 = p1.M / BM;
  const int nt0 = tiles_m0 * (p0.N / BN);
  const int ntiles = nt0 + nt1;
  const int nt = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;  // >= 1 (grid <= ntiles)
  const int nk = p0.K / 64;
  // tile i of this workgroup: origin and which GEMM it belongs to (uniform per workgroup)
  auto tile_origin = [&](int i, int& m0, int& n0) -> int {
    int g = (int)blockIdx.x + i * (int)gridDim.x;
    const int sel = g >= nt0;
    if (sel) g -= nt0;
    const int tm = sel ? tiles_m1 : tiles_m0;
    m0 = (g % tm) * BM;
    n0 = (g / tm) * BN;
    return sel;
  };
  const pipe::Params& p = p0;  // K, alpha, lr, momentum, wd: shared by both GEMMs

  if (wave < 4) {
    // ------------------------------------------------------------------ math waves
    const int wm = wave >> 1, wn = wave & 1;
    const __amdgpu_buffer_rsrc_t ra0 = __builtin_amdgcn_make_buffer_rsrc((void*)p0.A, 0, p0.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb0 = __builtin_amdgcn_make_buffer_rsrc((void*)p0.B, 0, p0.b_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ra1 = __builtin_amdgcn_make_buffer_rsrc((void*)p1.A, 0, p1.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb1 = __builtin_amdgcn_make_buffer_rsrc((void*)p1.B, 0, p1.b_bytes, 0x00020000);
    for (int i = 0; i <= nt; ++i) {
      if (i == nt) {  // drain iteration: the stream waves finish the last tile
        for (int t = 0; t < nk; ++t) __builtin_amdgcn_s_barrier();
      } else {
        int m0, n0;
        const int sel = tile_origin(i, m0, n0);
        const __amdgpu_buffer_rsrc_t ra = sel ? ra1 : ra0, rb = sel ? rb1 : rb0;
        const int lda = sel ? p1.lda : p0.lda, ldb = sel ? p1.ldb : p0.ldb;
        const int Mg = sel ? p1.M : p0.M, Ng = sel ? p1.N : p0.N;
        auto issue = [&](int t) {
          char* slot = smem + (t % STAGES) * SLOT;
          pipe::stage_tile<BM, false, pipe::MODE_PLAIN, 4>(ra, slot, p.conv, lda, m0, Mg, t * 64, p.K, wave, lane);
          pipe::stage_tile<BN, false, pipe::MODE_PLAIN, 4>(rb, slot + A_SUB, p.conv, ldb, n0, Ng, t * 64, p.K,
                                                           wave, lane);
        };
        f32x4 acc[FM][FN];
#pragma unroll
        for (int a = 0; a < FM; ++a)
#pragma unroll
          for (int b = 0; b < FN; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < STAGES - 1; ++s)
          if (s < nk) issue(s);
        for (int t = 0; t < nk; ++t) {
          const int ahead = min(STAGES - 2, nk - 1 - t);
          // stage t landed: everything but the (up to STAGES - 2) younger stages' DMAs
          if (STAGES >= 4 && ahead >= 2) pipe::wait_vmcnt<2 * LPW>();
          else if (ahead >= 1) pipe::wait_vmcnt<LPW>();
          else pipe::wait_vmcnt<0>();
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
          if (t + STAGES - 1 < nk) issue(t + STAGES - 1);
          const char* sa = smem + (t % STAGES) * SLOT;
          const char* sb = sa + A_SUB;
#pragma unroll
          for (int kk = 0; kk < 64; kk += 32) {
            bf16x8 af[FM], bfr[FN];
            pipe::load_frags<BM, false, FM, BN, false, FN>(sa, wm * 32, sb, wn * 64, kk, lane, af, bfr);
#pragma unroll
            for (int a = 0; a < FM; ++a)
#pragma unroll
              for (int b = 0; b < FN; ++b)
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
          }
        }
        // accumulators -> tile buffer i&1 (C/D map: row 4*(lane>>4)+r, col lane&15 of each 16x16 block)
        float* T = accb + (i & 1) * (ACC_BYTES / 4);
        const int mr = wm * 32 + 4 * (lane >> 4), nc = wn * 64 + (lane & 15);
#pragma unroll
        for (int a = 0; a < FM; ++a)
#pragma unroll
          for (int b = 0; b < FN; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) T[(mr + a * 16 + r) * ALD + nc + b * 16] = acc[a][b][r] * p.alpha;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // hand-off: tile i's buffer complete, tile i-1's buffer released
    }
  } else {
    // ---------------------------------------------------------------- stream waves
    const int st = tid - 256;
    const int row0 = st >> 5, col = 4 * (st & 31);  // vector v: row row0 + 8 v, columns col..col+3
    const float lr = *p.sgd.lr;
    const float mom = p.sgd.mom, wd = p.sgd.wd;
    const bool has_mom = mom != 0.f;
    f32x4 pc[VPT], mc[VPT], pn[VPT], mn[VPT];
    auto load_tile = [&](int i, f32x4 (&pv)[VPT], f32x4 (&mv)[VPT]) {
      int m0, n0;
      const int sel = tile_origin(i, m0, n0);
      const SgdArgs& sg = sel ? p1.sgd : p0.sgd;
      const int ldc = sel ? p1.ldc : p0.ldc;
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const size_t off = (size_t)(m0 + row0 + 8 * v) * ldc + n0 + col;
        pv[v] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(sg.p + off));
        mv[v] = has_mom ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(sg.buf + off))
                        : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    };
    int pm0 = 0, pn0 = 0, psel = 0;  // origin / GEMM of the tile being updated (i - 1)
    for (int i = 0; i <= nt; ++i) {
      if (i < nt) load_tile(i, pn, mn);  // one iteration ahead of its update
      const float* T = accb + ((i - 1) & 1) * (ACC_BYTES / 4);
      for (int t = 0; t < nk; ++t) {
        __builtin_amdgcn_s_barrier();
        if (i == 0) continue;
        // this K-step's share of tile i-1's update
        // spread = 1: one share per K-step; spread = s > 1: the update in the first ceil(nk / s) K-steps
        // (more stores in flight early in the tile period)
        const int nks = (nk + spread - 1) / spread;
        const int v0 = t < nks ? t * VPT / nks : VPT, v1 = t < nks ? (t + 1) * VPT / nks : VPT;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
          if (v < v0 || v >= v1) continue;
          const f32x4 g = *reinterpret_cast<const f32x4*>(T + (row0 + 8 * v) * ALD + col);
          f32x4 po, bo;
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // sgd_apply's fma sequence
            float d = fmaf(wd, pc[v][q], g[q]);
            if (has_mom) {
              d = fmaf(mom, mc[v][q], d);
              bo[q] = d;
            }
            po[q] = fmaf(-lr, d, pc[v][q]);
          }
          const SgdArgs& sg = psel ? p1.sgd : p0.sgd;
          const size_t off = (size_t)(pm0 + row0 + 8 * v) * (psel ? p1.ldc : p0.ldc) + pn0 + col;
          __builtin_nontemporal_store(po, reinterpret_cast<f32x4*>(sg.p + off));
          if (has_mom) __builtin_nontemporal_store(bo, reinterpret_cast<f32x4*>(sg.buf + off));
          if (sg.shadow)
            *reinterpret_cast<u32x2*>(sg.shadow + off) = (u32x2){pack_bf2(po[0], po[1]), pack_bf2(po[2], po[3])};
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (i < nt) {
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
          pc[v] = pn[v];
          mc[v] = mn[v];
        }
        psel = tile_origin(i, pm0, pn0);
      }
    }
  }
}

// Eligible shapes: the plain weight-gradient layout (A M-contig, B N-contig), M % 64 == 0, N % 128 == 0,
// K % 64 == 0 (whole K-steps: the two roles' barrier counts are nk), ldc % 4 == 0.
static inline bool eligible(const pipe::Params& p, bool ak, bool bk) {
  return !ak && !bk && p.M % BM == 0 && p.N % BN == 0 && p.K % 64 == 0 && p.K >= 64 && (p.ldc & 3) == 0 &&
         p.sgd.p && p.sgd.lr && (p.sgd.mom == 0.f || p.sgd.buf);
}

// Ring depth: DDPX_WSGD_STAGES=3|4 forces it; by default 4 stages once every CU owns >= 64 tiles (wide MLP:
// 2.434 vs 2.469 ms/step) and 3 below (toy MLP, 14 tiles per CU: 0.2398 vs 0.2502 ms/step; profiles/r2_stages).
static inline int stages(long long ntiles = 0, int num_cus = 256) {
  static const int forced = [] {
    const char* e = getenv("DDPX_WSGD_STAGES");
    return e && e[0] == '3' ? 3 : (e && e[0] == '4' ? 4 : 0);
  }();
  if (forced) return forced;
  return ntiles >= 64LL * num_cus ? 4 : 3;
}

// DDPX_WSGD_SPREAD=s: the stream waves update each tile in the first ceil(nk / s) K-steps (default 1: one
// share per K-step; front-loading measured slower, profiles/r2_spread)
static inline int spread() {
  static const int v = [] {
    const char* e = getenv("DDPX_WSGD_SPREAD");
    const int x = e ? atoi(e) : 1;
    return x >= 1 ? x : 1;
  }();
  return v;
}

static inline hipError_t launch(const pipe::Params& p, int num_cus, hipStream_t s) {
  const int ntiles = (p.M / BM) * (p.N / BN);
  const int grid = ntiles < num_cus ? ntiles : num_cus;
  if (stages(ntiles, num_cus) == 4) hipLaunchKernelGGL(wgrad_sgd_ws_kernel<4>, dim3(grid), dim3(512), 0, s, p, p, 0, spread());
  else hipLaunchKernelGGL(wgrad_sgd_ws_kernel<3>, dim3(grid), dim3(512), 0, s, p, p, 0, spread());
  return hipGetLastError();
}

// Both weight gradients (+ their SGD updates) in one launch; the caller checked eligible() for both and equal
// K / alpha / lr / momentum / wd (pair_compatible).
static inline bool pair_compatible(const pipe::Params& a, const pipe::Params& b) {
  return a.K == b.K && a.alpha == b.alpha && a.sgd.lr == b.sgd.lr && a.sgd.mom == b.sgd.mom && a.sgd.wd == b.sgd.wd;
}

static inline hipError_t launch_pair(const pipe::Params& p0, const pipe::Params& p1, int num_cus, hipStream_t s) {
  const int nt1 = (p1.M / BM) * (p1.N / BN);
  const int ntiles = (p0.M / BM) * (p0.N / BN) + nt1;
  const int grid = ntiles < num_cus ? ntiles : num_cus;
  if (stages(ntiles, num_cus) == 4)
    hipLaunchKernelGGL(wgrad_sgd_ws_kernel<4>, dim3(grid), dim3(512), 0, s, p0, p1, nt1, spread());
  else hipLaunchKernelGGL(wgrad_sgd_ws_kernel<3>, dim3(grid), dim3(512), 0, s, p0, p1, nt1, spread());
  return hipGetLastError();
}

}  // namespace wsgd
}  // namespace ddpx
