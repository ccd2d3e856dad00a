// ddpx — a layer's data gradient folded into the warp-specialised weight-gradient + SGD launch (gfx950).
//
// The toy MLP's backward (batch 512, 3072-4096-4096-10) after the classifier head is, unfused,
//   dgrad(fc1):  dH0 = (dH1 W1) * (H0 > 0), fc0 bias gradient + SGD        (34.7 us, L2 -> CU bound GEMM)
//   pair:        W1 -= sgd(dH1^T H0), W0 -= sgd(dH0^T X)                     (116-127 us, HBM bound: the
//                optimizer streams 18 B per weight while the MFMA waves sit at barriers waiting for it)
// (profiles/r3_final/mlp_kernel_stats_v19.csv).  Here the data gradient runs on the SAME math waves as fc1's
// weight gradient, one K-step of each per barrier interval, so its MFMAs and operand loads fill the time the
// math waves spent waiting for the stream; fc0's weight-gradient tiles follow once every workgroup's share
// of dH0 is published.  One launch instead of two.
//
// Work per workgroup (one per CU, 4 math + NSW stream waves, the protocol of ddpx_wgrad_sgd.h):
//   phase 1: n1 fc1 weight-gradient tiles (64 x 128, K = batch = 512: 8 K-steps each) and nd data-gradient
//            tiles (64 x 128 of dH0, K = 4096: 64 K-steps each) with n1 * 8 == nd * 64 (the two GEMMs have
//            the same M*N*K), interleaved one K-step each per interval; a data-gradient tile's epilogue
//            (ReLU mask, bf16 store, column sums of the fc0 bias gradient, the bias SGD by the last row
//            tile of each column block) runs at the end of the weight-gradient tile in which it completes;
//   phase 2: n0 fc0 weight-gradient tiles (their A operand is dH0, written by every workgroup in phase 1).
// The stream waves update tile i-1 during tile i exactly as in the pair kernel (two accumulator buffers);
// the data-gradient epilogue stages through the buffer tile i's accumulators will go to, which nothing reads
// until then (LDS: 2 x 24 KiB + 2 x 24 KiB rings + 2 x 32 KiB buffers = all 160 KiB).
//
// Hazards and how they are met:
//   * W1 is read by the data gradient while the stream waves rewrite it: the stream writes the new bf16
//     compute copy of W1 into the OTHER buffer of a ping-pong pair (FlatParams ping-pong parity), so the data
//     gradient reads the copy the forward used; the fp32 master / momentum are not read by any GEMM;
//   * dH0 crosses workgroups (fc0's tile (i, *) needs dH0[:, 64i .. 64i+63] from 8 row tiles on other CUs):
//     the data-gradient tiles store it write-through (sc1), every storing wave drains (vmcnt(0)), then one
//     lane adds to a launch-wide counter; before the first fc0 operand load every math wave polls that
//     counter (relaxed sc1 loads, bounded spin) and takes ONE agent-scope acquire (MI355X_MICROARCH.md
//     "Valid forms", Guideline 16).  The counter, the column tickets and the timeout word are zeroed by a
//     memset node ahead of every launch.  Every workgroup is resident (grid = CUs, one 512-thread workgroup
//     per CU), so the wait always ends;
//   * barrier counts: both roles execute, per weight-gradient tile, nk K-step barriers + (EB epilogue
//     barriers when a data-gradient tile completes in it) + 1 hand-off barrier, for nt + 1 iterations.
// Arithmetic: the data gradient accumulates in the same k order as the 64x64 pipe tile and its epilogue
// (mask, bf16 rounding, per-64-column quad / row-group column sums, row-tile-order finish, sgd_apply) is
// the standalone dgrad kernel's, and the stream's update is sgd_apply's: bitwise equal to dgrad + pair.
#pragma once

#include "ddpx_wgrad_sgd.h"

namespace ddpx {
namespace wsgdd {

using wsgd::A_SUB;
using wsgd::B_SUB;
using wsgd::BM;
using wsgd::BN;
using wsgd::SLOT;
using wsgd::VPT;

constexpr int ALD = BN;                           // accumulator row stride (floats): unpadded, 2 buffers fit
constexpr int ACC_BYTES = BM * ALD * 4;           // 32 KiB per buffer
constexpr int WRING = 0, DRING = 2 * SLOT, ACCB = 4 * SLOT;
constexpr int LDS_BYTES = 4 * SLOT + 2 * ACC_BYTES;  // 163,840 B: the whole LDS
static_assert(LDS_BYTES <= 160 * 1024, "LDS");
constexpr int EB = 9;                            // barriers of one data-gradient epilogue (both roles)
constexpr unsigned kSpinMax = 1u << 22;          // ~ seconds of s_sleep polling before the give-up code

struct DgArgs {
  const unsigned short* A;    // dY [M = batch][K] bf16 (K-contig)
  const unsigned short* B;    // W [K][N] bf16 (N-contig: the weight's compute copy the forward read)
  unsigned short* C;          // dX [M][N] bf16 (the next weight-gradient's A operand)
  const unsigned short* aux;  // ReLU mask source [M][N] bf16
  int M, N, K, lda, ldb, ldc, ldaux;
  unsigned a_bytes, b_bytes;
  float* colsum;              // [M / 64][N] fp32 per-row-tile column sums (write-through)
  int* tickets;               // [N / 128] per column block; zeroed before every launch
  int* done;                  // [1] data-gradient tiles published; zeroed before every launch
  int* err;                   // [1] spin give-up flag; zeroed before every launch
  SgdArgs bias;               // the bias of the layer below (fused SGD of its gradient)
};

__device__ __forceinline__ void bar() { __builtin_amdgcn_s_barrier(); }

template <bool FP8, int NSW>
__global__ void __launch_bounds__(256 + 64 * NSW)
wgrad_sgd_dgrad_kernel(pipe::Params p1, pipe::Params p0, DgArgs d) {
  constexpr int FM = 2, FN = 4;  // math wave tile 32 x 64 (both GEMMs)
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  float* const accb = reinterpret_cast<float*>(smem + ACCB);  // two accumulator buffers (tile i -> i & 1)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = (int)gridDim.x, b = (int)blockIdx.x;
  const int tn1 = p1.N / BN, tn0 = p0.N / BN;
  const int nt1 = (p1.M / BM) * tn1, nt0 = (p0.M / BM) * tn0;
  const int n1 = nt1 / G;                                   // exact (host-checked)
  const int n0 = (nt0 - b + G - 1) / G;
  const int nt = n1 + n0;
  const int nk = p1.K / 64;                                 // == VPT (8)
  const int tmd = d.M / BM;                                 // data-gradient row tiles (8)
  const int nkd = d.K / 64;
  const int ndw = (n1 * nk) / nkd;                          // data-gradient tiles per workgroup
  const int nd = ndw * G;
  // wgrad tile i: origin, GEMM (1: fc1, 0: fc0); n-fastest (ddpx_wgrad_sgd.h NORD)
  auto wtile = [&](int i, int& m0, int& n0_) -> int {
    if (i < n1) {
      const int g = b + i * G;
      m0 = (g / tn1) * BM;
      n0_ = (g % tn1) * BN;
      return 1;
    }
    const int g = b + (i - n1) * G;
    m0 = (g / tn0) * BM;
    n0_ = (g % tn0) * BN;
    return 0;
  };
  // data-gradient tile j of this workgroup.  The tmd row tiles of one column block read the same W1 column
  // panel (K x 128 bf16, 1 MiB for the toy MLP): they are given workgroup ids of equal id % 8 — one XCD under
  // round-robin placement (speed only, never correctness: MI355X_MICROARCH.md) — so the panel comes from
  // that XCD's L2 after its first reader instead of 8 times from the Infinity Cache / HBM.
  const int ncb = d.N / BN;
  const bool xcd_map = (ncb % 8) == 0 && ((ndw * G) % 8) == 0;
  auto dtile = [&](int j, int& m0, int& n0_) {
    const int g = b + j * G;
    if (xcd_map) {
      const int x = g & 7, s = g >> 3;  // (id % 8, id / 8)
      m0 = (s % tmd) * BM;
      n0_ = (x * (ncb / 8) + s / tmd) * BN;
    } else {
      m0 = (g % tmd) * BM;
      n0_ = (g / tmd) * BN;
    }
  };
  // a data-gradient tile completes at the end of weight-gradient iteration i (phase 1 only)
  auto dg_done_at = [&](int i) -> bool { return i < n1 && ((i + 1) * nk) % nkd == 0; };

  if (wave < 4) {
    // ------------------------------------------------------------------ math waves
    const int wm = wave >> 1, wn = wave & 1;
    const __amdgpu_buffer_rsrc_t ra1 = __builtin_amdgcn_make_buffer_rsrc((void*)p1.A, 0, p1.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb1 = __builtin_amdgcn_make_buffer_rsrc((void*)p1.B, 0, p1.b_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ra0 = __builtin_amdgcn_make_buffer_rsrc((void*)p0.A, 0, p0.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb0 = __builtin_amdgcn_make_buffer_rsrc((void*)p0.B, 0, p0.b_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rda = __builtin_amdgcn_make_buffer_rsrc((void*)d.A, 0, d.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rdb = __builtin_amdgcn_make_buffer_rsrc((void*)d.B, 0, d.b_bytes, 0x00020000);
    const int GW = nt * nk;      // weight-gradient K-steps of this workgroup
    const int GD = n1 * nk;      // data-gradient K-steps (== ndw * nkd), interleaved with the first GD
    const int G1 = n1 * nk;      // first fc0 K-step (phase boundary: no DMA look-ahead across it)
    auto issue_w = [&](int g) {
      int m0, n0_;
      const int sel = wtile(g / nk, m0, n0_);
      const int kt = g % nk;
      char* slot = smem + WRING + (g & 1) * SLOT;
      const pipe::Params& p = sel ? p1 : p0;
      pipe::stage_tile<BM, false, pipe::MODE_PLAIN, 4>(sel ? ra1 : ra0, slot, p.conv, p.lda, m0, p.M, kt * 64, p.K,
                                                       wave, lane);
      pipe::stage_tile<BN, false, pipe::MODE_PLAIN, 4>(sel ? rb1 : rb0, slot + A_SUB, p.conv, p.ldb, n0_, p.N, kt * 64,
                                                       p.K, wave, lane);
    };
    auto issue_d = [&](int h) {
      int m0, n0_;
      dtile(h / nkd, m0, n0_);
      const int kt = h % nkd;
      char* slot = smem + DRING + (h & 1) * SLOT;
      pipe::stage_tile<BM, true, pipe::MODE_PLAIN, 4>(rda, slot, p1.conv, d.lda, m0, d.M, kt * 64, d.K, wave, lane);
      pipe::stage_tile<BN, false, pipe::MODE_PLAIN, 4>(rdb, slot + A_SUB, p1.conv, d.ldb, n0_, d.N, kt * 64, d.K, wave,
                                                       lane);
    };
    // the launch-wide "every data-gradient tile published" wait, then one agent-scope acquire: the fc0
    // operand loads that follow read dH0 bytes other CUs stored write-through (bounded spin: give-up code)
    auto wait_published = [&]() {
      unsigned spins = 0;
      while (__hip_atomic_load(d.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nd) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > kSpinMax) {
          if (lane == 0) __hip_atomic_store(d.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };

    if (GW > 0 && G1 > 0) issue_w(0);
    if (GD > 0) issue_d(0);
    // data-gradient accumulators: one tile spans nkd / nk weight-gradient tiles, reset after its epilogue
    f32x4 ad[FM][FN];
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
      for (int c = 0; c < FN; ++c) ad[a][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i <= nt; ++i) {
      if (i == nt) {  // drain iteration: the stream waves finish the last tile
        for (int t = 0; t < nk; ++t) bar();
        bar();
        break;
      }
      f32x4 aw[FM][FN];
#pragma unroll
      for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int c = 0; c < FN; ++c) aw[a][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
      for (int t = 0; t < nk; ++t) {
        const int g = i * nk + t;
        if (g == G1) {  // first fc0 K-step: its operand was not prefetched across the phase boundary
          wait_published();
          issue_w(g);
        }
        pipe::wait_vmcnt<0>();  // stage g (both rings) landed: the only DMA in flight
        bar();
        asm volatile("" ::: "memory");
        if (g + 1 < GW && g + 1 != G1) issue_w(g + 1);
        const bool dg = g < GD;
        if (dg && g + 1 < GD) issue_d(g + 1);
        const char* sa = smem + WRING + (g & 1) * SLOT;
        const char* da = smem + DRING + (g & 1) * SLOT;
#pragma unroll
        for (int kk = 0; kk < 64; kk += 32) {
          bf16x8 af[FM], bfr[FN];
          pipe::load_frags<BM, false, FM, BN, false, FN>(sa, wm * 32, sa + A_SUB, wn * 64, kk, lane, af, bfr);
#pragma unroll
          for (int a = 0; a < FM; ++a)
#pragma unroll
            for (int c = 0; c < FN; ++c)
              aw[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfr[c], aw[a][c], 0, 0, 0);
          if (dg) {
            bf16x8 xf[FM], yf[FN];
            pipe::load_frags<BM, true, FM, BN, false, FN>(da, wm * 32, da + A_SUB, wn * 64, kk, lane, xf, yf);
#pragma unroll
            for (int a = 0; a < FM; ++a)
#pragma unroll
              for (int c = 0; c < FN; ++c)
                ad[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[a], yf[c], ad[a][c], 0, 0, 0);
          }
        }
      }
      if (dg_done_at(i)) {
        // ---------------- data-gradient epilogue: 64 x 128 tile j, staged in two 64-column halves through T
        int dm0, dn0;
        const int j = ((i + 1) * nk) / nkd - 1;
        dtile(j, dm0, dn0);
        const int tm = dm0 / BM;
        const int cq = tid & 15, r0 = tid >> 4;  // the 64x64 pipe tile's epilogue map (NT 256, BN 64)
        // scratch: accumulator buffer i & 1 (the stream waves last read it during tile i - 1; tile i's
        // accumulators go there only after this epilogue)
        float* const T = accb + (i & 1) * (ACC_BYTES / 4);
        float* red = T + BM * 68;                 // [16][64] row-group partials
        int* flag = reinterpret_cast<int*>(red + 16 * 64);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (wn == h) {
            const int mr = wm * 32 + 4 * (lane >> 4), nc = lane & 15;
#pragma unroll
            for (int a = 0; a < FM; ++a)
#pragma unroll
              for (int c = 0; c < FN; ++c)
#pragma unroll
                for (int r = 0; r < 4; ++r) T[(mr + a * 16 + r) * 68 + nc + c * 16] = ad[a][c][r];
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          bar();  // (1, 4) staged half complete
          const int n = dn0 + 64 * h + 4 * cq;
          u32x2 av[4];
#pragma unroll
          for (int v = 0; v < 4; ++v)  // all mask loads in flight first (epilogue_vec phase 1)
            av[v] = *reinterpret_cast<const u32x2*>(d.aux + (size_t)(dm0 + r0 + 16 * v) * d.ldaux + n);
          float cs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int r = r0 + 16 * v;
            const f32x4 x = *reinterpret_cast<const f32x4*>(T + r * 68 + 4 * cq);
            float st[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const unsigned short m = (unsigned short)((q & 1) ? (av[v][q >> 1] >> 16) : (av[v][q >> 1] & 0xffffu));
              const bool pos = (m & 0x8000u) == 0 && (m & 0x7fffu) != 0;
              st[q] = pos ? bf2f(f2bf(x[q])) : 0.f;
              cs[q] += st[q];
            }
            const unsigned long long packed =
                (unsigned long long)pack_bf2(st[0], st[1]) | ((unsigned long long)pack_bf2(st[2], st[3]) << 32);
            // write-through: fc0's tiles on other CUs read these bytes after the published-counter wait
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(d.C + (size_t)(dm0 + r) * d.ldc + n), packed,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) red[r0 * 64 + 4 * cq + q] = cs[q];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          bar();  // (2, 5) row-group partials complete
          if (tid < 64) {
            float s = 0.f;
            for (int gr = 0; gr < 16; ++gr) s += red[gr * 64 + tid];
            __hip_atomic_store(d.colsum + (size_t)tm * d.N + dn0 + 64 * h + tid, s, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          bar();  // (3, 6) T / red free for the next half
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
        bar();                                            // (7)
        if (tid == 0) {
          *flag = __hip_atomic_fetch_add(d.tickets + dn0 / BN, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add(d.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar();  // (8) ticket visible to the workgroup
        const bool last_row_tile = *flag == tmd - 1;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar();  // (9) every wave read the ticket: the buffer may take tile i's accumulators
        if (last_row_tile && tid < BN) {
          // last row tile of this column block: the bias gradient in row-tile order, applied as SGD
          const __amdgpu_buffer_rsrc_t rcs = __builtin_amdgcn_make_buffer_rsrc(
              (void*)d.colsum, 0, (unsigned)((size_t)tmd * d.N * 4), 0x00020000);
          float tot = 0.f;
          for (int t0 = 0; t0 < tmd; t0 += 8) {
            float v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q)
              v[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                  rcs, (unsigned)(((size_t)(t0 + q) * d.N + dn0 + tid) * 4), 0, 16 /* sc1 */));
#pragma unroll
            for (int q = 0; q < 8; ++q) tot += v[q];
          }
          sgd_apply(d.bias, dn0 + tid, tot, *d.bias.lr);
        }
#pragma unroll
        for (int a = 0; a < FM; ++a)
#pragma unroll
          for (int c = 0; c < FN; ++c) ad[a][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
      // weight-gradient accumulators -> buffer i & 1 (the stream waves update tile i - 1 from the other one)
      {
        float* const T = accb + (i & 1) * (ACC_BYTES / 4);
        const int mr = wm * 32 + 4 * (lane >> 4), nc = wn * 64 + (lane & 15);
#pragma unroll
        for (int a = 0; a < FM; ++a)
#pragma unroll
          for (int c = 0; c < FN; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) T[(mr + a * 16 + r) * ALD + nc + c * 16] = aw[a][c][r] * p1.alpha;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar();  // hand-off
    }
  } else {
    // ---------------------------------------------------------------- stream waves (ddpx_wgrad_sgd.h)
    constexpr int DIST = 4;
    constexpr int SV = BM * BN / 4 / (NSW * 64);
    constexpr int KPU = VPT / SV;
    constexpr int RSTEP = NSW * 2;
    static_assert(SV % DIST == 0 && VPT % SV == 0, "ring");
    const int st = tid - 256;
    const int row0 = st >> 5, col = 4 * (st & 31);
    const float lr = *p1.sgd.lr;
    const float mom = p1.sgd.mom, wd = p1.sgd.wd;
    const bool has_mom = mom != 0.f;
    f32x4 rp[DIST], rm[DIST];
    float* const P0 = p0.sgd.p;
    float* const P1 = p1.sgd.p;
    float* const M0 = has_mom ? p0.sgd.buf : p0.sgd.p;
    float* const M1 = has_mom ? p1.sgd.buf : p1.sgd.p;
    unsigned short* const S0 = p0.sgd.shadow;
    unsigned short* const S1 = p1.sgd.shadow;
    unsigned char* const Q0 = p0.sgd.q8;
    unsigned char* const Q1 = p1.sgd.q8;
    unsigned char* const E0 = p0.sgd.s8;
    unsigned char* const E1 = p1.sgd.s8;
    const int ldc0 = p0.ldc, ldc1 = p1.ldc;
    auto vec_off = [&](int j, int v, int& sel) -> size_t {
      int m0, n0_;
      sel = wtile(j, m0, n0_);
      return (size_t)(m0 + row0 + RSTEP * v) * (sel ? ldc1 : ldc0) + n0_ + col;
    };
    auto load_vec = [&](int j, int v, f32x4& pv, f32x4& mv) {
      int sel;
      const size_t off = vec_off(j, v, sel);
      pv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>((sel ? P1 : P0) + off));
      mv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>((sel ? M1 : M0) + off));
    };
    auto update_vec = [&](int j, int v, const float* T, f32x4& pv, f32x4& mv) {
      int sel;
      const size_t off = vec_off(j, v, sel);
      const f32x4 g = *reinterpret_cast<const f32x4*>(T + (row0 + RSTEP * v) * ALD + col);
      f32x4 po, bo;
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // sgd_apply's fma sequence
        float dd = fmaf(wd, pv[q], g[q]);
        if (has_mom) dd = fmaf(mom, mv[q], dd);
        po[q] = fmaf(-lr, dd, pv[q]);
        bo[q] = has_mom ? dd : po[q];
      }
      __builtin_nontemporal_store(po, reinterpret_cast<f32x4*>((sel ? P1 : P0) + off));
      __builtin_nontemporal_store(bo, reinterpret_cast<f32x4*>((sel ? M1 : M0) + off));
      *reinterpret_cast<u32x2*>((sel ? S1 : S0) + off) = (u32x2){pack_bf2(po[0], po[1]), pack_bf2(po[2], po[3])};
      if constexpr (FP8) {
        unsigned e8;
        const unsigned q = mx::e4m3_group8(po, &e8);
        *reinterpret_cast<unsigned*>((sel ? Q1 : Q0) + off) = q;
        const unsigned e1 = __shfl_down(e8, 8, 64), e2 = __shfl_down(e8, 16, 64), e3 = __shfl_down(e8, 24, 64);
        if ((lane & 31) == 0)
          *reinterpret_cast<unsigned*>((sel ? E1 : E0) + (off >> 5)) = e8 | (e1 << 8) | (e2 << 16) | (e3 << 24);
      }
      const int vn = v + DIST;
      const bool same = vn < SV, next = !same && j + 1 < nt;
      load_vec(same ? j : (next ? j + 1 : j), same ? vn : (next ? vn - SV : v), pv, mv);
    };
    if (nt > 0) {
#pragma unroll
      for (int v = 0; v < DIST; ++v) load_vec(0, v, rp[v], rm[v]);
    }
    // iteration 0: the math waves fill the first tile
    for (int t = 0; t < nk; ++t) bar();
    if (dg_done_at(0))
      for (int e = 0; e < EB; ++e) bar();
    bar();
    // trip r = DIST K-steps: iteration i = 1 + r / TPI updates tile i - 1, vectors (r % TPI) * DIST .. + DIST - 1
    // (ddpx_wgrad_sgd.h); the first trip is peeled so the loop is entered with the same memory operations in
    // flight as on its back edge (the compiler then counts every update's ring wait: vmcnt(15/16))
    constexpr int TPI = SV / DIST;
    auto trip = [&](int r) {
      const int i = 1 + r / TPI, t = (r % TPI) * DIST;
      const float* T = accb + ((i - 1) & 1) * (ACC_BYTES / 4);
#pragma unroll
      for (int u = 0; u < DIST; ++u) {
        bar();
        __builtin_amdgcn_sched_barrier(0);
        update_vec(i - 1, t + u, T, rp[u], rm[u]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 1; k < KPU; ++k) bar();
      }
      if (r % TPI == TPI - 1) {  // end of iteration i: its epilogue barriers (if any), then the hand-off
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (i < nt && dg_done_at(i))
          for (int e = 0; e < EB; ++e) bar();
        bar();
      }
    };
    if (nt >= 1) trip(0);
#pragma unroll 1
    for (int r = 1; r < TPI * nt; ++r) trip(r);
  }
}

// Eligible: both weight gradients are wsgd::eligible (K = 512), the data gradient is the fc1 layer's
// (d.M = batch, d.K = fc1's M, d.N = fc1's N ... i.e. dX = dY W with W [K][N] = fc1's weight), dX feeds fc0's
// weight gradient as its A operand, and the tiles divide evenly over the grid.
static inline bool eligible(const pipe::Params& p1, const pipe::Params& p0, const DgArgs& d, int grid) {
  if (!wsgd::eligible(p1, false, false) || !wsgd::eligible(p0, false, false) || !wsgd::pair_compatible(p1, p0))
    return false;
  if ((p1.sgd.q8 != nullptr) != (p0.sgd.q8 != nullptr)) return false;
  if (d.M != p1.K || d.M % BM || d.N % BN || d.K % 64 || d.K != p1.M || d.N != p1.N || d.N != p0.M) return false;
  if ((d.lda & 7) || (d.ldb & 7) || (d.ldc & 3) || (d.ldaux & 3)) return false;
  if (!d.colsum || !d.tickets || !d.done || !d.err || !d.bias.p || !d.bias.lr) return false;
  if ((d.bias.mom != 0.f) && !d.bias.buf) return false;
  const int nt1 = (p1.M / BM) * (p1.N / BN), nd = (d.M / BM) * (d.N / BN);
  const int nk = p1.K / 64, nkd = d.K / 64;
  if (grid <= 0 || nt1 % grid || nd % grid) return false;
  if ((nt1 / grid) * nk != (nd / grid) * nkd) return false;
  return true;
}

static inline hipError_t launch(const pipe::Params& p1, const pipe::Params& p0, const DgArgs& d, int grid,
                                size_t zero_bytes, hipStream_t s) {
  // every polled / counted word of this launch starts at zero: tickets, done, err (one block, 16-B multiple)
  hipError_t e = hipMemsetAsync(d.tickets, 0, zero_bytes, s);
  if (e != hipSuccess) return e;
  // 4 stream waves: the 8-wave variant's ring waits come out uncounted (vmcnt(4/8/12)) with the epilogue
  // barriers in its loop body
  const bool fp8 = p1.sgd.q8 != nullptr;
  if (fp8) hipLaunchKernelGGL((wgrad_sgd_dgrad_kernel<true, 4>), dim3(grid), dim3(512), 0, s, p1, p0, d);
  else hipLaunchKernelGGL((wgrad_sgd_dgrad_kernel<false, 4>), dim3(grid), dim3(512), 0, s, p1, p0, d);
  return hipGetLastError();
}

}  // namespace wsgdd
}  // namespace ddpx
