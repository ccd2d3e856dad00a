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
// Here every workgroup (one per CU, 4 + NSW waves) owns a list of 64x128 tiles (n-fastest over W, so the tiles
// in flight on the chip cover whole rows of W) and splits its waves by role:
//   * waves 0-3 (math): the LDS-DMA ring + v_mfma_f32_16x16x32_bf16 main loop of tile i (the pipe core of
//     ddpx_pipe.h), then its fp32 accumulators into one of two LDS tile buffers;
//   * waves 4.. (stream, NSW = 4 or 8): the optimizer update of tile i-1 from the other buffer, spread over
//     the K-steps, master / momentum loads a 4-vector ring ahead (non-temporal, counted vmcnt waits) — so a
//     CU's HBM stream runs while its matrix cores work on the next tile.
// Both roles execute exactly nk + 1 s_barriers per iteration (nk K-steps of 64, then the buffer hand-off)
// for nt + 1 iterations (one drain iteration), so the barrier sequence matches by construction.
// The update arithmetic is sgd_apply's fma sequence: bitwise equal to the stored-gradient + flat-SGD path.
#pragma once

#include <cstdlib>

#include "ddpx_mx.h"
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
//   SB (single hand-off buffer): the stream waves read each gradient vector one K-step ahead, so they never touch
//             the buffer in the K-step the math waves refill it: one fp32 tile buffer instead of two, which leaves
//             room for a 4-stage ring with padded rows (DDPX_WSGD_SB=1, 4 stream waves).
// Diagnostics (ddpx_gemm_set_stamps, benchmarks/pair_stamps.py): with p0.stamp set, lane 0 of wave 0 (math role)
// and of wave 4 (stream role) write s_memrealtime (10 ns ticks) at kernel start (slot 0), on ARRIVAL at each of the
// role's s_barriers (slots 1..), and at kernel end (last slot): stamp[(block * 2 + role) * kStampSlots + slot].  A
// barrier's departure is the later of the two roles' arrivals, so the per-barrier wait of each role shows which
// side sets the pace.  Off (a null pointer) it costs a scalar test per barrier.
constexpr int kStampSlots = 256;

template <int STAGES, int XTRA = 0, bool SB = false>
struct Cfg {
  static constexpr int ALD = (STAGES >= 4 && !SB) ? BN : BN + 4;
  static constexpr int ACC_BYTES = BM * ALD * 4;
  static constexpr int LDS_BYTES = STAGES * SLOT + (SB ? 1 : 2) * ACC_BYTES + (XTRA == 2 ? SLOT : 0);
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

// Two GEMMs may share one launch (p0's tiles, then p1's: the toy MLP's fc1 and fc0 weight gradients are
// independent once fc1's data gradient ran): one fill and one drain iteration instead of two, one launch
// boundary fewer.  Single GEMM: p1 = p0 and nt1 = 0.  Both must have the same K, lr, momentum, wd, alpha.
// XTRA (measurement only, DDPX_WSGD_XTRA): 3 = math only (the stream waves keep the barrier sequence but load,
// update and store nothing), 4 = stream only (the math waves issue no DMA and no MFMA: zero gradients);
// 1 = every K-step runs its MFMAs twice (the second set into a
// dead accumulator kept live), 2 = also a second operand stage of LDS-DMA per K-step into a dummy ring — the
// math and L2->LDS load a fused data-gradient GEMM would add beside the weight-gradient tiles.
// NMW: math waves, 4 (2 x 2 waves of 32 x 64) or 8 (2 x 4 waves of 32 x 32: two MFMA waves per SIMD, so one wave's
// fragment reads, DMA issue and barrier wait run under the other's MFMAs — the 4-wave math side ran its K-steps at
// 11 % MFMA busy with its waves waiting 62 % of their cycles, profiles/r6_pair).
// CP (cache policy of the optimizer stream, measurement: DDPX_WSGD_CACHE): 0 = master / momentum non-temporal loads
// and stores, shadow plain (default); 1 = everything plain (the 235 MB of toy-MLP master + momentum could stay in the
// 256 MB Infinity Cache between steps); 2 = the shadow store non-temporal too.
template <int STAGES, bool FP8, int NSW, bool NORD, int XTRA = 0, bool SB = false, int NMW = 4, int CP = 0>
__global__ void __launch_bounds__(64 * NMW + 64 * NSW) wgrad_sgd_ws_kernel(pipe::Params p0, pipe::Params p1, int nt1) {
  constexpr int ALD = Cfg<STAGES, XTRA, SB>::ALD, ACC_BYTES = Cfg<STAGES, XTRA, SB>::ACC_BYTES;
  constexpr int LDS_BYTES = Cfg<STAGES, XTRA, SB>::LDS_BYTES;
  static_assert(NMW == 4 || NMW == 8, "math waves");
  constexpr int WN = NMW / 2;                    // math waves along N
  constexpr int FM = 2, FN = BN / WN / 16;       // math wave tile 32 x (BN / WN)
  constexpr int LPW = (BM + BN) / (8 * NMW);     // LDS-DMA instructions per math wave per stage
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
  // NORD: the tiles running at once sweep whole rows of W (n fastest): the optimizer stream then reads and
  // writes every row's 512-B tile segments side by side instead of 64 rows x 4 segments scattered over W
  // (m fastest), which is what the HBM sees of 256 CUs streaming at once.
  auto tile_origin = [&](int i, int& m0, int& n0) -> int {
    int g = (int)blockIdx.x + i * (int)gridDim.x;
    const int sel = g >= nt0;
    if (sel) g -= nt0;
    if constexpr (NORD) {
      const int tn = (sel ? p1.N : p0.N) / BN;
      m0 = (g / tn) * BM;
      n0 = (g % tn) * BN;
    } else {
      const int tm = sel ? tiles_m1 : tiles_m0;
      m0 = (g % tm) * BM;
      n0 = (g / tm) * BN;
    }
    return sel;
  };
  const pipe::Params& p = p0;  // K, alpha, lr, momentum, wd: shared by both GEMMs
  long long* const stp = (p0.stamp && (tid == 0 || tid == 64 * NMW))
                             ? p0.stamp + ((size_t)blockIdx.x * 2 + (wave < NMW ? 0 : 1)) * kStampSlots
                             : nullptr;
  int nstamp = 1;
  auto mark = [&]() {  // arrival at the role's next barrier
    if (stp) {
      stp[nstamp < kStampSlots - 1 ? nstamp : kStampSlots - 2] = (long long)__builtin_amdgcn_s_memrealtime();
      ++nstamp;
    }
  };
  if (stp) stp[0] = (long long)__builtin_amdgcn_s_memrealtime();

  if (wave < NMW) {
    // ------------------------------------------------------------------ math waves
    const int wm = wave / WN, wn = wave % WN;
    const __amdgpu_buffer_rsrc_t ra0 = __builtin_amdgcn_make_buffer_rsrc((void*)p0.A, 0, p0.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb0 = __builtin_amdgcn_make_buffer_rsrc((void*)p0.B, 0, p0.b_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ra1 = __builtin_amdgcn_make_buffer_rsrc((void*)p1.A, 0, p1.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb1 = __builtin_amdgcn_make_buffer_rsrc((void*)p1.B, 0, p1.b_bytes, 0x00020000);
    // One LDS-DMA ring across ALL of this workgroup's tiles: K-step g of the workgroup's sequence is K-step
    // g % nk of its tile g / nk, and stage g + STAGES - 1 is issued during K-step g even when it belongs to
    // the next tile, so the ring never drains and refills at a tile boundary (with K = 512 a tile is only
    // nk = 8 K-steps: a per-tile refill cost ~2 of every 10 K-steps of L2 latency).
    const int G = nt * nk;
    // the issuer walks g = 0, 1, 2, ... in order: the tile origin (integer divisions) is computed once per tile
    int iss_i = -1, iss_kt = nk - 1, iss_m0 = 0, iss_n0 = 0, iss_sel = 0;
    auto issue = [&](int g) {
      if constexpr (XTRA == 4) return;  // measurement: stream only
      if (++iss_kt >= nk) {
        iss_kt = 0;
        iss_sel = tile_origin(++iss_i, iss_m0, iss_n0);
      }
      const int m0 = iss_m0, n0 = iss_n0, sel = iss_sel, kt = iss_kt;
      const __amdgpu_buffer_rsrc_t ra = sel ? ra1 : ra0, rb = sel ? rb1 : rb0;
      const int lda = sel ? p1.lda : p0.lda, ldb = sel ? p1.ldb : p0.ldb;
      const int Mg = sel ? p1.M : p0.M, Ng = sel ? p1.N : p0.N;
      char* slot = smem + (g % STAGES) * SLOT;
      pipe::stage_tile<BM, false, pipe::MODE_PLAIN, NMW>(ra, slot, p.conv, lda, m0, Mg, kt * 64, p.K, wave, lane);
      pipe::stage_tile<BN, false, pipe::MODE_PLAIN, NMW>(rb, slot + A_SUB, p.conv, ldb, n0, Ng, kt * 64, p.K, wave,
                                                         lane);
      if constexpr (XTRA == 2) {  // dummy second stage (same operands, other k rows) into the extra ring
        char* x = smem + STAGES * SLOT + 2 * ACC_BYTES;  // one dummy slot (its contents are never used)
        const int kx = ((kt + 3) % (p.K / 64)) * 64;
        pipe::stage_tile<BM, false, pipe::MODE_PLAIN, NMW>(ra, x, p.conv, lda, m0, Mg, kx, p.K, wave, lane);
        pipe::stage_tile<BN, false, pipe::MODE_PLAIN, NMW>(rb, x + A_SUB, p.conv, ldb, n0, Ng, kx, p.K, wave, lane);
      }
    };
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < G) issue(s);
    for (int i = 0; i <= nt; ++i) {
      if (i == nt) {  // drain iteration: the stream waves finish the last tile
        for (int t = 0; t < nk; ++t) {
          mark();
          __builtin_amdgcn_s_barrier();
        }
      } else {
        f32x4 acc[FM][FN], acc2[FM][FN];
#pragma unroll
        for (int a = 0; a < FM; ++a)
#pragma unroll
          for (int b = 0; b < FN; ++b) acc[a][b] = acc2[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
        for (int t = 0; t < nk; ++t) {
          const int g = i * nk + t;
          const int ahead = min(STAGES - 2, G - 1 - g);
          constexpr int LW = XTRA == 2 ? 2 * LPW : LPW;
          // stage g landed: everything but the (up to STAGES - 2) younger stages' DMAs
          if (STAGES >= 5 && ahead >= 3) pipe::wait_vmcnt<3 * LW>();
          else if (STAGES >= 4 && ahead >= 2) pipe::wait_vmcnt<2 * LW>();
          else if (ahead >= 1) pipe::wait_vmcnt<LW>();
          else pipe::wait_vmcnt<0>();
          mark();
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
          if (g + STAGES - 1 < G) issue(g + STAGES - 1);
          const char* sa = smem + (g % STAGES) * SLOT;
          const char* sb = sa + A_SUB;
#pragma unroll
          for (int kk = 0; kk < (XTRA == 4 ? 0 : 64); kk += 32) {
            bf16x8 af[FM], bfr[FN];
            pipe::load_frags<BM, false, FM, BN, false, FN>(sa, wm * 32, sb, wn * (BN / WN), kk, lane, af, bfr);
#pragma unroll
            for (int a = 0; a < FM; ++a)
#pragma unroll
              for (int b = 0; b < FN; ++b)
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
            if constexpr (XTRA == 1 || XTRA == 2) {
              const char* xa = XTRA == 2 ? smem + STAGES * SLOT + 2 * ACC_BYTES : sa;
              bf16x8 af2[FM], bf2[FN];
              pipe::load_frags<BM, false, FM, BN, false, FN>(xa, wm * 32, xa + A_SUB, wn * (BN / WN), kk, lane, af2,
                                                             bf2);
#pragma unroll
              for (int a = 0; a < FM; ++a)
#pragma unroll
                for (int b = 0; b < FN; ++b)
                  acc2[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af2[a], bf2[b], acc2[a][b], 0, 0, 0);
            }
          }
        }
        if constexpr (XTRA == 1 || XTRA == 2) {
#pragma unroll
          for (int a = 0; a < FM; ++a)
#pragma unroll
            for (int b = 0; b < FN; ++b) asm volatile("" ::"v"(acc2[a][b]));
        }
        // accumulators -> tile buffer i&1 (C/D map: row 4*(lane>>4)+r, col lane&15 of each 16x16 block)
        float* T = accb + (SB ? 0 : (i & 1) * (ACC_BYTES / 4));
        const int mr = wm * 32 + 4 * (lane >> 4), nc = wn * (BN / WN) + (lane & 15);
#pragma unroll
        for (int a = 0; a < FM; ++a)
#pragma unroll
          for (int b = 0; b < FN; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) T[(mr + a * 16 + r) * ALD + nc + b * 16] = acc[a][b][r] * p.alpha;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      mark();
      __builtin_amdgcn_s_barrier();  // hand-off: tile i's buffer complete, tile i-1's buffer released
    }
    if (stp) stp[kStampSlots - 1] = (long long)__builtin_amdgcn_s_memrealtime();
  } else {
    // ---------------------------------------------------------------- stream waves
    // Vector v of tile i-1 (row row0 + 8 v, columns col..col+3 of the tile) is updated in K-step v of
    // iteration i (nk == VPT: one vector per K-step).  Its master / momentum loads are issued DIST K-steps
    // earlier — for the first DIST vectors of a tile, in the last K-steps of the previous iteration — into a
    // ring of DIST register slots.  Profiled on MI355X (benchmarks/stream_probe.hip): 4 waves per CU stream the
    // optimizer's 18 B per weight at 6.2 TB/s with 4 vectors in flight per thread, against 3.5 TB/s holding a
    // whole tile (8 vectors, 128 VGPRs of state) ahead, which also pushed this kernel into register spills.
    // NSW stream waves (4, or 8 with DDPX_WSGD_STREAM_WAVES=8): SV vectors per stream thread per tile, one
    // update every KPU K-steps; a ring of DIST = 4 vectors in flight per thread (a ring of 8 measured no faster).
    constexpr int DIST = 4;
    constexpr int SV = BM * BN / 4 / (NSW * 64);  // 8 (NSW 4) or 4 (NSW 8)
    constexpr int KPU = VPT / SV;                 // K-steps per update: 1 or 2
    constexpr int RSTEP = NSW * 2;                // tile rows between a thread's consecutive vectors
    static_assert(SV % DIST == 0 && VPT % SV == 0, "ring");
    const int st = tid - 64 * NMW;
    const int row0 = st >> 5, col = 4 * (st & 31);  // row0 < RSTEP
    const float lr = *p.sgd.lr;
    const float mom = p.sgd.mom, wd = p.sgd.wd;
    const bool has_mom = mom != 0.f;
    f32x4 rp[DIST], rm[DIST];  // the ring (statically indexed: every loop over it is unrolled)
    // per-GEMM pointers selected as scalars (a reference to p0.sgd / p1.sgd picked at run time put the structs
    // on the stack: scratch loads, which also count in vmcnt)
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
    // transposed MX copy (FP8, 8 stream waves): each updated vector is staged as fp32 in the gradient tile it
    // replaced (the thread's own, already consumed slot), and once a 32-row block of the tile is complete (after
    // the barrier that follows its last vector's update) every stream thread quantises 8 rows of one column:
    // quad = 32 rows of a column = one MX block along M, its 4 lanes write 32 contiguous code bytes of W^T
    unsigned char* const QT0 = p0.sgd.q8t;
    unsigned char* const QT1 = p1.sgd.q8t;
    unsigned char* const ET0 = p0.sgd.s8t;
    unsigned char* const ET1 = p1.sgd.s8t;
    const bool qt_on = FP8 && NSW == 8 && (QT0 != nullptr || QT1 != nullptr);  // (either GEMM may skip its copy)
    unsigned qt_e0 = 0;  // block 0's E8M0 byte until block 1's: the column's two scales as one 2-byte store
    const int ldc0 = p0.ldc, ldc1 = p1.ldc;
    auto vec_off = [&](int j, int v, int& sel) -> size_t {
      int m0, n0;
      sel = tile_origin(j, m0, n0);
      return (size_t)(m0 + row0 + RSTEP * v) * (sel ? ldc1 : ldc0) + n0 + col;
    };
    // load vector v of tile j into a ring slot
    auto load_vec = [&](int j, int v, f32x4& pv, f32x4& mv) {
      int sel;
      const size_t off = vec_off(j, v, sel);
      if constexpr (CP == 1) {
        pv = *reinterpret_cast<const f32x4*>((sel ? P1 : P0) + off);
        mv = *reinterpret_cast<const f32x4*>((sel ? M1 : M0) + off);
      } else {
        pv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>((sel ? P1 : P0) + off));
        mv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>((sel ? M1 : M0) + off));
      }
    };
    auto grad_vec = [&](const float* T, int v) -> f32x4 {
      return *reinterpret_cast<const f32x4*>(T + (row0 + RSTEP * v) * ALD + col);
    };
    // update vector v of tile j with gradient g, then refill the slot with the vector DIST ahead
    auto update_vec_g = [&](int j, int v, const f32x4 g, f32x4& pv, f32x4& mv, float* stage) {
      int sel;
      const size_t off = vec_off(j, v, sel);
      f32x4 po, bo;
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // sgd_apply's fma sequence
        float d = fmaf(wd, pv[q], g[q]);
        if (has_mom) d = fmaf(mom, mv[q], d);
        po[q] = fmaf(-lr, d, pv[q]);
        bo[q] = has_mom ? d : po[q];
      }
      if (stage) *reinterpret_cast<f32x4*>(stage) = po;
      const u32x2 sh = (u32x2){pack_bf2(po[0], po[1]), pack_bf2(po[2], po[3])};
      if constexpr (CP == 1) {
        *reinterpret_cast<f32x4*>((sel ? P1 : P0) + off) = po;
        *reinterpret_cast<f32x4*>((sel ? M1 : M0) + off) = bo;
      } else {
        __builtin_nontemporal_store(po, reinterpret_cast<f32x4*>((sel ? P1 : P0) + off));
        __builtin_nontemporal_store(bo, reinterpret_cast<f32x4*>((sel ? M1 : M0) + off));
      }
      if constexpr (CP == 2) __builtin_nontemporal_store(sh, reinterpret_cast<u32x2*>((sel ? S1 : S0) + off));
      else *reinterpret_cast<u32x2*>((sel ? S1 : S0) + off) = sh;
      if constexpr (FP8) {  // MX-FP8 weight copy for the next forward: 8 lanes = one 32-column block
        unsigned e8;
        const unsigned q = mx::e4m3_group8(po, &e8);
        *reinterpret_cast<unsigned*>((sel ? Q1 : Q0) + off) = q;
        // the row's 4 block scales (lanes 0/8/16/24 of each half-wave) as two 2-byte stores by lanes 0 and 16 of
        // each half-wave, the neighbouring block's byte fetched by DPP row_ror:8 (plain VALU, no LDS permute on
        // the stream's per-update path); byte stores scattered over the tile's rows cost more than the codes
        const unsigned e1 = (unsigned)__builtin_amdgcn_update_dpp(0, (int)e8, 0x128, 0xF, 0xF, false);
        if ((lane & 15) == 0)
          *reinterpret_cast<unsigned short*>((sel ? E1 : E0) + (off >> 5)) = (unsigned short)(e8 | (e1 << 8));
      }
      // refill: vector v + DIST of tile j, or vector v + DIST - VPT of tile j + 1, or (past the last tile)
      // vector v of tile j again — a harmless reload that keeps the per-update operation count fixed
      const int vn = v + DIST;
      const bool same = vn < SV, next = !same && j + 1 < nt;
      load_vec(same ? j : (next ? j + 1 : j), same ? vn : (next ? vn - SV : v), pv, mv);
    };
    // update vector v of tile j from the gradient tile T
    auto update_vec = [&](int j, int v, const float* T, f32x4& pv, f32x4& mv) {
      if constexpr (FP8 && NSW == 8) {
        if (qt_on) {  // the updated vector back into its (consumed) gradient slot: the transposed copy's staging
          float* slot = const_cast<float*>(T) + (row0 + RSTEP * v) * ALD + col;
          const f32x4 g = *reinterpret_cast<const f32x4*>(slot);
          update_vec_g(j, v, g, pv, mv, slot);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // visible to the other waves after the next barrier
          return;
        }
      }
      update_vec_g(j, v, grad_vec(T, v), pv, mv, nullptr);
    };
    // quantise rows [32 b, 32 b + 32) of tile j (staged in T) into the transposed copy
    auto quant_t = [&](int j, int b, const float* T) {
      int m0, n0;
      const int sel = tile_origin(j, m0, n0);
      unsigned char* const qd = sel ? QT1 : QT0;
      if (!qd) return;  // uniform: this GEMM writes no transposed copy
      const int c = st >> 2, sub = st & 3;
      float v[8];
      float am = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        v[r] = bf2f(f2bf(T[(32 * b + 8 * sub + r) * ALD + c]));  // the bf16 copy's value, as the quantiser sees it
        am = fmaxf(am, fabsf(v[r]));
      }
      am = fmaxf(am, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, am), 0xB1, 0xF, 0xF, false)));
      am = fmaxf(am, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, am), 0x4E, 0xF, 0xF, false)));
      const int e = mx::block_exp(am, mx::kMaxE4M3);
      const float inv = ldexpf(1.f, -e);
      const unsigned lo = mx::quant4(v[0], v[1], v[2], v[3], inv, mx::kMaxE4M3, false);
      const unsigned hi = mx::quant4(v[4], v[5], v[6], v[7], inv, mx::kMaxE4M3, false);
      const int Mg = sel ? p1.M : p0.M;
      *reinterpret_cast<u32x2*>(qd + (size_t)(n0 + c) * Mg + m0 + 32 * b + 8 * sub) = (u32x2){lo, hi};
      unsigned char* const ed = sel ? ET1 : ET0;  // (null: codes only — measurement, benchmarks/pair_fp8t.py)
      if (sub == 0 && ed) {
        if (b == 0) {
          qt_e0 = (unsigned)(e + 127);
        } else {
          *reinterpret_cast<unsigned short*>(ed + (size_t)(n0 + c) * (Mg / 32) + m0 / 32) =
              (unsigned short)(qt_e0 | ((unsigned)(e + 127) << 8));
        }
      }
    };
    // iteration 0 (math fills the first tile): prefetch tile 0's first DIST vectors
#pragma unroll
    for (int v = 0; v < DIST; ++v)
      if constexpr (XTRA != 3) load_vec(0, v, rp[v], rm[v]);
    for (int t = 0; t < nk; ++t) {
      mark();
      __builtin_amdgcn_s_barrier();
    }
    mark();
    __builtin_amdgcn_s_barrier();
    // trip r = DIST K-steps: iteration i = 1 + r / TPI updates tile i - 1, vectors (r % TPI) * DIST .. + DIST - 1;
    // the first trip is peeled so the loop is entered with the same memory operations in flight as on its back
    // edge (the compiler then counts every update's ring wait, e.g. vmcnt(15) at DIST = 4, instead of the
    // entry path's smaller count)
    constexpr int TPI = SV / DIST;  // trips per iteration
    auto trip = [&](int r) {
      const int i = 1 + r / TPI, t = (r % TPI) * DIST;
      const float* T = accb + ((i - 1) & 1) * (ACC_BYTES / 4);
#pragma unroll
      for (int u = 0; u < DIST; ++u) {
        // sched_barrier: keep each update's register work (which waits for its ring slot) inside its K-step
        mark();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (XTRA != 3) update_vec(i - 1, t + u, T, rp[u], rm[u]);  // (3: measurement, math only)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 1; k < KPU; ++k) {
          mark();
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (FP8 && NSW == 8) {  // SV = 4, TPI = 1: rows 0-31 are vectors 0-1, rows 32-63 vectors 2-3
          if (qt_on && (t + u) % 2 == 1) {
            quant_t(i - 1, (t + u) / 2, T);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
        }
      }
      if (r % TPI == TPI - 1) {  // end of iteration i: the buffer hand-off barrier
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        mark();
        __builtin_amdgcn_s_barrier();
      }
    };
    if constexpr (SB) {
      // single hand-off buffer: vector v's gradient is read in the K-step before its update (vector 0 right after
      // the hand-off barrier), so the last K-step of an iteration — when the math waves overwrite the buffer with
      // the next tile — reads nothing; every read has landed before the next barrier (lgkmcnt(0))
      f32x4 gq = grad_vec(accb, 0);
      auto trip_sb = [&](int r) {
        const int i = 1 + r / TPI, t = (r % TPI) * DIST;
#pragma unroll
        for (int u = 0; u < DIST; ++u) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
          const f32x4 g = gq;
          if (t + u + 1 < SV) gq = grad_vec(accb, t + u + 1);
          update_vec_g(i - 1, t + u, g, rp[u], rm[u], nullptr);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int k = 1; k < KPU; ++k) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
          }
        }
        if (r % TPI == TPI - 1) {  // end of iteration i: the buffer hand-off barrier, then the next tile's vector 0
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          gq = grad_vec(accb, 0);
        }
      };
      trip_sb(0);
#pragma unroll 1
      for (int r = 1; r < TPI * nt; ++r) trip_sb(r);
    } else {
      trip(0);
#pragma unroll 1
      for (int r = 1; r < TPI * nt; ++r) trip(r);
    }
    if (stp) stp[kStampSlots - 1] = (long long)__builtin_amdgcn_s_memrealtime();
  }
}

// Eligible shapes: the plain weight-gradient layout (A M-contig, B N-contig), M % 64 == 0, N % 128 == 0,
// K == 512 (the batch: nk = 8 K-steps of 64, one optimizer vector per K-step; the two roles' barrier counts
// are nk + 1 per iteration), ldc % 4 == 0.
static inline bool eligible(const pipe::Params& p, bool ak, bool bk) {
  return !ak && !bk && p.M % BM == 0 && p.N % BN == 0 && p.K == 64 * VPT && (p.ldc & 3) == 0 && p.sgd.p &&
         p.sgd.lr && (p.sgd.mom == 0.f || p.sgd.buf) && p.sgd.shadow && (!p.sgd.q8 || (p.sgd.s8 && (p.ldc & 127) == 0 && !((uintptr_t)p.sgd.q8 & 3) && !((uintptr_t)p.sgd.s8 & 3))) &&
         (!p.sgd.q8t || (p.sgd.q8 && !((uintptr_t)p.sgd.q8t & 7) && !((uintptr_t)p.sgd.s8t & 1)));
}

// Ring depth: DDPX_WSGD_STAGES=3|4 forces it; by default 4 stages once every CU owns >= 64 tiles (wide MLP:
// 2.434 vs 2.469 ms/step) and 3 below (toy MLP, 14 tiles per CU: 0.2398 vs 0.2502 ms/step; profiles/r2_stages).
static inline int stages(long long ntiles = 0, int num_cus = 256) {
  static const int forced = [] {
    const char* e = getenv("DDPX_WSGD_STAGES");
    return e && e[0] == '2' ? 2 : (e && e[0] == '3' ? 3 : (e && e[0] == '4' ? 4 : 0));
  }();
  if (forced) return forced;
  return ntiles >= 64LL * num_cus ? 4 : 3;
}

// Stream waves per workgroup: DDPX_WSGD_STREAM_WAVES=4|8 forces it; by default 8 once every CU owns >= 64
// tiles (wide MLP, ~150 tiles per CU: 2.108 vs 2.175 ms/step) and 4 below (toy MLP, 14 tiles per CU: pair
// 115.9 vs 120.4 us; profiles/r3_wsgd).
// With the MX-FP8 copy (FP8) too since round 6 (wide MLP --fp8 1, one box: 8 stream waves 2.055 / 2.059 ms with 8 / 4
// math waves vs 4 stream waves 2.195 / 2.160 ms, profiles/r6_fp8; round 4 had measured 4 faster on the old pair).
static inline int stream_waves(long long ntiles, int num_cus, bool fp8) {
  (void)fp8;
  static const int forced = [] {
    const char* e = getenv("DDPX_WSGD_STREAM_WAVES");
    return e && e[0] == '8' ? 8 : (e && e[0] == '4' ? 4 : 0);
  }();
  if (forced) return forced;
  return ntiles >= 64LL * num_cus ? 8 : 4;
}
// Tile order: DDPX_WSGD_ORDER=n (n fastest, default) | m.
static inline bool n_order() {
  static const bool v = [] {
    const char* e = getenv("DDPX_WSGD_ORDER");
    return !(e && e[0] == 'm');
  }();
  return v;
}

// DDPX_WSGD_SB=1|5: single hand-off buffer + 4-stage (1) or 5-stage (5) padded ring (no MX-FP8 copy); 0 = off
static inline int single_buffer() {
  static const int v = [] {
    const char* e = getenv("DDPX_WSGD_SB");
    return (e && e[0] == '1') ? 4 : (e && e[0] == '5') ? 5 : 0;
  }();
  return v;
}

static inline int xtra() {
  static const int v = [] {
    const char* e = getenv("DDPX_WSGD_XTRA");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// Math waves: DDPX_WSGD_MATH_WAVES=4|8 (default 8: profiles/r6_pair).
static inline int math_waves() {
  static const int v = [] {
    const char* e = getenv("DDPX_WSGD_MATH_WAVES");
    return (e && e[0] == '4') ? 4 : 8;
  }();
  return v;
}

// Optimizer-stream cache policy (DDPX_WSGD_CACHE=0|1|2, see the kernel's CP; toy-MLP shapes only).
static inline int cache_policy() {
  static const int v = [] {
    const char* e = getenv("DDPX_WSGD_CACHE");
    return e ? atoi(e) : 0;
  }();
  return v;
}

template <int STAGES, bool FP8>
static inline void launch_dist(dim3 grid, hipStream_t s, const pipe::Params& p0, const pipe::Params& p1, int nt1,
                               int nsw) {
  const bool no = n_order();
  if constexpr (STAGES == 3 || STAGES == 4) {
    if (math_waves() == 8 && nsw == 4 && no && (FP8 || single_buffer() == 0)) {
      const int x = FP8 ? 0 : xtra();
      if constexpr (!FP8 && STAGES == 3) {  // measurement: math only / stream only (benchmarks/pair_stamps.py)
        if (x == 3) { hipLaunchKernelGGL((wgrad_sgd_ws_kernel<3, false, 4, true, 3, false, 8>), grid, dim3(768), 0, s, p0, p1, nt1); return; }
        if (x == 4) { hipLaunchKernelGGL((wgrad_sgd_ws_kernel<3, false, 4, true, 4, false, 8>), grid, dim3(768), 0, s, p0, p1, nt1); return; }
      }
      if (x == 0) {
        if constexpr (!FP8 && STAGES == 3) {
          const int cp = cache_policy();
          if (cp == 1) { hipLaunchKernelGGL((wgrad_sgd_ws_kernel<3, false, 4, true, 0, false, 8, 1>), grid, dim3(768), 0, s, p0, p1, nt1); return; }
          if (cp == 2) { hipLaunchKernelGGL((wgrad_sgd_ws_kernel<3, false, 4, true, 0, false, 8, 2>), grid, dim3(768), 0, s, p0, p1, nt1); return; }
        }
        hipLaunchKernelGGL((wgrad_sgd_ws_kernel<STAGES, FP8, 4, true, 0, false, 8>), grid, dim3(768), 0, s, p0, p1, nt1);
        return;
      }
    }
  }
  if constexpr (!FP8 && STAGES == 3) {
    // measurement variants: DDPX_WSGD_XTRA=3 math only, 4 stream only (benchmarks/pair_stamps.py)
    const int x = xtra();
    if (x == 3 && nsw == 4) { hipLaunchKernelGGL((wgrad_sgd_ws_kernel<3, false, 4, true, 3>), grid, dim3(512), 0, s, p0, p1, nt1); return; }
    if (x == 4 && nsw == 4) { hipLaunchKernelGGL((wgrad_sgd_ws_kernel<3, false, 4, true, 4>), grid, dim3(512), 0, s, p0, p1, nt1); return; }
  }
  if constexpr (!FP8 && STAGES == 2) {
    // measurement variants (DDPX_WSGD_XTRA=1|2, 2-stage ring so the dummy ring fits the LDS)
    const int x = xtra();
    if (x == 1) { hipLaunchKernelGGL((wgrad_sgd_ws_kernel<2, false, 4, true, 1>), grid, dim3(512), 0, s, p0, p1, nt1); return; }
    if (x == 2) { hipLaunchKernelGGL((wgrad_sgd_ws_kernel<2, false, 4, true, 2>), grid, dim3(512), 0, s, p0, p1, nt1); return; }
  }
  if constexpr (!FP8) {
    const int sb = no ? single_buffer() : 0;
    if (sb == 4 && nsw == 4) {
      hipLaunchKernelGGL((wgrad_sgd_ws_kernel<4, false, 4, true, 0, true>), grid, dim3(512), 0, s, p0, p1, nt1);
      return;
    }
    if (sb == 5 && nsw == 4) {
      hipLaunchKernelGGL((wgrad_sgd_ws_kernel<5, false, 4, true, 0, true>), grid, dim3(512), 0, s, p0, p1, nt1);
      return;
    }
    if (sb == 4 && nsw == 8) {
      hipLaunchKernelGGL((wgrad_sgd_ws_kernel<4, false, 8, true, 0, true>), grid, dim3(768), 0, s, p0, p1, nt1);
      return;
    }
    if (sb == 5 && nsw == 8) {
      hipLaunchKernelGGL((wgrad_sgd_ws_kernel<5, false, 8, true, 0, true>), grid, dim3(768), 0, s, p0, p1, nt1);
      return;
    }
  }
  if (nsw == 8) {
    if (no) hipLaunchKernelGGL((wgrad_sgd_ws_kernel<STAGES, FP8, 8, true>), grid, dim3(768), 0, s, p0, p1, nt1);
    else hipLaunchKernelGGL((wgrad_sgd_ws_kernel<STAGES, FP8, 8, false>), grid, dim3(768), 0, s, p0, p1, nt1);
  } else {
    if (no) hipLaunchKernelGGL((wgrad_sgd_ws_kernel<STAGES, FP8, 4, true>), grid, dim3(512), 0, s, p0, p1, nt1);
    else hipLaunchKernelGGL((wgrad_sgd_ws_kernel<STAGES, FP8, 4, false>), grid, dim3(512), 0, s, p0, p1, nt1);
  }
}

static inline hipError_t launch(const pipe::Params& p, int num_cus, hipStream_t s) {
  const int ntiles = (p.M / BM) * (p.N / BN);
  const int grid = ntiles < num_cus ? ntiles : num_cus;
  const bool fp8 = p.sgd.q8 != nullptr;
  const int nsw = stream_waves(ntiles, num_cus, fp8);
  if (stages(ntiles, num_cus) == 4) {
    if (fp8) launch_dist<4, true>(dim3(grid), s, p, p, 0, nsw);
    else launch_dist<4, false>(dim3(grid), s, p, p, 0, nsw);
  } else {
    if (fp8) launch_dist<3, true>(dim3(grid), s, p, p, 0, nsw);
    else launch_dist<3, false>(dim3(grid), s, p, p, 0, nsw);
  }
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
  if ((p0.sgd.q8 != nullptr) != (p1.sgd.q8 != nullptr)) return hipErrorInvalidValue;  // both or neither
  const bool fp8 = p0.sgd.q8 != nullptr;
  const bool qt = p0.sgd.q8t != nullptr || p1.sgd.q8t != nullptr;
  if (qt && !fp8) return hipErrorInvalidValue;
  // the transposed MX copy is emitted by the 8-stream-wave layout only
  const int nsw = qt ? 8 : stream_waves(ntiles, num_cus, fp8);
  if (stages(ntiles, num_cus) == 4) {
    if (fp8) launch_dist<4, true>(dim3(grid), s, p0, p1, nt1, nsw);
    else launch_dist<4, false>(dim3(grid), s, p0, p1, nt1, nsw);
  } else if (stages(ntiles, num_cus) == 2 && !fp8) {
    launch_dist<2, false>(dim3(grid), s, p0, p1, nt1, nsw);
  } else {
    if (fp8) launch_dist<3, true>(dim3(grid), s, p0, p1, nt1, nsw);
    else launch_dist<3, false>(dim3(grid), s, p0, p1, nt1, nsw);
  }
  return hipGetLastError();
}

}  // namespace wsgd
}  // namespace ddpx
