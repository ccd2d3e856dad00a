// ddpx — weight gradient + SGD with the MFMA side and the optimizer stream in DIFFERENT workgroups (gfx950).
//
// The one-workgroup pair (ddpx_wgrad_sgd.h) couples its two roles at every 64-deep K-step: both pass the same
// s_barrier sequence, so each K-step lasts max(MFMA step, one optimizer vector).  Measured on the toy MLP's
// pair (profiles/r6_pair, benchmarks/pair_stamps.py): math alone 79 us, stream alone 80 us, together 107 us —
// a quarter of the kernel is the lock-step, not either role.  Here a launch holds 2G workgroups of 8 waves:
//
//   * math workgroup m < G: 8 MFMA waves run the LDS-DMA ring + v_mfma_f32_16x16x32_bf16 main loop of its
//     64x128 tiles (the same K order as the one-workgroup kernel: the same gradient bits), transpose each
//     16x16 accumulator quad-wise (DPP) so a lane holds 4 consecutive columns, and store the tile row-major into
//     global slot (m, i % 2) with sc1 (write-through) stores; each math wave publishes with one no-return atomic
//     (produced[m] += 1, 8 per tile) once its counted vmcnt shows the stores done — one K-step later, inside
//     the ring's own waits.  Before rewriting a slot the math side checks that the stream side has read it, from
//     an LDS-DMA of consumed[m] issued inside the ring (vmcnt is in order: a load a wave waited on directly
//     would drain its ring).
//   * stream workgroup G + m: a poller wave waits for produced[m], copies the tile into one of two LDS buffers
//     with sc1 LDS-DMA, counts consumed[m] += 1 and releases 4 stream waves with ONE barrier per tile; they
//     apply sgd_apply's fma sequence to 8 vectors per thread per tile with 4 master / momentum vectors in flight
//     (non-temporal), the one-workgroup kernel's arithmetic.  Its 3 spare waves exit at once.
//
// Every poll is bounded (error word set, kernel still ends).  Two workgroups of 8 waves (2 per SIMD each, <= 128
// VGPRs, 73 KiB LDS each) always fit one CU together, so the 2G = 2 x #CUs workgroups are all resident at once.
// Cross-workgroup visibility is the split-K combine's proven form (sc1 stores, drained, agent-scope counters,
// sc1 loads), correct whichever XCDs the two workgroups land on.  The poller resets the two counters at the end
// for the next launch.
#pragma once

#include "ddpx_wgrad_sgd.h"

namespace ddpx {
namespace wsgd {
namespace xwg {

constexpr int NW = 8;                     // waves per workgroup: 2 per SIMD, so two workgroups always share a CU
constexpr int STAGES = 3;
constexpr int TILE_F = BM * BN;           // floats per gradient tile
constexpr int NB = 2;                     // global gradient slots per math workgroup
constexpr int kPolls = 1 << 21;           // poll bound (s_sleep 2: ~0.1 s)
constexpr int CNT_OFF = STAGES * SLOT;    // LDS word: the math side's view of consumed[m]
constexpr int LDS_BYTES = STAGES * SLOT + 1024;

struct Scratch {
  float* T;         // [G][NB][BM][BN] fp32 gradient tiles
  int* produced;    // [G] math-wave publications (8 per tile); zero between launches
  int* consumed;    // [G] tiles read by the stream side; zero between launches
  int* err;         // poll timeouts (0 = healthy)
};

__device__ __forceinline__ bool poll_ge(int* c, int target, int* err) {
  for (int it = 0; it < kPolls; ++it) {
    if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    __builtin_amdgcn_s_sleep(2);
  }
  __hip_atomic_fetch_add(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return false;
}

// 4x4 transpose across each quad of lanes: in, lane i holds rows 0..3 of column i; out, lane i holds columns
// 0..3 of row i (two DPP butterfly steps, xor 1 then xor 2)
__device__ __forceinline__ f32x4 quad_transpose(f32x4 v, int lane) {
  const bool b0 = lane & 1, b1 = lane & 2;
  float r[4] = {v[0], v[1], v[2], v[3]};
#pragma unroll
  for (int b = 0; b < 2; ++b) {  // 2x2 blocks: swap r[2b+1] of even lanes with r[2b] of odd lanes
    const float send = b0 ? r[2 * b] : r[2 * b + 1];
    const float recv = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send), 0xB1, 0xF, 0xF, false));
    if (b0) r[2 * b] = recv;
    else r[2 * b + 1] = recv;
  }
  const float s0 = b1 ? r[0] : r[2], s1 = b1 ? r[1] : r[3];
  const float q0 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s0), 0x4E, 0xF, 0xF, false));
  const float q1 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s1), 0x4E, 0xF, 0xF, false));
  if (b1) {
    r[0] = q0;
    r[1] = q1;
  } else {
    r[2] = q0;
    r[3] = q1;
  }
  return (f32x4){r[0], r[1], r[2], r[3]};
}

template <int V>
__device__ __forceinline__ void vmwait() {
  pipe::wait_vmcnt<V>();
}

// LOCAL (measurement, DDPX_WSGD_XWG_LOCAL=1): the tile exchange with default-policy stores and sc0 loads (L2-local,
// coherent only when the two workgroups of a pair share an XCD) instead of sc1 on both sides.
template <bool LOCAL>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(4)))
wgrad_sgd_xwg_kernel(pipe::Params p0, pipe::Params p1, int nt1, int G, Scratch sc) {
  constexpr int CP_ST = LOCAL ? 0 : 16, CP_LD = LOCAL ? 1 : 16;
  constexpr int NMW = 8, WN = 4, FM = 2, FN = 2;   // math waves 2 (M) x 4 (N), 32 x 32 each
  constexpr int LPW = (BM + BN) / (8 * NMW);       // LDS-DMA instructions per math wave per stage (3)
  constexpr int NST = FM * FN;                     // gradient-slot stores per math wave per tile (4)
  constexpr int NSWV = 4;                          // stream waves of a stream workgroup (+ 1 poller)
  constexpr int SV = TILE_F / 4 / (NSWV * 64);     // vectors per stream thread per tile (8)
  constexpr int RSTEP = NSWV * 64 / (BN / 4);      // rows between a stream thread's vectors (8)
  constexpr int DIST = 4;                          // master / momentum vectors in flight per stream thread
  static_assert(NB * TILE_F * 4 <= STAGES * SLOT, "stream tile buffers");
  static_assert(SV % DIST == 0, "ring");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool math_wg = (int)blockIdx.x < G;
  const int m = math_wg ? (int)blockIdx.x : (int)blockIdx.x - G;  // this pair's index
  const int tiles_m0 = p0.M / BM;
  const int nt0 = tiles_m0 * (p0.N / BN);
  const int ntiles = nt0 + nt1;
  const int nt = (ntiles - m + G - 1) / G;  // >= 1 (G <= ntiles)
  const int nk = p0.K / 64;                 // >= 6 (launch_pair)
  auto tile_origin = [&](int i, int& m0, int& n0) -> int {  // n-fastest (ddpx_wgrad_sgd.h NORD)
    int g = m + i * G;
    const int sel = g >= nt0;
    if (sel) g -= nt0;
    const int tn = (sel ? p1.N : p0.N) / BN;
    m0 = (g / tn) * BM;
    n0 = (g % tn) * BN;
    return sel;
  };
  const pipe::Params& p = p0;
  float* const Tg = sc.T + (size_t)m * NB * TILE_F;
  int* const produced = sc.produced + m;
  int* const consumed = sc.consumed + m;
  const __amdgpu_buffer_rsrc_t rt =
      __builtin_amdgcn_make_buffer_rsrc((void*)Tg, 0, (unsigned)(NB * TILE_F * 4), 0x00020000);
  // diagnostics (ddpx_gemm_set_stamps; benchmarks/pair_stamps.py --xwg): per workgroup [HW_ID, XCC_ID, start, end of
  // wave 0] so the placement (which CU holds which role) and each workgroup's span can be read back
  long long* const dbg = (p0.stamp && tid == 0) ? p0.stamp + (size_t)blockIdx.x * 4 : nullptr;
  if (dbg) {
    dbg[0] = (long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
    dbg[1] = (long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));   // HW_REG_XCC_ID
    dbg[2] = (long long)__builtin_amdgcn_s_memrealtime();
  }

  if (math_wg) {
    // ====================================================================== math workgroup
    const int G_ = nt * nk;
    const int wm = wave / WN, wn = wave % WN;
    const __amdgpu_buffer_rsrc_t ra0 = __builtin_amdgcn_make_buffer_rsrc((void*)p0.A, 0, p0.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb0 = __builtin_amdgcn_make_buffer_rsrc((void*)p0.B, 0, p0.b_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ra1 = __builtin_amdgcn_make_buffer_rsrc((void*)p1.A, 0, p1.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb1 = __builtin_amdgcn_make_buffer_rsrc((void*)p1.B, 0, p1.b_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rc =
        __builtin_amdgcn_make_buffer_rsrc((void*)consumed, 0, 4u, 0x00020000);
    int* const cnt_lds = reinterpret_cast<int*>(smem + CNT_OFF);
    int iss_i = -1, iss_kt = nk - 1, iss_m0 = 0, iss_n0 = 0, iss_sel = 0;
    auto issue = [&](int g) {
      if (++iss_kt >= nk) {
        iss_kt = 0;
        iss_sel = tile_origin(++iss_i, iss_m0, iss_n0);
      }
      const int sel = iss_sel, kt = iss_kt;
      const __amdgpu_buffer_rsrc_t ra = sel ? ra1 : ra0, rb = sel ? rb1 : rb0;
      const int lda = sel ? p1.lda : p0.lda, ldb = sel ? p1.ldb : p0.ldb;
      const int Mg = sel ? p1.M : p0.M, Ng = sel ? p1.N : p0.N;
      char* slot = smem + (g % STAGES) * SLOT;
      pipe::stage_tile<BM, false, pipe::MODE_PLAIN, NMW>(ra, slot, p.conv, lda, iss_m0, Mg, kt * 64, p.K, wave, lane);
      pipe::stage_tile<BN, false, pipe::MODE_PLAIN, NMW>(rb, slot + A_SUB, p.conv, ldb, iss_n0, Ng, kt * 64, p.K,
                                                         wave, lane);
    };
    auto publish = [&]() {
      if (lane == 0) __hip_atomic_fetch_add(produced, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    const int TC = nk - 4;  // K-step whose barrier is followed by wave 0's LDS-DMA of consumed[m]
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < G_) issue(s);
    for (int i = 0; i < nt; ++i) {
      f32x4 acc[FM][FN];
#pragma unroll
      for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
      for (int t = 0; t < nk; ++t) {
        const int g = i * nk + t;
        const bool ahead = g + 1 < G_;  // stage g + 1 in flight (STAGES = 3: at most one younger stage)
        // in-order vmcnt: stage g must have landed.  Younger than it: stage g + 1, plus tile i - 1's slot stores
        // (t = 0: issued after stage g + 1), tile i - 1's publish (t = 2: issued before stage g + 1) or wave 0's
        // counter DMA (t = TC + 1: issued before stage g + 1)
        if (i > 0 && t == 0) {
          if (ahead) vmwait<LPW + NST>(); else vmwait<NST>();
        } else if ((i > 0 && t == 2) || (wave == 0 && i >= NB && t == TC + 1)) {
          if (ahead) vmwait<LPW + 1>(); else vmwait<1>();
        } else {
          if (ahead) vmwait<LPW>(); else vmwait<0>();
        }
        if (i > 0 && t == 1) publish();  // tile i - 1's slot stores are older than stage g: done
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // slot i % NB is rewritten at the end of this tile: read consumed[m] into LDS now (sc1), in the ring's own
        // vmcnt order, so no wave ever waits on a global load of its own (vmcnt is in order: a dependent load
        // would drain the ring)
        if (wave == 0 && i >= NB && t == TC && lane == 0)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (LDS_AS void*)cnt_lds, 4, 0u, 0, 0, 16);
        if (g + STAGES - 1 < G_) issue(g + STAGES - 1);
        const char* sa = smem + (g % STAGES) * SLOT;
        const char* sb = sa + A_SUB;
#pragma unroll
        for (int kk = 0; kk < 64; kk += 32) {
          bf16x8 af[FM], bfr[FN];
          pipe::load_frags<BM, false, FM, BN, false, FN>(sa, wm * 32, sb, wn * (BN / WN), kk, lane, af, bfr);
#pragma unroll
          for (int a = 0; a < FM; ++a)
#pragma unroll
            for (int b = 0; b < FN; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
        }
      }
      if (i >= NB) {
        // the counter DMA (K-step TC) landed before stage TC + 1 did, and every wave has passed a barrier since:
        // the slot is free when the stream side has read tile i - NB out of it
        int seen = *cnt_lds;
        if (seen < i - NB + 1) {  // rare: the stream side is NB tiles behind — wait on the global counter
          if (lane == 0) poll_ge(consumed, i - NB + 1, sc.err);
          asm volatile("" ::: "memory");
        }
      }
      // tile i -> slot i % NB: lane (16 q + 4 j + r) of 16x16 block (a, b) stores row 4 q + r, columns 4 j .. 4 j + 3
      // after the quad transpose
      const int q = lane >> 4, j = (lane >> 2) & 3, r = lane & 3;
#pragma unroll
      for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b) {
          const f32x4 v = quad_transpose(acc[a][b] * p.alpha, lane);
          const int row = wm * 32 + a * 16 + 4 * q + r, col = wn * (BN / WN) + b * 16 + 4 * j;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rt,
                                                 (unsigned)((((i % NB) * BM + row) * BN + col) * 4), 0,
                                                 CP_ST /* sc1 */);
        }
    }
    vmwait<0>();  // the last tile's stores
    publish();
    if (dbg) dbg[3] = (long long)__builtin_amdgcn_s_memrealtime();
    return;
  }

  // ====================================================================== stream workgroup
  if (wave > NSWV) return;  // spare waves: the stream needs 4 + the poller
  float* const Tl = reinterpret_cast<float*>(smem);  // [NB][BM][BN]
  if (wave == NSWV) {
    // ---------------------------------------------------------------- poller
    for (int i = 0; i < nt; ++i) {
      if (lane == 0) poll_ge(produced, NMW * (i + 1), sc.err);
      asm volatile("" ::: "memory");
      char* dst = reinterpret_cast<char*>(Tl) + (i % NB) * TILE_F * 4;
#pragma unroll 4
      for (int c = 0; c < TILE_F * 4 / 1024; ++c)  // 32 x 1 KiB, lane-linear, sc1 (the slot was rewritten)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (LDS_AS void*)(dst + c * 1024), 16,
                                                 (unsigned)(((i % NB) * TILE_F * 4) + c * 1024 + lane * 16), 0, 0,
                                                 CP_LD);
      vmwait<0>();
      if (lane == 0) __hip_atomic_fetch_add(consumed, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_barrier();  // B_i: tile i is in LDS buffer i % NB
    }
    __builtin_amdgcn_s_barrier();  // B_nt
    // every publication and every slot read of this pair is done: reset for the next launch
    if (lane == 0) {
      __hip_atomic_store(produced, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(consumed, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  // -------------------------------------------------------------------- stream waves
  const int st = tid;  // 0 .. 255
  const int row0 = st >> 5, col = 4 * (st & 31);
  const float lr = *p.sgd.lr;
  const float mom = p.sgd.mom, wd = p.sgd.wd;
  const bool has_mom = mom != 0.f;
  float* const P0 = p0.sgd.p;
  float* const P1 = p1.sgd.p;
  float* const M0 = has_mom ? p0.sgd.buf : p0.sgd.p;
  float* const M1 = has_mom ? p1.sgd.buf : p1.sgd.p;
  unsigned short* const S0 = p0.sgd.shadow;
  unsigned short* const S1 = p1.sgd.shadow;
  const int ldc0 = p0.ldc, ldc1 = p1.ldc;
  f32x4 rp[DIST], rm[DIST];
  auto vec_off = [&](int j, int v, int& sel) -> size_t {
    int m0, n0;
    sel = tile_origin(j, m0, n0);
    return (size_t)(m0 + row0 + RSTEP * v) * (sel ? ldc1 : ldc0) + n0 + col;
  };
  auto load_vec = [&](int j, int v, f32x4& pv, f32x4& mv) {
    int sel;
    const size_t off = vec_off(j, v, sel);
    pv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>((sel ? P1 : P0) + off));
    mv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>((sel ? M1 : M0) + off));
  };
#pragma unroll
  for (int v = 0; v < DIST; ++v) load_vec(0, v, rp[v], rm[v]);
  auto do_tile = [&](int i) {
    __builtin_amdgcn_s_barrier();  // B_i
    asm volatile("" ::: "memory");
    const float* T = Tl + (i % NB) * TILE_F;
    int sel;
    const size_t off0 = vec_off(i, 0, sel);
    const int ldc = sel ? ldc1 : ldc0;
    float* const Pp = sel ? P1 : P0;
    float* const Mp = sel ? M1 : M0;
    unsigned short* const Sp = sel ? S1 : S0;
    const bool next = i + 1 < nt;
#pragma unroll
    for (int v = 0; v < SV; ++v) {
      const size_t off = off0 + (size_t)RSTEP * v * ldc;
      const f32x4 g = *reinterpret_cast<const f32x4*>(T + (row0 + RSTEP * v) * BN + col);
      const f32x4 pv = rp[v % DIST], mv = rm[v % DIST];
      f32x4 po, bo;
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // sgd_apply's fma sequence
        float d = fmaf(wd, pv[q], g[q]);
        if (has_mom) d = fmaf(mom, mv[q], d);
        po[q] = fmaf(-lr, d, pv[q]);
        bo[q] = has_mom ? d : po[q];
      }
      __builtin_nontemporal_store(po, reinterpret_cast<f32x4*>(Pp + off));
      __builtin_nontemporal_store(bo, reinterpret_cast<f32x4*>(Mp + off));
      *reinterpret_cast<u32x2*>(Sp + off) = (u32x2){pack_bf2(po[0], po[1]), pack_bf2(po[2], po[3])};
      // refill: vector v + DIST of this tile, or v + DIST - SV of the next (past the last tile: this one again,
      // a harmless reload that keeps the per-update operation count fixed)
      const int vn = v + DIST;
      if (vn < SV) load_vec(i, vn, rp[v % DIST], rm[v % DIST]);
      else load_vec(next ? i + 1 : i, next ? vn - SV : v, rp[v % DIST], rm[v % DIST]);
    }
  };
  do_tile(0);  // peeled: the loop is entered with the same memory operations in flight as on its back edge
#pragma unroll 1
  for (int i = 1; i < nt; ++i) do_tile(i);
  __builtin_amdgcn_s_barrier();  // B_nt
  if (dbg) dbg[3] = (long long)__builtin_amdgcn_s_memrealtime();
}

// Launch (the caller checked eligible() / pair_compatible(), no MX-FP8 copy).  G = #CUs workgroup pairs (fewer when
// there are fewer tiles); returns hipErrorInvalidValue when the scratch holds fewer than G pairs.
static inline hipError_t launch_pair(const pipe::Params& p0, const pipe::Params& p1, int num_cus, const Scratch& sc,
                                     int g_cap, hipStream_t s) {
  const int nt1 = p1.M / BM * (p1.N / BN);
  const int ntiles = p0.M / BM * (p0.N / BN) + nt1;
  const int G = ntiles < num_cus ? ntiles : num_cus;
  if (G > g_cap || p0.K / 64 < 6) return hipErrorInvalidValue;
  static const bool local = [] {
    const char* e = getenv("DDPX_WSGD_XWG_LOCAL");
    return e && e[0] == '1';
  }();
  if (local) hipLaunchKernelGGL(wgrad_sgd_xwg_kernel<true>, dim3(2 * G), dim3(64 * NW), 0, s, p0, p1, nt1, G, sc);
  else hipLaunchKernelGGL(wgrad_sgd_xwg_kernel<false>, dim3(2 * G), dim3(64 * NW), 0, s, p0, p1, nt1, G, sc);
  return hipGetLastError();
}

}  // namespace xwg
}  // namespace wsgd
}  // namespace ddpx
