// ddpx — pipelined bf16 MFMA GEMM for gfx950: LDS-DMA multi-stage ring.
//
// Operand layouts (chosen per call so forward, dgrad and wgrad of a Linear never
// materialise a transpose; reference equivalent: the implicit cuBLAS addmm/mm of
// nn.Linear, /root/reference/singlegpu.py:73):
//   A "K-contig" A[m*lda + k] / "M-contig" A[k*lda + m];  B "K-contig" B[n*ldb + k] / "N-contig" B[k*ldb + n]
//   forward Y = X W^T (A=X K-contig, B=W K-contig); dgrad dX = dY W (A=dY K-contig, B=W N-contig);
//   wgrad dW = dY^T X (A=dY M-contig, B=X N-contig).
// Built for the regime the MLP shapes live in (M = 512 rows against N, K = 3-16 K):
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
//    swizzles (K-contig [row][64] tiles: 16-B chunk ^= (row>>1)&7; M/N-contig
//    [k][row] tiles read by ds_read_b64_tr_b16: a 32-B-chunk XOR per row
//    stride) are applied to the per-lane SOURCE address and undone on the
//    read (rule 21).
//  * Buffer-resource bounds checking returns zeros for out-of-range lanes
//    (voffset forced past num_records), which handles ragged M/N/K tails with
//    no branches in the load path.
//  * XCD-aware workgroup remap (T1): tiles sharing a B panel run on one XCD.
//  * Epilogues: bias (+ReLU) -> bf16, fp32 (+accumulate) for gradients
//    written straight into DDP buckets, bf16 (+accumulate), ReLU-mask
//    backward, and an optional per-tile column sum of the stored output (the
//    bias gradient of the layer below) written as [tiles_m][N] partials.
#include <cstdlib>

#include "ddpx_gemm_dispatch.h"
#include "ddpx_pipe.h"
#include "ddpx_wgrad_sgd.h"
#include "ddpx_wgrad_sgd_xwg.h"
#include "ddpx_wsgd_dgrad.h"

namespace ddpx {
namespace pipe {

// Default tile per operand-layout class, from the MI355X sweep of the MLP shapes
// (benchmarks/mlp_gemm_bench.py, benchmarks/sgd_bw.py; profiles/r1_gemm2): the M=512-row products
// want 64x64 tiles with 128-wide K stages (fwd 27.1 vs 29.1 us, dgrad 36.5 vs 45.1 us at H=4096),
// the K=512 weight-gradient products 64x128/3 stages.
static int pick(int M, int N, int K, bool ak, bool bk) {
  auto tiles = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  if (!ak && !bk) return tiles(64, 128) >= 512 ? 5 : 7;      // wgrad-shaped (reduction over batch)
  // wide layers: 128x128 halves L2 traffic; two 2-stage workgroups per CU beat one 4-stage one on every wide-MLP
  // product (profiles/r6_gemm/sweep_wide.json, us: fc0 fwd 52.4 vs 82.5, fc1 fwd 298.3 vs 344.7, fc1 dgrad 308.0 vs
  // 406.4; hipBLASLt 62.1 / 260.7 / 352.0)
  if (tiles(128, 128) >= 512 && K >= 2048) return 21;
  return 12;  // M=512-row forward / dgrad: 64x64, BK=128 (one barrier per 128 of K), 2 WG/CU
}

// In-launch split-K plan for the M = 512-row products (forward, dgrad: A K-contiguous).  Their 64x64
// tiles are bound by L2 -> LDS operand traffic (each CU streams 2 MB of A/B panels for fc1 at ~78 GB/s;
// profiles/r1_pmc, r2_ab): 128x128 tiles halve the bytes per FLOP, and splitting K two ways keeps all 256
// CUs busy (128 tiles x 2), with the partial sums combined inside the same launch by the last split of
// each tile (64 KiB write-through slab per split, register layout).  The 128x128 tile needs 8 waves
// issuing LDS-DMA (4 waves at one workgroup per CU measured 28.9 / 32.3 / 46.2 us vs 21.8 / 26.8 / 34.8
// for the 64x64 tiles on fc0 fwd / fc1 fwd / fc1 dgrad).  Returns splits (1: no split), sets *cfg.
// Measured on MI355X in one process (benchmarks/mlp_step_kernels.py, profiles/r2_splitk): every split
// tile so far is slower than the 64x64 single-pass tile at M = 512 (fc1 fwd 26.7 us single-pass vs
// 28.9 on 8-wave 128x128 / 27.5 on 64x128 at 2 per CU / 37.3 on 256x128 split 4), so the plan is OFF by
// default.  DDPX_SPLITK=<cfg> enables it with that tile; DDPX_SPLITK_MAX caps the splits (default 2).
static int plan(int M, int N, int K, bool ak, bool bk, int epi, int* cfg) {
  *cfg = pick(M, N, K, ak, bk);
  static const int sk_cfg = [] {  // DDPX_SPLITK: 0 = off, else the split tile config (default 14)
    const char* e = getenv("DDPX_SPLITK");
    return e ? atoi(e) : 0;
  }();
  static const int sk_max = [] {
    const char* e = getenv("DDPX_SPLITK_MAX");
    return e ? atoi(e) : 2;
  }();
  if (sk_cfg <= 0 || !ak || epi == EPI_SGD || epi == EPI_BNSTAT_BF16 || K < 1024) return 1;
  int bm, bn;
  tile_of(sk_cfg, &bm, &bn);
  // workgroups that fill the chip: 2 per CU for the 4-wave tiles whose LDS ring fits twice per CU
  const int target = (sk_cfg == 5 || sk_cfg == 6 || sk_cfg == 7) ? 512 : 256;
  const int t = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  if (t * 4 >= target * 3) return 1;
  int s = target / t;
  if (s > sk_max) s = sk_max;
  while (s > 1 && (K / 64) / s < 8) --s;  // >= 8 K-steps of 64 per split
  if (s < 2) return 1;
  *cfg = sk_cfg;
  return s;
}

}  // namespace pipe
}  // namespace ddpx

using namespace ddpx;

static long long* g_stamp = nullptr;

// Scratch of the two-workgroup wgrad + SGD pair (ddpx_wgrad_sgd_xwg.h): gradient tile slots [cap][2][64x128] fp32 and
// counters [2 cap + 1] int (zeroed once; every launch leaves them zero); cap = workgroup pairs it holds.
static float* g_xwg_T = nullptr;
static int* g_xwg_cnt = nullptr;
static int g_xwg_cap = 0;
DDPX_API void ddpx_wsgd_set_xwg_scratch(float* T, int* counters, int cap) {
  g_xwg_T = T;
  g_xwg_cnt = counters;
  g_xwg_cap = (T && counters) ? cap : 0;
}
// DDPX_WSGD_XWG=1 (measurement): the two-workgroup pair.  Measured slower (profiles/r6_pair/NOTES.md: 178-186 vs
// 123 us back to back): unpaced, the optimizer stream's HBM traffic stalls the CU's texture-address path that the
// MFMA side's operand DMA shares, and the math side runs at half speed; the one-workgroup lock-step paces it.
static bool xwg_on() {
  static const bool v = [] {
    const char* e = getenv("DDPX_WSGD_XWG");
    return e && e[0] == '1';
  }();
  return v;
}

// Diagnostics: every following ddpx_gemm_pipe launch writes per-workgroup timestamps into buf
// ([workgroups][8] int64, s_memrealtime); nullptr turns it off (benchmarks/gemm_stamps.py).
DDPX_API void ddpx_gemm_set_stamps(long long* buf) { g_stamp = buf; }

// Number of row tiles (M direction) the kernel will use for cfg (for sizing colsum partials).
DDPX_API int ddpx_gemm_pipe_tiles_m(int M, int N, int K, int a_kcontig, int b_kcontig, int tile_cfg) {
  int cfg = tile_cfg;
  if (cfg < 0) pipe::plan(M, N, K, a_kcontig, b_kcontig, pipe::EPI_BF16, &cfg);
  int bm, bn;
  pipe::tile_of(cfg, &bm, &bn);
  return (M + bm - 1) / bm;
}

DDPX_API void ddpx_gemm_tile_dims(int cfg, int* bm, int* bn) { pipe::tile_of(cfg, bm, bn); }

// Launch plan for ddpx_gemm_pipe with tile_cfg = -1: splits (> 1: in-launch split-K, needing a slab of
// *slab_floats floats and *tickets zeroed ints), and the tile config.
DDPX_API int ddpx_gemm_pipe_plan(int M, int N, int K, int a_kcontig, int b_kcontig, int epi, int* cfg,
                                 long long* slab_floats, int* tickets) {
  const int s = pipe::plan(M, N, K, a_kcontig, b_kcontig, epi, cfg);
  int bm, bn;
  pipe::tile_of(*cfg, &bm, &bn);
  const long long tiles = (long long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  *slab_floats = s > 1 ? (long long)s * tiles * bm * bn : 0;
  *tickets = s > 1 ? (int)tiles : 0;
  return s;
}

DDPX_API int ddpx_gemm_pipe(const void* A, const void* B, void* C, const float* bias, const void* aux, float* colsum,
                            int M, int N, int K, int lda, int ldb, int ldc, int ldaux, int a_kcontig, int b_kcontig,
                            int epi, int accumulate, float alpha, int tile_cfg, float* sgd_p, float* sgd_buf,
                            void* sgd_shadow, const float* sgd_lr, float sgd_mom, float sgd_wd, int splits,
                            float* slab, long long slab_floats, int* tcnt, void* cs_out, int cs_flags,
                            int* cs_tcnt, hipStream_t stream) {
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
                 pipe::make_geom(0, 0, 0, 0), 0, 0, 0, nullptr, 0u, nullptr, cs_out, cs_flags, cs_tcnt};
  p.stamp = g_stamp;
  if (cs_tcnt && (!colsum || epi == pipe::EPI_SGD || epi == pipe::EPI_BNSTAT_BF16 || (!cs_out && !sgd_p) ||
                  (sgd_p && !sgd_lr)))
    return -10;
  if (epi == pipe::EPI_SGD && (!sgd_p || !sgd_lr || (sgd_mom != 0.f && !sgd_buf))) return -5;
  static const int sgd_plain = [] {
    const char* e = getenv("DDPX_SGD_PLAIN");
    return e && e[0] == '1' ? 1 : 0;
  }();
  p.sgd_plain = sgd_plain;
  int cfg = tile_cfg >= 0 ? tile_cfg : pipe::pick(M, N, K, a_kcontig, b_kcontig);
  if (cs_tcnt && pipe::eight_wave(cfg)) return -11;  // in-launch column sums: 4-wave tiles only
  if (cfg >= 16 && cfg <= 20 && (epi == pipe::EPI_SGD || epi == pipe::EPI_BNSTAT_BF16)) return -12;
  if (splits > 1) {  // in-launch split-K (ddpx_gemm_pipe_plan): the caller's cfg, slab and zeroed tickets
    if (epi == pipe::EPI_SGD || epi == pipe::EPI_BNSTAT_BF16 || !slab || !tcnt || tile_cfg < 0 || !a_kcontig)
      return -7;
    int bm, bn;
    pipe::tile_of(cfg, &bm, &bn);
    const long long tiles = (long long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    if (slab_floats < (long long)splits * tiles * bm * bn || slab_floats * 4 >= 0x80000000ll) return -8;
    int klen = (K + splits - 1) / splits;
    klen = (klen + 63) / 64 * 64;
    if ((K + klen - 1) / klen != splits) return -9;
    p.klen = klen;
    p.slab = slab;
    p.slab_bytes = (unsigned)(slab_floats * 4);
    p.tcnt = tcnt;
  }
  // Weight gradients stored to a buffer (DDP path: bf16 / fp32 gradient output, no fused optimizer):
  // the 256x256 8-wave tile moves a quarter of the 64x128 tile's L2->LDS operand bytes and is faster
  // once it fills half the chip (MI355X, K = 512: 35.4 vs 46.1 us on 4096x4096, 30.9 vs 38.6 us on
  // 4096x3072, fp32 out; benchmarks/wgrad_probe.py, profiles/r1_wgrad).  The fused-SGD epilogue keeps
  // 64x128 (its HBM stream wants two resident workgroups per CU: 78.9 vs 72.8 us).
  if (tile_cfg < 0 && !a_kcontig && !b_kcontig && epi != pipe::EPI_SGD && !colsum &&
      ((M + 255) / 256) * ((N + 255) / 256) >= 128)
    cfg = 13;
  // Weight gradient with the SGD update: the warp-specialised persistent kernel (MFMA waves + optimizer
  // stream waves per CU, ddpx_wgrad_sgd.h) when the shape allows; DDPX_WGRAD_WS=0 keeps the tile kernel.
  static const int wgrad_ws = [] {
    const char* e = getenv("DDPX_WGRAD_WS");
    return e && e[0] == '0' ? 0 : 1;
  }();
  if (epi == pipe::EPI_SGD && wgrad_ws && tile_cfg < 0 && splits <= 1 && wsgd::eligible(p, a_kcontig, b_kcontig)) {
    static const int cus = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
        n = 256;
      return n;
    }();
    return (int)wsgd::launch(p, cus, stream);
  }
  // Master/momentum LDS prefetch for the fused-SGD tiles: opt-in (DDPX_SGD_PREFETCH=1).  Measured
  // slower on MI355X (toy fc1 64x128: 112 vs 77 us; profiles/r1_epi): the 64 KiB side buffer halves
  // occupancy and the prefetch lands on the critical path of short (K = 512) main loops.
  static const int sgd_pf = [] {
    const char* e = getenv("DDPX_SGD_PREFETCH");
    return e && e[0] == '1' ? 1 : 0;
  }();
  if (epi == pipe::EPI_SGD && sgd_pf && !a_kcontig && !b_kcontig && (ldc & 3) == 0 &&
      (size_t)M * ldc * 4 < 0x80000000ull && (cfg == 3 || cfg == 5 || cfg == 7 || cfg == 12)) {
    return (int)pipe::dispatch_sgd_prefetch_mn(p, cfg, stream);
  }
  hipError_t e;
  if (splits > 1) {
    e = b_kcontig ? pipe::dispatch_sk_kk(p, cfg, splits, stream) : pipe::dispatch_sk_kn(p, cfg, splits, stream);
    return (int)e;
  }
  const int S = 1;
  if (a_kcontig && b_kcontig) e = pipe::dispatch_kk(p, cfg, S, stream);
  else if (a_kcontig) e = pipe::dispatch_kn(p, cfg, S, stream);
  else if (b_kcontig) e = pipe::dispatch_mk(p, cfg, S, stream);
  else e = pipe::dispatch_mn(p, cfg, S, stream);
  return (int)e;
}

// Two fused weight-gradient + SGD GEMMs in ONE warp-specialised launch (dW_i = A_i^T-contig x B_i, M_i x N_i,
// shared K = batch): the toy MLP's fc1 and fc0 updates, independent once fc1's data gradient has run.
// Returns -20 when the pair is not eligible (the caller then launches them one by one).
// q8t_i / s8t_i (optional, with q8_i; each GEMM may skip its own): the transposed MX-FP8 copy of W_i (W_i^T [N_i][M_i],
// 32-blocks along M_i: the data gradient's B operand), written by the stream waves too (8 stream waves).
DDPX_API int ddpx_wgrad_sgd_pair_t(const void* A0, const void* B0, int M0, int N0, int lda0, int ldb0, int ldc0,
                                   float* p0, float* buf0, void* sh0, void* q80, void* s80, void* q8t0, void* s8t0,
                                   const void* A1, const void* B1, int M1, int N1, int lda1, int ldb1, int ldc1,
                                   float* p1, float* buf1, void* sh1, void* q81, void* s81, void* q8t1, void* s8t1,
                                   int K, const float* lr, float mom, float wd, hipStream_t stream) {
  // q8_i / s8_i (optional): MX-FP8 codes + E8M0 scales of the updated W_i, written by the stream waves
  auto make = [&](const void* A, const void* B, int M, int N, int lda, int ldb, int ldc, float* pp, float* buf,
                  void* sh, void* q8, void* s8, void* q8t, void* s8t) {
    const size_t a_bytes = ((size_t)(K - 1) * lda + M) * 2, b_bytes = ((size_t)(K - 1) * ldb + N) * 2;
    return pipe::Params{(const unsigned short*)A, (const unsigned short*)B, pp, nullptr, nullptr, nullptr,
                        M, N, K, lda, ldb, ldc, 0, pipe::EPI_SGD, 0, 1.f, (unsigned)a_bytes, (unsigned)b_bytes,
                        SgdArgs{pp, buf, (unsigned short*)sh, lr, mom, wd, (unsigned char*)q8, (unsigned char*)s8,
                                (unsigned char*)q8t, (unsigned char*)s8t},
                        pipe::make_geom(0, 0, 0, 0), 0, 0, 0, nullptr, 0u, nullptr, nullptr, 0, nullptr};
  };
  if (K <= 0 || lda0 % 8 || ldb0 % 8 || lda1 % 8 || ldb1 % 8 || M0 % 8 || N0 % 8 || M1 % 8 || N1 % 8) return -20;
  if (((uintptr_t)A0 | (uintptr_t)B0 | (uintptr_t)A1 | (uintptr_t)B1) & 15) return -20;
  if ((q8t0 || q8t1) && (!q80 || !q81)) return -20;  // the transposed copies ride on the fp8 pair
  pipe::Params q0 = make(A0, B0, M0, N0, lda0, ldb0, ldc0, p0, buf0, sh0, q80, s80, q8t0, s8t0);
  const pipe::Params q1 = make(A1, B1, M1, N1, lda1, ldb1, ldc1, p1, buf1, sh1, q81, s81, q8t1, s8t1);
  q0.stamp = g_stamp;  // diagnostics: per-role barrier arrival stamps (ddpx_wgrad_sgd.h kStampSlots) / xwg placement
  if ((size_t)q0.a_bytes != ((size_t)(K - 1) * lda0 + M0) * 2 || (size_t)q1.b_bytes != ((size_t)(K - 1) * ldb1 + N1) * 2)
    return -20;  // 32-bit buffer offsets
  if (!wsgd::eligible(q0, false, false) || !wsgd::eligible(q1, false, false) || !wsgd::pair_compatible(q0, q1))
    return -20;
  if ((q80 != nullptr) != (q81 != nullptr)) return -20;  // one launch writes both MX-FP8 copies or neither
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  if (xwg_on() && g_xwg_cap > 0 && !q80 && wsgd::xwg::launch_pair(q0, q1, cus,
                                                                  wsgd::xwg::Scratch{g_xwg_T, g_xwg_cnt,
                                                                                     g_xwg_cnt + g_xwg_cap,
                                                                                     g_xwg_cnt + 2 * g_xwg_cap},
                                                                  g_xwg_cap, stream) == hipSuccess)
    return 0;
  return (int)wsgd::launch_pair(q0, q1, cus, stream);
}

DDPX_API int ddpx_wgrad_sgd_pair(const void* A0, const void* B0, int M0, int N0, int lda0, int ldb0, int ldc0,
                                 float* p0, float* buf0, void* sh0, void* q80, void* s80, const void* A1,
                                 const void* B1, int M1, int N1, int lda1, int ldb1, int ldc1, float* p1, float* buf1,
                                 void* sh1, void* q81, void* s81, int K, const float* lr, float mom, float wd,
                                 hipStream_t stream) {
  return ddpx_wgrad_sgd_pair_t(A0, B0, M0, N0, lda0, ldb0, ldc0, p0, buf0, sh0, q80, s80, nullptr, nullptr, A1, B1,
                               M1, N1, lda1, ldb1, ldc1, p1, buf1, sh1, q81, s81, nullptr, nullptr, K, lr, mom, wd,
                               stream);
}

// fc1's data gradient folded into the fc1 + fc0 weight-gradient + SGD launch (ddpx_wsgd_dgrad.h):
//   dX = relu_mask(aux) * (dY1 W1)  [batch x N1]  (W1: the bf16 copy the forward read, [M1][N1] row-major),
//   its column sums applied as SGD of the layer below's bias, then W1 -= sgd(dY1^T X1), W0 -= sgd(dX^T X0)
//   with W1's new bf16 copy written to sh1 (the other buffer of W1's ping-pong pair).
// scratch: colsum [batch / 64][N1] fp32; words: int32 [N1 / 128 + 2] rounded up to 4 (tickets, done, err),
// zeroed by the launch.  Returns -20 when not eligible (nothing launched).
DDPX_API int ddpx_wgrad_sgd_dgrad(const void* dY1, const void* X1, int M1, int N1, int ldy1, int ldx1, float* p1,
                                  float* buf1, void* sh1, void* q81, void* s81, const void* W1, int ldw1,
                                  void* dX, const void* aux, int ldaux, const void* X0, int N0, int ldx0, float* p0,
                                  float* buf0, void* sh0, void* q80, void* s80, float* bp, float* bbuf, void* bsh,
                                  float* colsum, int* words, int K, const float* lr, float mom, float wd,
                                  hipStream_t stream) {
  if (K <= 0 || M1 <= 0 || N1 <= 0 || N0 <= 0) return -20;
  if (ldy1 % 8 || ldx1 % 8 || ldx0 % 8 || ldw1 % 8 || ldaux % 8 || M1 % 8 || N1 % 8 || N0 % 8) return -20;
  if (((uintptr_t)dY1 | (uintptr_t)X1 | (uintptr_t)X0 | (uintptr_t)W1 | (uintptr_t)dX | (uintptr_t)aux) & 15)
    return -20;
  auto wp = [&](const void* A, const void* B, int M, int N, int lda, int ldb, float* pp, float* buf, void* sh,
                void* q8, void* s8) {
    const size_t a_bytes = ((size_t)(K - 1) * lda + M) * 2, b_bytes = ((size_t)(K - 1) * ldb + N) * 2;
    return pipe::Params{(const unsigned short*)A, (const unsigned short*)B, pp, nullptr, nullptr, nullptr,
                        M, N, K, lda, ldb, N, 0, pipe::EPI_SGD, 0, 1.f, (unsigned)a_bytes, (unsigned)b_bytes,
                        SgdArgs{pp, buf, (unsigned short*)sh, lr, mom, wd, (unsigned char*)q8, (unsigned char*)s8},
                        pipe::make_geom(0, 0, 0, 0), 0, 0, 0, nullptr, 0u, nullptr, nullptr, 0, nullptr};
  };
  // fc1: W1 [M1][N1], dY1 [K][M1], X1 [K][N1];  fc0: W0 [N1][N0] (its outputs are fc1's inputs), A = dX [K][N1]
  const pipe::Params q1 = wp(dY1, X1, M1, N1, ldy1, ldx1, p1, buf1, sh1, q81, s81);
  const pipe::Params q0 = wp(dX, X0, N1, N0, N1, ldx0, p0, buf0, sh0, q80, s80);
  if ((size_t)q1.a_bytes != ((size_t)(K - 1) * ldy1 + M1) * 2 || (size_t)q1.b_bytes != ((size_t)(K - 1) * ldx1 + N1) * 2 ||
      (size_t)q0.b_bytes != ((size_t)(K - 1) * ldx0 + N0) * 2)
    return -20;  // 32-bit buffer offsets
  const int nb = N1 / wsgdd::BN;
  wsgdd::DgArgs d{(const unsigned short*)dY1, (const unsigned short*)W1, (unsigned short*)dX,
                  (const unsigned short*)aux, K, N1, M1, ldy1, ldw1, N1, ldaux,
                  (unsigned)(((size_t)(K - 1) * ldy1 + M1) * 2), (unsigned)(((size_t)(M1 - 1) * ldw1 + N1) * 2),
                  colsum, words, words + nb, words + nb + 1, SgdArgs{bp, bbuf, (unsigned short*)bsh, lr, mom, wd}};
  if ((size_t)d.b_bytes != ((size_t)(M1 - 1) * ldw1 + N1) * 2) return -20;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  if (!wsgdd::eligible(q1, q0, d, cus)) return -20;
  const size_t zero_bytes = (size_t)((nb + 2 + 3) / 4 * 4) * 4;
  return (int)wsgdd::launch(q1, q0, d, cus, zero_bytes, stream);
}

DDPX_API int ddpx_wgrad_sgd_dgrad_words(int N1) { return (N1 / wsgdd::BN + 2 + 3) / 4 * 4; }
