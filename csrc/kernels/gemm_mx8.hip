// ddpx — MXFP8 GEMM and quantisation for gfx950 (the wide-MLP fp8 path, BASELINE config 5).
//
// CDNA4 runs the NON-scaled fp8 MFMA (16x16x32_fp8_fp8) at the bf16 rate; only the block-scaled
// `v_mfma_scale_f32_16x16x128_f8f6f4` reaches 2x bf16 per clock (MI355X_MICROARCH "Matrix cores").
// So fp8 here is OCP MX-FP8: every 32 consecutive K-elements of a row share one E8M0 power-of-two
// scale, applied by the MFMA itself — no per-tensor amax reduction, no delayed-scaling history,
// and quantisation is a local 32-element operation that can live in any producer kernel.
//
//   C[M][N] = epilogue( sum_k  A8[m][k] 2^(sa[m][k/32]-127)  *  B8[n][k] 2^(sb[n][k/32]-127) )
//
// Operands are K-contiguous ("NT"): A8 [M][K], B8 [N][K] (lda/ldb in bytes), scales [rows][K/32].
// Transposed operands (wgrad's dY^T, X^T) are produced by the transposing quantiser below, which
// costs the same bytes as a plain one.  A = e4m3 or e5m2 (gradients), B = e4m3.
//
// Kernel structure = the bf16 pipe (ddpx_pipe.h): 128x128 tile, 4 waves (2x2, 64x64 each),
// STAGES-deep LDS-DMA ring with counted vmcnt waits; one stage = 128 K-bytes = one MFMA K-step.
// The fp8 tile rows are 128 B, byte-identical to the bf16 pipe's [row][64 x bf16] images, so the
// same staging code and XOR swizzle serve both.  Each wave additionally DMAs 256 B of scales per
// stage (waves 0/1: A rows, 2/3: B rows; 4 E8M0 bytes per row per stage).  Operand map of the
// scaled MFMA (measured on MI355X with per-block scales, tools/mx_probe.py): lane l holds row l&15,
// its bytes 0-15 are K [16g, 16g+16) and bytes 16-31 are K [64+16g, 64+16g+16) (g = l>>4), and the
// scale byte lane-group g supplies (opsel 0) applies to K-block g = [32g, 32g+32) — so a block's
// data sits in two lane groups.  Epilogues are the bf16 pipe's (bias/ReLU/bf16/f32/SGD).
#include "ddpx_mx.h"
#include "ddpx_pipe.h"

namespace ddpx {
namespace mx8 {

using namespace pipe;
using mx::block_exp;
using mx::cvt_pk;
using mx::kMaxE4M3;
using mx::kMaxE5M2;
typedef int i32x8 __attribute__((ext_vector_type(8)));

// Quantise 32 values (one MX block) to 8 packed dwords.
__device__ __forceinline__ void quant32(const float* v, float inv, float maxv, bool e5m2, unsigned* out) {
#pragma unroll
  for (int w = 0; w < 8; ++w) out[w] = mx::quant4(v[4 * w], v[4 * w + 1], v[4 * w + 2], v[4 * w + 3], inv, maxv, e5m2);
}

// Row-direction quantiser: x bf16 [R][C] (ld elems) -> q [R][C] (ldq bytes), s [R][C/32].
// One thread per 32-element block.
__global__ void __launch_bounds__(256) quant_rows_kernel(const unsigned short* __restrict__ x, int R, int C, int ld,
                                                         unsigned char* __restrict__ q, int ldq,
                                                         unsigned char* __restrict__ s, int e5m2) {
  const int nb = C >> 5;
  const long long blk = (long long)blockIdx.x * 256 + threadIdx.x;
  if (blk >= (long long)R * nb) return;
  const int r = (int)(blk / nb), b = (int)(blk - (long long)r * nb);
  const u32x4* src = reinterpret_cast<const u32x4*>(x + (size_t)r * ld + b * 32);
  float v[32];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u32x4 w = src[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[8 * i + 2 * j] = __uint_as_float(w[j] << 16);
      v[8 * i + 2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
      amax = fmaxf(amax, fmaxf(fabsf(v[8 * i + 2 * j]), fabsf(v[8 * i + 2 * j + 1])));
    }
  }
  const float maxv = e5m2 ? kMaxE5M2 : kMaxE4M3;
  const int e = block_exp(amax, maxv);
  unsigned out[8];
  quant32(v, ldexpf(1.f, -e), maxv, e5m2, out);
  u32x4* dst = reinterpret_cast<u32x4*>(q + (size_t)r * ldq + b * 32);
  dst[0] = (u32x4){out[0], out[1], out[2], out[3]};
  dst[1] = (u32x4){out[4], out[5], out[6], out[7]};
  s[(size_t)r * nb + b] = (unsigned char)(e + 127);
}

// Transposing quantiser: x bf16 [R][C] -> qt [C][R] (ldq bytes) with blocks of 32 along R, st [C][R/32].
// A 512-thread workgroup stages a 128-row x 128-column slab in LDS (rows read as whole 256-B segments); thread
// (column t / 4, block t % 4) quantises one 32-row block of one column, so the 4 threads of a column write its
// 128 consecutive output bytes (one full line) and its 4 scale bytes together.  (A 32-row x 256-column slab with
// one thread per column wrote 32-B pieces 16 KB apart: 258 us for the wide MLP's 16384 x 16384 weight; 128 x 64
// slabs: 203 us.)
constexpr int kQcR = 128, kQcC = 128;
__global__ void __launch_bounds__(512) quant_cols_kernel(const unsigned short* __restrict__ x, int R, int C, int ld,
                                                         unsigned char* __restrict__ qt, int ldq,
                                                         unsigned char* __restrict__ st, int e5m2) {
  // row r sits at column offset 2 (r / 32): the 4 32-row blocks a wave reads in one instruction land in 4 different
  // banks (a plain row stride put them all on one)
  __shared__ unsigned short tile[kQcR][kQcC + 8];
  const int r0 = blockIdx.y * kQcR, c0 = blockIdx.x * kQcC;
  const int t = threadIdx.x;
  // load: 128 rows x 16 chunks of 8 bf16; 512 threads x 4 chunks (16 consecutive threads read one row's 256 B)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int chunk = i * 512 + t;
    const int rr = chunk >> 4, cc = (chunk & 15) * 8;
    u32x4 w = (u32x4){0u, 0u, 0u, 0u};
    if (r0 + rr < R && c0 + cc < C) w = *reinterpret_cast<const u32x4*>(x + (size_t)(r0 + rr) * ld + c0 + cc);
    unsigned* d = reinterpret_cast<unsigned*>(&tile[rr][cc + 2 * (rr >> 5)]);
    d[0] = w[0];
    d[1] = w[1];
    d[2] = w[2];
    d[3] = w[3];
  }
  __syncthreads();
  const int cl = t >> 2, q = t & 3;
  const int c = c0 + cl, rb = r0 + q * 32;
  if (c >= C || rb >= R) return;
  float v[32];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    v[i] = bf2f(tile[q * 32 + i][cl + 2 * q]);
    amax = fmaxf(amax, fabsf(v[i]));
  }
  const float maxv = e5m2 ? kMaxE5M2 : kMaxE4M3;
  const int e = block_exp(amax, maxv);
  unsigned out[8];
  quant32(v, ldexpf(1.f, -e), maxv, e5m2, out);
  u32x4* dst = reinterpret_cast<u32x4*>(qt + (size_t)c * ldq + rb);
  dst[0] = (u32x4){out[0], out[1], out[2], out[3]};
  dst[1] = (u32x4){out[4], out[5], out[6], out[7]};
  st[(size_t)c * (R >> 5) + (rb >> 5)] = (unsigned char)(e + 127);
}

// Single-wave probe of the scaled MFMA's operand map: A8/B8 [16][128], scales [16][4] -> C [16][16].
template <int FA, int FB>
__global__ void probe_kernel(const unsigned char* A, const unsigned char* B, const unsigned char* sa,
                             const unsigned char* sb, float* C) {
  const int l = threadIdx.x;
  const int row = l & 15, g = l >> 4;
  const u32x4 alo = *reinterpret_cast<const u32x4*>(A + row * 128 + 16 * g);
  const u32x4 ahi = *reinterpret_cast<const u32x4*>(A + row * 128 + 64 + 16 * g);
  const u32x4 blo = *reinterpret_cast<const u32x4*>(B + row * 128 + 16 * g);
  const u32x4 bhi = *reinterpret_cast<const u32x4*>(B + row * 128 + 64 + 16 * g);
  const i32x8 a = {(int)alo[0], (int)alo[1], (int)alo[2], (int)alo[3], (int)ahi[0], (int)ahi[1], (int)ahi[2], (int)ahi[3]};
  const i32x8 b = {(int)blo[0], (int)blo[1], (int)blo[2], (int)blo[3], (int)bhi[0], (int)bhi[1], (int)bhi[2], (int)bhi[3]};
  const int xa = sa[row * 4 + g], xb = sb[row * 4 + g];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, FA, FB, 0, xa, 0, xb);
#pragma unroll
  for (int r = 0; r < 4; ++r) C[(4 * g + r) * 16 + (l & 15)] = acc[r];
}

struct MxParams {
  Params base;               // C, bias, epi, alpha, sgd, M, N, K (K in elements = bytes), ldc ...
  const unsigned char* sa;   // [M][K/32]
  const unsigned char* sb;   // [N][K/32]
  unsigned sa_bytes, sb_bytes;
};

template <int STAGES, int FA>
__global__ void __launch_bounds__(256) gemm_mx8_kernel(MxParams mp) {
  constexpr int BM = 128, BN = 128, BKB = 128;  // BKB: K-bytes per stage
  constexpr int A_BYTES = BM * BKB, B_BYTES = BN * BKB, S_BYTES = (BM + BN) * 4;
  constexpr int SLOT = A_BYTES + B_BYTES + S_BYTES;
  constexpr int FM = 4, FN = 4;
  constexpr int LPW = BM / 32 + BN / 32 + 1;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * SLOT];
  const Params& p = mp.base;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = wg % tiles_m, tn = wg / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nkb = p.K >> 5;  // scale blocks per row

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, 0, p.b_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)mp.sa, 0, mp.sa_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)mp.sb, 0, mp.sb_bytes, 0x00020000);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BKB;
  // byte-addressed operands staged as "pairs" by the bf16 staging code: ld and K halved
  const int lda2 = p.lda >> 1, ldb2 = p.ldb >> 1, kend2 = p.K >> 1;
  const bool s_is_a = wave < 2;
  const int srow = (wave & 1) * 64 + lane;

  auto issue = [&](int t) {
    char* slot = smem + (t % STAGES) * SLOT;
    const int k2 = t * (BKB / 2);
    stage_tile<BM, true, MODE_PLAIN>(ra, slot, p.conv, lda2, m0, p.M, k2, kend2, wave, lane);
    stage_tile<BN, true, MODE_PLAIN>(rb, slot + A_BYTES, p.conv, ldb2, n0, p.N, k2, kend2, wave, lane);
    const int grow = (s_is_a ? m0 : n0) + srow;
    const int lim = s_is_a ? p.M : p.N;
    const unsigned voff = grow < lim ? (unsigned)(grow * nkb + t * 4) : kOOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(s_is_a ? rsa : rsb,
                                             (LDS_AS void*)(slot + A_BYTES + B_BYTES + (wave * 256)), 4, voff, 0,
                                             0, 0);
  };

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s);

  const int g = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    const int ahead = min(STAGES - 2, nk - 1 - t);
    if (ahead >= 2) wait_vmcnt<2 * LPW>();
    else if (ahead == 1) wait_vmcnt<LPW>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1);

    const char* sa = smem + (t % STAGES) * SLOT;
    const char* sb = sa + A_BYTES;
    const unsigned char* ss = reinterpret_cast<const unsigned char*>(sb + B_BYTES);
    i32x8 a[FM], b[FN];
    int xa[FM], xb[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * 64 + i * 16 + (lane & 15);
      const int sw = (row >> 1) & 7;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(sa + row * 128 + ((g ^ sw) << 4));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(sa + row * 128 + (((g + 4) ^ sw) << 4));
      a[i] = (i32x8){(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      xa[i] = ss[row * 4 + g];
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * 64 + j * 16 + (lane & 15);
      const int sw = (row >> 1) & 7;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(sb + row * 128 + ((g ^ sw) << 4));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(sb + row * 128 + (((g + 4) ^ sw) << 4));
      b[j] = (i32x8){(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      xb[j] = ss[BM * 4 + row * 4 + g];
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b[j], acc[i][j], FA, 0, 0, xa[i], 0,
                                                                     xb[j]);
  }

  constexpr int TLD = BN + 4;
  float* T = reinterpret_cast<float*>(smem);
  static_assert(BM * TLD * 4 <= STAGES * SLOT, "epilogue LDS overflow");
  __builtin_amdgcn_s_barrier();
  {
    const int mr = wm * 64 + 4 * (lane >> 4);
    const int nc = wn * 64 + (lane & 15);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) T[(mr + i * 16 + r) * TLD + nc + j * 16] = acc[i][j][r];
  }
  __syncthreads();
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  void* Cbase = p.C;
  switch (p.epi) {
    case EPI_F32: epilogue_vec<EPI_F32, BM, BN>(p, Cbase, T, m0, n0, tid, cs); break;
    case EPI_BF16: epilogue_vec<EPI_BF16, BM, BN>(p, Cbase, T, m0, n0, tid, cs); break;
    case EPI_BIAS_BF16: epilogue_vec<EPI_BIAS_BF16, BM, BN>(p, Cbase, T, m0, n0, tid, cs); break;
    case EPI_BIAS_RELU_BF16: epilogue_vec<EPI_BIAS_RELU_BF16, BM, BN>(p, Cbase, T, m0, n0, tid, cs); break;
    case EPI_BIAS_F32: epilogue_vec<EPI_BIAS_F32, BM, BN>(p, Cbase, T, m0, n0, tid, cs); break;
    case EPI_SGD: epilogue_vec<EPI_SGD, BM, BN>(p, Cbase, T, m0, n0, tid, cs); break;
    default: epilogue_vec<EPI_RELUMASK_BF16, BM, BN>(p, Cbase, T, m0, n0, tid, cs); break;
  }
}

}  // namespace mx8
}  // namespace ddpx

using namespace ddpx;

// x bf16 [R][C] -> MX-fp8 rows (q [R][C], s [R][C/32]) and/or transposed (qt [C][R], st [C][R/32]).
DDPX_API int ddpx_mx8_quant(const void* x, int R, int C, int ld, void* q, int ldq, void* s, void* qt, int ldqt,
                            void* st, int e5m2, hipStream_t stream) {
  if (R <= 0 || C <= 0) return 0;
  if (q) {
    if (C % 32 || ld % 8 || ldq % 16) return -1;
    const long long nb = (long long)R * (C / 32);
    hipLaunchKernelGGL(mx8::quant_rows_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, stream,
                       (const unsigned short*)x, R, C, ld, (unsigned char*)q, ldq, (unsigned char*)s, e5m2);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  if (qt) {
    if (R % 32 || ld % 8 || ldqt % 16) return -2;
    hipLaunchKernelGGL(mx8::quant_cols_kernel, dim3((C + mx8::kQcC - 1) / mx8::kQcC, (R + mx8::kQcR - 1) / mx8::kQcR),
                       dim3(512), 0, stream,
                       (const unsigned short*)x, R, C, ld, (unsigned char*)qt, ldqt, (unsigned char*)st, e5m2);
    return (int)hipGetLastError();
  }
  return 0;
}

DDPX_API int ddpx_mx8_probe(const void* A, const void* B, const void* sa, const void* sb, float* C, int fa,
                            int fb, hipStream_t s) {
  const unsigned char *a = (const unsigned char*)A, *b = (const unsigned char*)B;
  const unsigned char *xa = (const unsigned char*)sa, *xb = (const unsigned char*)sb;
  if (fa == 0 && fb == 0) hipLaunchKernelGGL((mx8::probe_kernel<0, 0>), dim3(1), dim3(64), 0, s, a, b, xa, xb, C);
  else if (fa == 1 && fb == 0) hipLaunchKernelGGL((mx8::probe_kernel<1, 0>), dim3(1), dim3(64), 0, s, a, b, xa, xb, C);
  else return -1;
  return (int)hipGetLastError();
}

// C = epi( A8 . B8^T ) with MX scales.  A8 [M][K] (lda bytes, fmt fa: 0 e4m3 / 1 e5m2), B8 [N][K] e4m3.
DDPX_API int ddpx_gemm_mx8(const void* A, const void* sa, const void* B, const void* sb, void* C, const float* bias,
                           const void* aux, int M, int N, int K, int lda, int ldb, int ldc, int ldaux, int fa,
                           int epi, int accumulate, float alpha, float* sgd_p, float* sgd_buf, void* sgd_shadow,
                           const float* sgd_lr, float sgd_mom, float sgd_wd, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % 128 || lda % 16 || ldb % 16) return -1;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -3;
  if ((reinterpret_cast<uintptr_t>(sa) | reinterpret_cast<uintptr_t>(sb)) & 3) return -3;
  if (epi == pipe::EPI_BNSTAT_BF16) return -6;
  const size_t a_bytes = (size_t)(M - 1) * lda + K, b_bytes = (size_t)(N - 1) * ldb + K;
  if (a_bytes >= 0x80000000ull || b_bytes >= 0x80000000ull) return -4;
  if (epi == pipe::EPI_SGD && (!sgd_p || !sgd_lr || (sgd_mom != 0.f && !sgd_buf))) return -5;
  mx8::MxParams mp;
  mp.base = pipe::Params{(const unsigned short*)A, (const unsigned short*)B, C, bias, (const unsigned short*)aux,
                         nullptr, M, N, K, lda, ldb, ldc, ldaux, epi, accumulate, alpha, (unsigned)a_bytes,
                         (unsigned)b_bytes, SgdArgs{sgd_p, sgd_buf, (unsigned short*)sgd_shadow, sgd_lr, sgd_mom,
                                                     sgd_wd},
                         pipe::make_geom(0, 0, 0, 0), 0, 0};
  mp.sa = (const unsigned char*)sa;
  mp.sb = (const unsigned char*)sb;
  mp.sa_bytes = (unsigned)((size_t)M * (K / 32));
  mp.sb_bytes = (unsigned)((size_t)N * (K / 32));
  const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
  // ring depth (DDPX_MX8_STAGES=2|3): 2 stages = 66 KiB, two workgroups per CU (default: wide-MLP products 7-24 %
  // faster than one 3-stage workgroup of 99 KiB per CU, profiles/r6_fp8/fp8_table_s{2,3}.json)
  static const int stages = [] {
    const char* e = getenv("DDPX_MX8_STAGES");
    return e && e[0] == '3' ? 3 : 2;
  }();
  if (stages == 2) {
    if (fa) hipLaunchKernelGGL((mx8::gemm_mx8_kernel<2, 1>), dim3(tiles), dim3(256), 0, stream, mp);
    else hipLaunchKernelGGL((mx8::gemm_mx8_kernel<2, 0>), dim3(tiles), dim3(256), 0, stream, mp);
  } else {
    if (fa) hipLaunchKernelGGL((mx8::gemm_mx8_kernel<3, 1>), dim3(tiles), dim3(256), 0, stream, mp);
    else hipLaunchKernelGGL((mx8::gemm_mx8_kernel<3, 0>), dim3(tiles), dim3(256), 0, stream, mp);
  }
  return (int)hipGetLastError();
}
