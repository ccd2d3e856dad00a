// ddpx — 3x3 / stride 1 / pad 1 convolutions as implicit GEMMs on the
// pipelined MFMA core (ddpx_pipe.h), NHWC bf16 activations.
//
// Replaces MIOpen's conv fwd / dgrad / wgrad for the reference's VGG
// (/root/reference/singlegpu.py:64 `nn.Conv2d(in, x, 3, padding=1, bias=False)`;
// SURVEY §2.2 N7, §2.3 shape table).  With P = N*H*W pixels:
//   forward : y[P][Co]        = im2col(x)[P][9Ci]      . Wf[Co][9Ci]^T   (A: IM2COL_FWD, B: K-contig)
//   dgrad   : dx[P][Ci]       = im2col~(dy)[P][9Co]    . Wd[9Co][Ci]     (A: IM2COL_BWD, B: N-contig)
//   wgrad   : dW[Co][9Ci]     = dy[P][Co]^T            . im2col(x)[P][9Ci] (A: M-contig, B: IM2COL_COL)
// where the K index is (tap, channel) with channel fastest, so every 16-B
// DMA chunk is 8 consecutive channels of one pixel.  Padding taps are zero
// through the buffer bounds check.  Wf = W permuted to [Co][3][3][Ci],
// Wd = W permuted to [3][3][Co][Ci] (ddpx_conv_weight_prep, one pass per
// step, channels padded to a multiple of 8 with zeros — conv0's Ci = 3).
// The weight gradient (K = P up to 524288) is split over blockIdx.y into
// fp32 slabs reduced in fixed order by ddpx_conv_wgrad_reduce, which also
// permutes back to torch's [Co][Ci][3][3] layout (checkpoint format) and
// either stores the gradient or applies the fused SGD update.
// The forward epilogue can emit per-tile BatchNorm statistics (mean, M2 of
// the stored bf16 outputs) for the fused BN that follows (bn.hip).
#include "ddpx_gemm_dispatch.h"
#include "ddpx_pipe.h"

namespace ddpx {
namespace conv {

using namespace pipe;

// fp32 torch weight [Co][Cr][3][3] -> Wf bf16 [Co][9][Cp], Wd bf16 [9][Co][Cp]  (Cp >= Cr, zero padded)
__global__ void __launch_bounds__(256) weight_prep_kernel(const float* __restrict__ w, int Co, int Cr, int Cp,
                                                          unsigned short* __restrict__ wf,
                                                          unsigned short* __restrict__ wd) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // over Co*9*Cp, output-major (c fastest)
  if (i >= Co * 9 * Cp) return;
  const int c = i % Cp;
  const int t = (i / Cp) % 9;
  const int o = i / (9 * Cp);
  const float v = c < Cr ? w[((size_t)o * Cr + c) * 9 + t] : 0.f;
  const unsigned short h = f2bf(v);
  if (wf) wf[i] = h;
  if (wd) wd[((size_t)t * Co + o) * Cp + c] = h;
}

// out (torch layout [Co][Cr][3][3]) (=|+=) sum_s part[s][Co][9*Cp]   or fused SGD on the parameter.
// Workgroup = (output channel o, 64-channel tile): the S partial slabs are read tap-major with the
// channel index fastest (coalesced, 4 slabs' loads in flight per thread), the sums are transposed
// through LDS, and the [c][tap] run of the torch layout — 64 x 9 consecutive floats — is written (or
// SGD-updated) contiguously.  Fixed summation order: deterministic.
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ part, int S, int Co, int Cr,
                                                           int Cp, void* __restrict__ out, int out_bf16,
                                                           int accumulate, SgdArgs sgd,
                                                           unsigned short* __restrict__ wf,
                                                           unsigned short* __restrict__ wd) {
  constexpr int CT = 64;
  __shared__ float red[9][CT + 1];
  __shared__ float sred[256];
  const int o = blockIdx.x;
  const int c0 = blockIdx.y * CT;
  const int nc = min(CT, Cr - c0);
  const size_t slab = (size_t)Co * 9 * Cp;
  const int items = 9 * nc;
  // few outputs per workgroup (thin layers, e.g. 3 input channels) but many slabs: TS threads share an
  // output, each summing every TS-th slab, then a fixed-order combine (deterministic)
  int TS = 1;
  while (TS < 16 && items * TS * 2 <= 256) TS *= 2;
  if (TS == 1) {
    // one thread per output, up to 3 outputs per thread (9 x 64 items): the loads of 8 slabs for ALL of a
    // thread's outputs go out together (24 in flight instead of 4: the reduce was latency-bound at ~2 TB/s),
    // then each output adds its slabs in slab order (the same sum, bit for bit, as one slab at a time)
    constexpr int MI = (9 * CT + 255) / 256;
    float acc[MI];
    const float* src[MI];
#pragma unroll
    for (int ii = 0; ii < MI; ++ii) {
      acc[ii] = 0.f;
      const int j = threadIdx.x + ii * 256;
      const int jj = j < items ? j : 0;
      src[ii] = part + (size_t)o * 9 * Cp + (size_t)(jj / nc) * Cp + c0 + jj % nc;
    }
    for (int k0 = 0; k0 < S; k0 += 8) {
      float v[MI][8];
#pragma unroll
      for (int ii = 0; ii < MI; ++ii)
#pragma unroll
        for (int q = 0; q < 8; ++q)
          v[ii][q] = (k0 + q < S && threadIdx.x + ii * 256 < items) ? src[ii][(size_t)(k0 + q) * slab] : 0.f;
#pragma unroll
      for (int ii = 0; ii < MI; ++ii)
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (k0 + q < S) acc[ii] += v[ii][q];
    }
#pragma unroll
    for (int ii = 0; ii < MI; ++ii) {
      const int j = threadIdx.x + ii * 256;
      if (j < items) red[j / nc][j % nc] = acc[ii];
    }
  }
  for (int j0 = 0; TS > 1 && j0 < items; j0 += 256 / TS) {
    const int j = j0 + threadIdx.x / TS, sub = threadIdx.x % TS;
    float s = 0.f;
    if (j < items && threadIdx.x / TS < 256 / TS) {
      const int t = j / nc, cc = j % nc;
      const float* src = part + (size_t)o * 9 * Cp + (size_t)t * Cp + c0 + cc;
      int k = sub;
      for (; k + 3 * TS < S; k += 4 * TS) {
        const float a0 = src[(size_t)k * slab], a1 = src[(size_t)(k + TS) * slab];
        const float a2 = src[(size_t)(k + 2 * TS) * slab], a3 = src[(size_t)(k + 3 * TS) * slab];
        s += a0;
        s += a1;
        s += a2;
        s += a3;
      }
      for (; k < S; k += TS) s += src[(size_t)k * slab];
    }
    if (TS == 1) {
      if (j < items) red[j / nc][j % nc] = s;
    } else {
      sred[threadIdx.x] = s;
      __syncthreads();
      if (sub == 0 && j < items) {
        float v = 0.f;
        for (int q = 0; q < TS; ++q) v += sred[threadIdx.x + q];
        red[j / nc][j % nc] = v;
      }
      __syncthreads();
    }
  }
  __syncthreads();
  const size_t base = ((size_t)o * Cr + c0) * 9;
  for (int q = threadIdx.x; q < nc * 9; q += 256) {
    const int cc = q / 9, t = q % 9;
    const float v = red[t][cc];
    const size_t i = base + q;
    if (sgd.p) {
      const float pn = sgd_apply(sgd, i, v, *sgd.lr);
      if (wf) red[t][cc] = pn;  // (this thread's own element) -> the layout writes below
    } else if (out_bf16) {
      unsigned short* d = reinterpret_cast<unsigned short*>(out) + i;
      *d = f2bf(accumulate ? v + bf2f(*d) : v);
    } else {
      float* d = reinterpret_cast<float*>(out) + i;
      *d = accumulate ? v + *d : v;
    }
  }
  if (sgd.p && wf) {
    // the forward / dgrad GEMM layouts of the updated weight (weight_prep's output), channel-fastest: a wave
    // writes 128 contiguous bytes of each [.][tap][channel] row instead of 2-byte stores 9 taps apart
    __syncthreads();
    for (int q = threadIdx.x; q < nc * 9; q += 256) {
      const int t = q / nc, cc = q - t * nc;
      const unsigned short h = f2bf(red[t][cc]);
      wf[((size_t)o * 9 + t) * Cp + c0 + cc] = h;
      wd[((size_t)t * Co + o) * Cp + c0 + cc] = h;
    }
  }
}

// Tile picks from the per-layer MI355X sweep after the fast-division addressing (benchmarks/conv_sweep.py,
// profiles/r1_fdiv/conv_sweep_fdiv.json): the 8-wave 256x256 tile (cfg 13) wins every >= 128-channel
// layer at 16x16 and 8x8 (fwd 512->512@8: 151 vs 198 us for 256x128); the 32x32 layers keep 256x128
// (cfg 8); 4x4 layers (P = 8192) want 64x128; <= 64-channel outputs stay on 64x64.
// Picks re-measured in round 5 with the 2-deep 128x128 rings (configs 21 / 22: two workgroups per CU, so one
// workgroup's ring fill and epilogue run under the other's main loop; profiles/r5_conv/NOTES.md).
// DDPX_CONV_PICKS=r4 restores the round-4 picks (A/B runs).
static int g_picks_r4 = -1;
static bool picks_r4() {
  if (g_picks_r4 < 0) {
    const char* e = getenv("DDPX_CONV_PICKS");
    g_picks_r4 = (e && e[0] == 'r' && e[1] == '4') ? 1 : 0;
  }
  return g_picks_r4 == 1;
}
static int pick_fwd(int P, int C, int Co) {
  // 64-channel outputs at 32x32 (VGG conv0, DeepNN 128->64): 256x64, 2-deep (47.9 vs 53.4 us, 120.7 vs 159.9 us)
  if (Co <= 64 && P >= 524288 && !picks_r4()) return 23;
  if (Co <= 64) return 7;     // DeepNN's 64/32-channel layers at 16x16: 64x64, 3 stages
  if (P <= 8192) return picks_r4() ? 5 : 14;  // 4x4 layers: 128x128 / 8 waves / 3 stages (55.1 vs 61.7 us for cfg 5)
  if (picks_r4()) return P >= 524288 ? 8 : 13;
  if (C <= 128) return 22;    // K <= 1152 (VGG conv1 @32, conv2 @16): 115.6 vs 149.3 us (cfg 8) on conv1
  return 13;                  // 256x256, 8 waves
}
// Data-gradient picks do not change any result bit (every tile sums K in the same order, no statistics), so
// they follow the measurements directly: VGG conv1's dx 128x64 with the cached im2col rows (141 vs 153 us
// for 64x64, profiles/r4_vgg/probe_*.jsonl).
static int pick_dgrad(int P, int C, int Co) {
  if (C <= 64 && P >= 524288 && !picks_r4()) return 23;  // VGG conv1's dx @32: 256x64, 2-deep (116.6 vs 144.5 us)
  if (C <= 64) return 6;      // dx of a 64-channel input (DeepNN @16): 128x64, 3 stages
  if (picks_r4()) return P <= 8192 ? 15 : (Co <= 64 || Co > C) ? 8 : 13;
  // 4x4 layers: 8-wave 128x128 / 4 stages (the 2-deep cfg 22 is faster alone, 56.5 vs 63.1 us, but slower with
  // the fused BatchNorm sums in its epilogue, 78.4 vs 68.5 us in the step, profiles/r5_conv)
  if (P <= 8192) return 15;
  if (Co <= 64 || Co > C) return 22;  // widening layers (dx narrower than dy), thin DeepNN layers: 124 vs 140 us
  return 13;
}

}  // namespace conv
}  // namespace ddpx

using namespace ddpx;
using namespace ddpx::pipe;

static bool chk16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// DDPX_IM2COL_ROWCACHE=0: per-chunk im2col addressing for the forward / data-gradient A operand (A/B checks)
static int g_im_slow = -1;
static int im_slow() {
  if (g_im_slow < 0) {
    const char* e = getenv("DDPX_IM2COL_ROWCACHE");
    g_im_slow = (e && e[0] == '0') ? 1 : 0;
  }
  return g_im_slow;
}
// 1: cached row addressing (default), 0: per-chunk addressing, < 0: back to the environment / default
DDPX_API void ddpx_conv_set_rowcache(int on) { g_im_slow = on < 0 ? -1 : (on ? 0 : 1); }


DDPX_API int ddpx_conv_weight_prep(const float* w, int Co, int Cr, int Cp, void* wf, void* wd, hipStream_t s) {
  if (Cp % 8 || Cp < Cr) return -1;
  const int n = Co * 9 * Cp;
  hipLaunchKernelGGL(conv::weight_prep_kernel, dim3((n + 255) / 256), dim3(256), 0, s, w, Co, Cr, Cp,
                     (unsigned short*)wf, (unsigned short*)wd);
  return (int)hipGetLastError();
}

// Row tiles the forward GEMM uses (for sizing the BatchNorm statistics partials).
DDPX_API int ddpx_conv_fwd_tiles_m(int P, int C, int Co, int tile_cfg) {
  const int cfg = tile_cfg >= 0 ? tile_cfg : conv::pick_fwd(P, C, Co);
  int bm, bn;
  tile_of(cfg, &bm, &bn);
  return (P + bm - 1) / bm;  // one statistics row per row tile (the epilogue merges its row parts)
}

DDPX_API int ddpx_conv_fwd_tile_rows(int P, int C, int Co, int tile_cfg) {
  const int cfg = tile_cfg >= 0 ? tile_cfg : conv::pick_fwd(P, C, Co);
  int bm, bn;
  tile_of(cfg, &bm, &bn);
  return bm;
}

// y[P][Co] = conv(x, W).  x NHWC [N][H][W][C] bf16 (C % 8 == 0), wf [Co][9][C].
// stats (optional): [tiles_m][2][Co] per-tile (mean, M2) of the stored bf16 outputs.
DDPX_API int ddpx_conv_fwd(const void* x, const void* wf, void* y, float* stats, int N, int H, int W, int C, int Co,
                           int tile_cfg, hipStream_t s) {
  if (C % 8 || Co % 8) return -1;
  if (!chk16(x) || !chk16(wf) || !chk16(y)) return -3;
  const int P = N * H * W, K = 9 * C;
  Params p{};
  p.A = (const unsigned short*)x;
  p.B = (const unsigned short*)wf;
  p.C = y;
  p.colsum = stats;
  p.M = P; p.N = Co; p.K = K;
  p.lda = C; p.ldb = K; p.ldc = Co;
  p.epi = stats ? EPI_BNSTAT_BF16 : EPI_BF16;
  p.alpha = 1.f;
  p.im_slow = im_slow();
  const size_t ab = (size_t)P * C * 2, bb = (size_t)Co * K * 2;
  if (ab >= 0x80000000ull || bb >= 0x80000000ull) return -4;
  p.a_bytes = (unsigned)ab; p.b_bytes = (unsigned)bb;
  p.conv = make_geom(H, W, C, P);
  const int cfg = tile_cfg >= 0 ? tile_cfg : conv::pick_fwd(P, C, Co);
  return (int)dispatch_conv_fwd(p, cfg, s);
}

// DeepNN's conv blocks (no BatchNorm, /root/reference/singlegpu.py:18-44): act[P][Co] = relu(conv(x, W) + bias) in
// the GEMM epilogue (EPI_BIAS_RELU_BF16), so no separate bias/ReLU pass reads the conv output back.
DDPX_API int ddpx_conv_fwd_act(const void* x, const void* wf, void* act, const float* bias, int N, int H, int W, int C,
                               int Co, int tile_cfg, hipStream_t s) {
  if (C % 8 || Co % 8 || !bias) return -1;
  if (!chk16(x) || !chk16(wf) || !chk16(act)) return -3;
  const int P = N * H * W, K = 9 * C;
  Params p{};
  p.A = (const unsigned short*)x;
  p.B = (const unsigned short*)wf;
  p.C = act;
  p.bias = bias;
  p.M = P; p.N = Co; p.K = K;
  p.lda = C; p.ldb = K; p.ldc = Co;
  p.epi = EPI_BIAS_RELU_BF16;
  p.alpha = 1.f;
  p.im_slow = im_slow();
  const size_t ab = (size_t)P * C * 2, bb = (size_t)Co * K * 2;
  if (ab >= 0x80000000ull || bb >= 0x80000000ull) return -4;
  p.a_bytes = (unsigned)ab; p.b_bytes = (unsigned)bb;
  p.conv = make_geom(H, W, C, P);
  const int cfg = tile_cfg >= 0 ? tile_cfg : conv::pick_fwd(P, C, Co);
  return (int)dispatch_conv_fwd(p, cfg, s);
}

// Row tiles of the data-gradient GEMM (rows of ddpx_conv_dgrad_act's column-sum partials).
DDPX_API int ddpx_conv_dgrad_tiles_m(int N, int H, int W, int C, int Co, int tile_cfg) {
  const int P = N * H * W;
  const int cfg = tile_cfg >= 0 ? tile_cfg : conv::pick_dgrad(P, C, Co);
  int bm, bn;
  tile_of(cfg, &bm, &bn);
  return (P + bm - 1) / bm;
}

// Data gradient straight into the pre-activation gradient of the (un-pooled) ReLU block below:
// dz[P][C] = dgrad(dy, W) * (act[P][C] > 0) (EPI_RELUMASK_BF16, act = relu(conv + bias) of that block), plus
// colsum[T][C] = per-row-tile column sums of the stored dz (its bias gradient, finished in fixed order by
// ddpx_colsum_finish).  One launch replaces the plain data gradient and a reduce + apply pass over dz.
DDPX_API int ddpx_conv_dgrad_act(const void* dy, const void* wd, void* dz, int N, int H, int W, int C, int Co,
                                 int tile_cfg, const void* act, float* colsum, hipStream_t s) {
  if (C % 8 || Co % 8 || !act || !colsum) return -1;
  if (!chk16(dy) || !chk16(wd) || !chk16(dz) || !chk16(act)) return -3;
  const int P = N * H * W, K = 9 * Co;
  Params p{};
  p.A = (const unsigned short*)dy;
  p.B = (const unsigned short*)wd;
  p.C = dz;
  p.aux = (const unsigned short*)act;
  p.ldaux = C;
  p.colsum = colsum;
  p.M = P; p.N = C; p.K = K;
  p.lda = Co; p.ldb = C; p.ldc = C;
  p.epi = EPI_RELUMASK_BF16;
  p.alpha = 1.f;
  p.im_slow = im_slow();
  const size_t ab = (size_t)P * Co * 2, bb = (size_t)K * C * 2;
  if (ab >= 0x80000000ull || bb >= 0x80000000ull) return -4;
  p.a_bytes = (unsigned)ab; p.b_bytes = (unsigned)bb;
  p.conv = make_geom(H, W, Co, P);
  const int cfg = tile_cfg >= 0 ? tile_cfg : conv::pick_dgrad(P, C, Co);
  return (int)dispatch_conv_dgrad(p, cfg, s);
}

namespace ddpx {
namespace conv {
// out[c] (=|+=) sum_t part[t][c], or the fused SGD of the parameter out points at.  Two fixed-order levels (the
// partials can be 4096 rows: one thread per channel walking them all took 237 us): split sp of S sums rows
// [sp * RS, (sp + 1) * RS) as 4 interleaved row groups merged in group order, then one thread per channel adds
// the S split sums in split order.  Deterministic.
constexpr int kColsumRows = 64;  // rows per split
__global__ void __launch_bounds__(256) colsum_split_kernel(const float* __restrict__ part, int T, int C,
                                                           float* __restrict__ ws) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, sp = blockIdx.y;
  const int t0 = sp * kColsumRows, t1 = min(T, t0 + kColsumRows);
  float s = 0.f;
  if (c < C) {
    float v[kColsumRows / 4];
#pragma unroll
    for (int u = 0; u < kColsumRows / 4; ++u) {
      const int t = t0 + g + 4 * u;
      v[u] = t < t1 ? part[(size_t)t * C + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kColsumRows / 4; ++u) s += v[u];
  }
  red[g][cl] = s;
  __syncthreads();
  if (g == 0 && c < C) ws[(size_t)sp * C + c] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
}

__global__ void __launch_bounds__(256) colsum_finish_kernel(const float* __restrict__ ws, int S, int C,
                                                            void* __restrict__ out, int out_bf16, int accumulate,
                                                            SgdArgs sgd) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  int t = 0;
  for (; t + 8 <= S; t += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ws[(size_t)(t + u) * C + c];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; t < S; ++t) s += ws[(size_t)t * C + c];
  if (sgd.p) {
    sgd_apply(sgd, c, s, *sgd.lr);
  } else if (out_bf16) {
    unsigned short* d = reinterpret_cast<unsigned short*>(out) + c;
    *d = f2bf(accumulate ? s + bf2f(*d) : s);
  } else {
    float* d = reinterpret_cast<float*>(out) + c;
    *d = accumulate ? s + *d : s;
  }
}
}  // namespace conv
}  // namespace ddpx

// Workspace floats ddpx_colsum_finish needs for T partial rows of C columns.
DDPX_API long long ddpx_colsum_ws_floats(int T, int C) {
  return (long long)((T + conv::kColsumRows - 1) / conv::kColsumRows) * C;
}

DDPX_API int ddpx_colsum_finish(const float* part, int T, int C, float* ws, void* out, int out_bf16, int accumulate,
                                float* sgd_p, float* sgd_buf, void* sgd_shadow, const float* sgd_lr, float sgd_mom,
                                float sgd_wd, hipStream_t s) {
  if (T < 1 || C < 1 || !ws || (!out && !sgd_p) || (sgd_p && !sgd_lr)) return -1;
  const int S = (T + conv::kColsumRows - 1) / conv::kColsumRows;
  hipLaunchKernelGGL(conv::colsum_split_kernel, dim3((C + 63) / 64, S), dim3(256), 0, s, part, T, C, ws);
  hipLaunchKernelGGL(conv::colsum_finish_kernel, dim3((C + 255) / 256), dim3(256), 0, s, ws, S, C, out, out_bf16,
                     accumulate, SgdArgs{sgd_p, sgd_buf, (unsigned short*)sgd_shadow, sgd_lr, sgd_mom, sgd_wd});
  return (int)hipGetLastError();
}

// dx[P][C] = dgrad(dy, W) (optionally times relu mask of aux — unused by VGG, whose
// ReLU sits behind BN).  dy [P][Co] bf16, wd [9][Co][C] bf16.
DDPX_API int ddpx_conv_dgrad(const void* dy, const void* wd, void* dx, int N, int H, int W, int C, int Co,
                             int tile_cfg, hipStream_t s) {
  if (C % 8 || Co % 8) return -1;
  if (!chk16(dy) || !chk16(wd) || !chk16(dx)) return -3;
  const int P = N * H * W, K = 9 * Co;
  Params p{};
  p.A = (const unsigned short*)dy;
  p.B = (const unsigned short*)wd;
  p.C = dx;
  p.M = P; p.N = C; p.K = K;
  p.lda = Co; p.ldb = C; p.ldc = C;
  p.epi = EPI_BF16;
  p.alpha = 1.f;
  p.im_slow = im_slow();
  const size_t ab = (size_t)P * Co * 2, bb = (size_t)K * C * 2;
  if (ab >= 0x80000000ull || bb >= 0x80000000ull) return -4;
  p.a_bytes = (unsigned)ab; p.b_bytes = (unsigned)bb;
  p.conv = make_geom(H, W, Co, P);
  const int cfg = tile_cfg >= 0 ? tile_cfg : conv::pick_dgrad(P, C, Co);
  return (int)dispatch_conv_dgrad(p, cfg, s);
}

// Data gradient fused with the BatchNorm backward sums of the block below (EPI_BNBWD_BF16): dx as ddpx_conv_dgrad,
// plus part[B][2][C] = per-row-tile (sum dz, sum dz*xhat) of the routed, ReLU-masked gradient, B =
// ddpx_conv_dgrad_parts(...).  bn_y: the block below's pre-BN activation [N][H'][W'][C] (H' = 2H when pooled).
// Returns 0 when the picked tile has no fused variant (the caller then runs the plain data gradient and the
// separate reduce).
DDPX_API int ddpx_conv_dgrad_parts(int N, int H, int W, int C, int Co, int tile_cfg) {
  const int P = N * H * W;
  const int cfg = tile_cfg >= 0 ? tile_cfg : conv::pick_dgrad(P, C, Co);
  if (cfg != 8 && cfg != 15 && cfg != 22) return 0;  // the configs instantiating EPI_BNBWD_BF16 (ddpx_pipe.h)
  int bm, bn;
  tile_of(cfg, &bm, &bn);
  return (P + bm - 1) / bm * epilogue_halves(cfg);
}

DDPX_API int ddpx_conv_dgrad_bn(const void* dy, const void* wd, void* dx, int N, int H, int W, int C, int Co,
                                int tile_cfg, const void* bn_y, const float* a, const float* b, const float* mean,
                                const float* rstd, int pool, float* part, hipStream_t s) {
  if (C % 8 || Co % 8 || !bn_y || !a || !b || !mean || !rstd || !part) return -1;
  if (!chk16(dy) || !chk16(wd) || !chk16(dx) || !chk16(bn_y)) return -3;
  const int P = N * H * W, K = 9 * Co;
  Params p{};
  p.A = (const unsigned short*)dy;
  p.B = (const unsigned short*)wd;
  p.C = dx;
  p.M = P; p.N = C; p.K = K;
  p.lda = Co; p.ldb = C; p.ldc = C;
  p.epi = EPI_BNBWD_BF16;
  p.alpha = 1.f;
  p.im_slow = im_slow();
  const size_t ab = (size_t)P * Co * 2, bb = (size_t)K * C * 2;
  if (ab >= 0x80000000ull || bb >= 0x80000000ull) return -4;
  p.a_bytes = (unsigned)ab; p.b_bytes = (unsigned)bb;
  p.conv = make_geom(H, W, Co, P);
  p.colsum = part;
  p.bn_y = (const unsigned short*)bn_y;
  p.bn_a = a; p.bn_b = b; p.bn_mean = mean; p.bn_rstd = rstd;
  p.bn_pool = pool;
  const int cfg = tile_cfg >= 0 ? tile_cfg : conv::pick_dgrad(P, C, Co);
  if (cfg != 8 && cfg != 15 && cfg != 22) return -5;
  return (int)dispatch_conv_dgrad(p, cfg, s);
}

static int pick_wgrad(int P, int C, int Co) {
  if (C <= 8) return 12;      // conv0 (K = 9 x 8): 64x64, BK 128
  // M = Co <= 64 (DeepNN's 128->64, 64->64, 64->32 layers): a 256-row tile would be 3/4 empty;
  // 64x64 / 3 stages measured 2.6x faster on 128->64@32 (profiles/r1_deepnn/conv_sweep_deepnn.json)
  if (Co <= 64) return 7;
  if (conv::picks_r4()) return C <= 64 ? 15 : 13;
  // (a different split-K summation order than round 4's picks, judged by the multi-seed tests/test_gpu_parity.py)
  // VGG conv1 (64->128 @32): 100.6 vs 133.0 us (cfg 15); conv2 (128->256 @16): 95.7 vs 99.0 us, and more splits
  // (two workgroups per CU) with a cheaper reduce (12.3 vs 16.6 us); in-step, profiles/r5_conv
  if (C <= 128) return 22;
  return 13;                  // 256x256, 8 waves (283 vs 393 us for 256x128 on 256->256@16)
}

// Workgroups of a tile config resident per CU (LDS-bound: STAGES x (BM+BN) x 64 x KSUB bf16 per
// workgroup out of 160 KiB; the 8-wave configs also hold one per CU by registers).
static int wgs_per_cu(int cfg) {
  static const int t[14] = {1, 1, 1, 2, 1, 2, 2, 3, 1, 1, 1, 1, 2, 1};
  if (cfg == 21 || cfg == 22 || cfg == 23) return 2;
  return (cfg >= 0 && cfg <= 13) ? t[cfg] : 1;
}

// Number of K splits the weight-gradient GEMM uses for a tile config (cfg < 0: default).  Chosen so the
// tiles x splits workgroups fill whole rounds of the chip's resident slots (256 CUs x workgroups/CU):
// the candidate with the best last-round fill wins (smaller S on ties: less fp32 partial traffic),
// among S giving at least 3/4 of a round and at most ~2 rounds.
DDPX_API int ddpx_conv_wgrad_splits(int P, int C, int Co, int tile_cfg) {
  const int cfg = tile_cfg >= 0 ? tile_cfg : pick_wgrad(P, C, Co);
  int bm, bn;
  tile_of(cfg, &bm, &bn);
  const int tiles = ((Co + bm - 1) / bm) * ((9 * C + bn - 1) / bn);
  const int slots = 256 * wgs_per_cu(cfg);
  const int maxS = max(1, (P + 1023) / 1024);  // >= 16 K-steps per split
  const int S0 = min(maxS, max(1, (2 * slots + tiles - 1) / tiles));
  int best = S0;
  float best_eff = -1.f;
  for (int S = 1; S <= S0; ++S) {
    const long long w = (long long)tiles * S;
    if (4 * w < 3LL * slots && S < S0) continue;
    const long long rounds = (w + slots - 1) / slots;
    const float eff = (float)w / (float)(rounds * slots);
    if (eff > best_eff + 0.02f) {
      best_eff = eff;
      best = S;
    }
  }
  // the splits that actually get a K range (64-aligned split lengths can leave the last ones empty): the caller
  // sizes the partial slabs and the reduce by this, so no slab needs zeroing inside the step
  const int klen = ((P + best - 1) / best + 63) / 64 * 64;
  return (P + klen - 1) / klen;
}

// part[S][Co][9C] (fp32) = split-K partial weight gradients.  dy [P][Co], x NHWC [N][H][W][C].
DDPX_API int ddpx_conv_wgrad(const void* dy, const void* x, float* part, int S, int N, int H, int W, int C, int Co,
                             int tile_cfg, hipStream_t s) {
  if (C % 8 || Co % 8 || S < 1) return -1;
  if (!chk16(dy) || !chk16(x) || !chk16(part)) return -3;
  const int P = N * H * W;
  Params p{};
  p.A = (const unsigned short*)dy;
  p.B = (const unsigned short*)x;
  p.C = part;
  p.M = Co; p.N = 9 * C; p.K = P;
  p.lda = Co; p.ldb = C; p.ldc = 9 * C;
  p.epi = EPI_F32;
  p.alpha = 1.f;
  const size_t ab = (size_t)P * Co * 2, bb = (size_t)P * C * 2;
  if (ab >= 0x80000000ull || bb >= 0x80000000ull) return -4;
  p.a_bytes = (unsigned)ab; p.b_bytes = (unsigned)bb;
  p.conv = make_geom(H, W, C, P);
  p.im_slow = im_slow();
  p.klen = ((P + S - 1) / S + 63) / 64 * 64;
  p.split_stride = (long long)Co * 9 * C;
  const int Sreal = (P + p.klen - 1) / p.klen;
  if (Sreal != S) {
    // zero the slabs that get no K range so the reduce can always sum S
    hipMemsetAsync(part + (size_t)Sreal * p.split_stride, 0, (size_t)(S - Sreal) * p.split_stride * 4, s);
  }
  const int cfg = tile_cfg >= 0 ? tile_cfg : pick_wgrad(P, C, Co);
  return (int)dispatch_conv_wgrad(p, cfg, Sreal, s);
}

DDPX_API int ddpx_conv_wgrad_reduce(const float* part, int S, int Co, int Cr, int Cp, void* out, int out_bf16,
                                    int accumulate, float* sgd_p, float* sgd_buf, void* sgd_shadow,
                                    const float* sgd_lr, float sgd_mom, float sgd_wd, void* wf, void* wd,
                                    hipStream_t s) {
  // wf / wd (fused SGD only): also write the updated weight as the forward [Co][9][Cp] and dgrad [9][Co][Cp] bf16
  // layouts (their padded channels keep the zeros weight_prep wrote)
  if ((wf != nullptr) != (wd != nullptr) || (wf && !sgd_p)) return -1;
  hipLaunchKernelGGL(conv::wgrad_reduce_kernel, dim3(Co, (Cr + 63) / 64), dim3(256), 0, s, part, S, Co, Cr, Cp, out,
                     out_bf16, accumulate, SgdArgs{sgd_p, sgd_buf, (unsigned short*)sgd_shadow, sgd_lr, sgd_mom, sgd_wd},
                     (unsigned short*)wf, (unsigned short*)wd);
  return (int)hipGetLastError();
}
