// ddpx — fp32 Winograd F(2x2, 3x3) convolutions for the 3x3 / stride 1 / pad 1 layers of the reference's VGG at
// its own precision (/root/reference/singlegpu.py:60-70 conv blocks, :134 fp32 model).
//
// The stock fp32 recipe's forward and data-gradient convolutions are MIOpen's Winograd F(2,3) kernels
// (profiles/r4_f32: 2.25x fewer multiplies than the direct 3x3 product); this is the same algorithm on CDNA4
// directly, with the whole transform pipeline inside one GEMM launch:
//
//   Y = A^T [ sum_ci (G g G^T)[co,ci] (.) (B^T d B)[tile,ci] ] A        (per 2x2 output tile, 4x4 input patch)
//
//   * weights: U[xi][ci][co] = (G g G^T)[xi] once per step (wino_wprep_kernel; the data gradient's U is made
//     from the flipped, transposed kernel: the transposed 3x3/s1/p1 convolution is a convolution);
//   * one workgroup = 64 output tiles (256 pixels) x 32 output channels x all 16 transform positions xi:
//     16 independent 16x16x4 f32 MFMA chains per wave (v_mfma_f32_16x16x4_f32: f32 in, f32 accumulate);
//   * input patches (4x4 pixels x 4 channels per tile per K-step) go global -> LDS by LDS-DMA with the zero
//     padding from buffer bounds (an out-of-image pixel reads as 0); each wave fetches the patches of ITS OWN
//     16 tiles, so only the shared U slab needs the per-K-step barrier;
//   * the input transform B^T d B runs on the lane that feeds the MFMA: lane l = (channel l/16, tile l%16) is
//     exactly the A-fragment slot (row l%16, k l/16) of v_mfma_f32_16x16x4_f32, so V never touches LDS;
//   * the output transform A^T M A runs in the epilogue on the accumulators (each lane holds all 16 xi of its
//     4 tiles x 2 channels), writes the 2x2 pixels, and (forward) the BatchNorm tile statistics (mean, M2 per
//     channel over the workgroup's 256 pixels; merged by the existing Chan finalize).
// Requirements: C % 4 == 0, K % 32 == 0, H and W even (every VGG layer on CIFAR-10).
#include <cstdlib>

#include "ddpx_common.h"

namespace ddpx {
namespace wino {

constexpr int NT = 256;                  // 4 waves
constexpr int TP = 64;                   // output tiles per workgroup (16 per wave)
constexpr int TK = 32;                   // output channels per workgroup
constexpr int RAW_BYTES = TP * 16 * 16;  // 64 tiles x 16 pixels x 4 channels x 4 B = 16 KiB
constexpr int U_BYTES = 16 * 4 * TK * 4; // 16 xi x 4 channels x 32 out channels x 4 B = 8 KiB
constexpr int SLOT = RAW_BYTES + U_BYTES;
constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds_wave_base, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)lds_wave_base, 16, voff, 0, 0, 0);
}

// n / d for 0 <= n < 2^31 by multiply-high: s = ceil(log2 d), magic = ceil(2^(31+s) / d), n / d = umulhi(n, magic)
// >> (s - 1); d == 1: magic 0 (identity)
struct WDiv {
  unsigned magic;
  int shift;
};
static inline WDiv make_wdiv(int d) {
  WDiv f{0u, 0};
  if (d <= 1) return f;
  int s = 0;
  while ((1ll << s) < d) ++s;
  f.shift = s - 1;
  f.magic = (unsigned)(((1ull << (31 + s)) + (unsigned long long)d - 1) / (unsigned long long)d);
  return f;
}
__device__ __forceinline__ int wdiv(int n, WDiv f) {
  return f.magic ? (int)(__umulhi((unsigned)n, f.magic) >> f.shift) : n;
}

// One K-step of the forward's product with LDS reads the compiler does not see (inline asm, settled by explicit
// lgkmcnt waits that redefine their outputs, as frag_tr/frag_settle in ddpx_pipe.h).  With ordinary C++ loads
// hipcc (ROCm 7.2) takes the U-slab reads for possible readers of the LDS-DMA just issued for step t + 1 and puts
// an `s_waitcnt vmcnt(0)` in front of them: every K-step then waited out the whole global->LDS latency of the
// NEXT stage and the 2-stage ring (the one that fits 3 workgroups per CU) ran as a 1-stage one.  Here the ring's
// own vmcnt + barrier order reads against DMA; the U pairs are double-buffered (read of pair i + 1 in flight
// during pair i's four MFMAs) and the patch transform runs while the first U pair is in flight.
typedef float f32x2 __attribute__((ext_vector_type(2)));
#define WINO_RD_D(out, a, o0, o1) \
  asm volatile("ds_read2st64_b32 %0, %1 offset0:" #o0 " offset1:" #o1 : "=v"(out) : "v"(a) : "memory")
#define WINO_RD_B(out, a, o0, o1) \
  asm volatile("ds_read2st64_b64 %0, %1 offset0:" #o0 " offset1:" #o1 : "=v"(out) : "v"(a) : "memory")

// U rows q = 2i, 2i + 1 of this lane's channel: (b[2i].x, b[2i].y, b[2i+1].x, b[2i+1].y); row stride 512 B
__device__ __forceinline__ void rd_upair(f32x4& o, const LDS_AS char* a, int i) {
  switch (i) {
    case 0: WINO_RD_B(o, a, 0, 1); break;
    case 1: WINO_RD_B(o, a, 2, 3); break;
    case 2: WINO_RD_B(o, a, 4, 5); break;
    case 3: WINO_RD_B(o, a, 6, 7); break;
    case 4: WINO_RD_B(o, a, 8, 9); break;
    case 5: WINO_RD_B(o, a, 10, 11); break;
    case 6: WINO_RD_B(o, a, 12, 13); break;
    default: WINO_RD_B(o, a, 14, 15); break;
  }
}

__device__ __forceinline__ void step_asm(const float* dp, const float* bp, f32x4 (&acc)[16][2]) {
  const LDS_AS char* da = (const LDS_AS char*)(const char*)dp;  // patch pixel q at +256 q B
  const LDS_AS char* ba = (const LDS_AS char*)(const char*)bp;  // U row q at +512 q B
  f32x2 dd[8];
  WINO_RD_D(dd[0], da, 0, 1);
  WINO_RD_D(dd[1], da, 2, 3);
  WINO_RD_D(dd[2], da, 4, 5);
  WINO_RD_D(dd[3], da, 6, 7);
  WINO_RD_D(dd[4], da, 8, 9);
  WINO_RD_D(dd[5], da, 10, 11);
  WINO_RD_D(dd[6], da, 12, 13);
  WINO_RD_D(dd[7], da, 14, 15);
  f32x4 bb[2];
  rd_upair(bb[0], ba, 0);
  asm volatile("s_waitcnt lgkmcnt(1)"
               : "+v"(dd[0]), "+v"(dd[1]), "+v"(dd[2]), "+v"(dd[3]), "+v"(dd[4]), "+v"(dd[5]), "+v"(dd[6]),
                 "+v"(dd[7])::"memory");
  float tmp[16], v[16];
#pragma unroll
  for (int c = 0; c < 4; ++c) {  // the same B^T d B as the compiler-read path below
    const float d0 = dd[c >> 1][c & 1], d1 = dd[(4 + c) >> 1][c & 1];
    const float d2 = dd[(8 + c) >> 1][c & 1], d3 = dd[(12 + c) >> 1][c & 1];
    tmp[0 * 4 + c] = d0 - d2;
    tmp[1 * 4 + c] = d1 + d2;
    tmp[2 * 4 + c] = d2 - d1;
    tmp[3 * 4 + c] = d1 - d3;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    v[r * 4 + 0] = tmp[r * 4 + 0] - tmp[r * 4 + 2];
    v[r * 4 + 1] = tmp[r * 4 + 1] + tmp[r * 4 + 2];
    v[r * 4 + 2] = tmp[r * 4 + 2] - tmp[r * 4 + 1];
    v[r * 4 + 3] = tmp[r * 4 + 1] - tmp[r * 4 + 3];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    f32x4& b = bb[i & 1];
    if (i < 7) {
      rd_upair(bb[(i + 1) & 1], ba, i + 1);
      asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(b)::"memory");
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b)::"memory");
    }
    acc[2 * i][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[2 * i], b.x, acc[2 * i][0], 0, 0, 0);
    acc[2 * i][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[2 * i], b.y, acc[2 * i][1], 0, 0, 0);
    acc[2 * i + 1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[2 * i + 1], b.z, acc[2 * i + 1][0], 0, 0, 0);
    acc[2 * i + 1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[2 * i + 1], b.w, acc[2 * i + 1][1], 0, 0, 0);
  }
}

// y (+ stats) = conv3x3(x) through F(2,3).  x: NHWC [N][H][W][C]; U: [16][C][K]; y: [N*H*W][K].
// ASMRD: K-step reads through step_asm (default); false = compiler-visible LDS loads (DDPX_WINO_STAGES=2c).
template <int STAGES, int WAVES_PER_SIMD, bool ASMRD = true>
__global__ void __launch_bounds__(NT, WAVES_PER_SIMD)  // 2: <= 256 VGPR + AGPR (128 are accumulators); 3: <= 168
wino_f32_kernel(const float* __restrict__ x, const float* __restrict__ U, float* __restrict__ y,
                float* __restrict__ stats, const float* __restrict__ bias, int relu, int N, int H, int W, int C, int K,
                int tiles_p, unsigned x_bytes, unsigned u_bytes, const float* __restrict__ mask) {
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  // consecutive ids (one XCD's share) walk the tiles inside one output-channel block: its U slab stays in L2
  const int pb = bid % tiles_p, kb = bid / tiles_p;
  const int TH = H >> 1, TW = W >> 1, P = N * TH * TW;
  const int k0 = kb * TK;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc((void*)U, 0, u_bytes, 0x00020000);

  // patch DMA: instruction j = patch row dy, lane l = (patch column dx = l >> 4, tile l & 15 of this wave);
  // LDS image per wave [dy*4+dx][tile][4 ch] (16 B chunks): the transform's reads are conflict-free
  unsigned poff[4];
  {
    const int t = lane & 15, dx = lane >> 4;
    const int p = pb * TP + wave * 16 + t;
    const int pp = p < P ? p : 0;
    const int n = pp / (TH * TW), r = pp - n * (TH * TW);
    const int th = r / TW, tw = r - th * TW;
    const int w = 2 * tw + dx - 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int h = 2 * th + j - 1;
      const bool ok = p < P && h >= 0 && h < H && w >= 0 && w < W;
      poff[j] = ok ? (unsigned)((((size_t)n * H + h) * W + w) * C * 4) : kOOB;
    }
  }
  // U slab DMA: 8 wave-instructions per K-step, 2 per wave; chunk q = row (xi*4 + ci) * 8 + 16-B column
  // (instruction j = 1 is 32 rows = 8 xi further: a uniform 8 C K floats past instruction 0's lane offset)
  unsigned uoff;
  {
    const int q = wave * 64 + lane;
    const int row = q >> 3, ch = q & 7;
    const int xi = row >> 2, ci = row & 3;
    uoff = (unsigned)((((size_t)xi * C + ci) * K + k0 + ch * 4) * 4);
  }
  const unsigned u_j1 = (unsigned)((size_t)8 * C * K * 4);
  const int nk = C >> 2;
  auto issue = [&](int t) {
    char* slot = smem + (t % STAGES) * SLOT;
    const unsigned cx = (unsigned)(t * 16);  // 4 channels = 16 B further along every pixel
    char* raw = slot + wave * (RAW_BYTES / 4);
    // an out-of-image pixel's kOOB + cx (< 2^31 + 4C) stays past the buffer (x_bytes < 2^31): still reads 0
#pragma unroll
    for (int j = 0; j < 4; ++j) dma16(rx, raw + j * 1024, poff[j] + cx);
    const unsigned cu = (unsigned)((size_t)t * 4 * K * 4);  // 4 channels = 4 rows of K further
#pragma unroll
    for (int j = 0; j < 2; ++j) dma16(ru, slot + RAW_BYTES + (j * 4 + wave) * 1024, uoff + cu + j * u_j1);
  };

  f32x4 acc[16][2];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q][0] = acc[q][1] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s);
  constexpr int PER_STEP = 6;  // DMA instructions per wave per K-step
  const int ci = lane >> 4, tl = lane & 15;
  for (int t = 0; t < nk; ++t) {
    const int ahead = min(STAGES - 2, nk - 1 - t);
    if (STAGES >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_STEP) : "memory");
    else if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_STEP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1);
    const char* slot = smem + (t % STAGES) * SLOT;
    const float* raw = reinterpret_cast<const float*>(slot + wave * (RAW_BYTES / 4));
    const float* us = reinterpret_cast<const float*>(slot + RAW_BYTES);
    if constexpr (ASMRD) {
      step_asm(raw + tl * 4 + ci, us + ci * TK + 2 * tl, acc);
      continue;
    }
    float d[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) d[q] = raw[(q * 16 + tl) * 4 + ci];
    // B fragments: MFMA column tl of fragment j is output channel k0 + 2 tl + j, so a lane's two channels are
    // adjacent (one ds_read_b64, conflict-free; the epilogue stores them as one 8-B pair)
    float2 b[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) b[q] = *reinterpret_cast<const float2*>(us + (q * 4 + ci) * TK + 2 * tl);
    // V = B^T d B, B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]]
    float tmp[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      tmp[0 * 4 + c] = d[0 * 4 + c] - d[2 * 4 + c];
      tmp[1 * 4 + c] = d[1 * 4 + c] + d[2 * 4 + c];
      tmp[2 * 4 + c] = d[2 * 4 + c] - d[1 * 4 + c];
      tmp[3 * 4 + c] = d[1 * 4 + c] - d[3 * 4 + c];
    }
    float v[16];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r * 4 + 0] = tmp[r * 4 + 0] - tmp[r * 4 + 2];
      v[r * 4 + 1] = tmp[r * 4 + 1] + tmp[r * 4 + 2];
      v[r * 4 + 2] = tmp[r * 4 + 2] - tmp[r * 4 + 1];
      v[r * 4 + 3] = tmp[r * 4 + 1] - tmp[r * 4 + 3];
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      acc[q][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[q], b[q].x, acc[q][0], 0, 0, 0);
      acc[q][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[q], b[q].y, acc[q][1], 0, 0, 0);
    }
  }

  // epilogue: Y = A^T M A per (tile, channel), A^T = [[1,1,1,0],[0,1,-1,-1]]
  const int lr = lane >> 4;
  float out[4][2][4];  // [e (tile row of the fragment)][j (channel fragment)][pixel 2x2]
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float m[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) m[q] = acc[q][j][e];
      float t0[4], t1[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        t0[c] = m[0 * 4 + c] + m[1 * 4 + c] + m[2 * 4 + c];
        t1[c] = m[1 * 4 + c] - m[2 * 4 + c] - m[3 * 4 + c];
      }
      out[e][j][0] = t0[0] + t0[1] + t0[2];
      out[e][j][1] = t0[1] - t0[2] - t0[3];
      out[e][j][2] = t1[0] + t1[1] + t1[2];
      out[e][j][3] = t1[1] - t1[2] - t1[3];
    }
  if (bias || relu) {  // DeepNN's conv + bias + ReLU (y = relu(conv + b)); VGG's convolutions have neither
    const float b0 = bias ? bias[k0 + 2 * tl] : 0.f, b1 = bias ? bias[k0 + 2 * tl + 1] : 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        out[e][0][u] += b0;
        out[e][1][u] += b1;
        if (relu) {
          out[e][0][u] = fmaxf(out[e][0][u], 0.f);
          out[e][1][u] = fmaxf(out[e][1][u], 0.f);
        }
      }
  }
  bool valid[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int p = pb * TP + wave * 16 + lr * 4 + e;
    valid[e] = p < P;
    if (!valid[e]) continue;
    const int n = p / (TH * TW), r = p - n * (TH * TW);
    const int th = r / TW, tw = r - th * TW;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const size_t pix = ((size_t)n * H + 2 * th + i) * W + 2 * tw + jj;
        float2 v = make_float2(out[e][0][i * 2 + jj], out[e][1][i * 2 + jj]);
        if (mask) {  // data gradient through the ReLU below: zero where that layer's output mask[pix] <= 0
          const float2 mk = *reinterpret_cast<const float2*>(mask + pix * K + k0 + 2 * tl);
          if (!(mk.x > 0.f)) v.x = 0.f;
          if (!(mk.y > 0.f)) v.y = 0.f;
        }
        *reinterpret_cast<float2*>(y + pix * K + k0 + 2 * tl) = v;
      }
  }
  if (!stats) return;
  // BatchNorm chunk statistics over this workgroup's pixels (chunk = 256 rows; the last chunk may be short):
  // per channel, lanes sharing it (xor 16, 32), then the 4 waves in order through LDS; two passes (mean, M2)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave is done with the ring: reuse it
  float* red = reinterpret_cast<float*>(smem);  // [4 waves][32 channels] sums, then [4][32] M2
  const int rows = min(TP, P - pb * TP) * 4;
  float mean[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (valid[e]) s += (out[e][j][0] + out[e][j][1]) + (out[e][j][2] + out[e][j][3]);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (lr == 0) red[wave * TK + 2 * tl + j] = s;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = 2 * tl + j;
    mean[j] = (((red[col] + red[TK + col]) + red[2 * TK + col]) + red[3 * TK + col]) / (float)rows;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (valid[e])
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float dv = out[e][j][u] - mean[j];
          q = fmaf(dv, dv, q);
        }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    if (lr == 0) red[wave * TK + 2 * tl + j] = q;
  }
  __syncthreads();
  if (wave == 0 && lr == 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = 2 * tl + j;
      stats[(size_t)pb * 2 * K + k0 + col] = mean[j];
      stats[(size_t)pb * 2 * K + K + k0 + col] = ((red[col] + red[TK + col]) + red[2 * TK + col]) + red[3 * TK + col];
    }
  }
}

// U = G g G^T per (co, ci), G = [[1,0,0],[1/2,1/2,1/2],[1/2,-1/2,1/2],[0,0,1]].  w: torch [Co][Ci][3][3].
//   uf: [16][Cp][Co] (forward, channels Ci padded to Cp with zero kernels), ud: [16][Co][Ci] (data gradient:
//   the kernel flipped in both taps, input and output channels swapped), either may be null.
__device__ __forceinline__ void g_transform(const float (&g)[9], float (&u)[16]) {
  float t[4][3];  // G g
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    t[0][s] = g[0 * 3 + s];
    t[1][s] = 0.5f * ((g[0 * 3 + s] + g[1 * 3 + s]) + g[2 * 3 + s]);
    t[2][s] = 0.5f * ((g[0 * 3 + s] - g[1 * 3 + s]) + g[2 * 3 + s]);
    t[3][s] = g[2 * 3 + s];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    u[r * 4 + 0] = t[r][0];
    u[r * 4 + 1] = 0.5f * ((t[r][0] + t[r][1]) + t[r][2]);
    u[r * 4 + 2] = 0.5f * ((t[r][0] - t[r][1]) + t[r][2]);
    u[r * 4 + 3] = t[r][2];
  }
}

// One 256-thread block per 16 x 16 (co, ci) tile: w is read ci-fastest (9 contiguous floats per thread), ud is
// written ci-fastest, uf co-fastest through an LDS transpose — every store stream coalesced.
__global__ void __launch_bounds__(256)
wino_wprep_kernel(const float* __restrict__ w, int Co, int Ci, int Cp, float* __restrict__ uf, float* __restrict__ ud) {
  __shared__ float tr[16][16][17];
  const int t = threadIdx.x;
  const int ci = blockIdx.y * 16 + (t & 15), co = blockIdx.x * 16 + (t >> 4);
  const bool in = ci < Cp && co < Co, real = in && ci < Ci;
  float g[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) g[q] = real ? w[((size_t)co * Ci + ci) * 9 + q] : 0.f;
  float u[16];
  if (ud && real) {
    float gf[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) gf[q] = g[8 - q];
    g_transform(gf, u);
#pragma unroll
    for (int q = 0; q < 16; ++q) ud[((size_t)q * Co + co) * Ci + ci] = u[q];
  }
  if (!uf) return;
  g_transform(g, u);
#pragma unroll
  for (int q = 0; q < 16; ++q) tr[q][t & 15][t >> 4] = u[q];
  __syncthreads();
  const int co2 = blockIdx.x * 16 + (t & 15), ci2 = blockIdx.y * 16 + (t >> 4);
  if (co2 >= Co || ci2 >= Cp) return;
#pragma unroll
  for (int q = 0; q < 16; ++q) uf[((size_t)q * Cp + ci2) * Co + co2] = tr[q][t >> 4][t & 15];
}

// ---------------------------------------------------------------------------------------- weight gradient
// dW = G^T dU G,  dU[xi][co][ci] = sum over output tiles of (A dY A^T)[xi][tile][co] * (B^T d B)[xi][tile][ci]
// (A = (A^T)^T, 4x2): the forward's U = G g G^T enters Y = A^T (U (.) V) A linearly, so its gradient is the
// tile sum of the transformed output gradient times the transformed input patch, and g's is G^T dU G.  16
// GEMMs of [Co x tiles] x [tiles x Ci]: 4/9 of the direct weight gradient's multiplies.
//   * one workgroup = 64 output channels x 32 input channels x all 16 xi, over one split's range of tiles;
//     wave w owns output channels 16w..16w+15 and both 16-channel input halves: 32 f32 16x16x4 MFMA chains;
//   * K-step = 8 tiles (two MFMA k-steps of 4): the tiles' 4x4 input patches (32 channels) and 2x2 output
//     gradients (64 channels) go global -> LDS by LDS-DMA (zero padding from buffer bounds);
//   * lane l = (tile l/16, channel l%16) is the MFMA A slot (row = output channel) and B slot (column = input
//     channel) at once: each lane transforms its own dy 2x2 / patch 4x4 in registers, nothing else touches LDS;
//   * partial dU per split [S][16][Co][Cp]; ddpx_f32_wino_wgrad_reduce sums the splits in order and applies
//     G^T . G (fixed order: deterministic).
constexpr int WG_CO = 64, WG_CI = 32, WKT = 8;   // output channels, input channels, tiles per K-step
constexpr int XS_T = 16 * WG_CI + 16;             // floats per tile of the patch image (padded: bank shift 16)
constexpr int DS_T = 4 * WG_CO + 16;              // floats per tile of the dy image
constexpr int WX_BYTES = WKT * XS_T * 4, WD_BYTES = WKT * DS_T * 4;
constexpr int WSLOT = WX_BYTES + WD_BYTES;        // 25 KiB

// WS (wave split): 0 = wave w owns output channels 16w.. and both input-channel halves (each wave transforms
// all 32 channels' patches); 1 = wave w owns output channels 32(w/2).. and input channels 16(w%2).. (two dy
// transforms, one patch transform per MFMA k-step: a third fewer LDS reads)
template <int STAGES, int WS, int OCC = 2>
__global__ void __launch_bounds__(NT, OCC)  // OCC workgroups (waves per SIMD) per CU
wino_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ part, int H,
                  int W, int Cp, int Co, int Pt, int L, int nb_ci, unsigned x_bytes, unsigned dy_bytes, WDiv d_thw,
                  WDiv d_tw) {
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * WSLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nblk = nb_ci * (Co / WG_CO);
  const int blk = blockIdx.x % nblk, sp = blockIdx.x / nblk;
  const int ci0 = (blk % nb_ci) * WG_CI, co0 = (blk / nb_ci) * WG_CO;
  const int TH = H >> 1, TW = W >> 1;
  const int t_beg = sp * L, t_end = min(Pt, t_beg + L);
  const int nk = (t_end - t_beg + WKT - 1) / WKT;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)dy, 0, dy_bytes, 0x00020000);

  // DMA roles (per K-step): wave w fetches tiles 2w and 2w + 1: each tile's patch in two instructions of 8
  // pixels (lane = (pixel q%8 of the half, 16-B chunk c of the 32 channels)) and its dy in one (lane = (pixel q =
  // lane/16, 16-B chunk lane%16 of the 64 channels)).  A tile's (n, th, tw) by multiply-high division, once per
  // K-step (the v_rcp-based divisions per instruction were 4.6 VALU per MFMA, PMC in profiles/r5_wino)
  auto issue = [&](int k) {
    char* slot = smem + (k % STAGES) * WSLOT;
    const int tb = t_beg + k * WKT;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = 2 * wave + u, p = tb + t;
      const bool pv = p < t_end;
      int n = 0, th = 0, tw = 0;
      if (pv) {
        n = wdiv(p, d_thw);
        const int r = p - n * (TH * TW);
        th = wdiv(r, d_tw);
        tw = r - th * TW;
      }
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int q = half * 8 + (lane >> 3), c = lane & 7;
        const int h = 2 * th - 1 + (q >> 2), w = 2 * tw - 1 + (q & 3);
        const bool ok = pv && h >= 0 && h < H && w >= 0 && w < W;
        dma16(rx, slot + (t * XS_T + half * 8 * WG_CI) * 4,
              ok ? (unsigned)(((((size_t)n * H + h) * W + w) * Cp + ci0 + 4 * c) * 4) : kOOB);
      }
      const int q = lane >> 4, c = lane & 15;
      const size_t pix = ((size_t)n * H + 2 * th + (q >> 1)) * W + 2 * tw + (q & 1);
      dma16(rd, slot + WX_BYTES + t * DS_T * 4, pv ? (unsigned)((pix * Co + co0 + 4 * c) * 4) : kOOB);
    }
  };

  f32x4 acc[16][2];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q][0] = acc[q][1] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s);
  constexpr int PER_STEP = 6;  // DMA instructions per wave per K-step
  const int tl = lane >> 4, ch = lane & 15;
  for (int k = 0; k < nk; ++k) {
    const int ahead = min(STAGES - 2, nk - 1 - k);
    if (STAGES >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_STEP) : "memory");
    else if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_STEP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (k + STAGES - 1 < nk) issue(k + STAGES - 1);
    const char* slot = smem + (k % STAGES) * WSLOT;
    const float* xs = reinterpret_cast<const float*>(slot);
    const float* ds = reinterpret_cast<const float*>(slot + WX_BYTES);
    // A = [[1,0],[1,1],[1,-1],[0,-1]]: M = A dY A^T of (tile t, output channel col) from the 2x2 dy
    auto dy_transform = [&](int t, int col, float (&m)[16]) {
      float d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = ds[t * DS_T + q * WG_CO + col];
      float rr[4][2];  // A dY
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        rr[0][j] = d[0 * 2 + j];
        rr[1][j] = d[0 * 2 + j] + d[1 * 2 + j];
        rr[2][j] = d[0 * 2 + j] - d[1 * 2 + j];
        rr[3][j] = -d[1 * 2 + j];
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        m[a * 4 + 0] = rr[a][0];
        m[a * 4 + 1] = rr[a][0] + rr[a][1];
        m[a * 4 + 2] = rr[a][0] - rr[a][1];
        m[a * 4 + 3] = -rr[a][1];
      }
    };
    // V = B^T x B of (tile t, input channel col) from the 4x4 patch
    auto x_transform = [&](int t, int col, float (&v)[16]) {
      float xv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) xv[q] = xs[t * XS_T + q * WG_CI + col];
      float tmp[16];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        tmp[0 * 4 + c] = xv[0 * 4 + c] - xv[2 * 4 + c];
        tmp[1 * 4 + c] = xv[1 * 4 + c] + xv[2 * 4 + c];
        tmp[2 * 4 + c] = xv[2 * 4 + c] - xv[1 * 4 + c];
        tmp[3 * 4 + c] = xv[1 * 4 + c] - xv[3 * 4 + c];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r * 4 + 0] = tmp[r * 4 + 0] - tmp[r * 4 + 2];
        v[r * 4 + 1] = tmp[r * 4 + 1] + tmp[r * 4 + 2];
        v[r * 4 + 2] = tmp[r * 4 + 2] - tmp[r * 4 + 1];
        v[r * 4 + 3] = tmp[r * 4 + 1] - tmp[r * 4 + 3];
      }
    };
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int t = sub * 4 + tl;
      if constexpr (WS == 0) {
        float m[16];
        dy_transform(t, wave * 16 + ch, m);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          float v[16];
          x_transform(t, cb * 16 + ch, v);
#pragma unroll
          for (int q = 0; q < 16; ++q) acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(m[q], v[q], acc[q][cb], 0, 0, 0);
        }
      } else {
        float v[16];
        x_transform(t, (wave & 1) * 16 + ch, v);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {  // here cb = the output-channel half of the wave's 32
          float m[16];
          dy_transform(t, (wave >> 1) * 32 + cb * 16 + ch, m);
#pragma unroll
          for (int q = 0; q < 16; ++q) acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(m[q], v[q], acc[q][cb], 0, 0, 0);
        }
      }
    }
  }
  // partial dU[sp][xi][co][ci]: lane holds rows (output channels) 4 (lane/16) + r, column (input channel) lane%16
  const size_t plane = (size_t)Co * Cp;
  float* dst = part + (size_t)sp * 16 * plane;
#pragma unroll
  for (int q = 0; q < 16; ++q)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = WS == 0 ? co0 + wave * 16 + 4 * tl + r : co0 + (wave >> 1) * 32 + cb * 16 + 4 * tl + r;
        const int ci = WS == 0 ? ci0 + cb * 16 + ch : ci0 + (wave & 1) * 16 + ch;
        dst[(size_t)q * plane + (size_t)co * Cp + ci] = acc[q][cb][r];
      }
}

// dU[xi][co][ci] = sum over splits (in split order), 4 input channels per thread
__global__ void __launch_bounds__(256)
wino_wgrad_sum_kernel(const float* __restrict__ part, int S, size_t n4, float* __restrict__ du) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const f32x4* src = reinterpret_cast<const f32x4*>(part);
  f32x4 acc = src[i];
  int s = 1;
  // 16 splits' loads in flight while they last (small layers: 64 workgroups over ~100 splits were latency-bound at
  // 8, 24 us in the DeepNN fp32 step), then 8; added in split order either way
  for (; s + 15 < S; s += 16) {
    f32x4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = src[(size_t)(s + u) * n4 + i];
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += v[u];
  }
  for (; s + 7 < S; s += 8) {  // 8 splits' loads in flight, added in split order
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[(size_t)(s + u) * n4 + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; s < S; ++s) acc += src[(size_t)s * n4 + i];
  reinterpret_cast<f32x4*>(du)[i] = acc;
}

// grad[co][ci][3][3] (+)= G^T dU[.][co][ci] G, G = [[1,0,0],[1/2,1/2,1/2],[1/2,-1/2,1/2],[0,0,1]]; ci < Ci only
__global__ void __launch_bounds__(256)
wino_wgrad_out_kernel(const float* __restrict__ du, int Co, int Ci, int Cp, float* __restrict__ grad, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Co * Ci) return;
  const int co = i / Ci, ci = i - co * Ci;
  const size_t plane = (size_t)Co * Cp;
  float u[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) u[q] = du[(size_t)q * plane + (size_t)co * Cp + ci];
  float t[3][4];  // G^T dU
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    t[0][b] = u[0 * 4 + b] + 0.5f * (u[1 * 4 + b] + u[2 * 4 + b]);
    t[1][b] = 0.5f * (u[1 * 4 + b] - u[2 * 4 + b]);
    t[2][b] = 0.5f * (u[1 * 4 + b] + u[2 * 4 + b]) + u[3 * 4 + b];
  }
  float* g = grad + (size_t)i * 9;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const float g0 = t[r][0] + 0.5f * (t[r][1] + t[r][2]);
    const float g1 = 0.5f * (t[r][1] - t[r][2]);
    const float g2 = 0.5f * (t[r][1] + t[r][2]) + t[r][3];
    g[r * 3 + 0] = accumulate ? g[r * 3 + 0] + g0 : g0;
    g[r * 3 + 1] = accumulate ? g[r * 3 + 1] + g1 : g1;
    g[r * 3 + 2] = accumulate ? g[r * 3 + 2] + g2 : g2;
  }
}

}  // namespace wino
}  // namespace ddpx

using namespace ddpx;

// Winograd applies: 3x3 / s1 / p1, C % 4 == 0, K % 32 == 0, H and W even.
DDPX_API int ddpx_f32_wino_ok(int H, int W, int C, int K) {
  return (C >= 4 && C % 4 == 0 && K % 32 == 0 && H >= 2 && W >= 2 && H % 2 == 0 && W % 2 == 0) ? 1 : 0;
}

DDPX_API int ddpx_f32_wino_wprep(const float* w, int Co, int Ci, int Cp, float* uf, float* ud, hipStream_t s) {
  if (Cp < Ci) return -2;
  hipLaunchKernelGGL(wino::wino_wprep_kernel, dim3((Co + 15) / 16, (Cp + 15) / 16), dim3(256), 0, s, w, Co, Ci, Cp,
                     uf, ud);
  return -(int)hipGetLastError();
}

// y [N*H*W][K] = conv3x3(x [N][H][W][C]) with U [16][C][K] [+ bias[K]] [relu]; stats (nullable): [tiles_p][2][K]
// chunk statistics of 256-pixel chunks.  Returns the statistics chunk rows (256) or a negative error.
// mask (nullable, [N*H*W][K]): y is zeroed where mask <= 0 (the data gradient of a conv + ReLU block below)
DDPX_API int ddpx_f32_wino_conv_mask(const float* x, const float* U, float* y, float* stats, const float* bias,
                                     int relu, const float* mask, int N, int H, int W, int C, int K, hipStream_t s) {
  if (!ddpx_f32_wino_ok(H, W, C, K)) return -2;
  const size_t xb = (size_t)N * H * W * C * 4, ub = (size_t)16 * C * K * 4;
  if (xb >= 0x80000000ull || ub >= 0x80000000ull) return -3;  // 32-bit buffer offsets, top bit = out of bounds
  const int P = N * (H / 2) * (W / 2);
  const int tiles_p = (P + wino::TP - 1) / wino::TP;
  const int nwg = tiles_p * (K / wino::TK);
  // ring depth (DDPX_WINO_STAGES, default 2): 2 stages = 48 KiB, 3 workgroups per CU (8-10 % faster on every VGG
  // layer, profiles/r5_wino); 3 stages = 72 KiB, 2 per CU
  // (2c: the 2-stage ring with compiler-visible LDS reads, the round-5 kernel; see step_asm)
  static const int stages = [] {
    const char* e = getenv("DDPX_WINO_STAGES");
    return e && e[0] == '3' ? 3 : (e && e[0] == '2' && e[1] == 'c') ? 1 : 2;
  }();
  if (stages == 2)
    hipLaunchKernelGGL((wino::wino_f32_kernel<2, 3>), dim3(nwg), dim3(wino::NT), 0, s, x, U, y, stats, bias, relu, N,
                       H, W, C, K, tiles_p, (unsigned)xb, (unsigned)ub, mask);
  else if (stages == 1)
    hipLaunchKernelGGL((wino::wino_f32_kernel<2, 3, false>), dim3(nwg), dim3(wino::NT), 0, s, x, U, y, stats, bias,
                       relu, N, H, W, C, K, tiles_p, (unsigned)xb, (unsigned)ub, mask);
  else
    hipLaunchKernelGGL((wino::wino_f32_kernel<3, 2>), dim3(nwg), dim3(wino::NT), 0, s, x, U, y, stats, bias, relu, N,
                       H, W, C, K, tiles_p, (unsigned)xb, (unsigned)ub, mask);
  const int e = (int)hipGetLastError();
  return e ? -e : 4 * wino::TP;
}

DDPX_API int ddpx_f32_wino_conv(const float* x, const float* U, float* y, float* stats, const float* bias, int relu,
                                int N, int H, int W, int C, int K, hipStream_t s) {
  return ddpx_f32_wino_conv_mask(x, U, y, stats, bias, relu, nullptr, N, H, W, C, K, s);
}

// Winograd weight gradient applies: 3x3 / s1 / p1, H and W even, Cp % 32 == 0, Co % 64 == 0.
DDPX_API int ddpx_f32_wino_wgrad_ok(int H, int W, int Cp, int Co) {
  return (Cp >= 32 && Cp % wino::WG_CI == 0 && Co % wino::WG_CO == 0 && H >= 2 && W >= 2 && H % 2 == 0 &&
          W % 2 == 0) ? 1 : 0;
}

// Splits of the tile range: enough workgroups for one round of the chip (3 per CU), >= 16 K-steps each.
DDPX_API int ddpx_f32_wino_wgrad_splits(int N, int H, int W, int Cp, int Co) {
  const int Pt = N * (H / 2) * (W / 2);
  const int nblk = (Cp / wino::WG_CI) * (Co / wino::WG_CO);
  const int maxS = Pt / (16 * wino::WKT) > 1 ? Pt / (16 * wino::WKT) : 1;
  // DDPX_WINO_WGRAD_SLOTS: workgroups aimed for; default 768 = one round at three per CU (VGG layers 3.25 ms,
  // 1024: 3.40, 1536: 3.38; profiles/r5_wino)
  static const int slots = [] {
    const char* e = getenv("DDPX_WINO_WGRAD_SLOTS");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 768;
  }();
  int S = (slots + nblk - 1) / nblk;
  if (S > maxS) S = maxS;
  if (S < 1) S = 1;
  const int L = ((Pt + S - 1) / S + wino::WKT - 1) / wino::WKT * wino::WKT;
  return (Pt + L - 1) / L;  // the splits that get a tile range
}

// part [S][16][Co][Cp] = per-split dU; du [16][Co][Cp] (scratch) = their sum; grad [Co][Ci][3][3] (+)= G^T dU G.
// x NHWC [N][H][W][Cp], dy [N*H*W][Co].  S = ddpx_f32_wino_wgrad_splits(...).
DDPX_API int ddpx_f32_wino_wgrad(const float* x, const float* dy, float* part, float* du, int N, int H, int W, int Cp,
                                 int Co, int Ci, int S, float* grad, int accumulate, hipStream_t s) {
  if (!ddpx_f32_wino_wgrad_ok(H, W, Cp, Co) || Ci > Cp || S < 1) return -2;
  const size_t xb = (size_t)N * H * W * Cp * 4, db = (size_t)N * H * W * Co * 4;
  if (xb >= 0x80000000ull || db >= 0x80000000ull) return -3;
  if (S != ddpx_f32_wino_wgrad_splits(N, H, W, Cp, Co)) return -4;
  const int Pt = N * (H / 2) * (W / 2);
  const int L = ((Pt + S - 1) / S + wino::WKT - 1) / wino::WKT * wino::WKT;
  const int nb_ci = Cp / wino::WG_CI;
  const int nwg = nb_ci * (Co / wino::WG_CO) * S;
  const wino::WDiv dthw = wino::make_wdiv((H / 2) * (W / 2)), dtw = wino::make_wdiv(W / 2);
  // DDPX_WINO_WGRAD_VARIANT: ring depth 2|3, wave split 0|1 (see wino_wgrad_kernel), "o3" = held to 168 VGPRs for
  // three workgroups per CU, e.g. "s3w1"; default s2w1o3 (VGG layers 3.42 ms; s2w1 3.55-3.60, s2w0 3.72; the ring
  // depth changed nothing; profiles/r5_wino)
  static const int variant = [] {
    const char* e = getenv("DDPX_WINO_WGRAD_VARIANT");
    if (!e || e[0] != 's' || !e[1] || e[2] != 'w' || !e[3]) return 121;
    if (e[4] == 'o' && e[5] == '3') return 121 + (e[3] == '1' ? 0 : -1);  // "s2w1o3": 3 workgroups per CU
    return (e[1] == '3' ? 30 : 20) + (e[3] == '1' ? 1 : 0);
  }();
  switch (variant) {
    case 21:
      hipLaunchKernelGGL((wino::wino_wgrad_kernel<2, 1>), dim3(nwg), dim3(wino::NT), 0, s, x, dy, part, H, W, Cp, Co,
                         Pt, L, nb_ci, (unsigned)xb, (unsigned)db, dthw, dtw);
      break;
    case 30:
      hipLaunchKernelGGL((wino::wino_wgrad_kernel<3, 0>), dim3(nwg), dim3(wino::NT), 0, s, x, dy, part, H, W, Cp, Co,
                         Pt, L, nb_ci, (unsigned)xb, (unsigned)db, dthw, dtw);
      break;
    case 31:
      hipLaunchKernelGGL((wino::wino_wgrad_kernel<3, 1>), dim3(nwg), dim3(wino::NT), 0, s, x, dy, part, H, W, Cp, Co,
                         Pt, L, nb_ci, (unsigned)xb, (unsigned)db, dthw, dtw);
      break;
    case 120:
      hipLaunchKernelGGL((wino::wino_wgrad_kernel<2, 0, 3>), dim3(nwg), dim3(wino::NT), 0, s, x, dy, part, H, W, Cp,
                         Co, Pt, L, nb_ci, (unsigned)xb, (unsigned)db, dthw, dtw);
      break;
    case 121:  // default
      hipLaunchKernelGGL((wino::wino_wgrad_kernel<2, 1, 3>), dim3(nwg), dim3(wino::NT), 0, s, x, dy, part, H, W, Cp,
                         Co, Pt, L, nb_ci, (unsigned)xb, (unsigned)db, dthw, dtw);
      break;
    case 20:
      hipLaunchKernelGGL((wino::wino_wgrad_kernel<2, 0>), dim3(nwg), dim3(wino::NT), 0, s, x, dy, part, H, W, Cp, Co,
                         Pt, L, nb_ci, (unsigned)xb, (unsigned)db, dthw, dtw);
      break;
    default:
      return -5;
  }
  const size_t n4 = (size_t)16 * Co * Cp / 4;
  hipLaunchKernelGGL(wino::wino_wgrad_sum_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, part, S, n4, du);
  hipLaunchKernelGGL(wino::wino_wgrad_out_kernel, dim3((Co * Ci + 255) / 256), dim3(256), 0, s, du, Co, Ci, Cp, grad,
                     accumulate);
  return -(int)hipGetLastError();
}
