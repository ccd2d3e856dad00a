// ddpx — fused classifier head: Linear(K -> C<=16) + softmax cross-entropy
// (forward), and its backward fused with the preceding ReLU's mask and bias
// gradient.
//
// Reference ops replaced:
//   classifier Linear  /root/reference/singlegpu.py:73,81 (`self.classifier(x)`)
//   F.cross_entropy    /root/reference/singlegpu.py:105
//   argmax/eq/sum eval /root/reference/singlegpu.py:200-206
//
// With C = 10 classes the head is skinny (N = 10): the work is a few MFLOP
// and a few MB of streaming, so the design goal is PARALLELISM and no long
// dependent chains:
//   forward  = split-K MFMA partial logits (16 rows x 16 padded classes per
//              workgroup slice, 4 waves split the slice's K) + a row-parallel
//              finalize (bias, log-softmax, NLL, dlogits, argmax) + a
//              deterministic mean;
//   backward = row-split x column-tile workgroups (>= 256 of them) that
//              each produce dH for their tile and partial dW / bias sums,
//              followed by a fixed-order reduction of the partials
//              (bitwise reproducible, no float atomics).
#include "ddpx_common.h"

namespace ddpx {

constexpr int kHeadC = 16;  // classes padded to one MFMA tile

// partial[ks][m][16] = sum_{k in slice ks} H[m][k] * W[c][k]   (c >= C -> 0)
__global__ void __launch_bounds__(256)
head_logits_partial_kernel(const unsigned short* __restrict__ H, const unsigned short* __restrict__ W, int M,
                           int K, int C, int ldh, int kslice, float* __restrict__ partial) {
  __shared__ float red[4][16][17];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 16, ks = blockIdx.y;
  const int kbeg = ks * kslice;
  const int kend = min(K, kbeg + kslice);
  const int wlen = (kslice + 3) / 4;
  const int wb = kbeg + wave * wlen;
  const int we = min(kend, wb + wlen);
  const int row = m0 + (lane & 15);
  const int cls = lane & 15;
  const int ko = 8 * (lane >> 4);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = wb; k < we; k += 32) {
    const int kk = k + ko;
    u32x4 av = {0u, 0u, 0u, 0u}, bv = {0u, 0u, 0u, 0u};
    if (row < M && kk < we) av = *reinterpret_cast<const u32x4*>(H + (size_t)row * ldh + kk);
    if (cls < C && kk < we) bv = *reinterpret_cast<const u32x4*>(W + (size_t)cls * K + kk);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av), __builtin_bit_cast(bf16x8, bv),
                                                  acc, 0, 0, 0);
  }
  // C/D map: col (class) = lane&15, row = 4*(lane>>4) + r
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][4 * (lane >> 4) + r][lane & 15] = acc[r];
  __syncthreads();
  const int t = threadIdx.x;
  const int rr = t >> 4, cc = t & 15;
  const float s = (red[0][rr][cc] + red[1][rr][cc]) + (red[2][rr][cc] + red[3][rr][cc]);
  if (m0 + rr < M) partial[((size_t)ks * M + m0 + rr) * kHeadC + cc] = s;
}

// Per row, given the summed logits z (bias not yet added): log-softmax, NLL, dlogits, argmax.
// Returns the row loss (0 for no target).
__device__ __forceinline__ float head_finish(float (&z)[kHeadC], const float* __restrict__ b,
                                             const int64_t* __restrict__ tgt, int C, float inv_m, int m,
                                             float* __restrict__ logits, float* __restrict__ dlogits, int* hit) {
  float mx = -INFINITY;
  int am = 0;
#pragma unroll
  for (int c = 0; c < kHeadC; ++c) {
    if (c < C) {
      z[c] += b[c];
      if (z[c] > mx) { mx = z[c]; am = c; }
    }
  }
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < kHeadC; ++c)
    if (c < C) se += __expf(z[c] - mx);
  const float lse = mx + __logf(se);
  const int t = tgt ? (int)tgt[m] : 0;
  float zt = 0.f;
#pragma unroll
  for (int c = 0; c < kHeadC; ++c) {
    if (c < C) {
      if (c == t) zt = z[c];
      if (logits) logits[(size_t)m * C + c] = z[c];
      if (dlogits) dlogits[(size_t)m * C + c] = (__expf(z[c] - lse) - (c == t ? 1.f : 0.f)) * inv_m;
    }
  }
  *hit = tgt ? (am == t) : 0;
  return lse - zt;
}

// Partial-logit slices ks = k0, k0 + kstep, ... of row m summed into z.
__device__ __forceinline__ void head_sum(const float* __restrict__ partial, int KS, int M, int m, int k0, int kstep,
                                         float (&z)[kHeadC]) {
#pragma unroll
  for (int c = 0; c < kHeadC; ++c) z[c] = 0.f;
  for (int ks = k0; ks < KS; ks += kstep) {
    const f32x4* pp = reinterpret_cast<const f32x4*>(partial + ((size_t)ks * M + m) * kHeadC);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 v = pp[q];
      z[4 * q] += v[0];
      z[4 * q + 1] += v[1];
      z[4 * q + 2] += v[2];
      z[4 * q + 3] += v[3];
    }
  }
}

__device__ __forceinline__ float head_row(const float* __restrict__ partial, int KS, const float* __restrict__ b,
                                          const int64_t* __restrict__ tgt, int M, int C, float inv_m, int m,
                                          float* __restrict__ logits, float* __restrict__ dlogits, int* hit) {
  float z[kHeadC];
  head_sum(partial, KS, M, m, 0, 1, z);
  return head_finish(z, b, tgt, C, inv_m, m, logits, dlogits, hit);
}

// One thread per row.
__global__ void __launch_bounds__(256)
head_finalize_kernel(const float* __restrict__ partial, int KS, const float* __restrict__ b,
                     const int64_t* __restrict__ tgt, int M, int C, float inv_m, float* __restrict__ logits,
                     float* __restrict__ loss_rows, float* __restrict__ dlogits, int* __restrict__ correct) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  int hit = 0;
  if (m < M) {
    const float l = head_row(partial, KS, b, tgt, M, C, inv_m, m, logits, dlogits, &hit);
    if (loss_rows) loss_rows[m] = l;
  }
  if (correct) {
    const unsigned long long bal = __ballot(hit);
    if ((threadIdx.x & 63) == 0 && bal) atomicAdd(correct, __popcll(bal));  // integer: deterministic
  }
}

// Single workgroup (M <= 8192): every row plus the mean loss in one launch.  TL lanes share a row
// (each sums every TL-th partial-logit slice, so the slice loads of a row are in flight together
// instead of in one thread's serial chain), a butterfly combines them, and the group's first lane
// finishes the row.  Rows are assigned in a fixed pattern and reduced in a fixed order: deterministic.
template <int TL>
__global__ void __launch_bounds__(1024)
head_finalize_mean_kernel(const float* __restrict__ partial, int KS, const float* __restrict__ b,
                          const int64_t* __restrict__ tgt, int M, int C, float inv_m, float* __restrict__ logits,
                          float* __restrict__ loss_rows, float* __restrict__ dlogits, int* __restrict__ correct,
                          float* __restrict__ loss_mean) {
  __shared__ float red[16];
  constexpr int RPP = 1024 / TL;  // rows per pass
  const int sub = threadIdx.x % TL, r = threadIdx.x / TL;
  float acc = 0.f;
  int hits = 0;
  for (int m0 = 0; m0 < M; m0 += RPP) {
    const int m = m0 + r;
    float z[kHeadC];
    if (m < M) head_sum(partial, KS, M, m, sub, TL, z);
    else {
#pragma unroll
      for (int c = 0; c < kHeadC; ++c) z[c] = 0.f;
    }
#pragma unroll
    for (int o = 1; o < TL; o <<= 1)
#pragma unroll
      for (int c = 0; c < kHeadC; ++c) z[c] += __shfl_xor(z[c], o, 64);
    if (m < M && sub == 0) {
      int hit = 0;
      const float l = head_finish(z, b, tgt, C, inv_m, m, logits, dlogits, &hit);
      if (loss_rows) loss_rows[m] = l;
      acc += l;
      hits += hit;
    }
  }
  if (correct) {
    int hsum = hits;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hsum += __shfl_xor(hsum, o, 64);
    if ((threadIdx.x & 63) == 0 && hsum) atomicAdd(correct, hsum);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = threadIdx.x < 16 ? red[threadIdx.x] : 0.f;
    t = wave_sum(t);
    if (threadIdx.x == 0) *loss_mean = t / (float)M;
  }
}

// Deterministic mean of loss_rows (single workgroup).
__global__ void __launch_bounds__(1024) mean_kernel(const float* __restrict__ x, int n, float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) s += x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = threadIdx.x < 16 ? red[threadIdx.x] : 0.f;
    t = wave_sum(t);
    if (threadIdx.x == 0) *out = t / (float)n;
  }
}

// Backward partials.  Workgroup (column tile ct of 64, row split rs):
//   g[m][k]  = go * sum_c dlogits[m][c] * W[c][k]
//   dH[m][k] = hscale * (relu_mask ? g * (H[m][k] > 0) : g)             (bf16, stored)
//   (hscale = 1/(1-p) when H is the output of an inverted Dropout(p) after a ReLU: H > 0 is then
//    exactly "kept and positive", so the dropout + ReLU backward costs nothing extra)
//   pdw[rs][c][k]  = go * sum_{m in split} dlogits[m][c] * H[m][k]
//   pdb[rs][k]     = sum_{m in split} dH[m][k]     (bias grad of the layer that produced H)
// 8 lanes x 8 columns per row, 32 rows per pass, ROWS_PER_SPLIT/32 passes.
template <int C>
__global__ void __launch_bounds__(256)
head_bwd_partial_kernel(const float* __restrict__ dlogits, const float* __restrict__ go_ptr,
                        const unsigned short* __restrict__ H, const unsigned short* __restrict__ W, int M, int K,
                        int ldh, int rows_per_split, unsigned short* __restrict__ dH, float* __restrict__ pdw,
                        float* __restrict__ pdb, float* __restrict__ pdbh, int relu_mask, float hscale) {
  __shared__ float red[4][64][C + 1];
  __shared__ float redh[16][C];
  const float go = go_ptr ? *go_ptr : 1.f;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int cg = tid & 7, r0 = tid >> 3;
  const int k = blockIdx.x * 64 + cg * 8;
  const int rs = blockIdx.y;
  const int mbeg = rs * rows_per_split;
  const int mend = min(M, mbeg + rows_per_split);
  float wv[C][8];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(W + (size_t)c * K + k);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wv[c][2 * j] = __uint_as_float(v[j] << 16);
      wv[c][2 * j + 1] = __uint_as_float(v[j] & 0xffff0000u);
    }
  }
  float dw[C][8], dbp[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    dbp[j] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) dw[c][j] = 0.f;
  }
  for (int m = mbeg + r0; m < mend; m += 32) {
    float dl[C];
#pragma unroll
    for (int c = 0; c < C; ++c) dl[c] = dlogits[(size_t)m * C + c] * go;
    const u32x4 hv = *reinterpret_cast<const u32x4*>(H + (size_t)m * ldh + k);
    float h[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      h[2 * j] = __uint_as_float(hv[j] << 16);
      h[2 * j + 1] = __uint_as_float(hv[j] & 0xffff0000u);
    }
    float g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) s = fmaf(dl[c], wv[c][j], s);
      if (relu_mask && !(h[j] > 0.f)) s = 0.f;
      g[j] = s * hscale;
#pragma unroll
      for (int c = 0; c < C; ++c) dw[c][j] = fmaf(dl[c], h[j], dw[c][j]);
    }
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = pack_bf2(g[2 * j], g[2 * j + 1]);
    if (dH) *reinterpret_cast<u32x4*>(dH + (size_t)m * ldh + k) = o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dbp[2 * j] += __uint_as_float(o[j] << 16);
      dbp[2 * j + 1] += __uint_as_float(o[j] & 0xffff0000u);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      dbp[j] += __shfl_xor(dbp[j], o, 64);
#pragma unroll
      for (int c = 0; c < C; ++c) dw[c][j] += __shfl_xor(dw[c][j], o, 64);
    }
  }
  if (lane < 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[w][lane * 8 + j][C] = dbp[j];
#pragma unroll
      for (int c = 0; c < C; ++c) red[w][lane * 8 + j][c] = dw[c][j];
    }
  }
  if (blockIdx.x == 0) {
    // head bias partial for this row split: pdbh[rs][c] = go * sum_m dlogits[m][c]
    const int c = tid & 15, rg = tid >> 4;
    float sh = 0.f;
    if (c < C)
      for (int m = mbeg + rg; m < mend; m += 16) sh += dlogits[(size_t)m * C + c];
    if (c < C) redh[rg][c] = sh * go;
  }
  __syncthreads();
  if (blockIdx.x == 0 && tid < C) {
    float sh = 0.f;
    for (int rg = 0; rg < 16; ++rg) sh += redh[rg][tid];
    pdbh[(size_t)rs * C + tid] = sh;
  }
  for (int i = tid; i < 64 * (C + 1); i += 256) {
    const int col = i % 64, c = i / 64;
    const float s = (red[0][col][c] + red[1][col][c]) + (red[2][col][c] + red[3][col][c]);
    const int kk = blockIdx.x * 64 + col;
    if (c < C) pdw[((size_t)rs * C + c) * K + kk] = s;
    else pdb[(size_t)rs * K + kk] = s;
  }
}

// Fixed-order reduction of the row-split partials into the gradient buffers
// (fp32 or bf16, write or accumulate) + the head bias gradient (workgroup 0).
template <int C>
__global__ void __launch_bounds__(256)
head_bwd_finalize_kernel(const float* __restrict__ pdw, const float* __restrict__ pdb,
                         const float* __restrict__ pdbh, int RS, int K, void* __restrict__ dW,
                         void* __restrict__ db, void* __restrict__ dbprev, int out_bf16, int accumulate,
                         SgdArgs sW, SgdArgs sB, SgdArgs sP) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // over (C+1)*K + C
  auto put = [&](const SgdArgs* sg, void* base, size_t idx, float v) {
    if (sg->p) {  // fused optimizer: update the parameter instead of storing its gradient
      sgd_apply(*sg, idx, v, *sg->lr);
    } else if (out_bf16) {
      unsigned short* o = reinterpret_cast<unsigned short*>(base) + idx;
      *o = f2bf(accumulate ? v + bf2f(*o) : v);
    } else {
      float* o = reinterpret_cast<float*>(base) + idx;
      *o = accumulate ? v + *o : v;
    }
  };
  if (i < C * K) {
    float s = 0.f;
    for (int r = 0; r < RS; ++r) s += pdw[(size_t)r * C * K + i];
    put(&sW, dW, i, s);
  } else if (i < (C + 1) * K) {
    if (!dbprev && !sP.p) return;
    const int kk = i - C * K;
    float s = 0.f;
    for (int r = 0; r < RS; ++r) s += pdb[(size_t)r * K + kk];
    put(&sP, dbprev, kk, s);
  } else if (i < (C + 1) * K + C) {
    if (!db && !sB.p) return;
    const int c = i - (C + 1) * K;
    float s = 0.f;
    for (int r = 0; r < RS; ++r) s += pdbh[(size_t)r * C + c];
    put(&sB, db, c, s);
  }
}

__global__ void __launch_bounds__(256)
accuracy_kernel(const float* __restrict__ logits, const int64_t* __restrict__ tgt, int M, int C,
                int* __restrict__ correct) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  int hit = 0;
  if (m < M) {
    const float* z = logits + (size_t)m * C;
    float mx = z[0];
    int am = 0;
    for (int c = 1; c < C; ++c)
      if (z[c] > mx) { mx = z[c]; am = c; }
    hit = (am == (int)tgt[m]);
  }
  const unsigned long long bal = __ballot(hit);
  if ((threadIdx.x & 63) == 0 && bal) atomicAdd(correct, __popcll(bal));
}

static int head_ksplit(int M, int K) {
  const int row_tiles = (M + 15) / 16;
  int ks = (256 + row_tiles - 1) / row_tiles;
  const int maxks = max(1, K / 128);
  if (ks > maxks) ks = maxks;
  if (ks < 1) ks = 1;
  return ks;
}

static int head_row_splits(int M, int K) {
  const int ctiles = K / 64;
  int rs = (256 + ctiles - 1) / ctiles;
  const int maxrs = max(1, M / 32);
  if (rs > maxrs) rs = maxrs;
  return max(rs, 1);
}

}  // namespace ddpx

using namespace ddpx;

// Scratch sizes (floats) the host must provide for the head kernels.
DDPX_API int64_t ddpx_head_fwd_scratch(int M, int K) { return (int64_t)head_ksplit(M, K) * M * kHeadC; }
DDPX_API int64_t ddpx_head_bwd_scratch(int M, int K, int C) {
  const int64_t rs = head_row_splits(M, K);
  return rs * (C + 1) * K + rs * C;
}

// loss_mean (optional): mean row loss written by the same launch (M <= 8192) or by a follow-up
// single-workgroup reduction (larger M); loss_rows may then be null for M <= 8192.
DDPX_API int ddpx_head_fwd(const void* H, const void* W, const float* b, const int64_t* tgt, int M, int K, int C,
                           int ldh, float inv_m, float* logits, float* loss_rows, float* dlogits, int* correct,
                           float* scratch, float* loss_mean, hipStream_t s) {
  if (M <= 0) return 0;
  if (C < 1 || C > kHeadC) return -1;
  if (K % 8 || ldh % 8) return -2;
  const int ks = head_ksplit(M, K);
  int kslice = (K + ks - 1) / ks;
  kslice = (kslice + 127) / 128 * 128;  // whole 32-k MFMA steps for each of the 4 waves
  hipLaunchKernelGGL(head_logits_partial_kernel, dim3((M + 15) / 16, ks), dim3(256), 0, s, (const unsigned short*)H,
                     (const unsigned short*)W, M, K, C, ldh, kslice, scratch);
  if (loss_mean && tgt && M <= 8192) {
    // lanes per row: as many as keep every row in ONE pass of the 1024 threads (M <= 1024 / TL), at most
    // one per partial-logit slice — more passes would each pay the load latency again
    int tl = 1;
    while (tl < 16 && tl < ks && M * tl * 2 <= 1024) tl *= 2;
    if (tl == 1)
      hipLaunchKernelGGL(head_finalize_mean_kernel<1>, dim3(1), dim3(1024), 0, s, scratch, ks, b, tgt, M, C, inv_m,
                         logits, loss_rows, dlogits, correct, loss_mean);
    else if (tl == 2)
      hipLaunchKernelGGL(head_finalize_mean_kernel<2>, dim3(1), dim3(1024), 0, s, scratch, ks, b, tgt, M, C, inv_m,
                         logits, loss_rows, dlogits, correct, loss_mean);
    else if (tl == 4)
      hipLaunchKernelGGL(head_finalize_mean_kernel<4>, dim3(1), dim3(1024), 0, s, scratch, ks, b, tgt, M, C, inv_m,
                         logits, loss_rows, dlogits, correct, loss_mean);
    else if (tl == 8)
      hipLaunchKernelGGL(head_finalize_mean_kernel<8>, dim3(1), dim3(1024), 0, s, scratch, ks, b, tgt, M, C, inv_m,
                         logits, loss_rows, dlogits, correct, loss_mean);
    else
      hipLaunchKernelGGL(head_finalize_mean_kernel<16>, dim3(1), dim3(1024), 0, s, scratch, ks, b, tgt, M, C, inv_m,
                         logits, loss_rows, dlogits, correct, loss_mean);
    return (int)hipGetLastError();
  }
  if (loss_mean && !loss_rows) return -3;
  hipLaunchKernelGGL(head_finalize_kernel, dim3((M + 255) / 256), dim3(256), 0, s, scratch, ks, b, tgt, M, C, inv_m,
                     logits, loss_rows, dlogits, correct);
  if (loss_mean && tgt) hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(1024), 0, s, loss_rows, M, loss_mean);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_mean(const float* x, int n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(1024), 0, s, x, n, out);
  return (int)hipGetLastError();
}

// Backward in two launches: the partials (dH for every row + per-row-split dW / bias partials) and
// the fixed-order finalize that stores or applies (fused SGD) the parameter gradients.  The finalize
// is tiny (a separate entry point so a caller can time or reorder it).
DDPX_API int ddpx_head_bwd_partial(const float* dlogits, const float* go, const void* H, const void* W, int M, int K,
                                   int C, int ldh, void* dH, int relu_mask, float hscale, float* scratch,
                                   hipStream_t s) {
  if (M <= 0) return 0;
  if (C != 10) return -1;
  if (K % 64 || ldh % 8) return -2;
  const int rs = head_row_splits(M, K);
  const int rps = (M + rs - 1) / rs;
  float* pdw = scratch;
  float* pdb = scratch + (size_t)rs * C * K;
  float* pdbh = pdb + (size_t)rs * K;
  hipLaunchKernelGGL(head_bwd_partial_kernel<10>, dim3(K / 64, rs), dim3(256), 0, s, dlogits, go,
                     (const unsigned short*)H, (const unsigned short*)W, M, K, ldh, rps, (unsigned short*)dH, pdw, pdb,
                     pdbh, relu_mask, hscale);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_head_bwd_finalize(int M, int K, int C, void* dW, void* db, void* dbprev, int out_bf16,
                                    int accumulate, const float* scratch, float* sw_p, float* sw_buf, void* sw_sh,
                                    float* sb_p, float* sb_buf, void* sb_sh, float* sp_p, float* sp_buf, void* sp_sh,
                                    const float* lr, float mom, float wd, hipStream_t s) {
  if (M <= 0) return 0;
  if (C != 10) return -1;
  const int rs = head_row_splits(M, K);
  const float* pdw = scratch;
  const float* pdb = scratch + (size_t)rs * C * K;
  const float* pdbh = pdb + (size_t)rs * K;
  hipLaunchKernelGGL(head_bwd_finalize_kernel<10>, dim3(((C + 1) * K + C + 255) / 256), dim3(256), 0, s, pdw, pdb,
                     pdbh, rs, K, dW, db, dbprev, out_bf16, accumulate,
                     SgdArgs{sw_p, sw_buf, (unsigned short*)sw_sh, lr, mom, wd},
                     SgdArgs{sb_p, sb_buf, (unsigned short*)sb_sh, lr, mom, wd},
                     SgdArgs{sp_p, sp_buf, (unsigned short*)sp_sh, lr, mom, wd});
  return (int)hipGetLastError();
}

DDPX_API int ddpx_accuracy(const float* logits, const int64_t* tgt, int M, int C, int* correct, hipStream_t s) {
  if (M <= 0) return 0;
  hipLaunchKernelGGL(accuracy_kernel, dim3((M + 255) / 256), dim3(256), 0, s, logits, tgt, M, C, correct);
  return (int)hipGetLastError();
}
