// ddpx — fused classifier head: Linear(K -> C) + softmax cross-entropy
// (forward) and its backward fused with the preceding ReLU's mask and bias
// gradient.
//
// Reference ops replaced:
//   classifier Linear  /root/reference/singlegpu.py:73,81 (`self.classifier(x)`)
//   F.cross_entropy    /root/reference/singlegpu.py:105
//   argmax/eq/sum eval /root/reference/singlegpu.py:200-206
// With C = 10 classes the head is far too skinny for MFMA tiles (N = 10): it is
// a streaming dot-product problem, so it runs one wave per sample row with
// 16-B vector loads, the 10 logits reduced across the 64 lanes by shuffles,
// and the whole softmax / NLL / dlogits / argmax done in registers.
#include "ddpx_common.h"

namespace ddpx {

// Forward: one wave per row m.
//   logits[m][c] = sum_k H[m][k] * W[c][k] + b[c]          (fp32 out, optional)
//   loss_rows[m] = logsumexp(logits[m]) - logits[m][t_m]   (optional)
//   dlogits[m][c] = (softmax[m][c] - [c==t_m]) * inv_m       (optional)
//   correct += [argmax(logits[m]) == t_m]                  (optional)
template <int C>
__global__ void __launch_bounds__(256)
head_fwd_kernel(const unsigned short* __restrict__ H, const unsigned short* __restrict__ W,
                const float* __restrict__ b, const int64_t* __restrict__ tgt, int M, int K, int ldh,
                float inv_m, float* __restrict__ logits, float* __restrict__ loss_rows,
                float* __restrict__ dlogits, int* __restrict__ correct) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  float acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = 0.f;
  const unsigned short* hrow = H + (size_t)m * ldh;
  for (int k = lane * 8; k < K; k += 512) {
    const u32x4 hv = *reinterpret_cast<const u32x4*>(hrow + k);
    float h[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      h[2 * j] = __uint_as_float(hv[j] << 16);
      h[2 * j + 1] = __uint_as_float(hv[j] & 0xffff0000u);
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const u32x4 wv = *reinterpret_cast<const u32x4*>(W + (size_t)c * K + k);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[c] = fmaf(h[2 * j], __uint_as_float(wv[j] << 16), acc[c]);
        acc[c] = fmaf(h[2 * j + 1], __uint_as_float(wv[j] & 0xffff0000u), acc[c]);
      }
    }
  }
  float z[C];
#pragma unroll
  for (int c = 0; c < C; ++c) z[c] = wave_sum(acc[c]) + b[c];
  // every lane now holds all C logits
  float mx = z[0];
  int am = 0;
#pragma unroll
  for (int c = 1; c < C; ++c)
    if (z[c] > mx) { mx = z[c]; am = c; }
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) se += __expf(z[c] - mx);
  const float lse = mx + __logf(se);
  const int t = tgt ? (int)tgt[m] : 0;
  if (lane < C) {
    float zc = z[0];
#pragma unroll
    for (int c = 1; c < C; ++c) zc = (lane == c) ? z[c] : zc;
    if (logits) logits[(size_t)m * C + lane] = zc;
    if (dlogits) {
      const float pr = __expf(zc - lse);
      dlogits[(size_t)m * C + lane] = (pr - (lane == t ? 1.f : 0.f)) * inv_m;
    }
  }
  if (lane == 0) {
    if (loss_rows) {
      float zt = z[0];
#pragma unroll
      for (int c = 1; c < C; ++c) zt = (t == c) ? z[c] : zt;
      loss_rows[m] = lse - zt;
    }
    if (correct && am == t) atomicAdd(correct, 1);
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

// Backward.  One workgroup per 64-column slice of K, looping over all M rows
// (8 lanes x 8 bf16 per row, 32 rows in flight per workgroup):
//   g[m][k]    = go * sum_c dlogits[m][c] * W[c][k]
//   dH[m][k]   = relu_mask ? g * (H[m][k] > 0) : g                  (bf16)
//   dW[c][k]  (=|+=) go * sum_m dlogits[m][c] * H[m][k]            (fp32)
//   dbprev[k] (=|+=) sum_m dH[m][k]        (bias grad of the layer that produced H)
//   db[c]     (=|+=) go * sum_m dlogits[m][c]                        (workgroup 0)
template <int C>
__global__ void __launch_bounds__(256)
head_bwd_kernel(const float* __restrict__ dlogits, const float* __restrict__ go_ptr,
                const unsigned short* __restrict__ H, const unsigned short* __restrict__ W, int M, int K,
                int ldh, unsigned short* __restrict__ dH, float* __restrict__ dW, float* __restrict__ db,
                float* __restrict__ dbprev, int relu_mask, int accumulate) {
  __shared__ float red[4][64][C + 1];
  const float go = go_ptr ? *go_ptr : 1.f;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int cg = tid & 7;         // column group: 8 columns
  const int r0 = tid >> 3;        // 0..31 row within a 32-row slab
  const int k = blockIdx.x * 64 + cg * 8;
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
  float dw[C][8];
  float dbp[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    dbp[j] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) dw[c][j] = 0.f;
  }
  for (int m = r0; m < M; m += 32) {
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
      g[j] = s;
#pragma unroll
      for (int c = 0; c < C; ++c) dw[c][j] = fmaf(dl[c], h[j], dw[c][j]);
    }
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = pack_bf2(g[2 * j], g[2 * j + 1]);
    if (dH) *reinterpret_cast<u32x4*>(dH + (size_t)m * ldh + k) = o;
    // bias grad of the producing layer from the bf16-rounded values actually stored
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dbp[2 * j] += __uint_as_float(o[j] << 16);
      dbp[2 * j + 1] += __uint_as_float(o[j] & 0xffff0000u);
    }
  }
  // reduce over the 8 row-lanes of a wave that share a column group (lane bits 3..5)
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
  __syncthreads();
  // 64 columns x (C + 1) outputs per workgroup
  for (int i = tid; i < 64 * (C + 1); i += 256) {
    const int col = i % 64, c = i / 64;
    const float s = (red[0][col][c] + red[1][col][c]) + (red[2][col][c] + red[3][col][c]);
    const int kk = blockIdx.x * 64 + col;
    if (c < C) {
      float* d = dW + (size_t)c * K + kk;
      *d = accumulate ? *d + s : s;
    } else if (dbprev) {
      dbprev[kk] = accumulate ? dbprev[kk] + s : s;
    }
  }
  if (blockIdx.x == 0 && db && w == 0) {
    // db[c] = go * sum_m dlogits[m][c]
    for (int c = 0; c < C; ++c) {
      float s = 0.f;
      for (int m = lane; m < M; m += 64) s += dlogits[(size_t)m * C + c];
      s = wave_sum(s) * go;
      if (lane == 0) db[c] = accumulate ? db[c] + s : s;
    }
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
  // wave-aggregated integer atomic (deterministic result)
  const unsigned long long bal = __ballot(hit);
  if ((threadIdx.x & 63) == 0 && bal) atomicAdd(correct, __popcll(bal));
}

}  // namespace ddpx

using namespace ddpx;

DDPX_API int ddpx_head_fwd(const void* H, const void* W, const float* b, const int64_t* tgt, int M, int K,
                           int C, int ldh, float inv_m, float* logits, float* loss_rows, float* dlogits,
                           int* correct, hipStream_t s) {
  if (M <= 0) return 0;
  if (C != 10) return -1;
  if (K % 8 || ldh % 8) return -2;
  hipLaunchKernelGGL(head_fwd_kernel<10>, dim3((M + 3) / 4), dim3(256), 0, s, (const unsigned short*)H,
                     (const unsigned short*)W, b, tgt, M, K, ldh, inv_m, logits, loss_rows, dlogits, correct);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_mean(const float* x, int n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(1024), 0, s, x, n, out);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_head_bwd(const float* dlogits, const float* go, const void* H, const void* W, int M, int K,
                           int C, int ldh, void* dH, float* dW, float* db, float* dbprev, int relu_mask,
                           int accumulate, hipStream_t s) {
  if (M <= 0) return 0;
  if (C != 10) return -1;
  if (K % 64 || ldh % 8) return -2;
  hipLaunchKernelGGL(head_bwd_kernel<10>, dim3(K / 64), dim3(256), 0, s, dlogits, go, (const unsigned short*)H,
                     (const unsigned short*)W, M, K, ldh, (unsigned short*)dH, dW, db, dbprev, relu_mask,
                     accumulate);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_accuracy(const float* logits, const int64_t* tgt, int M, int C, int* correct, hipStream_t s) {
  if (M <= 0) return 0;
  hipLaunchKernelGGL(accuracy_kernel, dim3((M + 255) / 256), dim3(256), 0, s, logits, tgt, M, C, correct);
  return (int)hipGetLastError();
}
