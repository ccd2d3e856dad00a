// ddpx — fused classifier head: Linear(K -> C<=16) + softmax cross-entropy
// (forward), and its backward fused with the preceding ReLU's mask and bias
// gradient.  ONE launch each way.
//
// Reference ops replaced:
//   classifier Linear  /root/reference/singlegpu.py:73,81 (`self.classifier(x)`)
//   F.cross_entropy    /root/reference/singlegpu.py:105
//   argmax/eq/sum eval /root/reference/singlegpu.py:200-206
//
// With C = 10 classes the head is skinny: a few MFLOP and a few MB of traffic, so what costs time
// is kernel boundaries, serial cross-workgroup reductions and idle CUs, not arithmetic (the r1
// split-K design took four launches and 28.5 us at M = 512, K = 4096):
//   forward  = (16-row block x K slice) workgroups; the last slice of a row block to arrive sums
//              the slices' partial logits and finishes its rows (bias, log-softmax, NLL, dlogits,
//              argmax), and the last row block sums the batch-mean loss (write-through partials +
//              agent-scope tickets, fixed summation orders);
//   backward = one workgroup per 16-column slab over ALL rows: dH for the slab, and the slab's
//              complete dW / previous-layer bias sums (reduced in registers + LDS in a fixed order),
//              stored or applied (fused SGD) directly.  Head bias gradient by workgroup 0.
#include "ddpx_common.h"

namespace ddpx {

constexpr int kHeadC = 16;      // classes padded to one MFMA tile
constexpr int kHeadCols = 16;   // backward: columns per workgroup

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

// Forward.  Workgroup (rb, ks) = 16 rows x one K slice (256 workgroups at M = 512: a 32-workgroup
// row-only split left 7/8 of the chip idle and ran 14.6 us); its 4 waves split the slice, issue all
// their loads first, and multiply on v_mfma_f32_16x16x32_bf16 (A = 16 rows of H, B = the 16 padded
// classes of W).  The [16][16] partial goes out write-through (sc1) and the workgroup takes the row
// block's agent-scope ticket; the last of the KS slices to arrive sums the partials in slice order
// (deterministic), finishes the 16 rows (bias, log-softmax, NLL, dlogits, argmax), stores their losses
// write-through and takes the batch ticket; the last row block sums every row loss in row order.
// Both hand-offs follow MI355X_MICROARCH.md "Valid forms", row 1 (sc1 stores drained before the
// ticket, sc1 loads after it): no release or acquire fence.  Each last arriver resets its ticket.
__global__ void __launch_bounds__(256)
head_fwd_kernel(const unsigned short* __restrict__ H, const unsigned short* __restrict__ W,
                const float* __restrict__ b, const int64_t* __restrict__ tgt, int M, int K, int C, int ldh, int KS,
                int kslice, float inv_m, float* __restrict__ logits, float* __restrict__ dlogits,
                int* __restrict__ correct, float* part, float* loss_rows, int* tickets, float* __restrict__ loss_mean,
                const float* __restrict__ lr_table, int lr_n, int* __restrict__ lr_counter, float* __restrict__ lr_out) {
  // one LDS object (cdna_hip_programming §5 item 4a): [4 waves][16][17] partials + [16][17] sums + flags
  __shared__ float lds[4 * 16 * 17 + 16 * 17 + 4];
  float* zs = lds + 4 * 16 * 17;
  int* flag = reinterpret_cast<int*>(zs + 16 * 17);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rb = blockIdx.x / KS, ks = blockIdx.x - rb * KS;
  const int nrb = gridDim.x / KS;
  const int m0 = rb * 16;
  const int kw = kslice / 4;  // multiple of 32
  const int kb = ks * kslice + wave * kw;
  const int ke = min(K, kb + kw);
  const int row = m0 + (lane & 15);
  const int cls = lane & 15;
  const int ko = 8 * (lane >> 4);
  // the LR-table advance at the very end reads counter -> table: both loaded now (by every workgroup: the last one
  // to arrive is not known yet), so the kernel's tail carries no dependent load round trips for it
  int lr_k = 0;
  float lr_next = 0.f;
  if (lr_counter && loss_mean) {
    lr_k = *lr_counter;
    lr_next = lr_table[lr_k < lr_n ? lr_k : lr_n - 1];
  }
  const bool rok = row < M, cok = cls < C;
  const unsigned short* hp = H + (size_t)(rok ? row : 0) * ldh;
  const unsigned short* wp = W + (size_t)(cok ? cls : 0) * K;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  constexpr int KST = 4;  // MFMA steps whose loads are in flight together
  for (int k = kb; k < ke; k += 32 * KST) {
    u32x4 av[KST], bv[KST];
#pragma unroll
    for (int i = 0; i < KST; ++i) {
      const int kk = k + 32 * i + ko;
      av[i] = bv[i] = (u32x4){0u, 0u, 0u, 0u};
      if (rok && kk < ke) av[i] = *reinterpret_cast<const u32x4*>(hp + kk);
      if (cok && kk < ke) bv[i] = *reinterpret_cast<const u32x4*>(wp + kk);
    }
#pragma unroll
    for (int i = 0; i < KST; ++i)
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av[i]),
                                                    __builtin_bit_cast(bf16x8, bv[i]), acc, 0, 0, 0);
  }
  // C/D map: col (class) = lane&15, row = 4*(lane>>4) + r
#pragma unroll
  for (int r = 0; r < 4; ++r) lds[(wave * 16 + 4 * (lane >> 4) + r) * 17 + (lane & 15)] = acc[r];
  __syncthreads();
  const int t = threadIdx.x;
  const int rr = t >> 4, cc = t & 15;
  float z = (lds[rr * 17 + cc] + lds[(16 + rr) * 17 + cc]) + (lds[(32 + rr) * 17 + cc] + lds[(48 + rr) * 17 + cc]);
  if (KS > 1) {
    __hip_atomic_store(part + (size_t)blockIdx.x * 256 + t, z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) *flag = __hip_atomic_fetch_add(tickets + rb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == KS - 1;
    __syncthreads();
    if (!*flag) return;
    // sc1 buffer loads, all in flight together (relaxed atomic loads were each waited for: 8 serial
    // round trips); summed in slice order, whichever slice arrived last
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void*)(part + (size_t)rb * KS * 256), 0,
                                                                          (unsigned)(KS * 256 * 4), 0x00020000);
    z = 0.f;
    for (int s0 = 0; s0 < KS; s0 += 8) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        v[q] = s0 + q < KS ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rp, ((s0 + q) * 256 + t) * 4, 0, 16))
                           : 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) z += v[q];
    }
    if (t == 0) __hip_atomic_store(tickets + rb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  zs[rr * 17 + cc] = z;
  __syncthreads();
  if (wave == 0) {
    int hit = 0;
    if (lane < 16 && m0 + lane < M) {
      const int m = m0 + lane;
      float zr[kHeadC];
#pragma unroll
      for (int c = 0; c < kHeadC; ++c) zr[c] = zs[lane * 17 + c];
      const float l = head_finish(zr, b, tgt, C, inv_m, m, logits, dlogits, &hit);
      if (loss_mean) __hip_atomic_store(loss_rows + m, l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (correct) {
      const unsigned long long bal = __ballot(hit);
      if (lane == 0 && bal) atomicAdd(correct, __popcll(bal));  // integer: deterministic
    }
  }
  if (!loss_mean) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the storing wave drains its sc1 stores
  __syncthreads();
  if (t == 0) flag[1] = __hip_atomic_fetch_add(tickets + nrb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nrb - 1;
  __syncthreads();
  if (!flag[1] || wave != 0) return;
  const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc((void*)loss_rows, 0, (unsigned)(M * 4), 0x00020000);
  float s = 0.f;
  for (int i0 = 0; i0 < M; i0 += 64 * 8) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)  // out-of-range lanes read zeros (buffer bounds check)
      v[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rl, (i0 + q * 64 + lane) * 4, 0, 16));
#pragma unroll
    for (int q = 0; q < 8; ++q) s += v[q];
  }
  s = wave_sum(s);  // fixed butterfly: the same order whichever row block is last
  if (lane == 0) {
    *loss_mean = s / (float)M;
    __hip_atomic_store(tickets + nrb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lr_counter) {
      // the training step's device LR schedule (SGD.device_lr_step): lr = table[step], step += 1.  Every
      // reader of the step counter (the batch gather) ran in an earlier kernel and every reader of lr (the
      // optimizer) runs in a later one, so this single thread saves the step its own 1-thread launch.
      *lr_out = lr_next;
      *lr_counter = lr_k + 1;
    }
  }
}

// Sum over the 32 lanes of each half-wave (every lane of the half gets it): DPP within 16-lane rows
// (quad xor 1, quad xor 2, row rotate 4, row rotate 8: plain VALU), then one swap across the row pair.
// The DPP adds run in a fixed pattern, so the result does not depend on timing.
__device__ __forceinline__ float half_wave_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
  return v + __shfl_xor(v, 16, 64);
}

// Backward.  Workgroup = a 16-column slab [k0, k0+16) over all M rows (256 workgroups at K = 4096);
// thread (cg = half-wave, r0 = wave * 32 + lane % 32) owns 8 columns of rows r0, r0+256, ... (the two
// 16-B halves of a row come from lanes l and l+32 of one wave instruction) and issues the loads of
// RPT such rows before computing any of them (the 32-column, one-row-in-flight version was latency
// bound: 15.5 us at M = 512):
//   g[m][k]  = go * sum_c dlogits[m][c] * W[c][k]
//   dH[m][k] = hscale * (relu_mask ? g * (H[m][k] > 0) : g)             (bf16, stored)
//   (hscale = 1/(1-p) when H is the output of an inverted Dropout(p) after a ReLU: H > 0 is then
//    exactly "kept and positive", so the dropout + ReLU backward costs nothing extra)
//   dW[c][k]    = go * sum_m dlogits[m][c] * H[m][k]
//   dprev[k]    = sum_m dH[m][k]                  (bias gradient of the layer that produced H)
//   db[c]       = go * sum_m dlogits[m][c]        (workgroup 0)
// Column sums: registers over the thread's rows, then the 32 lanes of a half-wave (DPP row reduction +
// one cross-row swap; a 5-step ds_bpermute butterfly over 88 values per lane was LDS-issue bound),
// then the 8 waves in order through LDS — a fixed order, so the result is bitwise reproducible.
// Outputs are stored (fp32 / bf16, written or accumulated) or, with SgdArgs.p set, applied as an SGD
// update: each workgroup reads only its own columns of W, all before it updates them.
// NT threads, RPT rows per thread in flight: 256 x 4 (round 6) halves the per-block cross-lane reduction work of
// 512 x 2 (the 88 column sums' DPP butterflies dominated once the loads were in flight; wide MLP K = 16384: 1024
// blocks).
template <int C, int NT = 256, int RPT = 4>
__global__ void __launch_bounds__(NT)
head_bwd_kernel(const float* __restrict__ dlogits, const float* __restrict__ go_ptr,
                const unsigned short* __restrict__ H, const unsigned short* __restrict__ W, int M, int K, int ldh,
                unsigned short* __restrict__ dH, int relu_mask, float hscale, void* __restrict__ dW,
                void* __restrict__ db, void* __restrict__ dbprev, int out_bf16, int accumulate, SgdArgs sW,
                SgdArgs sB, SgdArgs sP) {
  constexpr int NWV = NT / 64;
  constexpr int TPR = kHeadCols / 8;  // threads per row
  constexpr int RL = NT / TPR;        // rows per pass (NT / 2)
  static_assert(C % 2 == 0, "dlogits rows are read as float2");
  __shared__ float lds[NWV * kHeadCols * (C + 1) + NWV * C];
  float* redh = lds + NWV * kHeadCols * (C + 1);
  const float go = go_ptr ? *go_ptr : 1.f;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  static_assert(TPR == 2, "half-wave column groups");
  const int cg = lane >> 5, r0 = w * 32 + (lane & 31);
  const int k0 = blockIdx.x * kHeadCols;
  const int k = k0 + cg * 8;
  // W packed bf16, widened at each use
  u32x4 wraw[C];
#pragma unroll
  for (int c = 0; c < C; ++c) wraw[c] = *reinterpret_cast<const u32x4*>(W + (size_t)c * K + k);
  auto wv = [&](int c, int j) -> float {
    return (j & 1) ? __uint_as_float(wraw[c][j >> 1] & 0xffff0000u) : __uint_as_float(wraw[c][j >> 1] << 16);
  };
  float dw[C][8], dbp[8], hb[C];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    dbp[j] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) dw[c][j] = 0.f;
  }
#pragma unroll
  for (int c = 0; c < C; ++c) hb[c] = 0.f;
  const bool head_bias = blockIdx.x == 0 && cg == 0;  // one thread per row sums dlogits for the head bias
  // fused SGD: the threads that finish a column's dW / previous-layer bias (tid < 16 (C + 1)) and the head bias
  // (block 0, tid < C) load their master / momentum now, under the main loop, not after the reduction
  float pre_p = 0.f, pre_m = 0.f, preh_p = 0.f, preh_m = 0.f;
  {
    const int col = tid % kHeadCols, c = tid / kHeadCols;
    if (tid < kHeadCols * (C + 1)) {
      const SgdArgs& sg = c < C ? sW : sP;
      const size_t idx = c < C ? (size_t)c * K + k0 + col : (size_t)(k0 + col);
      if (sg.p) {
        pre_p = __builtin_nontemporal_load(sg.p + idx);
        if (sg.mom != 0.f) pre_m = __builtin_nontemporal_load(sg.buf + idx);
      }
    }
    if (blockIdx.x == 0 && tid < C && sB.p) {
      preh_p = __builtin_nontemporal_load(sB.p + tid);
      if (sB.mom != 0.f) preh_m = __builtin_nontemporal_load(sB.buf + tid);
    }
  }
  const float lr = sW.p ? *sW.lr : 0.f;
  for (int mb = r0; mb < M; mb += RL * RPT) {
    float2 dn[RPT][C / 2];
    u32x4 hn[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int m = mb + q * RL;
      const int mm = m < M ? m : mb;  // rows past M re-read row mb and are skipped below
      const float2* dp = reinterpret_cast<const float2*>(dlogits + (size_t)mm * C);  // 8-B aligned rows
#pragma unroll
      for (int c = 0; c < C / 2; ++c) dn[q][c] = dp[c];
      hn[q] = *reinterpret_cast<const u32x4*>(H + (size_t)mm * ldh + k);
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int m = mb + q * RL;
      if (m >= M) break;
      float dl[C];
#pragma unroll
      for (int c = 0; c < C / 2; ++c) {
        dl[2 * c] = dn[q][c].x * go;
        dl[2 * c + 1] = dn[q][c].y * go;
      }
      if (head_bias) {
#pragma unroll
        for (int c = 0; c < C; ++c) hb[c] += dl[c];
      }
      float h[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        h[2 * j] = __uint_as_float(hn[q][j] << 16);
        h[2 * j + 1] = __uint_as_float(hn[q][j] & 0xffff0000u);
      }
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) s = fmaf(dl[c], wv(c, j), s);
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
      for (int j = 0; j < 4; ++j) {  // bias gradient of the stored (bf16-rounded) dH
        dbp[2 * j] += __uint_as_float(o[j] << 16);
        dbp[2 * j + 1] += __uint_as_float(o[j] & 0xffff0000u);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    dbp[j] = half_wave_sum(dbp[j]);
#pragma unroll
    for (int c = 0; c < C; ++c) dw[c][j] = half_wave_sum(dw[c][j]);
  }
  if (blockIdx.x == 0) {
#pragma unroll
    for (int c = 0; c < C; ++c) hb[c] = half_wave_sum(hb[c]);  // cg 1 lanes hold zeros
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < C; ++c) redh[w * C + c] = hb[c];
    }
  }
  if ((lane & 31) == 0) {  // lane 0: cg 0, lane 32: cg 1
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lds[(w * kHeadCols + cg * 8 + j) * (C + 1) + C] = dbp[j];
#pragma unroll
      for (int c = 0; c < C; ++c) lds[(w * kHeadCols + cg * 8 + j) * (C + 1) + c] = dw[c][j];
    }
  }
  __syncthreads();
  auto put = [&](const SgdArgs& sg, void* base, size_t idx, float v, float pv, float mv) {
    if (sg.p) {  // fused optimizer: update the parameter instead of storing its gradient
      sgd_apply_pre(sg, idx, v, lr, pv, mv);
    } else if (out_bf16) {
      unsigned short* o = reinterpret_cast<unsigned short*>(base) + idx;
      *o = f2bf(accumulate ? v + bf2f(*o) : v);
    } else {
      float* o = reinterpret_cast<float*>(base) + idx;
      *o = accumulate ? v + *o : v;
    }
  };
  if (tid < kHeadCols * (C + 1)) {
    const int col = tid % kHeadCols, c = tid / kHeadCols;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < NWV; ++ww) s += lds[(ww * kHeadCols + col) * (C + 1) + c];
    const int kk = k0 + col;
    if (c < C) {
      if (dW || sW.p) put(sW, dW, (size_t)c * K + kk, s, pre_p, pre_m);
    } else if (dbprev || sP.p) {
      put(sP, dbprev, kk, s, pre_p, pre_m);
    }
  }
  if (blockIdx.x == 0 && tid < C && (db || sB.p)) {  // head bias: db[c] = go * sum_m dlogits[m][c]
    float sh = 0.f;
#pragma unroll
    for (int ww = 0; ww < NWV; ++ww) sh += redh[ww * C + tid];
    put(sB, db, tid, sh, preh_p, preh_m);
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

}  // namespace ddpx

using namespace ddpx;

static int head_ksplit(int M, int K) {
  const int rbs = (M + 15) / 16;
  int ks = (256 + rbs - 1) / rbs;
  const int maxks = max(1, K / 128);  // >= one 32-wide MFMA step per wave
  return max(1, min(ks, maxks));
}

// Forward scratch (floats): slice partials [row blocks * KS][16][16] + row losses [M]; tickets (ints):
// row blocks + 1, zero before the first launch (every launch leaves them zero).
DDPX_API int64_t ddpx_head_fwd_scratch(int M, int K) {
  const int64_t rbs = (M + 15) / 16;
  return rbs * head_ksplit(M, K) * 256 + M;
}
DDPX_API int64_t ddpx_head_fwd_tickets(int M) { return (M + 15) / 16 + 1; }

// lr_table / lr_counter / lr_out (optional, with loss_mean): advance the device LR schedule in the launch.
DDPX_API int ddpx_head_fwd(const void* H, const void* W, const float* b, const int64_t* tgt, int M, int K, int C,
                           int ldh, float inv_m, float* logits, float* dlogits, int* correct, float* scratch,
                           int* tickets, float* loss_mean, const float* lr_table, int lr_n, int* lr_counter,
                           float* lr_out, hipStream_t s) {
  if (M <= 0) return 0;
  if (C < 1 || C > kHeadC) return -1;
  if (K % 8 || ldh % 8) return -2;
  if (!scratch || !tickets) return -3;
  if (loss_mean && !tgt) return -4;
  if (lr_counter && (!loss_mean || !lr_table || !lr_out || lr_n < 1)) return -5;
  const int rbs = (M + 15) / 16;
  const int ks = head_ksplit(M, K);
  int kslice = (K + ks - 1) / ks;
  kslice = (kslice + 127) / 128 * 128;  // whole 32-wide MFMA steps for each of the 4 waves
  float* part = scratch;
  float* loss_rows = scratch + (size_t)rbs * ks * 256;
  hipLaunchKernelGGL(head_fwd_kernel, dim3(rbs * ks), dim3(256), 0, s, (const unsigned short*)H,
                     (const unsigned short*)W, b, tgt, M, K, C, ldh, ks, kslice, inv_m, logits, dlogits, correct, part,
                     loss_rows, tickets, loss_mean, lr_table, lr_n, lr_counter, lr_out);
  return (int)hipGetLastError();
}

DDPX_API int ddpx_head_bwd(const float* dlogits, const float* go, const void* H, const void* W, int M, int K, int C,
                           int ldh, void* dH, int relu_mask, float hscale, void* dW, void* db, void* dbprev,
                           int out_bf16, int accumulate, float* sw_p, float* sw_buf, void* sw_sh, float* sb_p,
                           float* sb_buf, void* sb_sh, float* sp_p, float* sp_buf, void* sp_sh, const float* lr,
                           float mom, float wd, hipStream_t s) {
  if (M <= 0) return 0;
  if (C != 10) return -1;
  if (K % kHeadCols || ldh % 8) return -2;
  hipLaunchKernelGGL((head_bwd_kernel<10, 256, 4>), dim3(K / kHeadCols), dim3(256), 0, s, dlogits, go,
                     (const unsigned short*)H, (const unsigned short*)W, M, K, ldh, (unsigned short*)dH, relu_mask,
                     hscale, dW, db, dbprev, out_bf16, accumulate,
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
