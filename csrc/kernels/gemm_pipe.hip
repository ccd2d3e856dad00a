// ddpx — pipelined bf16 MFMA GEMM for gfx950: LDS-DMA multi-stage ring.
//
// Same contract and operand layouts as gemm_bf16.hip (see there), re-built
// for the regime the MLP shapes live in (M = 512 rows against N, K = 3-16 K):
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
//    swizzles of gemm_bf16.hip are applied to the per-lane SOURCE address and
//    undone on the read (rule 21): same images, same fragment readers.
//  * Buffer-resource bounds checking returns zeros for out-of-range lanes
//    (voffset forced past num_records), which handles ragged M/N/K tails with
//    no branches in the load path.
//  * XCD-aware workgroup remap (T1) as in v1.
//  * Epilogues: bias (+ReLU) -> bf16, fp32 (+accumulate) for gradients
//    written straight into DDP buckets, bf16 (+accumulate), ReLU-mask
//    backward, and an optional per-tile column sum of the stored output (the
//    bias gradient of the layer below) written as [tiles_m][N] partials.
#include "ddpx_common.h"

namespace ddpx {
namespace pipe {

enum Epi : int {
  EPI_F32 = 0,
  EPI_BF16 = 1,
  EPI_BIAS_BF16 = 2,
  EPI_BIAS_RELU_BF16 = 3,
  EPI_BIAS_F32 = 4,
  EPI_RELUMASK_BF16 = 5,
  EPI_SGD = 6,  // no C: the gradient tile updates master/momentum/shadow in place (fused optimizer)
};

struct Params {
  const unsigned short* A;
  const unsigned short* B;
  void* C;
  const float* bias;
  const unsigned short* aux;
  float* colsum;  // optional [tiles_m][N] partial column sums of the stored output
  int M, N, K;
  int lda, ldb, ldc, ldaux;
  int epi, accumulate;
  float alpha;
  unsigned a_bytes, b_bytes;  // buffer extents for the bounds-checked DMA
  SgdArgs sgd;
};

constexpr unsigned kOOB = 0x80000000u;

template <int ROWB>
__device__ __forceinline__ int tr_swz(int k) {
  if constexpr (ROWB >= 256) return (k & 3) | (((k >> 3) & 1) << 2);
  else if constexpr (ROWB == 128) return ((k >> 1) & 1) | (((k >> 3) & 1) << 1);
  else return (k >> 3) & 1;
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds_wave_base, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)lds_wave_base, 16, voff, 0, 0, 0);
}

// Stage one ROWS x 64 operand tile into an LDS slot with LDS-DMA.
// Each of the 4 waves issues ROWS/32 wave-instructions of 1 KiB.
template <int ROWS, bool KC>
__device__ __forceinline__ void stage_tile(__amdgpu_buffer_rsrc_t rs, char* slot, int ld, int row0, int nrows, int k0,
                                           int K, int wave, int lane) {
  constexpr int NI = ROWS / 32;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int inst = j * 4 + wave;
    if constexpr (KC) {
      // image [ROWS][64 bf16]: 128-B rows, an instruction covers 8 rows
      const int r = inst * 8 + (lane >> 3);
      const int p = lane & 7;
      const int c = p ^ ((r >> 1) & 7);  // logical 16-B chunk stored at physical p
      const int gr = row0 + r, gk = k0 + c * 8;
      const unsigned voff = (gr < nrows && gk < K) ? (unsigned)((gr * ld + gk) * 2) : kOOB;
      dma16(rs, slot + inst * 1024, voff);
    } else {
      // image [64 k][ROWS bf16]: ROWB-byte rows, an instruction covers 1024/ROWB k-rows
      constexpr int ROWB = ROWS * 2;
      constexpr int CPR = ROWB / 16;  // 16-B chunks per k-row
      const int kr = inst * (1024 / ROWB) + lane / CPR;
      const int q = lane % CPR;
      const int L = (q >> 1) ^ tr_swz<ROWB>(kr);
      const int col = L * 16 + (q & 1) * 8;
      const int gk = k0 + kr, gr = row0 + col;
      const unsigned voff = (gk < K && gr < nrows) ? (unsigned)((gk * ld + gr) * 2) : kOOB;
      dma16(rs, slot + inst * 1024, voff);
    }
  }
}

template <int ROWS, bool KC>
__device__ __forceinline__ bf16x8 frag(const char* lds, int rbase, int kbase, int lane) {
  if constexpr (KC) {
    const int row = rbase + (lane & 15);
    const int chunk = (kbase >> 3) + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
  } else {
    constexpr int ROWB = ROWS * 2;
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int chunk32 = rbase >> 4;
    const int k0 = kbase + 8 * g + q;
    const int k1 = k0 + 4;
    const int off0 = k0 * ROWB + ((chunk32 ^ tr_swz<ROWB>(k0)) << 5) + p * 8;
    const int off1 = k1 * ROWB + ((chunk32 ^ tr_swz<ROWB>(k1)) << 5) + p * 8;
    short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS short4v*)(lds + off0));
    short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS short4v*)(lds + off1));
    short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Store one wave's FM x FN fragments (C/D map of 16x16x32: col = lane&15,
// row = 4*(lane>>4) + r) through epilogue E; accumulate per-column sums of the
// stored values into csum (bias gradient of the layer below).
template <int E, int FM, int FN>
__device__ __forceinline__ void store_tile(const Params& p, const f32x4 (&acc)[FM][FN], int mb, int nb,
                                           float (&csum)[FN]) {
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = nb + j * 16;
    if (n >= p.N) continue;
    float bias = 0.f;
    if constexpr (E == EPI_BIAS_BF16 || E == EPI_BIAS_RELU_BF16 || E == EPI_BIAS_F32) bias = p.bias[n];
    float lr = 0.f;
    if constexpr (E == EPI_SGD) lr = *p.sgd.lr;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mb + i * 16 + r;
        if (m >= p.M) continue;
        const float v = acc[i][j][r];
        const size_t off = (size_t)m * p.ldc + n;
        float stored;
        if constexpr (E == EPI_F32) {
          float* c = reinterpret_cast<float*>(p.C) + off;
          stored = v * p.alpha;
          if (p.accumulate) stored += *c;
          *c = stored;
        } else if constexpr (E == EPI_BF16) {
          unsigned short* c = reinterpret_cast<unsigned short*>(p.C) + off;
          float x = v * p.alpha;
          if (p.accumulate) x += bf2f(*c);
          const unsigned short h = f2bf(x);
          *c = h;
          stored = bf2f(h);
        } else if constexpr (E == EPI_BIAS_BF16 || E == EPI_BIAS_RELU_BF16) {
          float x = v + bias;
          if constexpr (E == EPI_BIAS_RELU_BF16) x = fmaxf(x, 0.f);
          const unsigned short h = f2bf(x);
          reinterpret_cast<unsigned short*>(p.C)[off] = h;
          stored = bf2f(h);
        } else if constexpr (E == EPI_BIAS_F32) {
          stored = v + bias;
          reinterpret_cast<float*>(p.C)[off] = stored;
        } else if constexpr (E == EPI_SGD) {
          stored = v * p.alpha;
          sgd_apply(p.sgd, off, stored, lr);
        } else {  // EPI_RELUMASK_BF16
          const unsigned short hm = p.aux[(size_t)m * p.ldaux + n];
          const bool pos = (hm & 0x8000u) == 0 && (hm & 0x7fffu) != 0;
          const unsigned short h = pos ? f2bf(v) : (unsigned short)0;
          reinterpret_cast<unsigned short*>(p.C)[off] = h;
          stored = bf2f(h);
        }
        csum[j] += stored;
      }
    }
  }
}

template <int BM, int BN, int STAGES, bool AK, bool BKc>
__global__ void __launch_bounds__(256) gemm_pipe_kernel(Params p) {
  constexpr int BK = 64;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int SLOT = A_BYTES + B_BYTES;
  constexpr int FM = BM / 32, FN = BN / 32;     // 16x16 fragments per wave (2x2 waves)
  constexpr int LPW = BM / 32 + BN / 32;         // DMA instructions per wave per stage
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * SLOT];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = wg % tiles_m, tn = wg / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, 0, p.b_bytes, 0x00020000);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;

  auto issue = [&](int t) {
    char* slot = smem + (t % STAGES) * SLOT;
    stage_tile<BM, AK>(ra, slot, p.lda, m0, p.M, t * BK, p.K, wave, lane);
    stage_tile<BN, BKc>(rb, slot + A_BYTES, p.ldb, n0, p.N, t * BK, p.K, wave, lane);
  };

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s);

  for (int t = 0; t < nk; ++t) {
    // stages issued and not yet waited: t .. min(t+STAGES-2, nk-1); keep all but stage t in flight
    const int ahead = min(STAGES - 2, nk - 1 - t);
    if (ahead >= 2) wait_vmcnt<2 * LPW>();
    else if (ahead == 1) wait_vmcnt<LPW>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1);

    const char* sa = smem + (t % STAGES) * SLOT;
    const char* sb = sa + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = frag<BM, AK>(sa, wm * (BM / 2) + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = frag<BN, BKc>(sb, wn * (BN / 2) + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }

  // ---------------------------------------------------------------- epilogue
  // One wave-uniform dispatch on the epilogue kind; each kind is its own
  // straight-line store loop (no per-element switch).
  float csum[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) csum[j] = 0.f;
  const int mb = m0 + wm * (BM / 2) + 4 * (lane >> 4);
  const int nb = n0 + wn * (BN / 2) + (lane & 15);
  switch (p.epi) {
    case EPI_F32: store_tile<EPI_F32, FM, FN>(p, acc, mb, nb, csum); break;
    case EPI_BF16: store_tile<EPI_BF16, FM, FN>(p, acc, mb, nb, csum); break;
    case EPI_BIAS_BF16: store_tile<EPI_BIAS_BF16, FM, FN>(p, acc, mb, nb, csum); break;
    case EPI_BIAS_RELU_BF16: store_tile<EPI_BIAS_RELU_BF16, FM, FN>(p, acc, mb, nb, csum); break;
    case EPI_BIAS_F32: store_tile<EPI_BIAS_F32, FM, FN>(p, acc, mb, nb, csum); break;
    case EPI_SGD: store_tile<EPI_SGD, FM, FN>(p, acc, mb, nb, csum); break;
    default: store_tile<EPI_RELUMASK_BF16, FM, FN>(p, acc, mb, nb, csum); break;
  }
  if (p.colsum) {
    // reduce over the 4 row groups of the wave (lane bits 4,5), then the 2 row-waves via LDS
    __builtin_amdgcn_s_barrier();  // every wave is done with the last LDS slot
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float s = csum[j];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (lane < 16) red[(wm * 2 + wn) * (BN / 2) + j * 16 + lane] = s;
    }
    __syncthreads();
    if (tid < BN) {
      const int wnn = tid / (BN / 2), c = tid % (BN / 2);
      const float s = red[(0 * 2 + wnn) * (BN / 2) + c] + red[(1 * 2 + wnn) * (BN / 2) + c];
      const int n = n0 + tid;
      if (n < p.N) p.colsum[(size_t)tm * p.N + n] = s;
    }
  }
}

// out[n] (=|+=) sum_t partial[t][n]   (fixed order: deterministic)
__global__ void __launch_bounds__(256) reduce_partials_kernel(const float* __restrict__ part, int T, int N,
                                                              float* __restrict__ out, int out_bf16, int accumulate,
                                                              SgdArgs sgd) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int t = 0; t < T; ++t) s += part[(size_t)t * N + n];
  if (sgd.p) {
    sgd_apply(sgd, n, s, *sgd.lr);
  } else if (out_bf16) {
    unsigned short* o = reinterpret_cast<unsigned short*>(out);
    if (accumulate) s += bf2f(o[n]);
    o[n] = f2bf(s);
  } else {
    out[n] = accumulate ? out[n] + s : s;
  }
}

template <int BM, int BN, int STAGES, bool AK, bool BKc>
static hipError_t launch(const Params& p, hipStream_t s) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_pipe_kernel<BM, BN, STAGES, AK, BKc>), dim3(tiles), dim3(256), 0, s, p);
  return hipGetLastError();
}

template <bool AK, bool BKc>
static hipError_t dispatch(const Params& p, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: return launch<128, 128, 4, AK, BKc>(p, s);  // 128 KiB LDS, 1 WG/CU
    case 1: return launch<64, 128, 4, AK, BKc>(p, s);   //  96 KiB
    case 2: return launch<128, 64, 4, AK, BKc>(p, s);   //  96 KiB
    case 3: return launch<64, 64, 4, AK, BKc>(p, s);    //  64 KiB, 2 WG/CU
    case 4: return launch<128, 128, 3, AK, BKc>(p, s);  //  96 KiB
    case 5: return launch<64, 128, 3, AK, BKc>(p, s);   //  72 KiB, 2 WG/CU
    case 6: return launch<128, 64, 3, AK, BKc>(p, s);   //  72 KiB, 2 WG/CU
    default: return launch<64, 64, 3, AK, BKc>(p, s);   //  48 KiB, 3 WG/CU
  }
}

static void tile_of(int cfg, int* bm, int* bn) {
  static const int t[8][2] = {{128, 128}, {64, 128}, {128, 64}, {64, 64}, {128, 128}, {64, 128}, {128, 64}, {64, 64}};
  *bm = t[cfg & 7][0];
  *bn = t[cfg & 7][1];
}

// Default tile per operand-layout class, from the MI355X sweep of the MLP shapes
// (benchmarks/gemm_sweep.py; profiles/): M=512-row products want many small
// tiles (64x64, 2-3 WG/CU), the K=512 weight-gradient products 64x128/3 stages.
static int pick(int M, int N, int K, bool ak, bool bk) {
  auto tiles = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  if (!ak && !bk) return tiles(64, 128) >= 512 ? 5 : 7;      // wgrad-shaped (reduction over batch)
  if (ak && !bk) return 3;                                   // dgrad-shaped
  if (tiles(128, 128) >= 1024 && K >= 2048) return 0;        // big forward GEMMs
  return 7;                                                  // forward, small M
}

}  // namespace pipe
}  // namespace ddpx

using namespace ddpx;

// Number of row tiles (M direction) the kernel will use for cfg (for sizing colsum partials).
DDPX_API int ddpx_gemm_pipe_tiles_m(int M, int N, int K, int a_kcontig, int b_kcontig, int tile_cfg) {
  const int cfg = tile_cfg >= 0 ? tile_cfg : pipe::pick(M, N, K, a_kcontig, b_kcontig);
  int bm, bn;
  pipe::tile_of(cfg, &bm, &bn);
  return (M + bm - 1) / bm;
}

DDPX_API int ddpx_gemm_pipe(const void* A, const void* B, void* C, const float* bias, const void* aux, float* colsum,
                            int M, int N, int K, int lda, int ldb, int ldc, int ldaux, int a_kcontig, int b_kcontig,
                            int epi, int accumulate, float alpha, int tile_cfg, float* sgd_p, float* sgd_buf,
                            void* sgd_shadow, const float* sgd_lr, float sgd_mom, float sgd_wd, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (a_kcontig ? (K % 8 || lda % 8) : (M % 8 || lda % 8)) return -1;
  if (b_kcontig ? (K % 8 || ldb % 8) : (N % 8 || ldb % 8)) return -2;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -3;
  const size_t a_bytes = (size_t)(a_kcontig ? (size_t)(M - 1) * lda + K : (size_t)(K - 1) * lda + M) * 2;
  const size_t b_bytes = (size_t)(b_kcontig ? (size_t)(N - 1) * ldb + K : (size_t)(K - 1) * ldb + N) * 2;
  if (a_bytes >= 0x80000000ull || b_bytes >= 0x80000000ull) return -4;  // 32-bit buffer offsets
  pipe::Params p{(const unsigned short*)A, (const unsigned short*)B, C, bias, (const unsigned short*)aux, colsum,
                 M, N, K, lda, ldb, ldc, ldaux, epi, accumulate, alpha, (unsigned)a_bytes, (unsigned)b_bytes,
                 SgdArgs{sgd_p, sgd_buf, (unsigned short*)sgd_shadow, sgd_lr, sgd_mom, sgd_wd}};
  if (epi == pipe::EPI_SGD && (!sgd_p || !sgd_lr || (sgd_mom != 0.f && !sgd_buf))) return -5;
  const int cfg = tile_cfg >= 0 ? tile_cfg : pipe::pick(M, N, K, a_kcontig, b_kcontig);
  hipError_t e;
  if (a_kcontig && b_kcontig) e = pipe::dispatch<true, true>(p, cfg, stream);
  else if (a_kcontig) e = pipe::dispatch<true, false>(p, cfg, stream);
  else if (b_kcontig) e = pipe::dispatch<false, true>(p, cfg, stream);
  else e = pipe::dispatch<false, false>(p, cfg, stream);
  return (int)e;
}

DDPX_API int ddpx_reduce_partials(const float* part, int T, int N, void* out, int out_bf16, int accumulate,
                                  float* sgd_p, float* sgd_buf, void* sgd_shadow, const float* sgd_lr, float sgd_mom,
                                  float sgd_wd, hipStream_t s) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(pipe::reduce_partials_kernel, dim3((N + 255) / 256), dim3(256), 0, s, part, T, N, (float*)out,
                     out_bf16, accumulate, SgdArgs{sgd_p, sgd_buf, (unsigned short*)sgd_shadow, sgd_lr, sgd_mom, sgd_wd});
  return (int)hipGetLastError();
}
