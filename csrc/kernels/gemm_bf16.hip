// ddpx — bf16 MFMA GEMM for gfx950 (CDNA4) with fused epilogues.
//
//   C[M][N] = epilogue( sum_k A(m,k) * B(k,n) )
//
// Operand layouts (chosen per call so forward, dgrad and wgrad of a Linear
// never materialise a transpose):
//   A "K-contig" : A[m*lda + k]      A "M-contig" : A[k*lda + m]
//   B "K-contig" : B[n*ldb + k]      B "N-contig" : B[k*ldb + n]
// For nn.Linear (W stored [out][in]) with activations X [batch][in]:
//   forward  Y  = X  W^T : A=X  (K-contig), B=W   (K-contig)
//   dgrad    dX = dY W   : A=dY (K-contig), B=W   (N-contig)
//   wgrad    dW = dY^T X : A=dY (M-contig), B=X   (N-contig)
// (reference equivalent: the implicit cuBLAS addmm/mm of nn.Linear,
//  /root/reference/singlegpu.py:73 `nn.Linear(512, 10)`)
//
// Design (MI355X-first, cdna_hip_programming.md §3/§5):
//  * 256-thread workgroups = 4 waves in a 2x2 grid; every wave owns a
//    (16*FM) x (16*FN) output block of v_mfma_f32_16x16x32_bf16 tiles.
//  * BK = 64.  Tiles are staged global -> VGPR -> LDS (ds_write_b128) with
//    the next K-tile's global loads issued before the current tile's MFMAs
//    (issue-early / write-late, T14), two LDS buffers, ONE barrier per K-step.
//  * K-contig tiles live in LDS as [row][64] (128-B rows) with a 16-B-chunk
//    XOR swizzle chunk ^= (row>>1)&7 so every ds_read_b128 lane group hits
//    16 distinct bank slots.  M/N-contig tiles live as [k][row] and are read
//    with the CDNA4 hardware-transpose ds_read_b64_tr_b16 (T10) under a
//    32-B-chunk XOR swizzle chosen per row stride (conflict-free per half).
//  * Workgroup ids are remapped XCD-aware (T1) so the tiles that share a B
//    panel run on one XCD and hit its L2.
#include "ddpx_common.h"

namespace ddpx {

enum GemmEpilogue : int {
  EPI_F32 = 0,            // C(f32)  = alpha*acc (+ C if accumulate)
  EPI_BF16 = 1,           // C(bf16) = alpha*acc
  EPI_BIAS_BF16 = 2,      // C(bf16) = acc + bias[n]
  EPI_BIAS_RELU_BF16 = 3, // C(bf16) = max(acc + bias[n], 0)
  EPI_BIAS_F32 = 4,       // C(f32)  = acc + bias[n]
  EPI_RELUMASK_BF16 = 5,  // C(bf16) = acc * (aux[m][n] > 0)   (ReLU backward)
};

struct GemmParams {
  const unsigned short* A;
  const unsigned short* B;
  void* C;
  const float* bias;
  const unsigned short* aux;
  int M, N, K;
  int lda, ldb, ldc, ldaux;
  int epi;
  int accumulate;
  float alpha;
};

// 32-byte-chunk XOR swizzle for an LDS image [k][ROWB bytes] read with
// ds_read_b64_tr_b16: one 32-lane half of a tr-read touches rows
// k = 8g + q (+4) for g in {2s, 2s+1}, q in 0..3, all at one 32-B column
// chunk; the swizzle spreads those 8 rows over the 8 32-B bank slots.
template <int ROWB>
__device__ __forceinline__ int tr_swz(int k) {
  if constexpr (ROWB >= 256) {
    return (k & 3) | (((k >> 3) & 1) << 2);
  } else if constexpr (ROWB == 128) {
    return ((k >> 1) & 1) | (((k >> 3) & 1) << 1);
  } else {
    static_assert(ROWB == 64, "unsupported row stride");
    return (k >> 3) & 1;
  }
}

__device__ __forceinline__ int kc_swz_off(int row, int chunk) {
  // [row][64 bf16] image, 16-B chunk index 0..7.
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

template <int ROWS, bool KCONTIG>
struct TileLoader {
  // Stages a ROWS x 64 (rows x k) operand tile.  ROWS*8 16-byte chunks,
  // ROWS/32 per thread.
  static constexpr int kChunks = ROWS * 8 / 256;
  static constexpr int ROWB = ROWS * 2;  // bytes per k-row of the [k][row] image
  u32x4 reg[kChunks];

  __device__ __forceinline__ void load(const unsigned short* __restrict__ g, int ld, int row0,
                                       int nrows, int k0, int K, int tid) {
#pragma unroll
    for (int i = 0; i < kChunks; ++i) {
      const int c = tid + i * 256;
      int r, kk;
      if constexpr (KCONTIG) {
        r = c >> 3;
        kk = (c & 7) * 8;
      } else {
        constexpr int CPR = ROWS / 8;
        kk = c / CPR;
        r = (c % CPR) * 8;
      }
      const int gr = row0 + r, gk = k0 + kk;
      const bool ok = (gr < nrows) && (gk < K);
      u32x4 v = {0u, 0u, 0u, 0u};
      if (ok) {
        const unsigned short* p =
            KCONTIG ? (g + (size_t)gr * ld + gk) : (g + (size_t)gk * ld + gr);
        v = *reinterpret_cast<const u32x4*>(p);
      }
      reg[i] = v;
    }
  }

  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < kChunks; ++i) {
      const int c = tid + i * 256;
      int off;
      if constexpr (KCONTIG) {
        off = kc_swz_off(c >> 3, c & 7);
      } else {
        constexpr int CPR = ROWS / 8;
        const int k = c / CPR, rc = c % CPR;  // rc: 16-B chunk along the row
        off = k * ROWB + (((rc >> 1) ^ tr_swz<ROWB>(k)) << 5) + ((rc & 1) << 4);
      }
      *reinterpret_cast<u32x4*>(lds + off) = reg[i];
    }
  }

  // MFMA 16x16x32 operand fragment: lane l holds X[row = rbase + (l&15)][k = kbase + 8(l>>4) + j].
  __device__ __forceinline__ static bf16x8 frag(const char* lds, int rbase, int kbase, int lane) {
    if constexpr (KCONTIG) {
      const int row = rbase + (lane & 15);
      const int chunk = (kbase >> 3) + (lane >> 4);
      return *reinterpret_cast<const bf16x8*>(lds + kc_swz_off(row, chunk));
    } else {
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
};

template <int FM, int FN, bool AK, bool BK_>
__global__ void __launch_bounds__(256) gemm_bf16_kernel(GemmParams p) {
  constexpr int BM = 32 * FM, BN = 32 * FN, BK = 64;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = wg % tiles_m, tn = wg / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;

  TileLoader<BM, AK> la;
  TileLoader<BN, BK_> lb;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  la.load(p.A, p.lda, m0, p.M, 0, p.K, tid);
  lb.load(p.B, p.ldb, n0, p.N, 0, p.K, tid);
  la.store(smem, tid);
  lb.store(smem + A_BYTES, tid);
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const char* sa = smem + (t & 1) * STAGE;
    const char* sb = sa + A_BYTES;
    const bool more = (t + 1) < nk;
    if (more) {
      la.load(p.A, p.lda, m0, p.M, (t + 1) * BK, p.K, tid);
      lb.load(p.B, p.ldb, n0, p.N, (t + 1) * BK, p.K, tid);
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = TileLoader<BM, AK>::frag(sa, wm * (BM / 2) + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = TileLoader<BN, BK_>::frag(sb, wn * (BN / 2) + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      char* nxt = smem + ((t + 1) & 1) * STAGE;
      la.store(nxt, tid);
      lb.store(nxt + A_BYTES, tid);
    }
    __syncthreads();
  }

  // Epilogue.  C/D map of 16x16x32: col = lane&15, row = 4*(lane>>4) + r.
  const int epi = p.epi;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
      if (n >= p.N) continue;
      float bias = 0.f;
      if (epi == EPI_BIAS_BF16 || epi == EPI_BIAS_RELU_BF16 || epi == EPI_BIAS_F32) bias = p.bias[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + 4 * (lane >> 4) + r;
        if (m >= p.M) continue;
        float v = acc[i][j][r];
        const size_t off = (size_t)m * p.ldc + n;
        switch (epi) {
          case EPI_F32: {
            float* c = reinterpret_cast<float*>(p.C) + off;
            v *= p.alpha;
            *c = p.accumulate ? (*c + v) : v;
          } break;
          case EPI_BF16:
            reinterpret_cast<unsigned short*>(p.C)[off] = f2bf(v * p.alpha);
            break;
          case EPI_BIAS_BF16:
            reinterpret_cast<unsigned short*>(p.C)[off] = f2bf(v + bias);
            break;
          case EPI_BIAS_RELU_BF16:
            reinterpret_cast<unsigned short*>(p.C)[off] = f2bf(fmaxf(v + bias, 0.f));
            break;
          case EPI_BIAS_F32:
            reinterpret_cast<float*>(p.C)[off] = v + bias;
            break;
          case EPI_RELUMASK_BF16: {
            const unsigned short h = p.aux[(size_t)m * p.ldaux + n];
            const bool pos = (h & 0x8000u) == 0 && (h & 0x7fffu) != 0;
            reinterpret_cast<unsigned short*>(p.C)[off] = pos ? f2bf(v) : (unsigned short)0;
          } break;
          default:
            break;
        }
      }
    }
  }
}

template <int FM, int FN, bool AK, bool BK_>
static hipError_t launch(const GemmParams& p, hipStream_t s) {
  constexpr int BM = 32 * FM, BN = 32 * FN;
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_bf16_kernel<FM, FN, AK, BK_>), dim3(tiles), dim3(256), 0, s, p);
  return hipGetLastError();
}

template <bool AK, bool BK_>
static hipError_t dispatch_tile(const GemmParams& p, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: return launch<4, 4, AK, BK_>(p, s);  // 128 x 128
    case 1: return launch<2, 4, AK, BK_>(p, s);  //  64 x 128
    case 2: return launch<4, 2, AK, BK_>(p, s);  // 128 x  64
    default: return launch<2, 2, AK, BK_>(p, s); //  64 x  64
  }
}

static int pick_tile(int M, int N) {
  // Fill 256 CUs: prefer the largest tile that still yields >= 256 workgroups.
  auto tiles = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  if (tiles(128, 128) >= 256) return 0;
  if (tiles(64, 128) >= 256) return 1;
  if (tiles(128, 64) >= 256) return 2;
  return 3;
}

}  // namespace ddpx

using namespace ddpx;

// Returns 0 on success, a negative value on an unsupported shape, or a hipError_t.
// a_kcontig / b_kcontig select the operand layouts documented at the top.
// tile_cfg < 0 selects the tile automatically.
DDPX_API int ddpx_gemm_bf16(const void* A, const void* B, void* C, const float* bias, const void* aux,
                            int M, int N, int K, int lda, int ldb, int ldc, int ldaux, int a_kcontig,
                            int b_kcontig, int epi, int accumulate, float alpha, int tile_cfg,
                            hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  // 16-byte vector staging: the contiguous dimension of every operand must be
  // a multiple of 8 elements and 16-B aligned.
  if (a_kcontig ? (K % 8 || lda % 8) : (M % 8 || lda % 8)) return -1;
  if (b_kcontig ? (K % 8 || ldb % 8) : (N % 8 || ldb % 8)) return -2;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -3;
  GemmParams p{(const unsigned short*)A, (const unsigned short*)B, C, bias, (const unsigned short*)aux,
               M, N, K, lda, ldb, ldc, ldaux, epi, accumulate, alpha};
  const int cfg = tile_cfg >= 0 ? tile_cfg : pick_tile(M, N);
  hipError_t e;
  if (a_kcontig && b_kcontig) e = dispatch_tile<true, true>(p, cfg, stream);
  else if (a_kcontig) e = dispatch_tile<true, false>(p, cfg, stream);
  else if (b_kcontig) e = dispatch_tile<false, true>(p, cfg, stream);
  else e = dispatch_tile<false, false>(p, cfg, stream);
  return (int)e;
}
