// ddpx — pipelined bf16 MFMA GEMM core for gfx950 (shared by the plain GEMM and
// the implicit-GEMM 3x3 convolutions).
//
//   C[M][N] = epilogue( sum_k A(m,k) * B(k,n) )
//
// Operand storage: A "K-contig" A[m][k] / "M-contig" A[k][m]; B "K-contig"
// B[n][k] / "N-contig" B[k][n].  Addressing modes turn a (row, k) pair into a
// byte offset, so the same pipeline serves plain matrices and im2col views of
// NHWC activations without materialising them:
//   MODE_PLAIN      row-major matrix with leading dimension ld
//   MODE_IM2COL_FWD K-contig: row = output pixel, k = (tap, c)  -> x[pixel + off(tap)][c]
//   MODE_IM2COL_BWD K-contig: row = pixel,        k = (tap, c)  -> dy[pixel - off(tap)][c]
//   MODE_IM2COL_COL N-contig: k-row = pixel,      col = (tap,c) -> x[pixel + off(tap)][c]
// (off(tap) = (ky-1, kx-1) for a 3x3 / pad 1 / stride 1 convolution; taps
// falling outside the image are zero through the buffer bounds check.)
//
// Pipeline (cdna_hip_programming §5):
//  * operand tiles go HBM/L2 -> LDS by `buffer_load_dwordx4 ... lds` (LDS-DMA,
//    1 KiB per wave-instruction, no VGPR staging); out-of-range lanes get a
//    voffset past num_records and load zeros (ragged tiles, conv padding);
//  * STAGES-deep LDS ring, STAGES-1 K-tiles in flight; per iteration a counted
//    `s_waitcnt vmcnt(N)` for the oldest stage, a raw `s_barrier` (never
//    __syncthreads: its fence would drain the DMA queue), the next stage's DMA
//    into the slot freed one iteration ago, then ds_read + MFMA;
//  * LDS images are lane-linear, so bank swizzles are applied to the per-lane
//    SOURCE address and undone on the read (rule 21): K-contig tiles [row][64]
//    with chunk ^= (row>>1)&7 (conflict-free ds_read_b128), M/N-contig tiles
//    [k][row] with a 32-B-chunk XOR read by ds_read_b64_tr_b16 (T10);
//  * 4 waves (2x2), v_mfma_f32_16x16x32_bf16, XCD-aware workgroup remap (T1);
//  * optional split-K over blockIdx.y (fp32 partial slabs, reduced by a
//    separate fixed-order kernel: deterministic).
#pragma once

#include "ddpx_common.h"

namespace ddpx {
namespace pipe {

enum Epi : int {
  EPI_F32 = 0,            // C(f32)  = alpha*acc (+C)
  EPI_BF16 = 1,           // C(bf16) = alpha*acc (+C)
  EPI_BIAS_BF16 = 2,      // C(bf16) = acc + bias[n]
  EPI_BIAS_RELU_BF16 = 3, // C(bf16) = max(acc + bias[n], 0)
  EPI_BIAS_F32 = 4,       // C(f32)  = acc + bias[n]
  EPI_RELUMASK_BF16 = 5,  // C(bf16) = acc * (aux[m][n] > 0)
  EPI_SGD = 6,            // fused optimizer: acc is the gradient of the parameter at C's index
  EPI_BNSTAT_BF16 = 7,    // C(bf16) = acc; per-tile column (mean, M2) of the stored values -> colsum
  EPI_BNBWD_BF16 = 8,     // conv data gradient g (bf16) + the BatchNorm backward sums of the block below:
                          // per-tile column (sum dz, sum dz*xhat) -> colsum, dz = g routed / ReLU-masked by bn_y
};

enum Mode : int { MODE_PLAIN = 0, MODE_IM2COL_FWD = 1, MODE_IM2COL_BWD = 2, MODE_IM2COL_COL = 3 };

// Division by a runtime constant d >= 1 as a multiply-high and a shift (n < 2^31): the im2col
// address of every 16-B DMA chunk needs (tap, channel) = divmod(k, C) and (h, w) = divmod(pixel, W, H),
// and a v_rcp_iflag-based integer division is ~12 VALU instructions each — enough, 4 per chunk, to
// make the conv GEMMs VALU-issue-bound (ISA count of the 256x128 fwd kernel: 842 VALU per K-step
// against 32 MFMAs).  s = ceil(log2 d), magic = ceil(2^(31+s) / d) (< 2^32), n / d = umulhi(n, magic)
// >> (s - 1);  d == 1: magic 0 (identity).
struct FastDiv {
  unsigned magic;
  int shift;
};

static inline FastDiv make_fastdiv(int d) {
  FastDiv f{0u, 0};
  if (d <= 1) return f;
  int s = 0;
  while ((1ll << s) < d) ++s;
  f.shift = s - 1;
  f.magic = (unsigned)(((1ull << (31 + s)) + (unsigned long long)d - 1) / (unsigned long long)d);
  return f;
}

__device__ __forceinline__ int fdiv(int n, FastDiv f) {
  return f.magic ? (int)(__umulhi((unsigned)n, f.magic) >> f.shift) : n;
}

struct ConvGeom {
  int H, W, C;  // spatial size and channel count of the NHWC tensor being im2col'd
  int npix;     // N*H*W
  FastDiv dW, dH, dC;
};

static inline ConvGeom make_geom(int H, int W, int C, int npix) {
  return ConvGeom{H, W, C, npix, make_fastdiv(W), make_fastdiv(H), make_fastdiv(C)};
}

struct Params {
  const unsigned short* A;
  const unsigned short* B;
  void* C;
  const float* bias;
  const unsigned short* aux;
  float* colsum;   // [tiles_m][N] column sums (EPI_*) or [tiles_m][2][N] (mean, M2) for EPI_BNSTAT
  int M, N, K;
  int lda, ldb, ldc, ldaux;
  int epi, accumulate;
  float alpha;
  unsigned a_bytes, b_bytes;
  SgdArgs sgd;
  ConvGeom conv;
  int klen;        // split-K: K elements per split (0: no split)
  long long split_stride;  // elements between the output slabs of consecutive splits
  int sgd_plain;           // fused-SGD epilogue: 1 = ordinary (cached) loads/stores instead of non-temporal
  // In-launch split-K (gridDim.y = splits, klen set): each split's fp32 accumulators go write-through
  // (sc1) into slab[split][tile] in register layout, then the tile's ticket; the last split to arrive adds
  // every slab in split order and runs the epilogue (one launch, no partial-sum kernel).
  float* slab;
  unsigned slab_bytes;
  int* tcnt;               // per-tile tickets, zero between launches (the last arriver resets its own)
  // Column sums finished in-launch (the dgrad epilogue's bias gradient of the layer below): with cs_tcnt
  // set, every row tile writes its partial column sums write-through and takes its column tile's ticket;
  // the last row tile sums all partials in row-tile order and stores cs_out (fp32 / bf16, cs_flags bit 0;
  // accumulate, bit 1) or, with sgd.p set, applies them as an SGD update of that parameter.
  void* cs_out;
  int cs_flags;
  int* cs_tcnt;
  int im_slow;             // 1: im2col A operands use the per-chunk src_off path (A/B checks of ImRows)
  // diagnostics (ddpx_gemm_set_stamps): per-workgroup s_memrealtime stamps (100 MHz) at kernel start, main loop
  // end, split-K ticket taken, combine done, epilogue done: [workgroup][8] int64; nullptr = off
  long long* stamp;
  // EPI_BNBWD_BF16 (conv data gradient whose output g feeds the BatchNorm + ReLU [+ 2x2 max-pool] backward of
  // the block below): that block's pre-BN activation y (bf16, [P'][N], P' = 4 P when pooled) and per-channel
  // a = gamma*rstd, b = beta - mean*a, mean, rstd; bn_pool = 1 when a pool sits between y and g
  const unsigned short* bn_y;
  const float* bn_a;
  const float* bn_b;
  const float* bn_mean;
  const float* bn_rstd;
  int bn_pool;
};

__device__ __forceinline__ void stamp_at(const Params& p, int tid, int k) {
  if (p.stamp && tid == 0)
    p.stamp[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + k] = (long long)__builtin_amdgcn_s_memrealtime();
}

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

// Source byte offset of the 8-element chunk at (row, k) [K-contig] or (k-row, col) [M/N-contig].
template <int MODE, bool KC>
__device__ __forceinline__ unsigned src_off(const ConvGeom& g, int ld, int row, int k) {
  if constexpr (MODE == MODE_PLAIN) {
    return KC ? (unsigned)((row * ld + k) * 2) : (unsigned)((k * ld + row) * 2);
  } else {
    // pixel index p and (tap, channel) index q
    const int p = KC ? row : k;
    const int q = KC ? k : row;
    const int tap = fdiv(q, g.dC), c = q - tap * g.C;
    const int ky = (tap * 11) >> 5, kx = tap - ky * 3;  // tap / 3 for tap < 9 (tap >= 9 rejected below)
    int dy = ky - 1, dx = kx - 1;
    if constexpr (MODE == MODE_IM2COL_BWD) { dy = -dy; dx = -dx; }
    const int pw = fdiv(p, g.dW);
    const int w = p - pw * g.W;
    const int h = pw - fdiv(pw, g.dH) * g.H;
    const int hh = h + dy, ww = w + dx;
    if (tap >= 9 || hh < 0 || hh >= g.H || ww < 0 || ww >= g.W) return kOOB;
    return (unsigned)(((p + dy * g.W + dx) * g.C + c) * 2);
  }
}

// Source offset (bytes; kOOB = zero fill) of wave-instruction j of a ROWS x 64 operand tile: every
// wave-instruction moves 1 KiB, lane l its 16 B at LDS byte (j * NW + wave) * 1024 + 16 l of the slot.
template <int ROWS, bool KC, int MODE, int NW = 4>
__device__ __forceinline__ unsigned tile_voff(const ConvGeom& g, int ld, int row0, int nrows, int k0, int kend,
                                              int wave, int lane, int j) {
  const int inst = j * NW + wave;
  if constexpr (KC) {
    const int r = inst * 8 + (lane >> 3);
    const int pch = lane & 7;
    const int c = pch ^ ((r >> 1) & 7);
    const int gr = row0 + r, gk = k0 + c * 8;
    return (gr < nrows && gk < kend) ? src_off<MODE, true>(g, ld, gr, gk) : kOOB;
  } else {
    constexpr int ROWB = ROWS * 2;
    constexpr int CPR = ROWB / 16;
    const int kr = inst * (1024 / ROWB) + lane / CPR;
    const int q = lane % CPR;
    const int L = (q >> 1) ^ tr_swz<ROWB>(kr);
    const int col = L * 16 + (q & 1) * 8;
    const int gk = k0 + kr, gr = row0 + col;
    return (gk < kend && gr < nrows) ? src_off<MODE, false>(g, ld, gr, gk) : kOOB;
  }
}

// Stage one ROWS x 64 operand tile into an LDS slot with LDS-DMA (ROWS/8 wave-instructions of 1 KiB,
// spread over NW waves).
template <int ROWS, bool KC, int MODE, int NW = 4>
__device__ __forceinline__ void stage_tile(__amdgpu_buffer_rsrc_t rs, char* slot, const ConvGeom& g, int ld, int row0,
                                           int nrows, int k0, int kend, int wave, int lane) {
  constexpr int NI = ROWS / (8 * NW);
  static_assert(NI * 8 * NW == ROWS, "tile rows must split evenly over the waves");
#pragma unroll
  for (int j = 0; j < NI; ++j)
    dma16(rs, slot + (j * NW + wave) * 1024, tile_voff<ROWS, KC, MODE, NW>(g, ld, row0, nrows, k0, kend, wave, lane, j));
}

// im2col A operand (K-contig rows = output pixels) with C % 64 == 0: every 64-wide K-step lies inside ONE tap,
// so the tap, its pixel shift and the channel base are wave-uniform (scalar) per K-step, and everything that
// depends on the row — the pixel's (h, w) and its byte base — is computed once per tile.  The per-chunk work
// drops from two fast divisions, the tap divide and ~35 VALU (the 256x128 forward's K-step spent ~100 VALU on
// operand addresses between its barrier and its first MFMA, profiles/r4_vgg) to a bounds test and an add.
// Offsets are exactly src_off's (same bytes, same zero fill).
template <int ROWS, int NW>
struct ImRows {
  static constexpr int NI = ROWS / (8 * NW);
  int hw[NI];         // (h << 16) | w of the row's pixel; h = 0x4000 for rows past nrows (always out of bounds)
  unsigned base[NI];  // byte offset of (pixel, first channel of this lane's chunk) in the NHWC tensor
};

template <int ROWS, int NW>
__device__ __forceinline__ void im_rows_init(ImRows<ROWS, NW>& ir, const ConvGeom& g, int row0, int nrows, int wave,
                                             int lane) {
#pragma unroll
  for (int j = 0; j < ImRows<ROWS, NW>::NI; ++j) {
    const int r = (j * NW + wave) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int p = row0 + r;
    const int pw = fdiv(p, g.dW);
    const int w = p - pw * g.W;
    const int h = pw - fdiv(pw, g.dH) * g.H;
    ir.hw[j] = p < nrows ? ((h << 16) | w) : (0x4000 << 16);
    ir.base[j] = (unsigned)((p * g.C + c * 8) * 2);
  }
}

template <int ROWS, int MODE, int NW>
__device__ __forceinline__ void stage_tile_im(__amdgpu_buffer_rsrc_t rs, char* slot, const ConvGeom& g,
                                              const ImRows<ROWS, NW>& ir, int k0, int kend, int wave) {
  // K tail (k0 >= K = 9*C): zero fill like src_off's tap >= 9 (a wave-uniform scalar test); without it a
  // tap index of 9 would load real shifted pixels, and 0 * Inf in the product would turn into NaN
  if (k0 >= kend) {
#pragma unroll
    for (int j = 0; j < ImRows<ROWS, NW>::NI; ++j) dma16(rs, slot + (j * NW + wave) * 1024, kOOB);
    return;
  }
  // wave-uniform per K-step: tap, channel base, pixel shift
  const int tap = fdiv(k0, g.dC), c0 = k0 - tap * g.C;
  const int ky = (tap * 11) >> 5, kx = tap - ky * 3;
  int dy = ky - 1, dx = kx - 1;
  if constexpr (MODE == MODE_IM2COL_BWD) { dy = -dy; dx = -dx; }
  const int shift = ((dy * g.W + dx) * g.C + c0) * 2;
#pragma unroll
  for (int j = 0; j < ImRows<ROWS, NW>::NI; ++j) {
    const int hh = (ir.hw[j] >> 16) + dy, ww = (ir.hw[j] & 0xffff) + dx;
    const bool ok = (unsigned)hh < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
    dma16(rs, slot + (j * NW + wave) * 1024, ok ? ir.base[j] + (unsigned)shift : kOOB);
  }
}

// im2col N-contig operand of the weight gradient (k-rows = pixels, columns = (tap, channel)) when the image
// width divides 64: a lane's column, hence its tap shift, channel and column bounds, is fixed for the tile,
// and so is its pixel's w (k0 is a multiple of 64, so of W); per K-step only h = (k0 / W + kr / W) mod H and
// the K-tail test remain.  Two registers per wave-instruction: the byte offset relative to pixel k0, and
// kr | (kr / W) << 8 | (dy + 1) << 16 | column-valid << 24.  Offsets are exactly src_off's.
template <int ROWS, int NW>
struct ColRows {
  static constexpr int NI = ROWS / (8 * NW);
  unsigned base[NI];
  unsigned kv[NI];
};

template <int ROWS, int NW>
__device__ __forceinline__ void col_rows_init(ColRows<ROWS, NW>& cr, const ConvGeom& g, int col0, int ncols, int wave,
                                              int lane) {
  constexpr int ROWB = ROWS * 2;
  constexpr int CPR = ROWB / 16;
#pragma unroll
  for (int j = 0; j < ColRows<ROWS, NW>::NI; ++j) {
    const int inst = j * NW + wave;
    const int kr = inst * (1024 / ROWB) + lane / CPR;
    const int q = lane % CPR;
    const int L = (q >> 1) ^ tr_swz<ROWB>(kr);
    const int gr = col0 + L * 16 + (q & 1) * 8;
    const int tap = fdiv(gr, g.dC), c = gr - tap * g.C;
    const int ky = (tap * 11) >> 5, kx = tap - ky * 3;
    const int dy = ky - 1, dx = kx - 1;
    const int v = fdiv(kr, g.dW), w = kr - v * g.W;
    const bool ok = gr < ncols && tap < 9 && (unsigned)(w + dx) < (unsigned)g.W;
    cr.base[j] = (unsigned)(((kr + dy * g.W + dx) * g.C + c) * 2);
    cr.kv[j] = (unsigned)kr | ((unsigned)v << 8) | ((unsigned)(dy + 1) << 16) | ((unsigned)ok << 24);
  }
}

template <int ROWS, int NW>
__device__ __forceinline__ void stage_tile_col(__amdgpu_buffer_rsrc_t rs, char* slot, const ConvGeom& g,
                                               const ColRows<ROWS, NW>& cr, int k0, int kend, int wave) {
  const int pw0 = fdiv(k0, g.dW);                  // exact: W divides k0
  const int sH = pw0 - fdiv(pw0, g.dH) * g.H;      // h of pixel k0
  const unsigned kb = (unsigned)k0 * (unsigned)g.C * 2u;
  const int krem = kend - k0;
#pragma unroll
  for (int j = 0; j < ColRows<ROWS, NW>::NI; ++j) {
    const unsigned kv = cr.kv[j];
    const int t = sH + (int)((kv >> 8) & 0xffu);
    const int h = t - fdiv(t, g.dH) * g.H;
    const int hh = h + (int)((kv >> 16) & 3u) - 1;
    const bool ok = (kv >> 24) && (int)(kv & 0xffu) < krem && (unsigned)hh < (unsigned)g.H;
    dma16(rs, slot + (j * NW + wave) * 1024, ok ? kb + cr.base[j] : kOOB);
  }
}

// K-contig fragment (ds_read_b128 of the swizzled [row][64] image): an ordinary LDS load the compiler's
// waitcnt pass tracks.
template <int ROWS>
__device__ __forceinline__ bf16x8 frag_kc(const char* lds, int rbase, int kbase, int lane) {
  const int row = rbase + (lane & 15);
  const int chunk = (kbase >> 3) + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
}

// M/N-contig fragment: two ds_read_b64_tr_b16 of the [k][row] image, ISSUED here and settled by frag_settle.
// Inline asm, not __builtin_amdgcn_ds_read_tr16_b64: hipcc (ROCm 7.2) treats the builtin as a possible
// reader of every pending LDS-DMA write and puts an `s_waitcnt vmcnt(0)` in front of it, draining the
// stage that was just issued for t + STAGES - 1 and collapsing every >= 3-stage ring into a 1-stage one.
// The ring's own counted vmcnt + barrier order these reads against the DMA.
struct TrFrag {
  short4v lo, hi;
};

template <int ROWS>
__device__ __forceinline__ TrFrag frag_tr(const char* lds, int rbase, int kbase, int lane) {
  constexpr int ROWB = ROWS * 2;
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int chunk32 = rbase >> 4;
  const int k0 = kbase + 8 * g + q;
  const int k1 = k0 + 4;
  const int off0 = k0 * ROWB + ((chunk32 ^ tr_swz<ROWB>(k0)) << 5) + p * 8;
  const int off1 = k1 * ROWB + ((chunk32 ^ tr_swz<ROWB>(k1)) << 5) + p * 8;
  TrFrag f;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f.lo) : "v"((LDS_AS const char*)(lds + off0)) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f.hi) : "v"((LDS_AS const char*)(lds + off1)) : "memory");
  return f;
}

// The wait for a transposed fragment, in the SAME asm statement that redefines both of its halves: the
// compiler sees the halves' values come into existence only after `s_waitcnt lgkmcnt(0)`, so neither the
// combine below nor any copy or spill can read a VGPR the LDS read has not written yet (the asm outputs of
// frag_tr are otherwise "ready" the moment their asm line ends — round-2 advisor finding).  The first settle
// of a batch does the real wait; the rest find lgkmcnt already 0 (one issue cycle each).
__device__ __forceinline__ bf16x8 frag_settle(TrFrag& f) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f.lo), "+v"(f.hi) : : "memory");
  short8v v = {f.lo[0], f.lo[1], f.lo[2], f.lo[3], f.hi[0], f.hi[1], f.hi[2], f.hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Fragments of one K-slice for a wave: FA A-fragments (rows ra0 + 16 i) and FB B-fragments (rows rb0 + 16 j),
// every read issued before any wait; MFMAs are kept behind the settles.
template <int BMR, bool AKC, int FA, int BNR, bool BKC, int FB>
__device__ __forceinline__ void load_frags(const char* sa, int ra0, const char* sb, int rb0, int kk, int lane,
                                           bf16x8 (&a)[FA], bf16x8 (&b)[FB]) {
  TrFrag ta[AKC ? 1 : FA], tb[BKC ? 1 : FB];
#pragma unroll
  for (int i = 0; i < FA; ++i) {
    if constexpr (AKC) a[i] = frag_kc<BMR>(sa, ra0 + i * 16, kk, lane);
    else ta[i] = frag_tr<BMR>(sa, ra0 + i * 16, kk, lane);
  }
#pragma unroll
  for (int j = 0; j < FB; ++j) {
    if constexpr (BKC) b[j] = frag_kc<BNR>(sb, rb0 + j * 16, kk, lane);
    else tb[j] = frag_tr<BNR>(sb, rb0 + j * 16, kk, lane);
  }
  if constexpr (!AKC) {
#pragma unroll
    for (int i = 0; i < FA; ++i) a[i] = frag_settle(ta[i]);
  }
  if constexpr (!BKC) {
#pragma unroll
    for (int j = 0; j < FB; ++j) b[j] = frag_settle(tb[j]);
  }
  if constexpr (!AKC || !BKC) __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Ring hand-off words of the warp-specialised pipeline (LW loader waves): monotone per-slot counters in the
// kernel's one LDS array.  A poll is a relaxed workgroup-scope load in an s_sleep loop, bounded so that a
// broken hand-off ends the kernel (wrong results, caught by the tests) instead of spinning forever
// (~2^20 polls x 64 clocks ~ 30 ms; a healthy wait is well under 100 us).
__device__ __forceinline__ void lds_wait_ge(int* c, int target) {
  for (int it = 0; it < (1 << 20); ++it) {
    if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) break;
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");  // no LDS read of the slot moves above the poll
}

// s_waitcnt vmcnt(n) for a run-time n (the ring's tail), n <= 63
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  switch (n) {
#define DDPX_VMC(i) case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
    DDPX_VMC(0) DDPX_VMC(1) DDPX_VMC(2) DDPX_VMC(3) DDPX_VMC(4) DDPX_VMC(5) DDPX_VMC(6) DDPX_VMC(7)
    DDPX_VMC(8) DDPX_VMC(9) DDPX_VMC(10) DDPX_VMC(11) DDPX_VMC(12) DDPX_VMC(13) DDPX_VMC(14) DDPX_VMC(15)
    DDPX_VMC(16) DDPX_VMC(17) DDPX_VMC(18) DDPX_VMC(19) DDPX_VMC(20) DDPX_VMC(21) DDPX_VMC(22) DDPX_VMC(23)
    DDPX_VMC(24) DDPX_VMC(25) DDPX_VMC(26) DDPX_VMC(27) DDPX_VMC(28) DDPX_VMC(29) DDPX_VMC(30) DDPX_VMC(31)
    DDPX_VMC(32) DDPX_VMC(33) DDPX_VMC(34) DDPX_VMC(35) DDPX_VMC(36) DDPX_VMC(37) DDPX_VMC(38) DDPX_VMC(39)
    DDPX_VMC(40) DDPX_VMC(41) DDPX_VMC(42) DDPX_VMC(43) DDPX_VMC(44) DDPX_VMC(45) DDPX_VMC(46) DDPX_VMC(47)
#undef DDPX_VMC
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

__device__ __forceinline__ void lds_signal(int* c, int lane) {
  asm volatile("" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ---------------------------------------------------------------- epilogue
// The accumulator tile is staged through LDS as fp32 [BM][BN+4]; every thread
// then owns one 4-column quad (BN/4 quads, 256 % (BN/4) == 0) for rows
// r = t/(BN/4) + i*(256/(BN/4)) and moves 16-B vectors: all global operand
// loads of a thread are issued before any result is computed (the fused SGD
// epilogue reads p and momentum, the ReLU-mask epilogue reads aux).

template <int E>
__device__ __forceinline__ float epi_one(const Params& p, void* Cbase, size_t off, int n, float v, float lr,
                                         float cin, unsigned short auxv, float pv, float bv, float* p_out,
                                         float* b_out, float bias_n) {
  float stored;
  if constexpr (E == EPI_F32) {
    stored = v * p.alpha + cin;
  } else if constexpr (E == EPI_BF16 || E == EPI_BNSTAT_BF16) {
    stored = bf2f(f2bf(v * p.alpha + cin));
  } else if constexpr (E == EPI_BIAS_BF16) {  // alpha: dequant scale of the fp8 GEMMs (1 for bf16)
    stored = bf2f(f2bf(fmaf(v, p.alpha, bias_n)));
  } else if constexpr (E == EPI_BIAS_RELU_BF16) {
    stored = bf2f(f2bf(fmaxf(fmaf(v, p.alpha, bias_n), 0.f)));
  } else if constexpr (E == EPI_BIAS_F32) {
    stored = fmaf(v, p.alpha, bias_n);
  } else if constexpr (E == EPI_SGD) {
    stored = v * p.alpha;
    float d = fmaf(p.sgd.wd, pv, stored);
    if (p.sgd.mom != 0.f) {
      d = fmaf(p.sgd.mom, bv, d);
      *b_out = d;
    }
    *p_out = fmaf(-lr, d, pv);
  } else {  // EPI_RELUMASK_BF16
    const bool pos = (auxv & 0x8000u) == 0 && (auxv & 0x7fffu) != 0;
    stored = pos ? bf2f(f2bf(v * p.alpha)) : 0.f;
  }
  return stored;
}

template <int E, int BM, int BN, int NT = 256>
__device__ __forceinline__ void epilogue_vec(const Params& p, void* Cbase, const float* T, int m0, int n0, int tid,
                                             float (&csum)[4], const float* pf = nullptr) {
  constexpr int Q = BN / 4;           // column quads per row
  constexpr int RSTEP = NT / Q;       // rows between a thread's consecutive vectors
  constexpr int NV = BM / RSTEP;      // vectors per thread
  constexpr int TLD = BN + 4;
  const int cq = tid % Q, r0 = tid / Q;
  const int n = n0 + 4 * cq;
  const bool vec = (n + 3 < p.N) && ((p.ldc & 3) == 0);
  float lr = 0.f;
  if constexpr (E == EPI_SGD) lr = *p.sgd.lr;
  // the thread's 4 columns are fixed: their bias is loaded once, not per row (the stores to C may alias p.bias
  // as far as the compiler knows, so it re-loaded bias[n] for every element)
  constexpr bool HAS_BIAS = E == EPI_BIAS_BF16 || E == EPI_BIAS_RELU_BF16 || E == EPI_BIAS_F32;
  float bq[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (HAS_BIAS) {
    if (vec && !(reinterpret_cast<uintptr_t>(p.bias + n) & 15)) {
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(p.bias + n);
#pragma unroll
      for (int q = 0; q < 4; ++q) bq[q] = b4[q];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) bq[q] = n + q < p.N ? p.bias[n + q] : 0.f;
    }
  }
  // vectors whose loads are in flight together: the fused-SGD epilogue is a pure stream (p, momentum
  // in; p, momentum, shadow out) and needs every byte in flight it can get; the others stay at 4
  constexpr int CH = E == EPI_SGD ? (NV < 8 ? NV : 8) : (NV < 4 ? NV : 4);
#pragma unroll
  for (int i0 = 0; i0 < NV; i0 += CH) {
  f32x4 pin[CH], bin[CH], cin[CH];
  u32x2 ain[CH];
  // phase 1: issue every global load of this chunk
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int m = m0 + r0 + (i0 + i) * RSTEP;
    pin[i] = bin[i] = cin[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    ain[i] = (u32x2){0u, 0u};
    if (m >= p.M) continue;
    const size_t off = (size_t)m * p.ldc + n;
    if (vec) {
      if constexpr (E == EPI_SGD) {  // read-once / write-once streams: non-temporal (default)
        if (pf) {  // p / momentum tile prefetched into LDS during the main loop
          const int r = r0 + (i0 + i) * RSTEP;
          pin[i] = *reinterpret_cast<const f32x4*>(pf + r * BN + 4 * cq);
          bin[i] = *reinterpret_cast<const f32x4*>(pf + BM * BN + r * BN + 4 * cq);
        } else if (p.sgd_plain) {
          pin[i] = *reinterpret_cast<const f32x4*>(p.sgd.p + off);
          if (p.sgd.mom != 0.f) bin[i] = *reinterpret_cast<const f32x4*>(p.sgd.buf + off);
        } else {
          pin[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p.sgd.p + off));
          if (p.sgd.mom != 0.f) bin[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p.sgd.buf + off));
        }
      } else if constexpr (E == EPI_F32) {
        if (p.accumulate) cin[i] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(Cbase) + off);
      } else if constexpr (E == EPI_BF16) {
        if (p.accumulate) {
          const u32x2 c = *reinterpret_cast<const u32x2*>(reinterpret_cast<const unsigned short*>(Cbase) + off);
          cin[i] = (f32x4){__uint_as_float(c[0] << 16), __uint_as_float(c[0] & 0xffff0000u),
                           __uint_as_float(c[1] << 16), __uint_as_float(c[1] & 0xffff0000u)};
        }
      } else if constexpr (E == EPI_RELUMASK_BF16) {
        ain[i] = *reinterpret_cast<const u32x2*>(p.aux + (size_t)m * p.ldaux + n);
      }
    }
  }
  // phase 2: compute and store
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int r = r0 + (i0 + i) * RSTEP;
    const int m = m0 + r;
    if (m >= p.M) continue;
    const f32x4 v = *reinterpret_cast<const f32x4*>(T + r * TLD + 4 * cq);
    const size_t off = (size_t)m * p.ldc + n;
    if (vec) {
      float st[4], po[4], bo[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const unsigned short av = (unsigned short)((q & 1) ? (ain[i][q >> 1] >> 16) : (ain[i][q >> 1] & 0xffffu));
        st[q] = epi_one<E>(p, Cbase, off + q, n + q, v[q], lr, cin[i][q], av, pin[i][q], bin[i][q], &po[q], &bo[q],
                           bq[q]);
        csum[q] += st[q];
      }
      if constexpr (E == EPI_F32 || E == EPI_BIAS_F32) {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Cbase) + off) = (f32x4){st[0], st[1], st[2], st[3]};
      } else if constexpr (E == EPI_SGD) {
        if (p.sgd_plain) {
          *reinterpret_cast<f32x4*>(p.sgd.p + off) = (f32x4){po[0], po[1], po[2], po[3]};
          if (p.sgd.mom != 0.f) *reinterpret_cast<f32x4*>(p.sgd.buf + off) = (f32x4){bo[0], bo[1], bo[2], bo[3]};
        } else {
          __builtin_nontemporal_store((f32x4){po[0], po[1], po[2], po[3]}, reinterpret_cast<f32x4*>(p.sgd.p + off));
          if (p.sgd.mom != 0.f)
            __builtin_nontemporal_store((f32x4){bo[0], bo[1], bo[2], bo[3]}, reinterpret_cast<f32x4*>(p.sgd.buf + off));
        }
        if (p.sgd.shadow)
          *reinterpret_cast<u32x2*>(p.sgd.shadow + off) = (u32x2){pack_bf2(po[0], po[1]), pack_bf2(po[2], po[3])};
      } else {
        *reinterpret_cast<u32x2*>(reinterpret_cast<unsigned short*>(Cbase) + off) =
            (u32x2){pack_bf2(st[0], st[1]), pack_bf2(st[2], st[3])};
      }
    } else {
      // ragged right edge / odd leading dimension: scalar path
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (n + q >= p.N) continue;
        const size_t o = off + q;
        float c0 = 0.f, pv = 0.f, bv = 0.f;
        unsigned short av = 0;
        if constexpr (E == EPI_F32) { if (p.accumulate) c0 = reinterpret_cast<const float*>(Cbase)[o]; }
        if constexpr (E == EPI_BF16) { if (p.accumulate) c0 = bf2f(reinterpret_cast<const unsigned short*>(Cbase)[o]); }
        if constexpr (E == EPI_RELUMASK_BF16) av = p.aux[(size_t)m * p.ldaux + n + q];
        if constexpr (E == EPI_SGD) { pv = p.sgd.p[o]; if (p.sgd.mom != 0.f) bv = p.sgd.buf[o]; }
        float po = 0.f, bo = 0.f;
        const float st = epi_one<E>(p, Cbase, o, n + q, v[q], lr, c0, av, pv, bv, &po, &bo, bq[q]);
        csum[q] += st;
        if constexpr (E == EPI_F32 || E == EPI_BIAS_F32) {
          reinterpret_cast<float*>(Cbase)[o] = st;
        } else if constexpr (E == EPI_SGD) {
          p.sgd.p[o] = po;
          if (p.sgd.mom != 0.f) p.sgd.buf[o] = bo;
          if (p.sgd.shadow) p.sgd.shadow[o] = f2bf(po);
        } else {
          reinterpret_cast<unsigned short*>(Cbase)[o] = f2bf(st);
        }
      }
    }
  }
}  // chunk
}

// EPI_BNBWD_BF16: store g = bf16(acc) like EPI_BF16 and accumulate, per column, the BatchNorm backward sums of
// the block below over this thread's rows: dz = g at the window's first max of relu(a*y+b) (pooled) / at its own
// pixel, zeroed where a*y+b <= 0 (the routing and mask of bn_pool.hip's grad_z / grad_window, recomputed from y),
// s1 += dz, s2 += dz * (y - mean) * rstd.  The standalone reduce pass over g and y is gone (g never re-read).
template <int BM, int BN, int NT = 256>
__device__ __forceinline__ void epilogue_bnbwd(const Params& p, void* Cbase, const float* T, int m0, int n0, int tid,
                                               float (&s1)[4], float (&s2)[4]) {
  constexpr int Q = BN / 4, RSTEP = NT / Q, NV = BM / RSTEP, TLD = BN + 4;
  const int cq = tid % Q, r0 = tid / Q;
  const int n = n0 + 4 * cq;
  if (n + 3 >= p.N) return;  // the host requires N % 8 == 0: a quad is all in or all out
  float av[4], bv[4], mu[4], rs[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    av[q] = p.bn_a[n + q];
    bv[q] = p.bn_b[n + q];
    mu[q] = p.bn_mean[n + q];
    rs[q] = p.bn_rstd[n + q];
  }
  const int Ho = p.conv.H, Wo = p.conv.W;  // g's spatial size (the dgrad's im2col'd dy)
  const int ldy = p.N;
  // rows whose y loads are in flight together: 2 (8 VGPRs of y per row when pooled; the 8-wave dgrad tiles
  // already spill in their plain epilogue)
  constexpr int CH = NV < 2 ? NV : 2;
#pragma unroll
  for (int i0 = 0; i0 < NV; i0 += CH) {
    u32x2 yv[CH][4];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int m = m0 + r0 + (i0 + i) * RSTEP;
#pragma unroll
      for (int k = 0; k < 4; ++k) yv[i][k] = (u32x2){0u, 0u};
      if (m >= p.M) continue;
      if (p.bn_pool) {
        const int wo = m % Wo, t = m / Wo, ho = t % Ho, img = t / Ho;
        const size_t base = ((size_t)img * 2 * Ho + 2 * ho) * (2 * Wo) + 2 * wo;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          yv[i][k] = *reinterpret_cast<const u32x2*>(p.bn_y + (base + (k >> 1) * 2 * Wo + (k & 1)) * ldy + n);
      } else {
        yv[i][0] = *reinterpret_cast<const u32x2*>(p.bn_y + (size_t)m * ldy + n);
      }
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int r = r0 + (i0 + i) * RSTEP;
      const int m = m0 + r;
      if (m >= p.M) continue;
      const f32x4 v = *reinterpret_cast<const f32x4*>(T + r * TLD + 4 * cq);
      float g[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) g[q] = bf2f(f2bf(v[q] * p.alpha));
      *reinterpret_cast<u32x2*>(reinterpret_cast<unsigned short*>(Cbase) + (size_t)m * p.ldc + n) =
          (u32x2){pack_bf2(g[0], g[1]), pack_bf2(g[2], g[3])};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float ysel, zsel;
        if (p.bn_pool) {
          float best = -INFINITY;
          ysel = 0.f;
          zsel = 0.f;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const unsigned w = yv[i][k][q >> 1];
            const float yk = __uint_as_float((q & 1) ? (w & 0xffff0000u) : (w << 16));
            const float z = fmaf(av[q], yk, bv[q]);
            const float zr = fmaxf(z, 0.f);
            if (zr > best) { best = zr; ysel = yk; zsel = z; }  // strict: the first max wins, as torch
          }
        } else {
          const unsigned w = yv[i][0][q >> 1];
          ysel = __uint_as_float((q & 1) ? (w & 0xffff0000u) : (w << 16));
          zsel = fmaf(av[q], ysel, bv[q]);
        }
        const float dz = zsel > 0.f ? g[q] : 0.f;
        s1[q] += dz;
        s2[q] = fmaf(dz, (ysel - mu[q]) * rs[q], s2[q]);
      }
    }
  }
}

// Column reductions of the stored tile: thread (cq, r0) holds partial sums of 4 columns.
template <int BN, int NT = 256>
__device__ __forceinline__ void quad_colsum(float* red, const float (&cs)[4], int tid, float* out /* BN */) {
  constexpr int Q = BN / 4, RG = NT / Q;
  const int cq = tid % Q, rg = tid / Q;
#pragma unroll
  for (int q = 0; q < 4; ++q) red[rg * BN + 4 * cq + q] = cs[q];
  __syncthreads();
  if (tid < BN) {
    float s = 0.f;
    for (int g = 0; g < RG; ++g) s += red[g * BN + tid];
    out[tid] = s;
  }
  __syncthreads();
}

// NW = 4: 2x2 waves; NW = 8: 4 (M) x 2 (N) waves.  Wave tile (BM/WGM) x (BN/2).
// KSUB: 64-wide K sub-tiles per stage (one barrier per 64*KSUB of K).
// SGDPF (fused-SGD wgrad only): the tile's fp32 master / momentum rows are LDS-DMA'd into a side
// buffer during the main loop, so the optimizer epilogue only streams writes.
// LW > 0: warp-specialised ring.  LW extra LOADER waves (the last ones of the workgroup) issue every K-step's
// LDS-DMA and publish it (counted vmcnt, then a FULL counter per slot); the NW MATH waves wait on FULL, read
// their fragments, release the slot (FREE counter) and run the MFMAs.  No workgroup barrier in the main loop:
// the math waves never wait for each other, and the loaders run up to STAGES - 1 K-steps ahead of the slowest
// math wave (the barrier-coupled ring lets 8 waves meet at every K-step: 52 vs 77 GB/s of L2 -> LDS per CU on
// the 128x128 tile, profiles/r2_splitk).  The loaders end after the last publish; the math waves then run the
// combine and epilogue (an s_barrier waits only for waves that have not ended).
// The 2-deep rings of configs 21 - 23 are built for several workgroups per CU: held to that register budget
// (waves per SIMD).
template <int BM, int BN, int STAGES, int NW, int KSUB, int LW>
constexpr int pipe_waves_per_eu() {
  if (LW != 0 || KSUB != 1 || STAGES != 2) return 1;
  if (BM == 128 && BN == 128) return NW / 2;         // 64 KiB: 2 per CU
  if (BM == 256 && BN == 64 && NW == 4) return 2;    // 80 KiB: 2 per CU
  return 1;
}

template <int BM, int BN, int STAGES, bool AK, bool BKc, int AMODE, int BMODE, int NW = 4, int KSUB = 1,
          bool SGDPF = false, bool SK = false, int LW = 0>
__global__ void __launch_bounds__((NW + LW) * 64)
__attribute__((amdgpu_waves_per_eu(pipe_waves_per_eu<BM, BN, STAGES, NW, KSUB, LW>())))
gemm_pipe_kernel(Params p) {
  constexpr int NT = NW * 64;
  constexpr int WGM = NW / 2;
  constexpr int BK = 64 * KSUB;
  constexpr int A_SUB = BM * 64 * 2, B_SUB = BN * 64 * 2;
  constexpr int A_BYTES = A_SUB * KSUB, B_BYTES = B_SUB * KSUB;
  constexpr int SLOT = A_BYTES + B_BYTES;
  constexpr int FM = BM / WGM / 16, FN = BN / 32;
  constexpr int LPW = KSUB * (BM + BN) / (8 * NW);  // DMA instructions per wave per stage
  constexpr int PF_BYTES = SGDPF ? 2 * BM * BN * 4 : 0;
  constexpr int PF_CPR = BN / 4, PF_RPI = 64 / PF_CPR;      // 16-B chunks per row, rows per wave-instruction
  constexpr int PF_PER_WAVE = SGDPF ? (BM / PF_RPI) / NW : 0;  // per array
  constexpr int PFW = 2 * PF_PER_WAVE;                        // prefetch DMA ops per wave
  static_assert(!SGDPF || (BM % (PF_RPI * NW) == 0 && 64 % PF_CPR == 0), "prefetch geometry");
  static_assert(LW == 0 || (!SGDPF && KSUB == 1 && AMODE == MODE_PLAIN && BMODE == MODE_PLAIN && STAGES <= 8),
                "warp-specialised ring: plain operands, one 64-deep K sub-tile per slot");
  constexpr int FLAG_BYTES = LW ? 64 : 0;  // FULL[8], FREE[8]
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * SLOT + PF_BYTES + FLAG_BYTES];
  int* const ring_full = reinterpret_cast<int*>(smem + STAGES * SLOT + PF_BYTES);
  int* const ring_free = ring_full + 8;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // wm in [0, WGM)
  stamp_at(p, tid, 0);

  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.N + BN - 1) / BN;
  // XCD-aware (tile, split) order.  With split-K the grid's linear workgroup id is remapped over ALL
  // workgroups, split-major: each XCD then owns whole K ranges (all tiles of a few splits), so a
  // split's slice of both operands is fetched from HBM into one XCD's L2 and reused by its tiles there.
  // Remapping only within a split spread every split's tiles over all 8 XCDs, and every XCD re-read
  // every split's slice (8x the HBM traffic on the conv weight-gradient GEMMs).
  const int ntiles = tiles_m * tiles_n;
  int wg, split;
  if (gridDim.y > 1) {
    const int lg = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, ntiles * gridDim.y);
    split = lg / ntiles;
    wg = lg - split * ntiles;
  } else {
    wg = xcd_remap(blockIdx.x, ntiles);
    split = 0;
  }
  const int tm = wg % tiles_m, tn = wg / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;

  const int kbeg = p.klen ? split * p.klen : 0;
  const int kend = p.klen ? min(p.K, kbeg + p.klen) : p.K;
  void* Cbase = p.C;
  if (p.klen && !SK) Cbase = reinterpret_cast<char*>(p.C) + (size_t)split * p.split_stride * (p.epi == EPI_F32 ? 4 : 2);

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, 0, p.b_bytes, 0x00020000);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + BK - 1) / BK;

  // im2col A operand with whole taps per K-step: row addressing cached for the tile (ImRows)
  constexpr bool A_IM = AK && (AMODE == MODE_IM2COL_FWD || AMODE == MODE_IM2COL_BWD);
  ImRows<A_IM ? BM : 8 * NW, NW> arow;
  const bool a_fast = A_IM && !p.im_slow && (p.conv.C & 63) == 0;
  if constexpr (A_IM) {
    if (a_fast) im_rows_init<BM, NW>(arow, p.conv, m0, p.M, wave, lane);
  }
  // weight-gradient im2col B operand with an image width dividing 64: column addressing cached (ColRows)
  constexpr bool B_COL = !BKc && BMODE == MODE_IM2COL_COL;
  ColRows<B_COL ? BN : 8 * NW, NW> bcol;
  const bool b_fast = B_COL && !p.im_slow && (64 % p.conv.W) == 0;
  if constexpr (B_COL) {
    if (b_fast) col_rows_init<BN, NW>(bcol, p.conv, n0, p.N, wave, lane);
  }

  auto issue = [&](int t) {
    char* slot = smem + (t % STAGES) * SLOT;
#pragma unroll
    for (int u = 0; u < KSUB; ++u) {
      const int k0 = kbeg + t * BK + u * 64;
      if constexpr (A_IM) {
        if (a_fast) stage_tile_im<BM, AMODE, NW>(ra, slot + u * A_SUB, p.conv, arow, k0, kend, wave);
        else stage_tile<BM, AK, AMODE, NW>(ra, slot + u * A_SUB, p.conv, p.lda, m0, p.M, k0, kend, wave, lane);
      } else {
        stage_tile<BM, AK, AMODE, NW>(ra, slot + u * A_SUB, p.conv, p.lda, m0, p.M, k0, kend, wave, lane);
      }
      if constexpr (B_COL) {
        if (b_fast) stage_tile_col<BN, NW>(rb, slot + A_BYTES + u * B_SUB, p.conv, bcol, k0, kend, wave);
        else stage_tile<BN, BKc, BMODE, NW>(rb, slot + A_BYTES + u * B_SUB, p.conv, p.ldb, n0, p.N, k0, kend, wave, lane);
      } else {
        stage_tile<BN, BKc, BMODE, NW>(rb, slot + A_BYTES + u * B_SUB, p.conv, p.ldb, n0, p.N, k0, kend, wave, lane);
      }
    }
  };

  auto prefetch_sgd = [&]() {
    if constexpr (SGDPF) {
      char* pfb = smem + STAGES * SLOT;
      const unsigned nbytes = (unsigned)((size_t)p.M * p.ldc * 4);
#pragma unroll
      for (int arr = 0; arr < 2; ++arr) {
        const float* src = (arr && p.sgd.buf) ? p.sgd.buf : p.sgd.p;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, nbytes, 0x00020000);
#pragma unroll
        for (int j = 0; j < PF_PER_WAVE; ++j) {
          const int inst = j * NW + wave;
          const int r = inst * PF_RPI + lane / PF_CPR, c = lane % PF_CPR;
          const int gm = m0 + r, gn = n0 + 4 * c;
          const unsigned voff = (gm < p.M && gn + 3 < p.N) ? (unsigned)(((size_t)gm * p.ldc + gn) * 4) : kOOB;
          dma16(rs, pfb + arr * BM * BN * 4 + inst * 1024, voff);
        }
      }
    }
  };

  auto mma_slot = [&](int t) {
    const char* sa0 = smem + (t % STAGES) * SLOT;
    const char* sb0 = sa0 + A_BYTES;
#pragma unroll
    for (int k2 = 0; k2 < BK; k2 += 32) {
      const int u = k2 >> 6, kk = k2 & 63;
      const char* sa = sa0 + u * A_SUB;
      const char* sb = sb0 + u * B_SUB;
      bf16x8 a[FM], b[FN];
      load_frags<BM, AK, FM, BN, BKc, FN>(sa, wm * (BM / WGM), sb, wn * (BN / 2), kk, lane, a, b);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };

  if constexpr (LW > 0) {
    if (tid < 16) ring_full[tid] = 0;  // FULL[0..7], FREE[0..7]
    __syncthreads();
    if (wave >= NW) {
      // ------------------------------------------------------------ loader waves
      const int lw = wave - NW;
      constexpr int LPL = (BM + BN) / (8 * LW);  // LDS-DMA instructions per loader wave per K-step
      // K-steps kept in flight before one is published: STAGES - 2 (one slot of slack for the math waves)
      constexpr int D = STAGES > 2 ? STAGES - 2 : 1;
      static_assert(D * LPL <= 47, "vmcnt range");
      for (int t = 0; t < nk; ++t) {
        const int sl = t % STAGES;
        if (t >= STAGES) lds_wait_ge(ring_free + sl, (t / STAGES) * NW);  // every math wave read step t - STAGES
        char* slot = smem + sl * SLOT;
        const int k0 = kbeg + t * 64;
        stage_tile<BM, AK, AMODE, LW>(ra, slot, p.conv, p.lda, m0, p.M, k0, kend, lw, lane);
        stage_tile<BN, BKc, BMODE, LW>(rb, slot + A_BYTES, p.conv, p.ldb, n0, p.N, k0, kend, lw, lane);
        if (t >= D) {  // this wave's share of step t - D has landed (D younger steps may still fly): publish it
          wait_vmcnt<D * LPL>();
          lds_signal(ring_full + (t - D) % STAGES, lane);
        }
      }
      for (int j = nk > D ? nk - D : 0; j < nk; ++j) {  // the last D steps, oldest first
        wait_vmcnt_rt((nk - 1 - j) * LPL);
        lds_signal(ring_full + j % STAGES, lane);
      }
      return;
    }
    // --------------------------------------------------------------- math waves
    for (int t = 0; t < nk; ++t) {
      const int sl = t % STAGES;
      lds_wait_ge(ring_full + sl, (t / STAGES + 1) * LW);
      mma_slot(t);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the slot are done
      lds_signal(ring_free + sl, lane);
    }
  } else {
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s);

  for (int t = 0; t < nk; ++t) {
    const int ahead = min(STAGES - 2, nk - 1 - t);
    // stages 1..STAGES-1 were issued before the prefetch (t = 0): its PFW ops are younger than them
    const bool pf_young = SGDPF && t >= 1 && t <= STAGES - 1;
    // deep rings (configs 24 / 25: 6 stages) keep up to STAGES - 2 younger stages in flight past the barrier
    if (STAGES >= 6 && !SGDPF && ahead >= 4) wait_vmcnt<(STAGES >= 6 ? 4 : 0) * LPW>();
    else if (STAGES >= 5 && !SGDPF && ahead >= 3) wait_vmcnt<(STAGES >= 5 ? 3 : 0) * LPW>();
    else if (ahead >= 2) { if (pf_young) wait_vmcnt<2 * LPW + PFW>(); else wait_vmcnt<2 * LPW>(); }
    else if (ahead == 1) { if (pf_young) wait_vmcnt<LPW + PFW>(); else wait_vmcnt<LPW>(); }
    else { if (pf_young) wait_vmcnt<PFW>(); else wait_vmcnt<0>(); }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1);
    if (t == 0) prefetch_sgd();
    mma_slot(t);
  }
  }

  stamp_at(p, tid, 1);
  // ---- in-launch split-K combine (cdna_hip_programming §5 "Projection GEMM" item 2, sc1 form) ----
  if constexpr (SK) {
    constexpr int NF = FM * FN;
    const int S = gridDim.y;
    const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc((void*)p.slab, 0, p.slab_bytes, 0x00020000);
    // slab (split, tile): NF blocks of NT x 16 B, lane-linear -> every store / load is a whole 1 KiB per wave
    auto slab_off = [&](int sp, int f) -> unsigned {
      return (unsigned)((((size_t)(sp * ntiles + wg) * NF + f) * NT + tid) * 16);
    };
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rsl, slab_off(split, i * FN + j),
                                               0, 16 /* sc1: write-through */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the ticket
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (tid == 0) *flag = __hip_atomic_fetch_add(p.tcnt + wg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    stamp_at(p, tid, 2);
    if (*flag != S - 1) return;  // not the last split of this tile
    if (tid == 0) __hip_atomic_store(p.tcnt + wg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // sum in split order, every partial (this split's too) read back from its slab: the same bits whichever split
    // arrives last, and the accumulators are the running sum (no second tile of registers: the 8-wave tiles
    // would spill); one split's fragments are in flight together
    for (int sp = 0; sp < S; ++sp) {
      f32x4 v[FM][FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          v[i][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsl, slab_off(sp, i * FN + j), 0,
                                                                                    16 /* sc1 */));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = sp == 0 ? v[i][j] : acc[i][j] + v[i][j];
    }
    stamp_at(p, tid, 3);
  }

  // ---- stage the accumulator tile through LDS (all DMA has landed: last wait was vmcnt(0)) ----
  // The fp32 tile is staged through LDS in EH row-parts when BM x BN does not fit beside the
  // reduction scratch (256x256: 4 parts of 64 rows): waves owning the part's rows write it, every
  // thread runs the epilogue on it.
  constexpr int TLD = BN + 4;
  constexpr int SCR = (NT / (BN / 4) + 2) * BN * 4;
  constexpr int EH = (BM * TLD * 4 + SCR <= STAGES * SLOT) ? 1 : ((BM / 2) * TLD * 4 + SCR <= STAGES * SLOT) ? 2 : 4;
  static_assert(WGM % EH == 0, "epilogue parts must align with wave rows");
  constexpr int BMH = BM / EH;
  constexpr int WPH = WGM / EH;  // wave rows per half
  float* T = reinterpret_cast<float*>(smem);
  static_assert(BMH * TLD * 4 + SCR <= STAGES * SLOT, "epilogue LDS overflow");
  static_assert(EH == 1 || !SGDPF, "prefetch needs a single-pass epilogue");
  if constexpr (SGDPF) wait_vmcnt<0>();  // the prefetch (if the loop ended before waiting on it)
  float* red = T + BMH * TLD;
  float* colres = red + (NT / (BN / 4)) * BN;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  float st_n = 0.f, st_mean = 0.f, st_m2 = 0.f;  // EPI_BNSTAT: the tile's statistics merged over its row parts
#pragma unroll
  for (int h = 0; h < EH; ++h) {
    if (h == 0) __builtin_amdgcn_s_barrier();  // every wave is done reading the last LDS slot
    else __syncthreads();                      // the previous half's epilogue is done with T
    if (wm / WPH == h) {
      const int mr = (wm % WPH) * (BM / WGM) + 4 * (lane >> 4);
      const int nc = wn * (BN / 2) + (lane & 15);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) T[(mr + i * 16 + r) * TLD + nc + j * 16] = acc[i][j][r];
    }
    __syncthreads();
    const int mh = m0 + h * BMH;
    float ch[4] = {0.f, 0.f, 0.f, 0.f};
    switch (p.epi) {
      case EPI_F32: epilogue_vec<EPI_F32, BMH, BN, NT>(p, Cbase, T, mh, n0, tid, ch); break;
      case EPI_BF16: epilogue_vec<EPI_BF16, BMH, BN, NT>(p, Cbase, T, mh, n0, tid, ch); break;
      case EPI_BIAS_BF16: epilogue_vec<EPI_BIAS_BF16, BMH, BN, NT>(p, Cbase, T, mh, n0, tid, ch); break;
      case EPI_BIAS_RELU_BF16: epilogue_vec<EPI_BIAS_RELU_BF16, BMH, BN, NT>(p, Cbase, T, mh, n0, tid, ch); break;
      case EPI_BIAS_F32: epilogue_vec<EPI_BIAS_F32, BMH, BN, NT>(p, Cbase, T, mh, n0, tid, ch); break;
      case EPI_SGD:  // (not instantiated in the warp-specialised kernels: their register budget is 168)
        if constexpr (LW == 0)
          epilogue_vec<EPI_SGD, BMH, BN, NT>(p, Cbase, T, mh, n0, tid, ch,
                                             SGDPF ? reinterpret_cast<const float*>(smem + STAGES * SLOT) : nullptr);
        break;
      case EPI_BNSTAT_BF16:
        if constexpr (LW == 0) epilogue_vec<EPI_BNSTAT_BF16, BMH, BN, NT>(p, Cbase, T, mh, n0, tid, ch);
        break;
      case EPI_BNBWD_BF16:
        // conv data-gradient kernels, only the tiles where the fused sums measured faster than the separate
        // reduce pass (256x128 / 3 stages and 128x128 / 4 or 2 stages / 8 waves, profiles/r5_vgg/NOTES.md): the
        // others do not carry the epilogue's registers
        if constexpr (LW == 0 && AMODE == MODE_IM2COL_BWD &&
                      ((NW == 8 && BM == 256 && BN == 128 && STAGES == 3) ||
                       (NW == 8 && BM == 128 && BN == 128 && STAGES != 3))) {
          // (256x64 / cfg 23 measured 129 -> 190 us with it, more than the 35 us reduce it removes)
          float s2[4] = {0.f, 0.f, 0.f, 0.f};
          epilogue_bnbwd<BMH, BN, NT>(p, Cbase, T, mh, n0, tid, ch, s2);
          __syncthreads();
          quad_colsum<BN, NT>(red, ch, tid, colres);
          const size_t st = (size_t)tm * EH + h;
          if (tid < BN && n0 + tid < p.N) p.colsum[(st * 2) * p.N + n0 + tid] = colres[tid];
          quad_colsum<BN, NT>(red, s2, tid, colres);
          if (tid < BN && n0 + tid < p.N) p.colsum[(st * 2 + 1) * p.N + n0 + tid] = colres[tid];
#pragma unroll
          for (int q = 0; q < 4; ++q) ch[q] = 0.f;
        }
        break;
      default: epilogue_vec<EPI_RELUMASK_BF16, BMH, BN, NT>(p, Cbase, T, mh, n0, tid, ch); break;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) cs[q] += ch[q];
    if (LW == 0 && p.colsum && p.epi == EPI_BNSTAT_BF16) {
      // BatchNorm statistics of the stored (bf16-rounded) values of the BMH-row part: its mean, then M2 = sum
      // (y - mean)^2 over its rows; the parts are Chan-merged in order in registers and the tile writes ONE
      // statistics row (tm): a quarter / half of the tiles to merge for the 256x256 / 2-deep 128x128 tiles
      __syncthreads();
      quad_colsum<BN, NT>(red, ch, tid, colres);
      const int rows_valid = min(BMH, p.M - mh);
      float* tmean = colres + BN;
      if (tid < BN) tmean[tid] = rows_valid > 0 ? colres[tid] / (float)rows_valid : 0.f;
      __syncthreads();
      {
        constexpr int Q = BN / 4, RSTEP = NT / Q, NV = BMH / RSTEP;
        const int cq = tid % Q, r0 = tid / Q;
        float m2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int r = r0 + i * RSTEP;
          if (mh + r >= p.M) continue;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float y = bf2f(f2bf(T[r * TLD + 4 * cq + q] * p.alpha));
            const float d = y - tmean[4 * cq + q];
            m2[q] += d * d;
          }
        }
        quad_colsum<BN, NT>(red, m2, tid, colres);
      }
      if (tid < BN) {
        const float nb = (float)max(rows_valid, 0);
        if (nb > 0.f) {
          const float mb = tmean[tid], qb = colres[tid];
          if (st_n == 0.f) {
            st_n = nb;
            st_mean = mb;
            st_m2 = qb;
          } else {
            const float nn = st_n + nb, d = mb - st_mean;
            st_mean += d * (nb / nn);
            st_m2 += qb + d * d * (st_n * nb / nn);
            st_n = nn;
          }
        }
        if (h == EH - 1 && n0 + tid < p.N) {
          p.colsum[((size_t)tm * 2) * p.N + n0 + tid] = st_mean;
          p.colsum[((size_t)tm * 2 + 1) * p.N + n0 + tid] = st_m2;
        }
      }
    }
  }
  stamp_at(p, tid, 4);
  if (!p.colsum || p.epi == EPI_BNSTAT_BF16 || p.epi == EPI_BNBWD_BF16) return;

  // ---- per-tile column sums (bias gradient) ----
  __syncthreads();
  quad_colsum<BN, NT>(red, cs, tid, colres);
  if ((NW != 4 && LW == 0) || !p.cs_tcnt) {  // (the in-launch finish is built for the 4-wave tiles and the
                                            // warp-specialised ones: it adds spills to the register-bound
                                            // barrier-coupled 8-wave ones, which no dgrad picks)
    if (tid < BN && n0 + tid < p.N) p.colsum[(size_t)tm * p.N + n0 + tid] = colres[tid];
    return;
  }
  // in-launch finish (MI355X_MICROARCH.md "Valid forms", row 1): sc1 partials, drained, then the column
  // tile's ticket; the last row tile reads every partial with sc1 loads, in row-tile order
  if (tid < BN && n0 + tid < p.N)
    __hip_atomic_store(p.colsum + (size_t)tm * p.N + n0 + tid, colres[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* csflag = reinterpret_cast<int*>(colres + BN);
  if (tid == 0)
    *csflag = __hip_atomic_fetch_add(p.cs_tcnt + tn, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tiles_m - 1;
  __syncthreads();
  if (!*csflag) return;
  if (tid == 0) __hip_atomic_store(p.cs_tcnt + tn, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid >= BN || n0 + tid >= p.N) return;
  const __amdgpu_buffer_rsrc_t rcs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.colsum, 0, (unsigned)((size_t)tiles_m * p.N * 4), 0x00020000);
  // fused bias SGD: master / momentum / lr loads go out with the partials' (one round trip, not two)
  float pv = 0.f, mv = 0.f, lrv = 0.f;
  if (p.sgd.p) {
    pv = __builtin_nontemporal_load(p.sgd.p + n0 + tid);
    if (p.sgd.mom != 0.f) mv = __builtin_nontemporal_load(p.sgd.buf + n0 + tid);
    lrv = *p.sgd.lr;
  }
  float tot = 0.f;
  for (int t0 = 0; t0 < tiles_m; t0 += 8) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)  // all in flight together; rows past tiles_m read zeros (bounds check)
      v[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          rcs, (unsigned)(((size_t)(t0 + q) * p.N + n0 + tid) * 4), 0, 16 /* sc1 */));
#pragma unroll
    for (int q = 0; q < 8; ++q) tot += v[q];
  }
  const int n = n0 + tid;
  if (p.sgd.p) {
    sgd_apply_pre(p.sgd, n, tot, lrv, pv, mv);
  } else if (p.cs_flags & 1) {
    unsigned short* o = reinterpret_cast<unsigned short*>(p.cs_out) + n;
    *o = f2bf((p.cs_flags & 2) ? tot + bf2f(*o) : tot);
  } else {
    float* o = reinterpret_cast<float*>(p.cs_out) + n;
    *o = (p.cs_flags & 2) ? tot + *o : tot;
  }
}

template <int BM, int BN, int STAGES, bool AK, bool BKc, int AMODE, int BMODE, int NW = 4, int KSUB = 1,
          bool SGDPF = false, bool SK = false, int LW = 0>
static hipError_t launch(const Params& p, int splits, hipStream_t s) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_pipe_kernel<BM, BN, STAGES, AK, BKc, AMODE, BMODE, NW, KSUB, SGDPF, SK, LW>),
                     dim3(tiles, splits), dim3((NW + LW) * 64), 0, s, p);
  return hipGetLastError();
}

// cfg 16 - 20: warp-specialised rings (LW = 4 loader waves) for the M = 512-row products
constexpr int kNumCfgs = 26;
// 8-wave configs whose register budget has no room for the in-launch column-sum finish
static inline bool eight_wave(int cfg) {
  return cfg == 8 || cfg == 13 || cfg == 14 || cfg == 15 || cfg == 22 || cfg == 25;
}

// Row-parts the epilogue stages the tile in (the data gradient's BatchNorm backward sums come out per part; the
// forward statistics are merged to one row per tile).
static inline int epilogue_halves(int cfg) { return cfg == 13 ? 4 : (cfg == 21 || cfg == 22) ? 2 : 1; }

static inline void tile_of(int cfg, int* bm, int* bn) {
  static const int t[kNumCfgs][2] = {{128, 128}, {64, 128}, {128, 64}, {64, 64},  {128, 128}, {64, 128}, {128, 64},
                                     {64, 64},   {256, 128}, {64, 64},  {64, 128}, {128, 64}, {64, 64},  {256, 256},
                                     {128, 128}, {128, 128}, {256, 128}, {128, 128}, {64, 128}, {128, 64},
                                     {64, 64},   {128, 128}, {128, 128}, {256, 64}, {128, 64}, {128, 64}};
  const int c = (cfg >= 0 && cfg < kNumCfgs) ? cfg : 7;
  *bm = t[c][0];
  *bn = t[c][1];
}

template <bool AK, bool BKc, int AMODE, int BMODE>
static hipError_t dispatch(const Params& p, int cfg, int splits, hipStream_t s) {
  switch (cfg) {
    case 8: return launch<256, 128, 3, AK, BKc, AMODE, BMODE, 8>(p, splits, s);  // 8 waves, 144 KiB LDS
    case 9: return launch<64, 64, 3, AK, BKc, AMODE, BMODE, 4, 2>(p, splits, s);  // BK 128, 96 KiB
    case 10: return launch<64, 128, 2, AK, BKc, AMODE, BMODE, 4, 2>(p, splits, s); // BK 128, 96 KiB
    case 11: return launch<128, 64, 2, AK, BKc, AMODE, BMODE, 4, 2>(p, splits, s); // BK 128, 96 KiB
    case 12: return launch<64, 64, 2, AK, BKc, AMODE, BMODE, 4, 2>(p, splits, s);  // BK 128, 64 KiB (2 WG/CU)
    case 13: return launch<256, 256, 2, AK, BKc, AMODE, BMODE, 8>(p, splits, s);   // 8 waves, 64x128 each, 128 KiB
    case 14: return launch<128, 128, 3, AK, BKc, AMODE, BMODE, 8>(p, splits, s);   // 8 waves, 32x64 each, 96 KiB
    case 15: return launch<128, 128, 4, AK, BKc, AMODE, BMODE, 8>(p, splits, s);   // 8 waves, 32x64 each, 128 KiB
    // 128x128 with a 2-deep ring (64 KiB): two workgroups per CU, one's epilogue / ring fill under the other's loop
    case 21: return launch<128, 128, 2, AK, BKc, AMODE, BMODE, 4>(p, splits, s);   // 4 waves, 64x64 each
    case 22: return launch<128, 128, 2, AK, BKc, AMODE, BMODE, 8>(p, splits, s);   // 8 waves, 32x64 each
    // narrow (N = 64) products: 256x64, 2-deep (80 KiB, 2 per CU), 4 waves of 128x32 (8 waves would need 128
    // VGPRs each and spilled)
    case 23: return launch<256, 64, 2, AK, BKc, AMODE, BMODE, 4>(p, splits, s);
    // one 128x64 tile per CU at M = 512 (256 tiles: 25 % fewer operand bytes per CU than two 64x64 tiles) on a
    // barrier-coupled 6 x 24 KiB ring: 5 K-steps (120 KiB) of LDS-DMA in flight per CU, against config 12's 64 KiB
    // (PMC, profiles/r6_gemm: config 12's waves wait 53 % of their cycles with the TA path 53 % busy)
    case 24: return launch<128, 64, 6, AK, BKc, AMODE, BMODE, 4>(p, splits, s);  // 4 waves, 64x32 each
    case 25: return launch<128, 64, 6, AK, BKc, AMODE, BMODE, 8>(p, splits, s);  // 8 waves, 32x32 each
    case 16:  // warp-specialised (plain operands only)
      if constexpr (AMODE == MODE_PLAIN && BMODE == MODE_PLAIN)
        return launch<256, 128, 3, AK, BKc, AMODE, BMODE, 8, 1, false, false, 4>(p, splits, s);
      return hipErrorInvalidValue;
    case 17:
      if constexpr (AMODE == MODE_PLAIN && BMODE == MODE_PLAIN)
        return launch<128, 128, 4, AK, BKc, AMODE, BMODE, 4, 1, false, false, 4>(p, splits, s);
      return hipErrorInvalidValue;
    // one tile per CU at M = 512 (256 tiles), 6 x 24 KiB ring: 5 K-steps of LDS-DMA in flight per CU
    case 18:
      if constexpr (AMODE == MODE_PLAIN && BMODE == MODE_PLAIN)
        return launch<64, 128, 6, AK, BKc, AMODE, BMODE, 4, 1, false, false, 4>(p, splits, s);
      return hipErrorInvalidValue;
    case 19:
      if constexpr (AMODE == MODE_PLAIN && BMODE == MODE_PLAIN)
        return launch<128, 64, 6, AK, BKc, AMODE, BMODE, 4, 1, false, false, 4>(p, splits, s);
      return hipErrorInvalidValue;
    // the 64x64 tile (two per CU) with a 4 x 16 KiB warp-specialised ring
    case 20:
      if constexpr (AMODE == MODE_PLAIN && BMODE == MODE_PLAIN)
        return launch<64, 64, 4, AK, BKc, AMODE, BMODE, 4, 1, false, false, 4>(p, splits, s);
      return hipErrorInvalidValue;
    case 0: return launch<128, 128, 4, AK, BKc, AMODE, BMODE>(p, splits, s);  // 128 KiB LDS, 1 WG/CU
    case 1: return launch<64, 128, 4, AK, BKc, AMODE, BMODE>(p, splits, s);   //  96 KiB
    case 2: return launch<128, 64, 4, AK, BKc, AMODE, BMODE>(p, splits, s);   //  96 KiB
    case 3: return launch<64, 64, 4, AK, BKc, AMODE, BMODE>(p, splits, s);    //  64 KiB, 2 WG/CU
    case 4: return launch<128, 128, 3, AK, BKc, AMODE, BMODE>(p, splits, s);  //  96 KiB
    case 5: return launch<64, 128, 3, AK, BKc, AMODE, BMODE>(p, splits, s);   //  72 KiB, 2 WG/CU
    case 6: return launch<128, 64, 3, AK, BKc, AMODE, BMODE>(p, splits, s);   //  72 KiB, 2 WG/CU
    default: return launch<64, 64, 3, AK, BKc, AMODE, BMODE>(p, splits, s);   //  48 KiB, 3 WG/CU
  }
}

// In-launch split-K variants (Params.slab / tcnt / klen set, gridDim.y = splits >= 2).
template <bool AK, bool BKc>
static hipError_t dispatch_sk(const Params& p, int cfg, int splits, hipStream_t s) {
  switch (cfg) {
    case 0: return launch<128, 128, 4, AK, BKc, MODE_PLAIN, MODE_PLAIN, 4, 1, false, true>(p, splits, s);
    case 5: return launch<64, 128, 3, AK, BKc, MODE_PLAIN, MODE_PLAIN, 4, 1, false, true>(p, splits, s);
    case 6: return launch<128, 64, 3, AK, BKc, MODE_PLAIN, MODE_PLAIN, 4, 1, false, true>(p, splits, s);
    case 10: return launch<64, 128, 2, AK, BKc, MODE_PLAIN, MODE_PLAIN, 4, 2, false, true>(p, splits, s);
    case 8: return launch<256, 128, 3, AK, BKc, MODE_PLAIN, MODE_PLAIN, 8, 1, false, true>(p, splits, s);
    case 14: return launch<128, 128, 3, AK, BKc, MODE_PLAIN, MODE_PLAIN, 8, 1, false, true>(p, splits, s);
    case 15: return launch<128, 128, 4, AK, BKc, MODE_PLAIN, MODE_PLAIN, 8, 1, false, true>(p, splits, s);
    // warp-specialised: 8 math waves (64x64 each) + 4 loaders, 3 x 48 KiB ring / 4 math waves + 4 loaders
    case 16: return launch<256, 128, 3, AK, BKc, MODE_PLAIN, MODE_PLAIN, 8, 1, false, true, 4>(p, splits, s);
    case 17: return launch<128, 128, 4, AK, BKc, MODE_PLAIN, MODE_PLAIN, 4, 1, false, true, 4>(p, splits, s);
    default: return hipErrorInvalidValue;
  }
}

// Fused-SGD weight-gradient tiles with the master/momentum prefetch (plain A/B layouts only).
// Returns hipErrorInvalidValue for configs without a prefetch variant.
template <bool AK, bool BKc>
static hipError_t dispatch_sgd_prefetch(const Params& p, int cfg, hipStream_t s) {
  switch (cfg) {
    case 3: return launch<64, 64, 4, AK, BKc, MODE_PLAIN, MODE_PLAIN, 4, 1, true>(p, 1, s);   //  96 KiB
    case 5: return launch<64, 128, 3, AK, BKc, MODE_PLAIN, MODE_PLAIN, 4, 1, true>(p, 1, s);  // 136 KiB
    case 7: return launch<64, 64, 3, AK, BKc, MODE_PLAIN, MODE_PLAIN, 4, 1, true>(p, 1, s);   //  80 KiB, 2 WG/CU
    case 12: return launch<64, 64, 2, AK, BKc, MODE_PLAIN, MODE_PLAIN, 4, 2, true>(p, 1, s);  //  96 KiB
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pipe
}  // namespace ddpx
