// Per-CU read rate of MFMA-fragment-shaped register loads on MI355X (gfx950).
//
// The hybrid-operand GEMM (csrc/include/ddpx_hyb.h) loads a K-contiguous operand straight into
// v_mfma_f32_16x16x32_bf16 fragments: one 16-B load per lane at row (lane & 15), k-chunk (lane >> 4), so each
// wave-instruction touches 16 rows x 64 B.  This probe times that access shape against 8 rows x 128 B
// (whole lines) and 1 KiB contiguous per instruction, with the GEMM's geometry: one 4-wave workgroup per CU,
// each wave sweeping its own 64-row strip of a [rows][K] bf16 matrix in 64-deep K-steps, DEPTH K-steps of
// loads in flight.
//
//   hipcc -O3 --offload-arch=gfx950 -o build/frag_probe benchmarks/frag_probe.hip && build/frag_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

// SHAPE 0: fragment (16 rows x 64 B per instruction; 8 instructions per wave per K-step: 4 row groups x 2 halves)
// SHAPE 1: lines    (8 rows x 128 B per instruction; 8 instructions cover the same 64 rows x 128 B)
// SHAPE 2: flat     (1 KiB contiguous per instruction; same bytes per step, no row structure)
template <int SHAPE, int DEPTH>
__global__ void __launch_bounds__(256) probe(const char* __restrict__ src, unsigned bytes, int ld, int nk, int strips,
                                             unsigned* sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, bytes, 0x00020000);
  const int strip = blockIdx.x % strips;  // 256-row strip of this workgroup
  const int row0 = strip * 256 + wave * 64;
  unsigned base;
  if constexpr (SHAPE == 0) base = (unsigned)(((row0 + (lane & 15)) * ld + 8 * (lane >> 4)) * 2);
  else if constexpr (SHAPE == 1) base = (unsigned)(((row0 + (lane >> 3)) * ld + 8 * (lane & 7)) * 2);
  else base = (unsigned)((row0 * ld) * 2 + lane * 16);
  u32x4 acc = {0u, 0u, 0u, 0u};
  u32x4 ring[DEPTH][8];
  auto issue = [&](int t, u32x4 (&d)[8]) {
    const unsigned kb = (unsigned)(t * 128);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      unsigned off;
      if constexpr (SHAPE == 0) off = base + kb + (i >> 1) * 16 * ld * 2 + (i & 1) * 64;
      else if constexpr (SHAPE == 1) off = base + kb + i * 8 * ld * 2;
      else off = base + (unsigned)t * 8192u + i * 1024;
      d[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
  };
#pragma unroll
  for (int s = 0; s < DEPTH - 1; ++s) issue(s, ring[s]);
  for (int t0 = 0; t0 < nk; t0 += DEPTH) {
#pragma unroll
    for (int r = 0; r < DEPTH; ++r) {
      const int t = t0 + r;
      issue(t + DEPTH - 1 < nk ? t + DEPTH - 1 : 0, ring[(r + DEPTH - 1) % DEPTH]);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc ^= ring[r][i];
    }
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9e3779b9u) sink[0] = 1;
}

template <typename F>
static float time_ms(F launch, int iters) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

template <int SHAPE, int DEPTH>
static void run(const char* name, const char* src, unsigned bytes, int rows, int ld, int ncu, unsigned* sink) {
  const int nk = ld / 64;  // 64-wide K-steps over the whole row
  const int strips = rows / 256;
  const int grid = ncu;
  const double moved = (double)grid * 256 * ld * 2;
  float t = time_ms([&] { probe<SHAPE, DEPTH><<<grid, 256>>>(src, bytes, ld, nk, strips, sink); }, 20);
  printf("%-6s depth %d  rows %5d ld %5d : %8.1f us  %6.1f GB/s/CU  %6.2f TB/s\n", name, DEPTH, rows, ld, t * 1e3,
         moved / t / 1e6 / ncu, moved / t / 1e9);
}

int main() {
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  unsigned* sink;
  CHECK(hipMalloc(&sink, 64));
  for (int ld : {3072, 4096, 4160}) {
    const int rows = 4096;
    const unsigned bytes = (unsigned)rows * ld * 2;
    char* src;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMemset(src, 1, bytes));
    run<0, 3>("frag", src, bytes, rows, ld, ncu, sink);
    run<0, 4>("frag", src, bytes, rows, ld, ncu, sink);
    run<0, 6>("frag", src, bytes, rows, ld, ncu, sink);
    run<1, 4>("lines", src, bytes, rows, ld, ncu, sink);
    run<1, 6>("lines", src, bytes, rows, ld, ncu, sink);
    run<2, 4>("flat", src, bytes, rows, ld, ncu, sink);
    CHECK(hipFree(src));
  }
  return 0;
}
