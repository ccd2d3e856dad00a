// How many waves per CU, and how much ILP per wave, does the SGD optimizer's HBM stream (fp32 master +
// momentum in; master + momentum + bf16 shadow out: 18 B per weight) need on MI355X?  The warp-specialised
// weight-gradient + SGD kernel (csrc/include/ddpx_wgrad_sgd.h) gives the stream 4 waves per CU and reaches
// ~3.4-4.6 TB/s; this separates "waves" from "bytes in flight per wave".
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/stream_probe benchmarks/stream_probe.hip && /tmp/stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__device__ __forceinline__ unsigned pack_bf2(float a, float b) {
  return (unsigned)__builtin_bit_cast(unsigned short, (__bf16)a) |
         ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)b) << 16);
}

// U vectors (16 B) per thread per iteration, all loads of an iteration issued before any store.
// PF: the next iteration's loads are issued before this iteration's stores (software pipelining).
template <int U, bool PF>
__global__ void stream(float* __restrict__ p, float* __restrict__ m, unsigned short* __restrict__ sh, size_t n4,
                       float lr) {
  const size_t nthr = (size_t)gridDim.x * blockDim.x;
  const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t chunk = nthr * U;
  f32x4 pv[U], mv[U], pn[U], mn[U];
  auto load = [&](size_t base, f32x4 (&a)[U], f32x4 (&b)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * nthr + tid;
      if (i < n4) {
        a[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p) + i);
        b[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(m) + i);
      }
    }
  };
  size_t base = 0;
  if (PF) load(0, pv, mv);
  for (; base < n4; base += chunk) {
    if (PF) {
      if (base + chunk < n4) load(base + chunk, pn, mn);
    } else {
      load(base, pv, mv);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * nthr + tid;
      if (i >= n4) continue;
      f32x4 g = pv[u] * 1e-3f;
      f32x4 mo = mv[u] * 0.9f + g;
      f32x4 po = pv[u] - lr * mo;
      __builtin_nontemporal_store(po, reinterpret_cast<f32x4*>(p) + i);
      __builtin_nontemporal_store(mo, reinterpret_cast<f32x4*>(m) + i);
      reinterpret_cast<u32x2*>(sh)[i] = (u32x2){pack_bf2(po[0], po[1]), pack_bf2(po[2], po[3])};
    }
    if (PF) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        pv[u] = pn[u];
        mv[u] = mn[u];
      }
    }
  }
}

// The same stream in the order the warp-specialised weight-gradient kernel walks it: tiles of TR rows x TC
// columns of a row-major [rows][cols] fp32 matrix, tile g at (g % tiles_m, g / tiles_m), each thread owning
// 16-B column groups of every (256 / (TC / 4))-th row; a workgroup sweeps its tiles g = blockIdx.x + i gridDim.x.
template <int TR, int TC>
__global__ void __launch_bounds__(256) stream_tiled(float* __restrict__ p, float* __restrict__ m,
                                                    unsigned short* __restrict__ sh, int rows, int cols, float lr) {
  constexpr int TPR = TC / 4;            // threads per tile row
  constexpr int RSTEP = 256 / TPR;       // rows between a thread's vectors
  constexpr int VPT = TR / RSTEP;        // vectors per thread per tile
  const int tiles_m = rows / TR, ntiles = tiles_m * (cols / TC);
  const int r0 = threadIdx.x / TPR, c = 4 * (threadIdx.x % TPR);
  for (int g = blockIdx.x; g < ntiles; g += gridDim.x) {
    const int m0 = (g % tiles_m) * TR, n0 = (g / tiles_m) * TC;
    f32x4 pv[VPT], mv[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      const size_t off = (size_t)(m0 + r0 + RSTEP * v) * cols + n0 + c;
      pv[v] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + off));
      mv[v] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(m + off));
    }
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      const size_t off = (size_t)(m0 + r0 + RSTEP * v) * cols + n0 + c;
      f32x4 g4 = pv[v] * 1e-3f;
      f32x4 mo = mv[v] * 0.9f + g4;
      f32x4 po = pv[v] - lr * mo;
      __builtin_nontemporal_store(po, reinterpret_cast<f32x4*>(p + off));
      __builtin_nontemporal_store(mo, reinterpret_cast<f32x4*>(m + off));
      *reinterpret_cast<u32x2*>(sh + off) = (u32x2){pack_bf2(po[0], po[1]), pack_bf2(po[2], po[3])};
    }
  }
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

template <int U, bool PF>
static void run(int ncu, float* p, float* m, unsigned short* sh, size_t n, const char* tag) {
  const double bytes = (double)n * 18;
  for (int wpc : {4, 8, 16}) {  // waves per CU, one workgroup per CU
    const int thr = 64 * wpc;
    float t = time_ms([&] { stream<U, PF><<<ncu, thr>>>(p, m, sh, n / 4, 0.01f); }, 20);
    printf("%-8s U=%d waves/CU %2d: %7.1f us %5.2f TB/s\n", tag, U, wpc, t * 1e3, bytes / t / 1e9);
  }
}

int main() {
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t n = 29425664;  // toy MLP parameter count (rounded to 64)
  float *p, *m;
  unsigned short* sh;
  CHECK(hipMalloc(&p, n * 4));
  CHECK(hipMalloc(&m, n * 4));
  CHECK(hipMalloc(&sh, n * 2));
  CHECK(hipMemset(p, 0, n * 4));
  CHECK(hipMemset(m, 0, n * 4));
  run<1, false>(ncu, p, m, sh, n, "plain");
  run<2, false>(ncu, p, m, sh, n, "plain");
  run<4, false>(ncu, p, m, sh, n, "plain");
  run<8, false>(ncu, p, m, sh, n, "plain");
  run<2, true>(ncu, p, m, sh, n, "pref");
  run<4, true>(ncu, p, m, sh, n, "pref");
  // tile-ordered sweeps of a [4096][7168] matrix (the toy MLP's fc1 | fc0 weights side by side)
  const int rows = 4096, cols = 7168;
  const double tb = (double)rows * cols * 18;
  for (int gm : {1, 2, 4}) {
    float t1 = time_ms([&] { stream_tiled<64, 128><<<ncu * gm, 256>>>(p, m, sh, rows, cols, 0.01f); }, 20);
    float t2 = time_ms([&] { stream_tiled<32, 256><<<ncu * gm, 256>>>(p, m, sh, rows, cols, 0.01f); }, 20);
    float t3 = time_ms([&] { stream_tiled<16, 512><<<ncu * gm, 256>>>(p, m, sh, rows, cols, 0.01f); }, 20);
    float t4 = time_ms([&] { stream_tiled<8, 1024><<<ncu * gm, 256>>>(p, m, sh, rows, cols, 0.01f); }, 20);
    printf("tiled wg/cu %d: 64x128 %.2f  32x256 %.2f  16x512 %.2f  8x1024 %.2f TB/s\n", gm, tb / t1 / 1e9,
           tb / t2 / 1e9, tb / t3 / 1e9, tb / t4 / 1e9);
  }
  return 0;
}
