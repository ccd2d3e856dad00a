// ddpx — fault-injection kernels for the failure-detection tests.
//
// spin_wait: one wave polls a host-mapped int32 flag until it equals `value` or `max_s` seconds have
// passed (s_memrealtime, 100 MHz), so it always terminates.  Inserted on a stream (or captured into a
// graph on the RCCL stream) it stands in for a collective whose peer never arrives: everything queued
// behind it stalls and the communicator watchdog must report the timeout.
#include "ddpx_common.h"

namespace {

__global__ void __launch_bounds__(64) spin_wait_kernel(const int* flag, int value, unsigned long long max_ticks,
                                                       int* status) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int ok = 0;
  while (true) {
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == value) {
      ok = 1;
      break;
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(127);
  }
  if (status) status[0] = ok ? 1 : 2;
}

}  // namespace

// Returns 0 on a successful launch; status[0] becomes 1 (flag seen) or 2 (gave up after max_s).
DDPX_API int ddpx_debug_spin_wait(const int* flag, int value, double max_s, int* status, hipStream_t s) {
  if (!flag || max_s <= 0.0 || max_s > 120.0) return -1;
  const unsigned long long ticks = (unsigned long long)(max_s * 1.0e8);
  hipLaunchKernelGGL(spin_wait_kernel, dim3(1), dim3(64), 0, s, flag, value, ticks, status);
  return (int)hipGetLastError();
}
