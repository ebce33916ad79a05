// Test-library kernels (libpow_gpu_test.so only; build.py TEST_ONLY).
//
// pow_test_stall: one wave that keeps the stream busy for a bounded time
// (POW_TEST_STALL_US), launched in front of a context's next kernel so that
// the host's wait for that kernel outlasts a short watchdog deadline
// (POW_WATCHDOG_MS): the watchdog tests of the HIP launch path.  The wave
// sleeps between reads of the constant-rate realtime counter and always ends.
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(64) void pow_test_stall(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

// us: stall time in microseconds, at most 5 s; realtime_khz: the counter's rate.
extern "C++" hipError_t pow_launch_test_stall(hipStream_t stream, unsigned us, int realtime_khz) {
  const unsigned long long capped = us > 5000000u ? 5000000u : us;
  hipLaunchKernelGGL(pow_test_stall, dim3(1), dim3(64), 0, stream, capped * (unsigned long long)realtime_khz / 1000ull);
  return hipGetLastError();
}
