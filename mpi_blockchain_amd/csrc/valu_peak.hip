// Int32 VALU peak microbenchmark for the roofline (include/pow_tools.h).
//
// 8 independent dependency chains per lane, each step one v_alignbit_b32,
// one v_bitop3_b32 and one v_add3_u32 — the three instruction kinds that make
// up ~97% of the SHA-256 kernel.  The instruction count per iteration is
// checked in tests/test_build.py against the disassembly (24 VALU + loop).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pow_gpu.h"
#include "../../include/pow_tools.h"

#define VP_ITERS 4096

__global__ __launch_bounds__(256) void valu_peak_kernel(uint32_t seed, uint32_t* out) {
  uint32_t x[8], y = seed ^ threadIdx.x, z = seed * 3u + blockIdx.x;
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = seed + (uint32_t)k * 0x9e3779b9u + threadIdx.x;
  for (int it = 0; it < VP_ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint32_t r = __builtin_amdgcn_alignbit(x[k], x[k], 7 + k);
      uint32_t b = __builtin_amdgcn_bitop3_b32(r, y, z, 0x96);
      x[k] = b + x[k] + r;  // v_add3_u32
    }
    asm volatile("" : "+v"(y), "+v"(z));
  }
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) acc ^= x[k];
  if (acc == 0x12345678u) out[0] = acc;  // keep the chains live
}

extern "C" int pow_valu_peak(int device, double* lane_ops_per_s, double* kernel_ms) {
  if (hipSetDevice(device) != hipSuccess) return POW_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return POW_EHIP;
  const unsigned grid = (unsigned)prop.multiProcessorCount * 8u;  // 32 waves per CU
  uint32_t* out = nullptr;
  hipEvent_t e0, e1;
  if (hipMalloc(&out, 4) != hipSuccess) return POW_EHIP;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {  // rep 0 warms up clocks
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(valu_peak_kernel, dim3(grid), dim3(256), 0, 0, 0x1234u + rep, out);
    (void)hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess) return POW_EHIP;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(out);
  const double ops = (double)grid * 256.0 * VP_ITERS * 8.0 * 3.0;  // lane-ops
  if (lane_ops_per_s) *lane_ops_per_s = ops / (best * 1e-3);
  if (kernel_ms) *kernel_ms = best;
  return POW_OK;
}
