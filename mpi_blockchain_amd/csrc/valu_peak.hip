// Int32 VALU issue-rate microbenchmarks for the roofline (include/pow_tools.h).
//
// Every CU runs 8 waves per SIMD of 8 independent dependency chains per lane,
// one of three instruction mixes:
//   POW_VALU_MIX   v_alignbit_b32 + v_bitop3_b32 + v_add3_u32 per step: the
//                  three instruction kinds that make up ~97% of the SHA-256
//                  kernel (2 half-rate : 1 full-rate on gfx950);
//   POW_VALU_FULL  v_bitop3_b32 + v_add_u32, VGPR operands only: the full-rate
//                  ceiling (SIMD-32: one wave64 instruction per 2 cycles);
//   POW_VALU_HALF  v_alignbit_b32 + v_add3_u32: the half-rate kinds alone.
// Each workgroup also stamps the shader clock (s_memtime) against the
// constant-rate realtime counter (s_memrealtime), so the clock the chip held
// during the run is measured, not assumed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "../../include/pow_gpu.h"
#include "../../include/pow_tools.h"

#define VP_ITERS 4096

template <int KIND>
__global__ __launch_bounds__(256) void valu_rate_kernel(uint32_t seed, uint32_t* out, unsigned long long* stamps) {
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  uint32_t x[8], y = seed ^ threadIdx.x, z = seed * 3u + blockIdx.x;
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = seed + (uint32_t)k * 0x9e3779b9u + threadIdx.x;
  for (int it = 0; it < VP_ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (KIND == POW_VALU_MIX) {
        const uint32_t r = __builtin_amdgcn_alignbit(x[k], x[k], 7 + k);
        const uint32_t b = __builtin_amdgcn_bitop3_b32(r, y, z, 0x96);
        x[k] = b + x[k] + r;  // v_add3_u32
      } else if (KIND == POW_VALU_FULL) {
        // v_bitop3_b32 then v_add_u32 ((x ^ y) + z would fuse into v_xad_u32, half rate)
        x[k] = __builtin_amdgcn_bitop3_b32(x[k], y, z, 0x96) + y;
      } else {
        const uint32_t r = __builtin_amdgcn_alignbit(x[k], x[k], 7 + k);
        x[k] = r + x[k] + y;  // v_add3_u32
      }
    }
    asm volatile("" : "+v"(y), "+v"(z));
  }
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) acc ^= x[k];
  if (acc == 0x12345678u) out[0] = acc;  // keep the chains live
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// VALU wave-instructions per lane-step of each kind (the loop's counter and
// branch are scalar): checked against the disassembly in tests/test_build.py.
static int instrs_per_step(int kind) { return kind == POW_VALU_MIX ? 3 : 2; }

extern "C" int pow_valu_rate(int device, int kind, pow_valu_result* res) {
  if (!res || kind < POW_VALU_MIX || kind > POW_VALU_HALF) return POW_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return POW_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return POW_EHIP;
  int rt_khz = 100000;
  (void)hipDeviceGetAttribute(&rt_khz, hipDeviceAttributeWallClockRate, device);
  const unsigned grid = (unsigned)prop.multiProcessorCount * 8u;  // 32 waves per CU
  uint32_t* out = nullptr;
  unsigned long long* stamps = nullptr;
  if (hipMalloc(&out, 4) != hipSuccess) return POW_EHIP;
  if (hipMalloc(&stamps, (size_t)grid * 16) != hipSuccess) {
    (void)hipFree(out);
    return POW_EHIP;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  double best_clock = 0;
  std::vector<unsigned long long> h(2 * (size_t)grid);
  int rc = POW_OK;
  for (int rep = 0; rep < 4 && rc == POW_OK; ++rep) {  // rep 0 warms up clocks
    (void)hipEventRecord(e0, 0);
    if (kind == POW_VALU_MIX)
      hipLaunchKernelGGL(valu_rate_kernel<POW_VALU_MIX>, dim3(grid), dim3(256), 0, 0, 0x1234u + rep, out, stamps);
    else if (kind == POW_VALU_FULL)
      hipLaunchKernelGGL(valu_rate_kernel<POW_VALU_FULL>, dim3(grid), dim3(256), 0, 0, 0x1234u + rep, out, stamps);
    else
      hipLaunchKernelGGL(valu_rate_kernel<POW_VALU_HALF>, dim3(grid), dim3(256), 0, 0, 0x1234u + rep, out, stamps);
    (void)hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess ||
        hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) {
      rc = POW_EHIP;
      break;
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // the clock each workgroup saw: shader cycles / realtime ticks x realtime rate
    std::vector<double> clk;
    clk.reserve(grid);
    for (unsigned b = 0; b < grid; ++b)
      if (h[2 * b + 1]) clk.push_back((double)h[2 * b] / (double)h[2 * b + 1] * rt_khz * 1e3);
    std::sort(clk.begin(), clk.end());
    if (rep > 0 && ms < best) {
      best = ms;
      best_clock = clk.empty() ? 0 : clk[clk.size() / 2];
    }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(out);
  (void)hipFree(stamps);
  if (rc != POW_OK) return rc;
  const double wave_instr = (double)grid * 4.0 * VP_ITERS * 8.0 * instrs_per_step(kind);
  res->lane_ops_per_s = wave_instr * 64.0 / (best * 1e-3);
  res->kernel_ms = best;
  res->clock_hz = best_clock;
  const double simds = (double)prop.multiProcessorCount * 4.0;
  res->cycles_per_instr = best_clock > 0 ? simds * best_clock * (best * 1e-3) / wave_instr : 0;
  return POW_OK;
}

extern "C" int pow_valu_peak(int device, double* lane_ops_per_s, double* kernel_ms) {
  pow_valu_result r{};
  const int rc = pow_valu_rate(device, POW_VALU_MIX, &r);
  if (rc == POW_OK) {
    if (lane_ops_per_s) *lane_ops_per_s = r.lane_ops_per_s;
    if (kernel_ms) *kernel_ms = r.kernel_ms;
  }
  return rc;
}
