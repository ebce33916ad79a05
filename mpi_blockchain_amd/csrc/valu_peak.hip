// Int32 VALU issue-rate microbenchmarks for the roofline (include/pow_tools.h).
//
// Every CU runs 8 waves per SIMD; each loop iteration is one asm block of
// 8-byte VALU instructions held 4 bytes past an 8-byte boundary (the phase
// K1's trial runs at), one of three streams:
//   POW_VALU_MIX   K1's SHA-256 round as it issues it (sha256_dev.h POW_R):
//                  8 rounds, 6 v_alignbit_b32 + 4 v_bitop3_b32 + 2 v_add3_u32
//                  + 2 v_add_u32_e64 each (8 half-rate : 6 full-rate);
//   POW_VALU_FULL  v_bitop3_b32 + v_add_u32_e64 over 8 independent chains,
//                  VGPR operands only: the full-rate ceiling (SIMD-32: one
//                  wave64 instruction per 2 cycles);
//   POW_VALU_HALF  v_alignbit_b32 + v_add3_u32 over 8 chains: half rate.
// Pure streams cost the same at either code phase; mixed ones do not
// (profiles/r03/probe/).  Each workgroup also stamps the shader clock
// (s_memtime) against the constant-rate realtime counter (s_memrealtime), so
// the clock the chip held during the run is measured, not assumed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/pow_gpu.h"
#include "../../include/pow_tools.h"
#include "pow_template.h"
#include "sha256_dev.h"

// iterations: ~2-3 ms per stream, long enough for a steady clock reading
#define VP_ITERS(kind) ((kind) == POW_VALU_MIX ? 2048 : 16384)

// one chain step: FULL x = bitop3(x, y, z) + y; HALF x = rotr(x, 7) + x + y
#define VP_F(x) "\tv_bitop3_b32 " x ", " x ", %[y], %[z] bitop3:0x96\n\tv_add_u32_e64 " x ", " x ", %[y]\n"
#define VP_H(x) "\tv_alignbit_b32 %[r], " x ", " x ", 7\n\tv_add3_u32 " x ", %[r], " x ", %[y]\n"
#define VP_CHAINS(M) M("%[x0]") M("%[x1]") M("%[x2]") M("%[x3]") M("%[x4]") M("%[x5]") M("%[x6]") M("%[x7]")

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
  for (int it = 0; it < VP_ITERS(KIND); ++it) {
    if (KIND == POW_VALU_MIX) {
      powdev::St s{x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]};
      uint32_t x0, x1, x2, x3, x4, x5, x6, x7;
      // 8 rounds: the state's names rotate by one per round, back to the start
      asm volatile(POW_PHASE
                   POW_R("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[y]")
                   POW_R("%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[y]")
                   POW_R("%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[y]")
                   POW_R("%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[y]")
                   POW_R("%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[y]")
                   POW_R("%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[y]")
                   POW_R("%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[y]")
                   POW_R("%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[y]")
                   : POW_STATE_OPS, POW_TEMPS
                   : [y] "v"(y));
      x[0] = s.a; x[1] = s.b; x[2] = s.c; x[3] = s.d; x[4] = s.e; x[5] = s.f; x[6] = s.g; x[7] = s.h;
    } else if (KIND == POW_VALU_FULL) {
      asm volatile(POW_PHASE VP_CHAINS(VP_F)
                   : [x0] "+v"(x[0]), [x1] "+v"(x[1]), [x2] "+v"(x[2]), [x3] "+v"(x[3]), [x4] "+v"(x[4]),
                     [x5] "+v"(x[5]), [x6] "+v"(x[6]), [x7] "+v"(x[7])
                   : [y] "v"(y), [z] "v"(z));
    } else {
      uint32_t rr;
      asm volatile(POW_PHASE VP_CHAINS(VP_H)
                   : [x0] "+v"(x[0]), [x1] "+v"(x[1]), [x2] "+v"(x[2]), [x3] "+v"(x[3]), [x4] "+v"(x[4]),
                     [x5] "+v"(x[5]), [x6] "+v"(x[6]), [x7] "+v"(x[7]), [r] "=&v"(rr)
                   : [y] "v"(y));
    }
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

// VALU wave-instructions per loop iteration of each kind (the loop's counter
// and branch are scalar): checked against the disassembly in tests/test_build.py.
static int instrs_per_iter(int kind) { return kind == POW_VALU_MIX ? 8 * 14 : 16; }

// The measurement on stream `st` of `device`.  Every launch, event and copy
// goes on that stream (never HIP's null stream: DESIGN.md §7, "Queue
// pressure"), and every wait is bounded (30 s).  *drained = false: a launch
// may still be running after a wait ran out; its events and buffers are then
// leaked rather than freed under it.
static int valu_rate_on(int device, hipStream_t st, int kind, pow_valu_result* res, bool* drained) {
  *drained = true;
  if (!res || kind < POW_VALU_MIX || kind > POW_VALU_HALF) return POW_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return POW_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return POW_EHIP;
  int rt_khz = 100000;
  (void)hipDeviceGetAttribute(&rt_khz, hipDeviceAttributeWallClockRate, device);
  const unsigned grid = (unsigned)prop.multiProcessorCount * 8u;  // 32 waves per CU
  uint32_t* out = nullptr;
  unsigned long long* stamps = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (hipMalloc(&out, 4) != hipSuccess || hipMalloc(&stamps, (size_t)grid * 16) != hipSuccess ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(out);
    (void)hipFree(stamps);
    return POW_EHIP;
  }
  auto wait = [&](hipEvent_t ev) {  // bounded: POW_OK, POW_EHIP on an error or after 30 s
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t q;
    while ((q = hipEventQuery(ev)) == hipErrorNotReady) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) return POW_EHIP;
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    return q == hipSuccess ? POW_OK : POW_EHIP;
  };
  float best = 1e30f;
  double best_clock = 0;
  std::vector<unsigned long long> h(2 * (size_t)grid);
  int rc = POW_OK;
  for (int rep = 0; rep < 4 && rc == POW_OK; ++rep) {  // rep 0 warms up clocks
    (void)hipEventRecord(e0, st);
    if (kind == POW_VALU_MIX)
      hipLaunchKernelGGL(valu_rate_kernel<POW_VALU_MIX>, dim3(grid), dim3(256), 0, st, 0x1234u + rep, out, stamps);
    else if (kind == POW_VALU_FULL)
      hipLaunchKernelGGL(valu_rate_kernel<POW_VALU_FULL>, dim3(grid), dim3(256), 0, st, 0x1234u + rep, out, stamps);
    else
      hipLaunchKernelGGL(valu_rate_kernel<POW_VALU_HALF>, dim3(grid), dim3(256), 0, st, 0x1234u + rep, out, stamps);
    (void)hipEventRecord(e1, st);
    if (hipMemcpyAsync(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost, st) != hipSuccess) {
      rc = POW_EHIP;
      *drained = wait(e1) == POW_OK;
      break;
    }
    if ((rc = wait(e1)) != POW_OK || (rc = hipStreamSynchronize(st) == hipSuccess ? POW_OK : POW_EHIP) != POW_OK) {
      *drained = hipEventQuery(e1) == hipSuccess;
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
  if (!*drained) return rc;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(out);
  (void)hipFree(stamps);
  if (rc != POW_OK) return rc;
  const double wave_instr = (double)grid * 4.0 * VP_ITERS(kind) * instrs_per_iter(kind);
  res->lane_ops_per_s = wave_instr * 64.0 / (best * 1e-3);
  res->kernel_ms = best;
  res->clock_hz = best_clock;
  const double simds = (double)prop.multiProcessorCount * 4.0;
  res->cycles_per_instr = best_clock > 0 ? simds * best_clock * (best * 1e-3) / wave_instr : 0;
  return POW_OK;
}

// A stream of this call's own.  HIP does not give the hardware queue behind
// it back when the stream is destroyed (hsa_queue_destroy is never called:
// tools/queue_trace.sh), so a process that has a pow_ctx should use
// pow_valu_rate_ctx instead.
extern "C" int pow_valu_rate(int device, int kind, pow_valu_result* res) {
  if (!res || kind < POW_VALU_MIX || kind > POW_VALU_HALF) return POW_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return POW_ENODEV;
  hipStream_t st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return POW_EHIP;
  bool drained = true;
  const int rc = valu_rate_on(device, st, kind, res, &drained);
  if (drained) (void)hipStreamDestroy(st);
  return rc;
}

// On the context's own stream: no hardware queue beyond the one the context
// already holds.
extern "C" int pow_valu_rate_ctx(pow_ctx* ctx, int kind, pow_valu_result* res) {
  if (!ctx) return POW_EINVAL;
  bool drained = true;
  return valu_rate_on(pow_ctx_device(ctx), (hipStream_t)pow_ctx_stream(ctx), kind, res, &drained);
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
