// VALU issue-pairing probe for gfx950: does the cost of a mixed stream of
// half-rate (v_alignbit_b32, v_add3_u32) and full-rate (v_bitop3_b32,
// v_add_u32) instructions depend on WHICH waves share a SIMD and whether they
// run in step?  (tools/valu_probe.hip measured: pure full 2.25 cycles per wave64
// instruction, pure half 4.14, but a 1:1 mix 3.7 instead of 3.2, and waves of
// different workgroups running pure-half / pure-full streams side by side 4.2.)
//
//   hipcc --offload-arch=gfx950 -O3 tools/issue_probe.hip -o tools/issue_probe && tools/issue_probe
//
// Variables: workgroup size (256 / 512 / 1024 threads: 1 / 2 / 4 waves of the
// same workgroup per SIMD), workgroups per CU, an s_barrier every B loop
// iterations (keeps a workgroup's waves in step), and s_setprio around runs.
// One JSON line per configuration.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define AB(v) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(v) : "v"(y));
#define B3(v) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v) : "v"(y), "v"(z));
#define A3(v) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v) : "v"(y), "v"(z));
#define AD(v) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(v) : "v"(y));
#define ALL8(M) M(x0) M(x1) M(x2) M(x3) M(x4) M(x5) M(x6) M(x7)
#define PRIO_HI asm volatile("s_setprio 3");
#define PRIO_LO asm volatile("s_setprio 0");

// 128 instructions per pattern step unless noted.
template <int P>
__device__ __forceinline__ void pattern(uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t& x3, uint32_t& x4,
                                        uint32_t& x5, uint32_t& x6, uint32_t& x7, uint32_t y, uint32_t z) {
  if constexpr (P == 0) {  // pure half
    ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB)
    ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB)
  }
  if constexpr (P == 1) {  // pure full
    ALL8(B3) ALL8(AD) ALL8(B3) ALL8(AD) ALL8(B3) ALL8(AD) ALL8(B3) ALL8(AD)
    ALL8(B3) ALL8(AD) ALL8(B3) ALL8(AD) ALL8(B3) ALL8(AD) ALL8(B3) ALL8(AD)
  }
  if constexpr (P == 2) {  // 1:1, runs of 8
    ALL8(AB) ALL8(B3) ALL8(AB) ALL8(AD) ALL8(AB) ALL8(B3) ALL8(AB) ALL8(AD)
    ALL8(AB) ALL8(B3) ALL8(AB) ALL8(AD) ALL8(AB) ALL8(B3) ALL8(AB) ALL8(AD)
  }
  if constexpr (P == 3) {  // 1:1, runs of 64
    ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB)
    ALL8(B3) ALL8(AD) ALL8(B3) ALL8(AD) ALL8(B3) ALL8(AD) ALL8(B3) ALL8(AD)
  }
  if constexpr (P == 4) {  // 1:1, runs of 64, full run at raised priority
    ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB) ALL8(AB)
    PRIO_HI
    ALL8(B3) ALL8(AD) ALL8(B3) ALL8(AD) ALL8(B3) ALL8(AD) ALL8(B3) ALL8(AD)
    PRIO_LO
  }
  if constexpr (P == 5) {  // SHA round mix (6 ab : 4 b3 : 2 a3 : 2 add) x 8 chains = 112
    ALL8(AB) ALL8(B3) ALL8(AB) ALL8(A3) ALL8(AB) ALL8(B3) ALL8(AD)
    ALL8(AB) ALL8(B3) ALL8(AB) ALL8(A3) ALL8(AB) ALL8(B3) ALL8(AD)
  }
  if constexpr (P == 6) {  // 1:1 strictly alternating single instructions (128)
#define HF(a, b) AB(a) B3(b)
    HF(x0, x1) HF(x2, x3) HF(x4, x5) HF(x6, x7) HF(x1, x0) HF(x3, x2) HF(x5, x4) HF(x7, x6)
    HF(x0, x1) HF(x2, x3) HF(x4, x5) HF(x6, x7) HF(x1, x0) HF(x3, x2) HF(x5, x4) HF(x7, x6)
    HF(x0, x1) HF(x2, x3) HF(x4, x5) HF(x6, x7) HF(x1, x0) HF(x3, x2) HF(x5, x4) HF(x7, x6)
    HF(x0, x1) HF(x2, x3) HF(x4, x5) HF(x6, x7) HF(x1, x0) HF(x3, x2) HF(x5, x4) HF(x7, x6)
    HF(x0, x1) HF(x2, x3) HF(x4, x5) HF(x6, x7) HF(x1, x0) HF(x3, x2) HF(x5, x4) HF(x7, x6)
    HF(x0, x1) HF(x2, x3) HF(x4, x5) HF(x6, x7) HF(x1, x0) HF(x3, x2) HF(x5, x4) HF(x7, x6)
    HF(x0, x1) HF(x2, x3) HF(x4, x5) HF(x6, x7) HF(x1, x0) HF(x3, x2) HF(x5, x4) HF(x7, x6)
    HF(x0, x1) HF(x2, x3) HF(x4, x5) HF(x6, x7) HF(x1, x0) HF(x3, x2) HF(x5, x4) HF(x7, x6)
#undef HF
  }
  if constexpr (P == 7) {  // 1:2 half:full, runs of 8 (F0-like weight of full ops, 192)
    ALL8(AB) ALL8(B3) ALL8(AD) ALL8(AB) ALL8(B3) ALL8(AD) ALL8(AB) ALL8(B3) ALL8(AD) ALL8(AB) ALL8(B3) ALL8(AD)
    ALL8(AB) ALL8(B3) ALL8(AD) ALL8(AB) ALL8(B3) ALL8(AD) ALL8(AB) ALL8(B3) ALL8(AD) ALL8(AB) ALL8(B3) ALL8(AD)
  }
}
static const int kPatLen[] = {128, 128, 128, 128, 128, 112, 128, 192};
static const char* kPatNames[] = {"pure half (alignbit)", "pure full (bitop3/add)", "1:1 runs of 8",
                                  "1:1 runs of 64", "1:1 runs of 64, full run at s_setprio 3",
                                  "SHA round mix 6ab:4b3:2a3:2add", "1:1 alternating singly",
                                  "1:2 runs of 8"};

// Odd workgroups run pattern Q instead of P when SPLIT (different streams side by side).
template <int P, int BAR>
__global__ void probe(uint32_t seed, int iters, uint32_t* out, unsigned long long* clk) {
  uint32_t x0 = seed + threadIdx.x, x1 = x0 * 3u, x2 = x0 * 5u, x3 = x0 * 7u, x4 = x0 * 11u,
           x5 = x0 * 13u, x6 = x0 * 17u, x7 = x0 * 19u;
  uint32_t y = seed ^ 0x5bd1e995u, z = blockIdx.x + 0x3f800000u;
  if (BAR) __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    pattern<P>(x0, x1, x2, x3, x4, x5, x6, x7, y, z);
    if (BAR && (i % BAR) == BAR - 1) __builtin_amdgcn_s_barrier();
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
  if (acc == 0x9e3779b9u) out[0] = acc;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int P, int BAR>
void run(int cus, int block, int wg_per_cu, uint32_t* out, unsigned long long* d_clk,
         unsigned long long* h_clk) {
  const int grid = cus * wg_per_cu, iters = 2000;
  const int waves_per_simd = wg_per_cu * block / 256;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  double clock_ghz = 0;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((probe<P, BAR>), dim3(grid), dim3(block), 0, 0, 0x1234u + rep, iters, out, d_clk);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) {
      best = ms;
      (void)hipMemcpy(h_clk, d_clk, 16 * grid, hipMemcpyDeviceToHost);
      double sc = 0, sr = 0;
      for (int b = 0; b < grid; ++b) { sc += (double)h_clk[2 * b]; sr += (double)h_clk[2 * b + 1]; }
      clock_ghz = sc / sr * 0.1;
    }
  }
  const double instr_per_simd = (double)waves_per_simd * iters * kPatLen[P];
  const double cyc = (best * 1e-3) * clock_ghz * 1e9 / instr_per_simd;
  printf("{\"pattern\": \"%s\", \"block\": %d, \"wg_per_cu\": %d, \"waves_per_simd\": %d, \"barrier_every\": %d, "
         "\"ms\": %.3f, \"clock_ghz\": %.3f, \"cycles_per_wave_instr\": %.3f}\n",
         kPatNames[P], block, wg_per_cu, waves_per_simd, BAR, best, clock_ghz, cyc);
  fflush(stdout);
}

template <int P, int BAR>
void sweep(int cus, uint32_t* out, unsigned long long* d_clk, unsigned long long* h_clk) {
  // 2, 4 and 8 waves per SIMD: from 256-thread WGs (waves of different WGs
  // share a SIMD) and from 512 / 1024-thread WGs (a WG's waves share SIMDs).
  run<P, BAR>(cus, 256, 2, out, d_clk, h_clk);
  run<P, BAR>(cus, 512, 1, out, d_clk, h_clk);
  run<P, BAR>(cus, 256, 4, out, d_clk, h_clk);
  run<P, BAR>(cus, 1024, 1, out, d_clk, h_clk);
  run<P, BAR>(cus, 256, 8, out, d_clk, h_clk);
  run<P, BAR>(cus, 1024, 2, out, d_clk, h_clk);
}

template <int P, int BAR>
void sweep_lockstep(int cus, uint32_t* out, unsigned long long* d_clk, unsigned long long* h_clk) {
  // waves of one workgroup share each SIMD (2 or 4 per SIMD), optionally re-aligned by s_barrier
  run<P, BAR>(cus, 512, 1, out, d_clk, h_clk);
  run<P, BAR>(cus, 1024, 1, out, d_clk, h_clk);
  run<P, BAR>(cus, 1024, 2, out, d_clk, h_clk);
}

int main() {
  int dev = 0;
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, dev);
  const int cus = prop.multiProcessorCount;
  printf("{\"device\": \"%s\", \"cus\": %d}\n", prop.gcnArchName, cus);
  uint32_t* out;
  unsigned long long *d_clk, *h_clk;
  (void)hipMalloc(&out, 64);
  (void)hipMalloc(&d_clk, 16 * cus * 16);
  h_clk = (unsigned long long*)malloc(16 * cus * 16);
  if (getenv("PROBE_LOCKSTEP")) {  // barrier cost on pure streams, and mixed streams in step
    sweep_lockstep<1, 0>(cus, out, d_clk, h_clk);
    sweep_lockstep<1, 4>(cus, out, d_clk, h_clk);
    sweep_lockstep<1, 16>(cus, out, d_clk, h_clk);
    sweep_lockstep<0, 16>(cus, out, d_clk, h_clk);
    sweep_lockstep<3, 0>(cus, out, d_clk, h_clk);
    sweep_lockstep<3, 4>(cus, out, d_clk, h_clk);
    sweep_lockstep<3, 16>(cus, out, d_clk, h_clk);
    sweep_lockstep<5, 4>(cus, out, d_clk, h_clk);
    sweep_lockstep<5, 16>(cus, out, d_clk, h_clk);
    return 0;
  }
  sweep<0, 0>(cus, out, d_clk, h_clk);
  sweep<1, 0>(cus, out, d_clk, h_clk);
  sweep<2, 0>(cus, out, d_clk, h_clk);
  sweep<2, 1>(cus, out, d_clk, h_clk);
  sweep<3, 0>(cus, out, d_clk, h_clk);
  sweep<3, 1>(cus, out, d_clk, h_clk);
  sweep<4, 0>(cus, out, d_clk, h_clk);
  sweep<5, 0>(cus, out, d_clk, h_clk);
  sweep<5, 1>(cus, out, d_clk, h_clk);
  sweep<6, 0>(cus, out, d_clk, h_clk);
  sweep<6, 1>(cus, out, d_clk, h_clk);
  sweep<7, 0>(cus, out, d_clk, h_clk);
  sweep<7, 1>(cus, out, d_clk, h_clk);
  return 0;
}
