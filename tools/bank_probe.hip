// VGPR-bank probe for gfx950: are the mixed-stream VALU costs of
// tools/issue_probe.hip (half-rate v_alignbit_b32 ~4.3 and full-rate
// v_bitop3_b32 ~3.1 cycles per wave64 instruction in a 1:1 mix, vs 4.1 / 2.2
// alone) a register-bank effect?  Every instruction here names its VGPRs
// explicitly: operands in 4 distinct banks (vN, N mod 4) vs all in one bank.
//
//   hipcc --offload-arch=gfx950 -O3 tools/bank_probe.hip -o tools/bank_probe && tools/bank_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

// 8 independent chains; destination d_k reads itself and two fixed sources.
// DIST: destinations v4..v11, sources v13 (bank 1) and v14 (bank 2) -> a
//       bitop3 of v4 (bank 0) reads banks 0,1,2; v5 reads 1,1,2 ...
// SAME: destinations v4,v8,...,v32 (all bank 0), sources v36, v40 (bank 0).
#define B3D(d) "v_bitop3_b32 v" #d ", v" #d ", v13, v14 bitop3:0x96\n"
#define ABD(d) "v_alignbit_b32 v" #d ", v" #d ", v13, 7\n"
#define B3S(d) "v_bitop3_b32 v" #d ", v" #d ", v36, v40 bitop3:0x96\n"
#define ABS(d) "v_alignbit_b32 v" #d ", v" #d ", v36, 7\n"
// distinct banks for all three operands of each instruction: dest bank k, sources banks k+1, k+2
#define B3X(d, s1, s2) "v_bitop3_b32 v" #d ", v" #d ", v" #s1 ", v" #s2 " bitop3:0x96\n"
#define ABX(d, s1) "v_alignbit_b32 v" #d ", v" #d ", v" #s1 ", 7\n"

#define DIST8(M) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11)
#define SAME8(M) M(4) M(8) M(12) M(16) M(20) M(24) M(28) M(32)
#define X8B3 B3X(4, 45, 46) B3X(5, 46, 47) B3X(6, 47, 44) B3X(7, 44, 45) \
             B3X(8, 45, 46) B3X(9, 46, 47) B3X(10, 47, 44) B3X(11, 44, 45)
#define X8AB ABX(4, 45) ABX(5, 46) ABX(6, 47) ABX(7, 44) ABX(8, 45) ABX(9, 46) ABX(10, 47) ABX(11, 44)

#define CLOB                                                                                        \
  "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v16", "v20", "v24", \
      "v28", "v32", "v36", "v40", "v44", "v45", "v46", "v47"

template <int P>
__device__ __forceinline__ void body() {
  if constexpr (P == 0)  // bitop3, distinct-ish banks (64)
    asm volatile(DIST8(B3D) DIST8(B3D) DIST8(B3D) DIST8(B3D) DIST8(B3D) DIST8(B3D) DIST8(B3D) DIST8(B3D) ::: CLOB);
  if constexpr (P == 1)  // bitop3, one bank
    asm volatile(SAME8(B3S) SAME8(B3S) SAME8(B3S) SAME8(B3S) SAME8(B3S) SAME8(B3S) SAME8(B3S) SAME8(B3S) ::: CLOB);
  if constexpr (P == 2)  // bitop3, three distinct banks per instruction
    asm volatile(X8B3 X8B3 X8B3 X8B3 X8B3 X8B3 X8B3 X8B3 ::: CLOB);
  if constexpr (P == 3)  // alignbit, distinct banks
    asm volatile(X8AB X8AB X8AB X8AB X8AB X8AB X8AB X8AB ::: CLOB);
  if constexpr (P == 4)  // alignbit, one bank
    asm volatile(SAME8(ABS) SAME8(ABS) SAME8(ABS) SAME8(ABS) SAME8(ABS) SAME8(ABS) SAME8(ABS) SAME8(ABS) ::: CLOB);
  if constexpr (P == 5)  // 1:1 runs of 8, distinct banks
    asm volatile(X8AB X8B3 X8AB X8B3 X8AB X8B3 X8AB X8B3 ::: CLOB);
  if constexpr (P == 6)  // 1:1 runs of 8, one bank
    asm volatile(SAME8(ABS) SAME8(B3S) SAME8(ABS) SAME8(B3S) SAME8(ABS) SAME8(B3S) SAME8(ABS) SAME8(B3S) ::: CLOB);
}
static const char* kNames[] = {"bitop3 banks(d,1,2)", "bitop3 one bank", "bitop3 3 distinct banks",
                               "alignbit 2 distinct banks", "alignbit one bank",
                               "1:1 runs of 8, distinct banks", "1:1 runs of 8, one bank"};

template <int P>
__global__ __launch_bounds__(256) void probe(int iters, unsigned long long* clk) {
  asm volatile(
      "v_mov_b32 v4, 1\n v_mov_b32 v5, 2\n v_mov_b32 v6, 3\n v_mov_b32 v7, 4\n"
      "v_mov_b32 v8, 5\n v_mov_b32 v9, 6\n v_mov_b32 v10, 7\n v_mov_b32 v11, 8\n"
      "v_mov_b32 v12, 9\n v_mov_b32 v13, 10\n v_mov_b32 v14, 11\n v_mov_b32 v16, 12\n"
      "v_mov_b32 v20, 13\n v_mov_b32 v24, 14\n v_mov_b32 v28, 15\n v_mov_b32 v32, 16\n"
      "v_mov_b32 v36, 17\n v_mov_b32 v40, 18\n v_mov_b32 v44, 19\n v_mov_b32 v45, 20\n"
      "v_mov_b32 v46, 21\n v_mov_b32 v47, 22\n" ::: CLOB);
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) body<P>();
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int P>
void run(int cus, int per_cu, unsigned long long* d_clk, unsigned long long* h_clk) {
  const int grid = cus * per_cu, iters = 4000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  double clock_ghz = 0;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(probe<P>, dim3(grid), dim3(256), 0, 0, iters, d_clk);
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
  const double instr_per_simd = (double)per_cu * iters * 64;
  const double cyc = (best * 1e-3) * clock_ghz * 1e9 / instr_per_simd;
  printf("{\"pattern\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"clock_ghz\": %.3f, "
         "\"cycles_per_wave_instr\": %.3f}\n", kNames[P], per_cu, best, clock_ghz, cyc);
  fflush(stdout);
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  unsigned long long *d_clk, *h_clk;
  (void)hipMalloc(&d_clk, 16 * cus * 8);
  h_clk = (unsigned long long*)malloc(16 * cus * 8);
  for (int w : {8, 2}) {
    run<0>(cus, w, d_clk, h_clk);
    run<1>(cus, w, d_clk, h_clk);
    run<2>(cus, w, d_clk, h_clk);
    run<3>(cus, w, d_clk, h_clk);
    run<4>(cus, w, d_clk, h_clk);
    run<5>(cus, w, d_clk, h_clk);
    run<6>(cus, w, d_clk, h_clk);
  }
  return 0;
}
