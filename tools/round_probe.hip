// SHA-256 round forms for gfx950 at the good code phase (round 3).
//
// tools/pattern_probe.hip showed that, with every instruction 8 bytes long and
// 4 bytes past an 8-byte boundary, a full-rate op right after a half-rate one
// is cheap only in some patterns: H F F issues at 3.06 cycles per instruction
// (isolated rates: 2.85), H F at 3.52 (3.18), and K1's round order
// F F H H H H H H F F F H F H at 3.66.  K1's round is 8 half-rate ops
// (6 v_alignbit_b32, 2 v_add3_u32) and 6 full-rate ones.  Here each wave runs
// a loop of 8 real SHA-256 rounds (true dependencies, K+W from a VGPR) in
// these forms; one JSON line per form: cycles per ROUND per SIMD (and per
// instruction), 8 waves per SIMD on every CU:
//   F = 0: K1 today, 14 ops:  Ch Maj ra ra ra re re re S0 S1 hk T1=add3 e' a'=add3
//          (F F H H H H H H F F F H F H)
//   F = 1: 16 ops, no v_add3: T1 = hk + (S1 + Ch), a' = T1 + (S0 + Maj), and the
//          NEXT round's hk = g + KW computed in this round:
//          re Ch Maj re hk' re S1 p ra T1 e' ra ra S0 q a'   (H F F H F H F F H F F H H F F F)
//   F = 2: the 16-op form with the a-rotations first:
//          ra Ch Maj ra hk' ra S0 q re ... (H F F H F H F F H H H F F F F F)
//   F = 3: 15 ops: a' = add3(T1, S0, Maj) kept, T1 = hk + (S1 + Ch) split, hk' in-round:
//          re Ch Maj re hk' re S1 p ra T1 e' ra ra S0 a'=add3  (H F F H F H F F H F F H H F H)
//   F = 4: 14 ops reordered: re Ch Maj re hk re S1 T1=add3 e' ra ra ra S0 a'=add3
//          (H F F H F H F H F H H H F H)
// The loop head is 4 bytes past an 8-byte boundary (F 0-4) or on one (F 5 = F 1 at phase 0).
//
//   hipcc --offload-arch=gfx950 -O3 tools/round_probe.hip -o tools/round_probe && tools/round_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define ITERS 2048

#define R0(a, b, c, d, e, f, g, h, HI, HO)                              \
  "v_bitop3_b32 %[t0], " e ", " f ", " g " bitop3:0xca\n"               \
  "v_bitop3_b32 %[t1], " a ", " b ", " c " bitop3:0xe8\n"               \
  "v_alignbit_b32 %[t2], " a ", " a ", 2\n"                             \
  "v_alignbit_b32 %[t3], " a ", " a ", 13\n"                            \
  "v_alignbit_b32 %[t4], " a ", " a ", 22\n"                            \
  "v_alignbit_b32 %[t5], " e ", " e ", 6\n"                             \
  "v_alignbit_b32 %[t6], " e ", " e ", 11\n"                            \
  "v_alignbit_b32 %[t7], " e ", " e ", 25\n"                            \
  "v_bitop3_b32 %[t2], %[t2], %[t3], %[t4] bitop3:0x96\n"               \
  "v_bitop3_b32 %[t5], %[t5], %[t6], %[t7] bitop3:0x96\n"               \
  "v_add_u32_e64 " h ", " h ", %[kw]\n"                                 \
  "v_add3_u32 " h ", " h ", %[t5], %[t0]\n"                             \
  "v_add_u32_e64 " d ", " d ", " h "\n"                                 \
  "v_add3_u32 " h ", " h ", %[t2], %[t1]\n"
// HI = this round's h + KW (computed by the previous round), HO = next round's
#define R1(a, b, c, d, e, f, g, h, HI, HO)                              \
  "v_alignbit_b32 %[t5], " e ", " e ", 6\n"                             \
  "v_bitop3_b32 %[t0], " e ", " f ", " g " bitop3:0xca\n"               \
  "v_bitop3_b32 %[t1], " a ", " b ", " c " bitop3:0xe8\n"               \
  "v_alignbit_b32 %[t6], " e ", " e ", 11\n"                            \
  "v_add_u32_e64 " HO ", " g ", %[kw]\n"                                \
  "v_alignbit_b32 %[t7], " e ", " e ", 25\n"                            \
  "v_bitop3_b32 %[t5], %[t5], %[t6], %[t7] bitop3:0x96\n"               \
  "v_add_u32_e64 %[t0], %[t0], %[t5]\n"                                 \
  "v_alignbit_b32 %[t2], " a ", " a ", 2\n"                             \
  "v_add_u32_e64 %[t0], " HI ", %[t0]\n"                                \
  "v_add_u32_e64 " d ", " d ", %[t0]\n"                                 \
  "v_alignbit_b32 %[t3], " a ", " a ", 13\n"                            \
  "v_alignbit_b32 %[t4], " a ", " a ", 22\n"                            \
  "v_bitop3_b32 %[t2], %[t2], %[t3], %[t4] bitop3:0x96\n"               \
  "v_add_u32_e64 %[t1], %[t1], %[t2]\n"                                 \
  "v_add_u32_e64 " h ", %[t0], %[t1]\n"
#define R2(a, b, c, d, e, f, g, h, HI, HO)                              \
  "v_alignbit_b32 %[t2], " a ", " a ", 2\n"                             \
  "v_bitop3_b32 %[t0], " e ", " f ", " g " bitop3:0xca\n"               \
  "v_bitop3_b32 %[t1], " a ", " b ", " c " bitop3:0xe8\n"               \
  "v_alignbit_b32 %[t3], " a ", " a ", 13\n"                            \
  "v_add_u32_e64 " HO ", " g ", %[kw]\n"                                \
  "v_alignbit_b32 %[t4], " a ", " a ", 22\n"                            \
  "v_bitop3_b32 %[t2], %[t2], %[t3], %[t4] bitop3:0x96\n"               \
  "v_add_u32_e64 %[t1], %[t1], %[t2]\n"                                 \
  "v_alignbit_b32 %[t5], " e ", " e ", 6\n"                             \
  "v_alignbit_b32 %[t6], " e ", " e ", 11\n"                            \
  "v_alignbit_b32 %[t7], " e ", " e ", 25\n"                            \
  "v_bitop3_b32 %[t5], %[t5], %[t6], %[t7] bitop3:0x96\n"               \
  "v_add_u32_e64 %[t0], %[t0], %[t5]\n"                                 \
  "v_add_u32_e64 %[t0], " HI ", %[t0]\n"                                \
  "v_add_u32_e64 " d ", " d ", %[t0]\n"                                 \
  "v_add_u32_e64 " h ", %[t0], %[t1]\n"
#define R3(a, b, c, d, e, f, g, h, HI, HO)                              \
  "v_alignbit_b32 %[t5], " e ", " e ", 6\n"                             \
  "v_bitop3_b32 %[t0], " e ", " f ", " g " bitop3:0xca\n"               \
  "v_bitop3_b32 %[t1], " a ", " b ", " c " bitop3:0xe8\n"               \
  "v_alignbit_b32 %[t6], " e ", " e ", 11\n"                            \
  "v_add_u32_e64 " HO ", " g ", %[kw]\n"                                \
  "v_alignbit_b32 %[t7], " e ", " e ", 25\n"                            \
  "v_bitop3_b32 %[t5], %[t5], %[t6], %[t7] bitop3:0x96\n"               \
  "v_add_u32_e64 %[t0], %[t0], %[t5]\n"                                 \
  "v_alignbit_b32 %[t2], " a ", " a ", 2\n"                             \
  "v_add_u32_e64 %[t0], " HI ", %[t0]\n"                                \
  "v_add_u32_e64 " d ", " d ", %[t0]\n"                                 \
  "v_alignbit_b32 %[t3], " a ", " a ", 13\n"                            \
  "v_alignbit_b32 %[t4], " a ", " a ", 22\n"                            \
  "v_bitop3_b32 %[t2], %[t2], %[t3], %[t4] bitop3:0x96\n"               \
  "v_add3_u32 " h ", %[t0], %[t2], %[t1]\n"
#define R4(a, b, c, d, e, f, g, h, HI, HO)                              \
  "v_alignbit_b32 %[t5], " e ", " e ", 6\n"                             \
  "v_bitop3_b32 %[t0], " e ", " f ", " g " bitop3:0xca\n"               \
  "v_bitop3_b32 %[t1], " a ", " b ", " c " bitop3:0xe8\n"               \
  "v_alignbit_b32 %[t6], " e ", " e ", 11\n"                            \
  "v_add_u32_e64 " h ", " h ", %[kw]\n"                                 \
  "v_alignbit_b32 %[t7], " e ", " e ", 25\n"                            \
  "v_bitop3_b32 %[t5], %[t5], %[t6], %[t7] bitop3:0x96\n"               \
  "v_add3_u32 " h ", " h ", %[t5], %[t0]\n"                             \
  "v_add_u32_e64 " d ", " d ", " h "\n"                                 \
  "v_alignbit_b32 %[t2], " a ", " a ", 2\n"                             \
  "v_alignbit_b32 %[t3], " a ", " a ", 13\n"                            \
  "v_alignbit_b32 %[t4], " a ", " a ", 22\n"                            \
  "v_bitop3_b32 %[t2], %[t2], %[t3], %[t4] bitop3:0x96\n"               \
  "v_add3_u32 " h ", " h ", %[t2], %[t1]\n"
#define R5 R1

// 8 rounds: the state's names rotate by one each round (a' lands in h's register, e' in d's)
#define EIGHT(R)                                                                          \
  R("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[k0]", "%[k1]")     \
  R("%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[k1]", "%[k0]")     \
  R("%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[k0]", "%[k1]")     \
  R("%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[k1]", "%[k0]")     \
  R("%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[k0]", "%[k1]")     \
  R("%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[k1]", "%[k0]")     \
  R("%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[k0]", "%[k1]")     \
  R("%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[k1]", "%[k0]")
static const int ops_per_round[6] = {14, 16, 16, 15, 14, 16};

#define KERNEL(F, PAD)                                                                                  \
  __global__ __launch_bounds__(256) void probe_##F(uint32_t seed, uint32_t* out, unsigned long long* stamps) { \
    unsigned long long t0 = 0, r0 = 0;                                                                   \
    if (threadIdx.x == 0) {                                                                              \
      t0 = __builtin_amdgcn_s_memtime();                                                                 \
      r0 = __builtin_amdgcn_s_memrealtime();                                                             \
    }                                                                                                    \
    uint32_t a = seed ^ threadIdx.x, b = a * 3u, c = a * 5u, d = a * 7u, e = a * 11u, f = a * 13u,       \
             g = a * 17u, h = a * 19u, kw = seed + blockIdx.x, k0 = a * 59u, k1 = a * 61u;               \
    uint32_t x0, x1, x2, x3, x4, x5, x6, x7;                                                             \
    uint32_t n = ITERS;                                                                                  \
    asm volatile(".p2align 6\n.rept " #PAD "\ns_nop 0\n.endr\n"                                          \
                 "1:\n" EIGHT(R##F) "s_sub_u32 %[n], %[n], 1\ns_cmp_lg_u32 %[n], 0\ns_cbranch_scc1 1b\n"  \
                 : [a] "+v"(a), [b] "+v"(b), [c] "+v"(c), [d] "+v"(d), [e] "+v"(e), [f] "+v"(f),        \
                   [g] "+v"(g), [h] "+v"(h), [k0] "+v"(k0), [k1] "+v"(k1), [t0] "=&v"(x0), [t1] "=&v"(x1), \
                   [t2] "=&v"(x2), [t3] "=&v"(x3), [t4] "=&v"(x4), [t5] "=&v"(x5), [t6] "=&v"(x6),        \
                   [t7] "=&v"(x7), [n] "+s"(n)                                                           \
                 : [kw] "v"(kw)                                                                          \
                 : "scc");                                                                               \
    if ((a ^ b ^ c ^ d ^ e ^ f ^ g ^ h ^ k0 ^ k1) == 0x12345678u) out[0] = a;                            \
    if (threadIdx.x == 0) {                                                                              \
      stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;                                        \
      stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;                                \
    }                                                                                                    \
  }
KERNEL(0, 1)
KERNEL(1, 1)
KERNEL(2, 1)
KERNEL(3, 1)
KERNEL(4, 1)
KERNEL(5, 0)

typedef void (*kfn)(uint32_t, uint32_t*, unsigned long long*);

int main() {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  int rt_khz = 100000;
  (void)hipDeviceGetAttribute(&rt_khz, hipDeviceAttributeWallClockRate, 0);
  const unsigned grid = (unsigned)prop.multiProcessorCount * 8u;
  uint32_t* out;
  unsigned long long* stamps;
  if (hipMalloc(&out, 4) != hipSuccess || hipMalloc(&stamps, (size_t)grid * 16) != hipSuccess) return 1;
  kfn k[6] = {probe_0, probe_1, probe_2, probe_3, probe_4, probe_5};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  std::vector<unsigned long long> h(2 * (size_t)grid);
  for (int round = 0; round < 3; ++round)
    for (int F = 0; F < 6; ++F) {
      float best = 1e30f;
      double clk = 0;
      for (int rep = 0; rep < 4; ++rep) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k[F], dim3(grid), dim3(256), 0, 0, 0x1234u + rep, out, stamps);
        (void)hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess) return 1;
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        std::vector<double> c;
        for (unsigned b = 0; b < grid; ++b)
          if (h[2 * b + 1]) c.push_back((double)h[2 * b] / (double)h[2 * b + 1] * rt_khz * 1e3);
        std::sort(c.begin(), c.end());
        if (rep > 0 && ms < best) {
          best = ms;
          clk = c.empty() ? 0 : c[c.size() / 2];
        }
      }
      const double wave_rounds = (double)grid * 4.0 * ITERS * 8.0;
      const double cpr = prop.multiProcessorCount * 4.0 * clk * best * 1e-3 / wave_rounds;
      printf("{\"round\": %d, \"form\": %d, \"ops_per_round\": %d, \"phase_mod8\": %d, \"ms\": %.4f, "
             "\"clock_ghz\": %.4f, \"cycles_per_round\": %.3f, \"cycles_per_instr\": %.4f}\n",
             round, F, ops_per_round[F], F == 5 ? 0 : 4, best, clk / 1e9, cpr, cpr / ops_per_round[F]);
      fflush(stdout);
    }
  return 0;
}
