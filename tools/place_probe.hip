// Code-placement probe for gfx950: does the issue cost of a SHA-256 round
// stream depend on where its instructions sit relative to 8/16/32/64-byte
// boundaries?  (K1's trial block ran 1.1% faster starting on an 8-byte
// boundary than 4 bytes past one: profiles/r03/ab/ab3_code_placement.log.)
//
// Each wave runs a loop of 8 SHA-256 rounds written in assembly in the order
// hipcc emits K1's rounds (Ch, Maj, 6 x v_alignbit_b32, 2 x xor3, h + Ch,
// T1 = v_add3, e' = d + T1, a' = v_add3), 14 VALU per round.  The loop head
// is placed at byte 4 * PAD past a 64-byte boundary (.p2align 6, then PAD
// s_nops, executed once).  Variants:
//   E = 0: the two plain adds as VOP2 (v_add_u32_e32, 4 bytes), as hipcc emits
//          them: a round is 104 bytes, and the instructions between the two
//          adds sit 4 bytes off the others' phase;
//   E = 1: the two adds as VOP3 (v_add_u32_e64, 8 bytes): every instruction
//          of the loop has the same phase mod 8.
// 8 waves per SIMD on every CU; one JSON line per (E, PAD): cycles per wave64
// VALU instruction per SIMD at the clock measured in the kernel.
//
//   hipcc --offload-arch=gfx950 -O3 tools/place_probe.hip -o tools/place_probe && tools/place_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define ITERS 2048

#define RND_E0(a, b, c, d, e, f, g, h)                                  \
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
  "v_add_u32_e32 " h ", %[t0], " h "\n"                                 \
  "v_add3_u32 " h ", " h ", %[t5], %[kw]\n"                             \
  "v_add_u32_e32 " d ", " h ", " d "\n"                                 \
  "v_add3_u32 " h ", %[t2], %[t1], " h "\n"
#define RND_E1(a, b, c, d, e, f, g, h)                                  \
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
  "v_add_u32_e64 " h ", %[t0], " h "\n"                                 \
  "v_add3_u32 " h ", " h ", %[t5], %[kw]\n"                             \
  "v_add_u32_e64 " d ", " h ", " d "\n"                                 \
  "v_add3_u32 " h ", %[t2], %[t1], " h "\n"
// 8 rounds: the state's names rotate by one each round (a' lands in h's register, e' in d's)
#define EIGHT(R)                                                                          \
  R("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]")                       \
  R("%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]")                       \
  R("%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]")                       \
  R("%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]")                       \
  R("%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]")                       \
  R("%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]")                       \
  R("%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]")                       \
  R("%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[a]")

#define STR2(x) #x
#define STR(x) STR2(x)

#define KERNEL(E, PAD)                                                                                  \
  __global__ __launch_bounds__(256) void probe_##E##_##PAD(uint32_t seed, uint32_t* out,                \
                                                           unsigned long long* stamps) {                 \
    unsigned long long t0 = 0, r0 = 0;                                                                   \
    if (threadIdx.x == 0) {                                                                              \
      t0 = __builtin_amdgcn_s_memtime();                                                                 \
      r0 = __builtin_amdgcn_s_memrealtime();                                                             \
    }                                                                                                    \
    uint32_t a = seed ^ threadIdx.x, b = a * 3u, c = a * 5u, d = a * 7u, e = a * 11u, f = a * 13u,       \
             g = a * 17u, h = a * 19u, kw = seed + blockIdx.x;                                           \
    uint32_t x0, x1, x2, x3, x4, x5, x6, x7;                                                             \
    uint32_t n = ITERS;                                                                                  \
    asm volatile(".p2align 6\n.rept " STR(PAD) "\ns_nop 0\n.endr\n"                                      \
                 "1:\n" EIGHT(RND_E##E) "s_sub_u32 %[n], %[n], 1\ns_cmp_lg_u32 %[n], 0\ns_cbranch_scc1 1b\n" \
                 : [a] "+v"(a), [b] "+v"(b), [c] "+v"(c), [d] "+v"(d), [e] "+v"(e), [f] "+v"(f),        \
                   [g] "+v"(g), [h] "+v"(h), [t0] "=&v"(x0), [t1] "=&v"(x1), [t2] "=&v"(x2),            \
                   [t3] "=&v"(x3), [t4] "=&v"(x4), [t5] "=&v"(x5), [t6] "=&v"(x6), [t7] "=&v"(x7),       \
                   [n] "+s"(n)                                                                           \
                 : [kw] "v"(kw)                                                                          \
                 : "scc");                                                                               \
    if ((a ^ b ^ c ^ d ^ e ^ f ^ g ^ h) == 0x12345678u) out[0] = a;                                      \
    if (threadIdx.x == 0) {                                                                              \
      stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;                                        \
      stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;                                \
    }                                                                                                    \
  }

#define ALLPAD(E)                                                                                     \
  KERNEL(E, 0) KERNEL(E, 1) KERNEL(E, 2) KERNEL(E, 3) KERNEL(E, 4) KERNEL(E, 5) KERNEL(E, 6)         \
  KERNEL(E, 7) KERNEL(E, 8) KERNEL(E, 9) KERNEL(E, 10) KERNEL(E, 11) KERNEL(E, 12) KERNEL(E, 13)     \
  KERNEL(E, 14) KERNEL(E, 15)
ALLPAD(0)
ALLPAD(1)

typedef void (*kfn)(uint32_t, uint32_t*, unsigned long long*);
#define PTRS(E)                                                                                        \
  {probe_##E##_0, probe_##E##_1, probe_##E##_2, probe_##E##_3, probe_##E##_4, probe_##E##_5,          \
   probe_##E##_6, probe_##E##_7, probe_##E##_8, probe_##E##_9, probe_##E##_10, probe_##E##_11,       \
   probe_##E##_12, probe_##E##_13, probe_##E##_14, probe_##E##_15}

int main() {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  int rt_khz = 100000;
  (void)hipDeviceGetAttribute(&rt_khz, hipDeviceAttributeWallClockRate, 0);
  const unsigned grid = (unsigned)prop.multiProcessorCount * 8u;
  uint32_t* out;
  unsigned long long* stamps;
  if (hipMalloc(&out, 4) != hipSuccess || hipMalloc(&stamps, (size_t)grid * 16) != hipSuccess) return 1;
  kfn k[2][16] = {PTRS(0), PTRS(1)};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  std::vector<unsigned long long> h(2 * (size_t)grid);
  const double wave_instr = (double)grid * 4.0 * ITERS * 8.0 * 14.0;
  for (int round = 0; round < 3; ++round) {  // the whole sweep 3 times: drift shows as spread
    for (int E = 0; E < 2; ++E)
      for (int pad = 0; pad < 16; ++pad) {
        float best = 1e30f;
        double clk = 0;
        for (int rep = 0; rep < 4; ++rep) {
          (void)hipEventRecord(e0, 0);
          hipLaunchKernelGGL(k[E][pad], dim3(grid), dim3(256), 0, 0, 0x1234u + rep, out, stamps);
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
        const double cpi = prop.multiProcessorCount * 4.0 * clk * best * 1e-3 / wave_instr;
        printf("{\"round\": %d, \"e64_adds\": %d, \"pad\": %d, \"loop_phase_mod64\": %d, \"ms\": %.4f, "
               "\"clock_ghz\": %.4f, \"cycles_per_instr\": %.4f}\n",
               round, E, pad, 4 * pad, best, clk / 1e9, cpi);
        fflush(stdout);
      }
  }
  return 0;
}
