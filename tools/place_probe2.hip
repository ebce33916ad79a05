// Code-placement probe 2 for gfx950 (round 3): K1's chunk 1-4 structure.
//
// tools/place_probe.hip found that a stream of 8-byte VALU instructions issues
// at ~3.67 cycles per instruction when the instructions start 4 bytes past an
// 8-byte boundary and at ~4.0-4.1 when they start ON one (profiles/r03/probe/).
// K1's chunks 1-4 read their K+W words from LDS once per 4 rounds, and the
// compiler's 4-byte s_waitcnt before the first use flips the phase of every
// later instruction; its 4-byte VOP2 adds do the same inside a round.  Here a
// loop of 2 groups x 4 rounds, each group reading 4 K+W words from LDS:
//   V = 0: as hipcc emits K1 today: h + Ch as v_add_u32_e32 right before the
//          s_waitcnt, e' as v_add_u32_e32 (a round: 104 bytes; a group flips
//          the phase);
//   V = 1: every add as v_add_u32_e64 except the group's first h + K+W, a
//          4-byte v_add_u32_e32 right after the 4-byte s_waitcnt: every VALU
//          instruction keeps one phase;
//   V = 2: every add e64, the s_waitcnt followed by a 4-byte s_nop 0: every
//          VALU instruction keeps one phase.
// The loop head sits 4 * PAD bytes past a 64-byte boundary.  One JSON line
// per (V, PAD): cycles per wave64 VALU instruction per SIMD.
//
//   hipcc --offload-arch=gfx950 -O3 tools/place_probe2.hip -o tools/place_probe2 && tools/place_probe2
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define ITERS 2048

// one round; KW = the K+W operand, HK = the h + K+W add, EN = the e' add, W = optional wait text
#define RND(a, b, c, d, e, f, g, h, KW, HKOP, ENOP, W)                   \
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
  W HKOP " " h ", " KW ", " h "\n"                                      \
  "v_add3_u32 " h ", " h ", %[t5], %[t0]\n"                             \
  ENOP " " d ", " h ", " d "\n"                                         \
  "v_add3_u32 " h ", %[t2], %[t1], " h "\n"

#define LD "ds_read_b32 %[k0], %[z]\nds_read_b32 %[k1], %[z] offset:4\nds_read_b32 %[k2], %[z] offset:8\nds_read_b32 %[k3], %[z] offset:12\n"
#define WAIT "s_waitcnt lgkmcnt(0)\n"
#define WAITNOP "s_waitcnt lgkmcnt(0)\ns_nop 0\n"
#define E32 "v_add_u32_e32"
#define E64 "v_add_u32_e64"

// a group of 4 rounds (names rotate); FIRST = the first round's (HK op, wait)
#define GROUP(HK0, W0, HK, EN, A, B, C, D, E_, F, G, H)                                      \
  LD RND(A, B, C, D, E_, F, G, H, "%[k0]", HK0, EN, W0)                                     \
  RND(H, A, B, C, D, E_, F, G, "%[k1]", HK, EN, "")                                        \
  RND(G, H, A, B, C, D, E_, F, "%[k2]", HK, EN, "")                                        \
  RND(F, G, H, A, B, C, D, E_, "%[k3]", HK, EN, "")
#define BODY(HK0, W0, HK, EN)                                                                  \
  GROUP(HK0, W0, HK, EN, "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]")       \
  GROUP(HK0, W0, HK, EN, "%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]")

#define BODY0 BODY(E32, WAIT, E32, E32)
#define BODY1 BODY(E32, WAIT, E64, E64)
#define BODY2 BODY(E64, WAITNOP, E64, E64)

#define STR2(x) #x
#define STR(x) STR2(x)

#define KERNEL(V, PAD)                                                                                   \
  __global__ __launch_bounds__(256) void probe2_##V##_##PAD(uint32_t seed, uint32_t* out,                \
                                                             unsigned long long* stamps) {                \
    __shared__ uint32_t lkw[64];                                                                          \
    if (threadIdx.x < 64) lkw[threadIdx.x] = seed * 0x9e3779b9u + threadIdx.x;                            \
    __syncthreads();                                                                                      \
    unsigned long long t0 = 0, r0 = 0;                                                                    \
    if (threadIdx.x == 0) {                                                                               \
      t0 = __builtin_amdgcn_s_memtime();                                                                  \
      r0 = __builtin_amdgcn_s_memrealtime();                                                              \
    }                                                                                                     \
    uint32_t a = seed ^ threadIdx.x, b = a * 3u, c = a * 5u, d = a * 7u, e = a * 11u, f = a * 13u,        \
             g = a * 17u, h = a * 19u;                                                                    \
    uint32_t x0, x1, x2, x3, x4, x5, x6, x7, k0, k1, k2, k3;                                              \
    uint32_t z = (uint32_t)(uintptr_t)lkw;                                                                \
    uint32_t n = ITERS;                                                                                   \
    asm volatile(".p2align 6\n.rept " STR(PAD) "\ns_nop 0\n.endr\n"                                       \
                 "1:\n" BODY##V "s_sub_u32 %[n], %[n], 1\ns_cmp_lg_u32 %[n], 0\ns_cbranch_scc1 1b\n"      \
                 : [a] "+v"(a), [b] "+v"(b), [c] "+v"(c), [d] "+v"(d), [e] "+v"(e), [f] "+v"(f),         \
                   [g] "+v"(g), [h] "+v"(h), [t0] "=&v"(x0), [t1] "=&v"(x1), [t2] "=&v"(x2),             \
                   [t3] "=&v"(x3), [t4] "=&v"(x4), [t5] "=&v"(x5), [t6] "=&v"(x6), [t7] "=&v"(x7),        \
                   [k0] "=&v"(k0), [k1] "=&v"(k1), [k2] "=&v"(k2), [k3] "=&v"(k3), [n] "+s"(n)            \
                 : [z] "v"(z)                                                                             \
                 : "scc", "memory");                                                                      \
    if ((a ^ b ^ c ^ d ^ e ^ f ^ g ^ h) == 0x12345678u) out[0] = a;                                       \
    if (threadIdx.x == 0) {                                                                               \
      stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;                                         \
      stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;                                 \
    }                                                                                                     \
  }

#define ALLPAD(V)                                                                                    \
  KERNEL(V, 0) KERNEL(V, 1) KERNEL(V, 2) KERNEL(V, 3) KERNEL(V, 4) KERNEL(V, 5) KERNEL(V, 6) KERNEL(V, 7)
ALLPAD(0)
ALLPAD(1)
ALLPAD(2)

typedef void (*kfn)(uint32_t, uint32_t*, unsigned long long*);
#define PTRS(V) \
  {probe2_##V##_0, probe2_##V##_1, probe2_##V##_2, probe2_##V##_3, probe2_##V##_4, probe2_##V##_5, probe2_##V##_6, probe2_##V##_7}

int main() {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  int rt_khz = 100000;
  (void)hipDeviceGetAttribute(&rt_khz, hipDeviceAttributeWallClockRate, 0);
  const unsigned grid = (unsigned)prop.multiProcessorCount * 8u;
  uint32_t* out;
  unsigned long long* stamps;
  if (hipMalloc(&out, 4) != hipSuccess || hipMalloc(&stamps, (size_t)grid * 16) != hipSuccess) return 1;
  kfn k[3][8] = {PTRS(0), PTRS(1), PTRS(2)};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  std::vector<unsigned long long> h(2 * (size_t)grid);
  const double wave_instr = (double)grid * 4.0 * ITERS * 8.0 * 14.0;  // VALU only
  for (int round = 0; round < 3; ++round)
    for (int V = 0; V < 3; ++V)
      for (int pad = 0; pad < 8; ++pad) {
        float best = 1e30f;
        double clk = 0;
        for (int rep = 0; rep < 4; ++rep) {
          (void)hipEventRecord(e0, 0);
          hipLaunchKernelGGL(k[V][pad], dim3(grid), dim3(256), 0, 0, 0x1234u + rep, out, stamps);
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
        printf("{\"round\": %d, \"variant\": %d, \"pad\": %d, \"loop_phase_mod64\": %d, \"ms\": %.4f, "
               "\"clock_ghz\": %.4f, \"cycles_per_valu_instr\": %.4f}\n",
               round, V, pad, 4 * pad, best, clk / 1e9, cpi);
        fflush(stdout);
      }
  return 0;
}
