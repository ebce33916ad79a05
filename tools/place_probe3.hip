// Code-placement probe 3 for gfx950 (round 3): is the phase effect of
// tools/place_probe.hip a property of each instruction class, or of the mix?
//
// place_probe found that a SHA-256 round stream of 8-byte VALU instructions
// issues at ~3.67 cycles per instruction when every instruction starts 4 bytes
// past an 8-byte boundary and at ~4.05 when it starts on one.  Here the loop
// body is one instruction class (or a fixed pattern of classes), every
// instruction 8 bytes long, 8 independent register chains, at phase 0 or 4:
//   K = 0  v_alignbit_b32                 (half rate)
//   K = 1  v_bitop3_b32                   (full rate)
//   K = 2  v_add_u32_e64                  (full rate)
//   K = 3  v_add3_u32                     (half rate)
//   K = 4  alignbit / bitop3 alternating  (1:1)
//   K = 5  alignbit, alignbit, bitop3     (2:1)
//   K = 6  SHA-256 rounds as K1 issues them (6 alignbit : 4 bitop3 : 2 add3 : 2 add)
// 8 waves per SIMD on every CU; one JSON line per (K, phase): cycles per
// wave64 VALU instruction per SIMD at the clock measured in the kernel.
//
//   hipcc --offload-arch=gfx950 -O3 tools/place_probe3.hip -o tools/place_probe3 && tools/place_probe3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define ITERS 2048

// 8 instructions over the rotating chains t0..t7
#define AL(d, s) "v_alignbit_b32 %[" d "], %[" s "], %[" s "], 7\n"
#define BO(d, s, u, v) "v_bitop3_b32 %[" d "], %[" s "], %[" u "], %[" v "] bitop3:0x96\n"
#define AD(d, s, u) "v_add_u32_e64 %[" d "], %[" s "], %[" u "]\n"
#define A3(d, s, u, v) "v_add3_u32 %[" d "], %[" s "], %[" u "], %[" v "]\n"
#define U_AL AL("t0", "t1") AL("t1", "t2") AL("t2", "t3") AL("t3", "t4") AL("t4", "t5") AL("t5", "t6") AL("t6", "t7") AL("t7", "t0")
#define U_BO                                                                                              \
  BO("t0", "t1", "t2", "t3") BO("t1", "t2", "t3", "t4") BO("t2", "t3", "t4", "t5") BO("t3", "t4", "t5", "t6") \
  BO("t4", "t5", "t6", "t7") BO("t5", "t6", "t7", "t0") BO("t6", "t7", "t0", "t1") BO("t7", "t0", "t1", "t2")
#define U_AD AD("t0", "t1", "t2") AD("t1", "t2", "t3") AD("t2", "t3", "t4") AD("t3", "t4", "t5") AD("t4", "t5", "t6") AD("t5", "t6", "t7") AD("t6", "t7", "t0") AD("t7", "t0", "t1")
#define U_A3                                                                                              \
  A3("t0", "t1", "t2", "t3") A3("t1", "t2", "t3", "t4") A3("t2", "t3", "t4", "t5") A3("t3", "t4", "t5", "t6") \
  A3("t4", "t5", "t6", "t7") A3("t5", "t6", "t7", "t0") A3("t6", "t7", "t0", "t1") A3("t7", "t0", "t1", "t2")
#define U_ALT AL("t0", "t1") BO("t1", "t2", "t3", "t4") AL("t2", "t3") BO("t3", "t4", "t5", "t6") AL("t4", "t5") BO("t5", "t6", "t7", "t0") AL("t6", "t7") BO("t7", "t0", "t1", "t2")
// 2:1, 24 instructions
#define U_HHF                                                                                            \
  AL("t0", "t1") AL("t1", "t2") BO("t2", "t3", "t4", "t5") AL("t3", "t4") AL("t4", "t5") BO("t5", "t6", "t7", "t0") \
  AL("t6", "t7") AL("t7", "t0") BO("t0", "t1", "t2", "t3") AL("t1", "t2") AL("t2", "t3") BO("t3", "t4", "t5", "t6") \
  AL("t4", "t5") AL("t5", "t6") BO("t6", "t7", "t0", "t1") AL("t7", "t0") AL("t0", "t1") BO("t1", "t2", "t3", "t4") \
  AL("t2", "t3") AL("t3", "t4") BO("t4", "t5", "t6", "t7") AL("t5", "t6") AL("t6", "t7") BO("t7", "t0", "t1", "t2")
#define X12(u) u u u u u u u u u u u u
#define X4(u) u u u u

#define RND(a, b, c, d, e, f, g, h)                                     \
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
#define EIGHT                                                                             \
  RND("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]")                     \
  RND("%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]")                     \
  RND("%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]")                     \
  RND("%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]")                     \
  RND("%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]")                     \
  RND("%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]")                     \
  RND("%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[a]", "%[b]")                     \
  RND("%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[a]")

// loop bodies: 96 instructions (K 0-5), 112 (K 6)
#define BODY0 X12(U_AL)
#define BODY1 X12(U_BO)
#define BODY2 X12(U_AD)
#define BODY3 X12(U_A3)
#define BODY4 X12(U_ALT)
#define BODY5 X4(U_HHF)
#define BODY6 EIGHT
static const int body_len[7] = {96, 96, 96, 96, 96, 96, 112};

// PH = 0: the loop's instructions start on 8-byte boundaries; PH = 1: 4 bytes past
#define KERNEL(K, PH)                                                                                   \
  __global__ __launch_bounds__(256) void probe_##K##_##PH(uint32_t seed, uint32_t* out,                 \
                                                          unsigned long long* stamps) {                  \
    unsigned long long t0 = 0, r0 = 0;                                                                   \
    if (threadIdx.x == 0) {                                                                              \
      t0 = __builtin_amdgcn_s_memtime();                                                                 \
      r0 = __builtin_amdgcn_s_memrealtime();                                                             \
    }                                                                                                    \
    uint32_t a = seed ^ threadIdx.x, b = a * 3u, c = a * 5u, d = a * 7u, e = a * 11u, f = a * 13u,       \
             g = a * 17u, h = a * 19u, kw = seed + blockIdx.x;                                           \
    uint32_t x0 = a * 23u, x1 = a * 29u, x2 = a * 31u, x3 = a * 37u, x4 = a * 41u, x5 = a * 43u,         \
             x6 = a * 47u, x7 = a * 53u;                                                                 \
    uint32_t n = ITERS;                                                                                  \
    asm volatile(".p2align 6\n.rept " #PH "\ns_nop 0\n.endr\n"                                           \
                 "1:\n" BODY##K "s_sub_u32 %[n], %[n], 1\ns_cmp_lg_u32 %[n], 0\ns_cbranch_scc1 1b\n"     \
                 : [a] "+v"(a), [b] "+v"(b), [c] "+v"(c), [d] "+v"(d), [e] "+v"(e), [f] "+v"(f),        \
                   [g] "+v"(g), [h] "+v"(h), [t0] "+v"(x0), [t1] "+v"(x1), [t2] "+v"(x2), [t3] "+v"(x3), \
                   [t4] "+v"(x4), [t5] "+v"(x5), [t6] "+v"(x6), [t7] "+v"(x7), [n] "+s"(n)              \
                 : [kw] "v"(kw)                                                                          \
                 : "scc");                                                                               \
    if ((a ^ b ^ c ^ d ^ e ^ f ^ g ^ h ^ x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7) == 0x12345678u) out[0] = a; \
    if (threadIdx.x == 0) {                                                                              \
      stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;                                        \
      stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;                                \
    }                                                                                                    \
  }
#define BOTH(K) KERNEL(K, 0) KERNEL(K, 1)
BOTH(0)
BOTH(1)
BOTH(2)
BOTH(3)
BOTH(4)
BOTH(5)
BOTH(6)

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
  kfn k[7][2] = {{probe_0_0, probe_0_1}, {probe_1_0, probe_1_1}, {probe_2_0, probe_2_1}, {probe_3_0, probe_3_1},
                 {probe_4_0, probe_4_1}, {probe_5_0, probe_5_1}, {probe_6_0, probe_6_1}};
  static const char* names[7] = {"alignbit", "bitop3", "add_e64", "add3", "alignbit_bitop3_1to1",
                                 "alignbit2_bitop3_2to1", "sha_rounds"};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  std::vector<unsigned long long> h(2 * (size_t)grid);
  for (int round = 0; round < 3; ++round) {
    for (int K = 0; K < 7; ++K)
      for (int ph = 0; ph < 2; ++ph) {
        float best = 1e30f;
        double clk = 0;
        for (int rep = 0; rep < 4; ++rep) {
          (void)hipEventRecord(e0, 0);
          hipLaunchKernelGGL(k[K][ph], dim3(grid), dim3(256), 0, 0, 0x1234u + rep, out, stamps);
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
        const double wave_instr = (double)grid * 4.0 * ITERS * body_len[K];
        const double cpi = prop.multiProcessorCount * 4.0 * clk * best * 1e-3 / wave_instr;
        printf("{\"round\": %d, \"stream\": \"%s\", \"phase_mod8\": %d, \"ms\": %.4f, \"clock_ghz\": %.4f, "
               "\"cycles_per_instr\": %.4f}\n",
               round, names[K], 4 * ph, best, clk / 1e9, cpi);
        fflush(stdout);
      }
  }
  return 0;
}
