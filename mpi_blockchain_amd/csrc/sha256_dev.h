// SHA-256 building blocks for gfx950 (CDNA4) device code.
//
// FIPS 180-4 SHA-256 as picosha2 implements it (picosha2.h:46-136): 64-round
// compression over big-endian words.  Every primitive maps to ONE gfx950 VALU
// instruction:
//   rotr            v_alignbit_b32  (x:x >> n)
//   3-way xor       v_bitop3_b32 0x96
//   Ch(e,f,g)       v_bitop3_b32 0xCA   (e ? f : g)
//   Maj(a,b,c)      v_bitop3_b32 0xE8
//   a+b+c           v_add3_u32          (formed by the compiler)
// so a round is 14 VALU ops and a schedule word 10 (DESIGN.md "op count").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace powdev {

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
__device__ __forceinline__ uint32_t bsig0(uint32_t a) { return xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)); }
__device__ __forceinline__ uint32_t bsig1(uint32_t e) { return xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)); }
__device__ __forceinline__ uint32_t ssig0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
__device__ __forceinline__ uint32_t ssig1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }

// picosha2.h:46-57
__device__ constexpr uint32_t K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
// picosha2.h:59-61
__device__ constexpr uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                       0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

// Working variables of one compression.  Rounds "rename" instead of moving:
// in the fully unrolled code the shifts below are SSA renames, not v_mov.
struct St {
  uint32_t a, b, c, d, e, f, g, h;
};

// One round with separate K (uniform) and W (per lane): add3(h,S1,Ch), add3(.,K,W).
__device__ __forceinline__ void round_k_w(St& s, uint32_t k, uint32_t w) {
  uint32_t t1 = s.h + bsig1(s.e) + ch(s.e, s.f, s.g) + k + w;
  uint32_t t2 = bsig0(s.a) + maj(s.a, s.b, s.c);
  s.h = s.g; s.g = s.f; s.f = s.e; s.e = s.d + t1;
  s.d = s.c; s.c = s.b; s.b = s.a; s.a = t1 + t2;
}

// The same rounds with their 14 VALU ops in a fixed issue order, pinned by
// scheduling barriers: the three bitop3/add ops that read only the round's
// inputs (Ch, Maj, h + K + W) first, then the six rotations (a's, then e's),
// the two Sigma xor3s, T1, e', a'.  Among 17 orders measured on the 2^32 sweep
// (profiles/r02/ab/ab5-ab7), this one was fastest: 2.0% less kernel time than
// the compiler's own order of the same instructions.
#define POW_SB() __builtin_amdgcn_sched_barrier(0)
// TWO_TERMS: h + k + w (v_add3; k and w separate), else h + kw (v_add).
template <bool TWO_TERMS>
__device__ __forceinline__ void round_ordered(St& s, uint32_t k, uint32_t w) {
  const uint32_t chv = ch(s.e, s.f, s.g); POW_SB();
  const uint32_t mj = maj(s.a, s.b, s.c); POW_SB();
  const uint32_t hk = TWO_TERMS ? s.h + k + w : s.h + k; POW_SB();
  const uint32_t r2 = rotr(s.a, 2); POW_SB();
  const uint32_t r13 = rotr(s.a, 13); POW_SB();
  const uint32_t r22 = rotr(s.a, 22); POW_SB();
  const uint32_t r6 = rotr(s.e, 6); POW_SB();
  const uint32_t r11 = rotr(s.e, 11); POW_SB();
  const uint32_t r25 = rotr(s.e, 25); POW_SB();
  const uint32_t S0 = xor3(r2, r13, r22); POW_SB();
  const uint32_t S1 = xor3(r6, r11, r25); POW_SB();
  const uint32_t t1 = hk + S1 + chv; POW_SB();
  const uint32_t en = s.d + t1; POW_SB();
  const uint32_t an = t1 + S0 + mj; POW_SB();
  s.h = s.g; s.g = s.f; s.f = s.e; s.e = en;
  s.d = s.c; s.c = s.b; s.b = s.a; s.a = an;
}
__device__ __forceinline__ void round_kw_o(St& s, uint32_t kw) { round_ordered<false>(s, kw, 0u); }
__device__ __forceinline__ void round_k_w_o(St& s, uint32_t k, uint32_t w) { round_ordered<true>(s, k, w); }

// Four rounds of a constant-schedule chunk (K+W from LDS) as ONE asm block:
// 56 VALU instructions, every one 8 bytes long (v_add_u32_e64, never the
// 4-byte VOP2 form hipcc picks).  Each round issues the e-path first, its
// full-rate ops between the rotations (rotr e 6, Ch, Maj, rotr e 11, h + K+W,
// rotr e 25, S1, T1, e'), then the a-path (three rotations, S0, a'):
// 0.22-0.31% less kernel time than round_ordered's order (Ch, Maj, the six
// rotations, S0, S1, then the adds) in three A/B runs at the pinned phase
// (profiles/r03/ab/ab17_*); every form measured within 2% in isolation
// (tools/round_probe.hip).
// Each block starts with `.p2align 3; s_nop 0`, so every VALU instruction of
// a chunk sits 4 bytes past an 8-byte boundary whatever the compiler puts
// before the block (its s_waitcnt for the LDS words, a hazard s_nop): on
// gfx950 that phase issues ~5% faster than the other for this stream
// (tools/place_probe*.hip, profiles/r03/probe/).
//   POW_RX(a, b, c, d, e, f, g, h, d', h', KW): one round reading a..h and
//   writing e' into d' and a' into h' (d' = d, h' = h for in-place).
#define POW_RX(a, b, c, d, e, f, g, h, dd, hh, KW)                     \
  "\tv_alignbit_b32 %[t5], " e ", " e ", 6\n"                           \
  "\tv_bitop3_b32 %[t0], " e ", " f ", " g " bitop3:0xca\n"             \
  "\tv_bitop3_b32 %[t1], " a ", " b ", " c " bitop3:0xe8\n"             \
  "\tv_alignbit_b32 %[t6], " e ", " e ", 11\n"                          \
  "\tv_add_u32_e64 " hh ", " h ", " KW "\n"                             \
  "\tv_alignbit_b32 %[t7], " e ", " e ", 25\n"                          \
  "\tv_bitop3_b32 %[t5], %[t5], %[t6], %[t7] bitop3:0x96\n"             \
  "\tv_add3_u32 " hh ", " hh ", %[t5], %[t0]\n"                         \
  "\tv_add_u32_e64 " dd ", " d ", " hh "\n"                             \
  "\tv_alignbit_b32 %[t2], " a ", " a ", 2\n"                           \
  "\tv_alignbit_b32 %[t3], " a ", " a ", 13\n"                          \
  "\tv_alignbit_b32 %[t4], " a ", " a ", 22\n"                          \
  "\tv_bitop3_b32 %[t2], %[t2], %[t3], %[t4] bitop3:0x96\n"             \
  "\tv_add3_u32 " hh ", " hh ", %[t2], %[t1]\n"
#define POW_R(a, b, c, d, e, f, g, h, KW) POW_RX(a, b, c, d, e, f, g, h, d, h, KW)
#define POW_PHASE "\t.p2align 3\n\ts_nop 0\n"
#define POW_TEMPS                                                                                    \
  [t0] "=&v"(x0), [t1] "=&v"(x1), [t2] "=&v"(x2), [t3] "=&v"(x3), [t4] "=&v"(x4), [t5] "=&v"(x5),   \
      [t6] "=&v"(x6), [t7] "=&v"(x7)
// Chunk 0's rounds, K+W (or K) from SGPRs (scalar loads of the template
// constants), W per lane, in the same e-path-first order.  The additions keep
// hipcc's forms (and rates):
//   rounds 4-15, K+W uniform:  h' = h + Ch (full rate);  T1 = h' + S1 + KW (v_add3, SGPR)
//   rounds 16-63, K uniform, W per lane: T1 = Ch + h + S1; T1 += K + W (two v_add3, SGPR)
#define POW_R_KWS(a, b, c, d, e, f, g, h, KWS)                          \
  "\tv_alignbit_b32 %[t5], " e ", " e ", 6\n"                         \
  "\tv_bitop3_b32 %[t0], " e ", " f ", " g " bitop3:0xca\n"           \
  "\tv_bitop3_b32 %[t1], " a ", " b ", " c " bitop3:0xe8\n"           \
  "\tv_alignbit_b32 %[t6], " e ", " e ", 11\n"                        \
  "\tv_add_u32_e64 " h ", " h ", %[t0]\n"                             \
  "\tv_alignbit_b32 %[t7], " e ", " e ", 25\n"                        \
  "\tv_bitop3_b32 %[t5], %[t5], %[t6], %[t7] bitop3:0x96\n"           \
  "\tv_add3_u32 " h ", " h ", %[t5], " KWS "\n"                       \
  "\tv_add_u32_e64 " d ", " d ", " h "\n"                             \
  "\tv_alignbit_b32 %[t2], " a ", " a ", 2\n"                         \
  "\tv_alignbit_b32 %[t3], " a ", " a ", 13\n"                        \
  "\tv_alignbit_b32 %[t4], " a ", " a ", 22\n"                        \
  "\tv_bitop3_b32 %[t2], %[t2], %[t3], %[t4] bitop3:0x96\n"           \
  "\tv_add3_u32 " h ", %[t2], %[t1], " h "\n"
#define POW_R_KS_W(a, b, c, d, e, f, g, h, KS, W)                       \
  "\tv_alignbit_b32 %[t5], " e ", " e ", 6\n"                         \
  "\tv_bitop3_b32 %[t0], " e ", " f ", " g " bitop3:0xca\n"           \
  "\tv_bitop3_b32 %[t1], " a ", " b ", " c " bitop3:0xe8\n"           \
  "\tv_alignbit_b32 %[t6], " e ", " e ", 11\n"                        \
  "\tv_alignbit_b32 %[t7], " e ", " e ", 25\n"                        \
  "\tv_bitop3_b32 %[t5], %[t5], %[t6], %[t7] bitop3:0x96\n"           \
  "\tv_add3_u32 " h ", %[t0], " h ", %[t5]\n"                         \
  "\tv_add3_u32 " h ", " h ", " KS ", " W "\n"                        \
  "\tv_add_u32_e64 " d ", " d ", " h "\n"                             \
  "\tv_alignbit_b32 %[t2], " a ", " a ", 2\n"                         \
  "\tv_alignbit_b32 %[t3], " a ", " a ", 13\n"                        \
  "\tv_alignbit_b32 %[t4], " a ", " a ", 22\n"                        \
  "\tv_bitop3_b32 %[t2], %[t2], %[t3], %[t4] bitop3:0x96\n"           \
  "\tv_add3_u32 " h ", %[t2], %[t1], " h "\n"
#define POW_STATE_OPS                                                                             \
  [a] "+v"(s.a), [b] "+v"(s.b), [c] "+v"(s.c), [d] "+v"(s.d), [e] "+v"(s.e), [f] "+v"(s.f),        \
      [g] "+v"(s.g), [h] "+v"(s.h)
// One-wave issue order (K2', round 4): with no other wave to issue between
// them, an instruction right after the one it depends on waits for its
// result, so the 14 ops of a round are spread to keep every operand at least
// two instructions old: the e rotations, Ch, then the a rotations interleaved
// with S1, h + K+W and T1, then Maj, S0, e', a'.  (The 8-wave order above
// groups the e-path first: other waves fill the gaps.)  K2' kernel 10.12 ->
// 10.04 us against the 8-wave order (profiles/r04/ab/ab2_*): one wave issues
// ~5 cycles per instruction either way, so the count, not the order, sets it.
#ifndef POW_1W_ORDER
#define POW_1W_ORDER 1
#endif
#if POW_1W_ORDER
#define POW_RX_1W(a, b, c, d, e, f, g, h, dd, hh, KW)                  \
  "\tv_alignbit_b32 %[t5], " e ", " e ", 6\n"                           \
  "\tv_alignbit_b32 %[t6], " e ", " e ", 11\n"                          \
  "\tv_alignbit_b32 %[t7], " e ", " e ", 25\n"                          \
  "\tv_bitop3_b32 %[t0], " e ", " f ", " g " bitop3:0xca\n"             \
  "\tv_alignbit_b32 %[t2], " a ", " a ", 2\n"                           \
  "\tv_bitop3_b32 %[t5], %[t5], %[t6], %[t7] bitop3:0x96\n"             \
  "\tv_alignbit_b32 %[t3], " a ", " a ", 13\n"                          \
  "\tv_add_u32_e64 " hh ", " h ", " KW "\n"                             \
  "\tv_alignbit_b32 %[t4], " a ", " a ", 22\n"                          \
  "\tv_add3_u32 " hh ", " hh ", %[t5], %[t0]\n"                         \
  "\tv_bitop3_b32 %[t1], " a ", " b ", " c " bitop3:0xe8\n"             \
  "\tv_bitop3_b32 %[t2], %[t2], %[t3], %[t4] bitop3:0x96\n"             \
  "\tv_add_u32_e64 " dd ", " d ", " hh "\n"                             \
  "\tv_add3_u32 " hh ", " hh ", %[t2], %[t1]\n"
#else
#define POW_RX_1W POW_RX
#endif
// Four rounds in the one-wave order, K+W in VGPRs (from LDS), in place;
// volatile: ordered with the explicit LDS reads and waits around them.
__device__ __forceinline__ void rounds4_kwv_asm_v(St& s, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  uint32_t x0, x1, x2, x3, x4, x5, x6, x7;
  asm volatile(POW_RX_1W("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[d]", "%[h]", "%[k0]")
               POW_RX_1W("%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[c]", "%[g]", "%[k1]")
               POW_RX_1W("%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[b]", "%[f]", "%[k2]")
               POW_RX_1W("%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[a]", "%[e]", "%[k3]")
               : POW_STATE_OPS, POW_TEMPS
               : [k0] "v"(k0), [k1] "v"(k1), [k2] "v"(k2), [k3] "v"(k3));
  s = St{s.e, s.f, s.g, s.h, s.a, s.b, s.c, s.d};
}
// ... and the first group of a chunk reading the chunk's input state without
// modifying it (the feed-forward needs it): no copies at the chunk boundary.
__device__ __forceinline__ St rounds4_asm_from_v(const St& in, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  uint32_t x0, x1, x2, x3, x4, x5, x6, x7;
  St o;
  asm volatile(POW_RX_1W("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[od]", "%[oh]", "%[k0]")
               POW_RX_1W("%[oh]", "%[a]", "%[b]", "%[c]", "%[od]", "%[e]", "%[f]", "%[g]", "%[oc]", "%[og]", "%[k1]")
               POW_RX_1W("%[og]", "%[oh]", "%[a]", "%[b]", "%[oc]", "%[od]", "%[e]", "%[f]", "%[ob]", "%[of]", "%[k2]")
               POW_RX_1W("%[of]", "%[og]", "%[oh]", "%[a]", "%[ob]", "%[oc]", "%[od]", "%[e]", "%[oa]", "%[oe]", "%[k3]")
               : [oa] "=&v"(o.a), [ob] "=&v"(o.b), [oc] "=&v"(o.c), [od] "=&v"(o.d), [oe] "=&v"(o.e),
                 [of] "=&v"(o.f), [og] "=&v"(o.g), [oh] "=&v"(o.h), POW_TEMPS
               : [a] "v"(in.a), [b] "v"(in.b), [c] "v"(in.c), [d] "v"(in.d), [e] "v"(in.e), [f] "v"(in.f),
                 [g] "v"(in.g), [h] "v"(in.h), [k0] "v"(k0), [k1] "v"(k1), [k2] "v"(k2), [k3] "v"(k3));
  return St{o.e, o.f, o.g, o.h, o.a, o.b, o.c, o.d};
}
// Four chunk-0 rounds with uniform K+W words (SGPR operands).
__device__ __forceinline__ void rounds4_kws_asm(St& s, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  uint32_t x0, x1, x2, x3, x4, x5, x6, x7;
  asm volatile(POW_PHASE
               POW_R_KWS("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[k0]")
               POW_R_KWS("%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[k1]")
               POW_R_KWS("%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[k2]")
               POW_R_KWS("%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[k3]")
               : POW_STATE_OPS, POW_TEMPS
               : [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3));
  s = St{s.e, s.f, s.g, s.h, s.a, s.b, s.c, s.d};
}
// The same for rounds 4-7, reading the state entering round 4 (most of it
// the per-prefix state, live across the j-loop) without writing it: each
// state word is written once, into a fresh register (no copies).
#define POW_R_KWS_X(a, b, c, d, e, f, g, h, dd, hh, KWS)                 \
  "\tv_alignbit_b32 %[t5], " e ", " e ", 6\n"                         \
  "\tv_bitop3_b32 %[t0], " e ", " f ", " g " bitop3:0xca\n"           \
  "\tv_bitop3_b32 %[t1], " a ", " b ", " c " bitop3:0xe8\n"           \
  "\tv_alignbit_b32 %[t6], " e ", " e ", 11\n"                        \
  "\tv_add_u32_e64 " hh ", " h ", %[t0]\n"                            \
  "\tv_alignbit_b32 %[t7], " e ", " e ", 25\n"                        \
  "\tv_bitop3_b32 %[t5], %[t5], %[t6], %[t7] bitop3:0x96\n"           \
  "\tv_add3_u32 " hh ", " hh ", %[t5], " KWS "\n"                     \
  "\tv_add_u32_e64 " dd ", " d ", " hh "\n"                           \
  "\tv_alignbit_b32 %[t2], " a ", " a ", 2\n"                         \
  "\tv_alignbit_b32 %[t3], " a ", " a ", 13\n"                        \
  "\tv_alignbit_b32 %[t4], " a ", " a ", 22\n"                        \
  "\tv_bitop3_b32 %[t2], %[t2], %[t3], %[t4] bitop3:0x96\n"           \
  "\tv_add3_u32 " hh ", %[t2], %[t1], " hh "\n"
__device__ __forceinline__ St rounds4_kws_asm_from(const St& in, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  uint32_t x0, x1, x2, x3, x4, x5, x6, x7;
  St o;
  asm volatile(POW_PHASE
               POW_R_KWS_X("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[od]", "%[oh]", "%[k0]")
               POW_R_KWS_X("%[oh]", "%[a]", "%[b]", "%[c]", "%[od]", "%[e]", "%[f]", "%[g]", "%[oc]", "%[og]", "%[k1]")
               POW_R_KWS_X("%[og]", "%[oh]", "%[a]", "%[b]", "%[oc]", "%[od]", "%[e]", "%[f]", "%[ob]", "%[of]", "%[k2]")
               POW_R_KWS_X("%[of]", "%[og]", "%[oh]", "%[a]", "%[ob]", "%[oc]", "%[od]", "%[e]", "%[oa]", "%[oe]", "%[k3]")
               : [oa] "=&v"(o.a), [ob] "=&v"(o.b), [oc] "=&v"(o.c), [od] "=&v"(o.d), [oe] "=&v"(o.e),
                 [of] "=&v"(o.f), [og] "=&v"(o.g), [oh] "=&v"(o.h), POW_TEMPS
               : [a] "v"(in.a), [b] "v"(in.b), [c] "v"(in.c), [d] "v"(in.d), [e] "v"(in.e), [f] "v"(in.f),
                 [g] "v"(in.g), [h] "v"(in.h), [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3));
  return St{o.e, o.f, o.g, o.h, o.a, o.b, o.c, o.d};
}
// A schedule word of chunk 0 (i >= 33): W = s1(W[i-2]) + W[i-7] + s0(W[i-15]) + W[i-16],
// every instruction 8 bytes (v_lshrrev_b32_e64).  Uses t0..t3.
#define POW_W(dst, wm2, wm7, wm15, wm16)                                \
  "\tv_alignbit_b32 %[t0], " wm2 ", " wm2 ", 17\n"                    \
  "\tv_alignbit_b32 %[t1], " wm2 ", " wm2 ", 19\n"                    \
  "\tv_lshrrev_b32_e64 %[t2], 10, " wm2 "\n"                          \
  "\tv_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n"           \
  "\tv_alignbit_b32 %[t1], " wm15 ", " wm15 ", 7\n"                   \
  "\tv_alignbit_b32 %[t2], " wm15 ", " wm15 ", 18\n"                  \
  "\tv_lshrrev_b32_e64 %[t3], 3, " wm15 "\n"                          \
  "\tv_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n"           \
  "\tv_add3_u32 %[t0], %[t0], " wm7 ", %[t1]\n"                       \
  "\tv_add_u32_e64 " dst ", %[t0], " wm16 "\n"
// Four chunk-0 rounds i..i+3 (i >= 36) with their schedule words computed in
// the same block, each just before its round.  W[i+k] is written over
// W[i-16+k] (dead once W[i+k] is formed; POW_W reads its W[i-16] last), so the
// block needs no registers beyond the window: w[0..3] = W[i-16..i-13] in,
// W[i..i+3] out; w4 = W[i-12], v7[k] = W[i-7+k], m2 = W[i-2], m1 = W[i-1].
__device__ __forceinline__ void rounds4_sched_asm(St& s, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3,
                                                  uint32_t* w, uint32_t w4, const uint32_t* v7, uint32_t m2,
                                                  uint32_t m1) {
  uint32_t x0, x1, x2, x3, x4, x5, x6, x7;
  asm volatile(POW_PHASE
               POW_W("%[o0]", "%[m2]", "%[v0]", "%[o1]", "%[o0]")
               POW_R_KS_W("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[k0]", "%[o0]")
               POW_W("%[o1]", "%[m1]", "%[v1]", "%[o2]", "%[o1]")
               POW_R_KS_W("%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[k1]", "%[o1]")
               POW_W("%[o2]", "%[o0]", "%[v2]", "%[o3]", "%[o2]")
               POW_R_KS_W("%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[k2]", "%[o2]")
               POW_W("%[o3]", "%[o1]", "%[v3]", "%[w4]", "%[o3]")
               POW_R_KS_W("%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[k3]", "%[o3]")
               : POW_STATE_OPS, POW_TEMPS, [o0] "+v"(w[0]), [o1] "+v"(w[1]), [o2] "+v"(w[2]), [o3] "+v"(w[3])
               : [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3), [w4] "v"(w4), [v0] "v"(v7[0]),
                 [v1] "v"(v7[1]), [v2] "v"(v7[2]), [v3] "v"(v7[3]), [m2] "v"(m2), [m1] "v"(m1));
  s = St{s.e, s.f, s.g, s.h, s.a, s.b, s.c, s.d};
}

// Chunk 0's schedule words 18-35 fold template-uniform and per-prefix terms
// (DESIGN.md §4): their forms, every instruction 8 bytes, t0..t2 temporaries.
//   POW_WA:  dst = x + y                       (y: VGPR or SGPR)
//   POW_WS:  dst = s1(x) + y
//   POW_WS3: dst = s1(x) + y + z
#define POW_SIG1(x)                                                     \
  "\tv_alignbit_b32 %[t0], " x ", " x ", 17\n"                        \
  "\tv_alignbit_b32 %[t1], " x ", " x ", 19\n"                        \
  "\tv_lshrrev_b32_e64 %[t2], 10, " x "\n"                            \
  "\tv_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n"
#define POW_WA(dst, x, y) "\tv_add_u32_e64 " dst ", " x ", " y "\n"
#define POW_WS(dst, x, y) POW_SIG1(x) "\tv_add_u32_e64 " dst ", %[t0], " y "\n"
#define POW_WS3(dst, x, y, z) POW_SIG1(x) "\tv_add3_u32 " dst ", %[t0], " y ", " z "\n"
// The four round slots of a group: state names rotate by one per round.
#define POW_R0(K, W) POW_R_KS_W("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", K, W)
#define POW_R1(K, W) POW_R_KS_W("%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", K, W)
#define POW_R2(K, W) POW_R_KS_W("%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", K, W)
#define POW_R3(K, W) POW_R_KS_W("%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", K, W)
#define POW_KS [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3)

// Chunk-0 rounds 16-35 in five groups G = 0..4 (rounds 16 + 4G .. 19 + 4G),
// each schedule word computed inside the group just before its round.  w[] is
// the chunk's schedule (w[16], w[17] given; the group writes its four words).
// The uniform terms (SGPRs) and per-prefix terms (VGPRs):
//   G = 0: ua = U18(j), ub = W3(j); pa = c18, pb = c19
//   G = 1: ua, ub, uc = U20..U22;    pa = c23
//   G = 2: ua, ub, uc = U25..U27;    pa = c24
//   G = 3: ua, ub, uc = U28..U30;    pa = c31
//   G = 4:                           pa = c32
template <int G>
__device__ __forceinline__ void rounds4_w_asm(St& s, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, uint32_t* w,
                                              uint32_t ua, uint32_t ub, uint32_t uc, uint32_t pa, uint32_t pb) {
  uint32_t x0, x1, x2, x3, x4, x5, x6, x7;
  if constexpr (G == 0) {
    (void)uc;
    asm volatile(POW_PHASE
                 POW_R0("%[k0]", "%[w16]") POW_R1("%[k1]", "%[w17]")
                 POW_WA("%[w18]", "%[pa]", "%[ua]") POW_R2("%[k2]", "%[w18]")
                 POW_WA("%[w19]", "%[pb]", "%[ub]") POW_R3("%[k3]", "%[w19]")
                 : POW_STATE_OPS, POW_TEMPS, [w18] "=&v"(w[18]), [w19] "=&v"(w[19])
                 : POW_KS, [w16] "v"(w[16]), [w17] "v"(w[17]), [pa] "v"(pa), [pb] "v"(pb), [ua] "s"(ua),
                   [ub] "s"(ub));
  } else if constexpr (G == 1) {
    (void)pb;
    asm volatile(POW_PHASE
                 POW_WS("%[w20]", "%[w18]", "%[ua]") POW_R0("%[k0]", "%[w20]")
                 POW_WS("%[w21]", "%[w19]", "%[ub]") POW_R1("%[k1]", "%[w21]")
                 POW_WS("%[w22]", "%[w20]", "%[uc]") POW_R2("%[k2]", "%[w22]")
                 POW_WS("%[w23]", "%[w21]", "%[pa]") POW_R3("%[k3]", "%[w23]")
                 : POW_STATE_OPS, POW_TEMPS, [w20] "=&v"(w[20]), [w21] "=&v"(w[21]), [w22] "=&v"(w[22]),
                   [w23] "=&v"(w[23])
                 : POW_KS, [w18] "v"(w[18]), [w19] "v"(w[19]), [pa] "v"(pa), [ua] "s"(ua), [ub] "s"(ub),
                   [uc] "s"(uc));
  } else if constexpr (G == 2) {
    (void)pb;
    asm volatile(POW_PHASE
                 POW_WS("%[w24]", "%[w22]", "%[pa]") POW_R0("%[k0]", "%[w24]")
                 POW_WS3("%[w25]", "%[w23]", "%[w18]", "%[ua]") POW_R1("%[k1]", "%[w25]")
                 POW_WS3("%[w26]", "%[w24]", "%[w19]", "%[ub]") POW_R2("%[k2]", "%[w26]")
                 POW_WS3("%[w27]", "%[w25]", "%[w20]", "%[uc]") POW_R3("%[k3]", "%[w27]")
                 : POW_STATE_OPS, POW_TEMPS, [w24] "=&v"(w[24]), [w25] "=&v"(w[25]), [w26] "=&v"(w[26]),
                   [w27] "=&v"(w[27])
                 : POW_KS, [w18] "v"(w[18]), [w19] "v"(w[19]), [w20] "v"(w[20]), [w22] "v"(w[22]),
                   [w23] "v"(w[23]), [pa] "v"(pa), [ua] "s"(ua), [ub] "s"(ub), [uc] "s"(uc));
  } else if constexpr (G == 3) {
    (void)pb;
    asm volatile(POW_PHASE
                 POW_WS3("%[w28]", "%[w26]", "%[w21]", "%[ua]") POW_R0("%[k0]", "%[w28]")
                 POW_WS3("%[w29]", "%[w27]", "%[w22]", "%[ub]") POW_R1("%[k1]", "%[w29]")
                 POW_WS3("%[w30]", "%[w28]", "%[w23]", "%[uc]") POW_R2("%[k2]", "%[w30]")
                 POW_WS3("%[w31]", "%[w29]", "%[w24]", "%[pa]") POW_R3("%[k3]", "%[w31]")
                 : POW_STATE_OPS, POW_TEMPS, [w28] "=&v"(w[28]), [w29] "=&v"(w[29]), [w30] "=&v"(w[30]),
                   [w31] "=&v"(w[31])
                 : POW_KS, [w21] "v"(w[21]), [w22] "v"(w[22]), [w23] "v"(w[23]), [w24] "v"(w[24]),
                   [w26] "v"(w[26]), [w27] "v"(w[27]), [pa] "v"(pa), [ua] "s"(ua), [ub] "s"(ub), [uc] "s"(uc));
  } else {
    // W33..35 are the generic form, into fresh registers: W17 is per prefix
    // (live across the j-loop) and W18, W19 are read again by W34, W35
    (void)ua, (void)ub, (void)uc, (void)pb;
    asm volatile(POW_PHASE
                 POW_WS3("%[w32]", "%[w30]", "%[w25]", "%[pa]") POW_R0("%[k0]", "%[w32]")
                 POW_W("%[w33]", "%[w31]", "%[w26]", "%[w18]", "%[w17]") POW_R1("%[k1]", "%[w33]")
                 POW_W("%[w34]", "%[w32]", "%[w27]", "%[w19]", "%[w18]") POW_R2("%[k2]", "%[w34]")
                 POW_W("%[w35]", "%[w33]", "%[w28]", "%[w20]", "%[w19]") POW_R3("%[k3]", "%[w35]")
                 : POW_STATE_OPS, POW_TEMPS, [w32] "=&v"(w[32]), [w33] "=&v"(w[33]), [w34] "=&v"(w[34]),
                   [w35] "=&v"(w[35])
                 : POW_KS, [w17] "v"(w[17]), [w18] "v"(w[18]), [w19] "v"(w[19]), [w20] "v"(w[20]),
                   [w25] "v"(w[25]), [w26] "v"(w[26]), [w27] "v"(w[27]), [w28] "v"(w[28]), [w30] "v"(w[30]),
                   [w31] "v"(w[31]), [pa] "v"(pa));
  }
  s = St{s.e, s.f, s.g, s.h, s.a, s.b, s.c, s.d};
}

// In place: the state is read and written in the same registers.
__device__ __forceinline__ void rounds4_asm(St& s, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  uint32_t x0, x1, x2, x3, x4, x5, x6, x7;
  asm volatile(POW_PHASE
               POW_R("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[k0]")
               POW_R("%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[k1]")
               POW_R("%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[k2]")
               POW_R("%[f]", "%[g]", "%[h]", "%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[k3]")
               : [a] "+v"(s.a), [b] "+v"(s.b), [c] "+v"(s.c), [d] "+v"(s.d), [e] "+v"(s.e), [f] "+v"(s.f),
                 [g] "+v"(s.g), [h] "+v"(s.h), POW_TEMPS
               : [k0] "v"(k0), [k1] "v"(k1), [k2] "v"(k2), [k3] "v"(k3));
  // after four rounds the state sits in the registers of (e, f, g, h, a, b, c, d)
  s = St{s.e, s.f, s.g, s.h, s.a, s.b, s.c, s.d};
}
// A chunk's first four rounds: the input state (the chaining value H, still
// needed for the feed-forward) is only read; each of the 8 state words is
// written once, into a fresh register, so no copies of H are needed.
__device__ __forceinline__ St rounds4_asm_from(const St& in, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  uint32_t x0, x1, x2, x3, x4, x5, x6, x7;
  St o;
  asm volatile(POW_PHASE
               POW_RX("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[od]", "%[oh]", "%[k0]")
               POW_RX("%[oh]", "%[a]", "%[b]", "%[c]", "%[od]", "%[e]", "%[f]", "%[g]", "%[oc]", "%[og]", "%[k1]")
               POW_RX("%[og]", "%[oh]", "%[a]", "%[b]", "%[oc]", "%[od]", "%[e]", "%[f]", "%[ob]", "%[of]", "%[k2]")
               POW_RX("%[of]", "%[og]", "%[oh]", "%[a]", "%[ob]", "%[oc]", "%[od]", "%[e]", "%[oa]", "%[oe]", "%[k3]")
               : [oa] "=&v"(o.a), [ob] "=&v"(o.b), [oc] "=&v"(o.c), [od] "=&v"(o.d), [oe] "=&v"(o.e),
                 [of] "=&v"(o.f), [og] "=&v"(o.g), [oh] "=&v"(o.h), POW_TEMPS
               : [a] "v"(in.a), [b] "v"(in.b), [c] "v"(in.c), [d] "v"(in.d), [e] "v"(in.e), [f] "v"(in.f),
                 [g] "v"(in.g), [h] "v"(in.h), [k0] "v"(k0), [k1] "v"(k1), [k2] "v"(k2), [k3] "v"(k3));
  return St{o.e, o.f, o.g, o.h, o.a, o.b, o.c, o.d};
}


// The previous chunk's feed-forward (H += t: 8 v_add_u32_e64) and the next
// chunk's first four rounds from the new H, in one group: t (the previous
// chunk's final state, dead once added) receives the new chunk's state, so
// the group needs no registers beyond H, t and the temporaries.
__device__ __forceinline__ void rounds4_asm_ff(St& H, St& t, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  uint32_t x0, x1, x2, x3, x4, x5, x6, x7;
  asm volatile(POW_PHASE
               "\tv_add_u32_e64 %[a], %[a], %[oa]\n\tv_add_u32_e64 %[b], %[b], %[ob]\n"
               "\tv_add_u32_e64 %[c], %[c], %[oc]\n\tv_add_u32_e64 %[d], %[d], %[od]\n"
               "\tv_add_u32_e64 %[e], %[e], %[oe]\n\tv_add_u32_e64 %[f], %[f], %[of]\n"
               "\tv_add_u32_e64 %[g], %[g], %[og]\n\tv_add_u32_e64 %[h], %[h], %[oh]\n"
               POW_RX("%[a]", "%[b]", "%[c]", "%[d]", "%[e]", "%[f]", "%[g]", "%[h]", "%[od]", "%[oh]", "%[k0]")
               POW_RX("%[oh]", "%[a]", "%[b]", "%[c]", "%[od]", "%[e]", "%[f]", "%[g]", "%[oc]", "%[og]", "%[k1]")
               POW_RX("%[og]", "%[oh]", "%[a]", "%[b]", "%[oc]", "%[od]", "%[e]", "%[f]", "%[ob]", "%[of]", "%[k2]")
               POW_RX("%[of]", "%[og]", "%[oh]", "%[a]", "%[ob]", "%[oc]", "%[od]", "%[e]", "%[oa]", "%[oe]", "%[k3]")
               : [oa] "+v"(t.a), [ob] "+v"(t.b), [oc] "+v"(t.c), [od] "+v"(t.d), [oe] "+v"(t.e), [of] "+v"(t.f),
                 [og] "+v"(t.g), [oh] "+v"(t.h), [a] "+v"(H.a), [b] "+v"(H.b), [c] "+v"(H.c), [d] "+v"(H.d),
                 [e] "+v"(H.e), [f] "+v"(H.f), [g] "+v"(H.g), [h] "+v"(H.h), POW_TEMPS
               : [k0] "v"(k0), [k1] "v"(k1), [k2] "v"(k2), [k3] "v"(k3));
  t = St{t.e, t.f, t.g, t.h, t.a, t.b, t.c, t.d};
}

// Generic compression of one chunk (used by the single-hash kernel K2; not on
// the mining hot loop).  The schedule is a 16-word ring computed just ahead
// of its round, and scheduling barriers every 4 rounds keep the compiler from
// running the schedule far ahead: K2 stays at 44 VGPRs (it must fit beside a
// running K1, which leaves one workgroup slot free for it) at the speed of a
// fully unrolled 78-VGPR version (19.9 us per hash, tools/k2_c.c).
__device__ __forceinline__ void compress(uint32_t h[8], const uint32_t win[16]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = win[i];
  St s{h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]};
#pragma unroll
  for (int r = 0; r < 4; ++r) {  // 4 x 16 rounds; ring indices are constants
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (r > 0) w[k] = ssig1(w[(k + 14) & 15]) + w[(k + 9) & 15] + ssig0(w[(k + 1) & 15]) + w[k];
      round_k_w(s, K[16 * r + k], w[k]);
      if ((k & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // keep the schedule from running ahead
    }
  }
  h[0] += s.a; h[1] += s.b; h[2] += s.c; h[3] += s.d;
  h[4] += s.e; h[5] += s.f; h[6] += s.g; h[7] += s.h;
}

}  // namespace powdev
