// gfx950 kernels of the proof-of-work hot path.
//
// K1  pow_search<MODE, FULL>  — the mining inner loop of proof_of_work
//     (node.cpp:302-308): nonce (block.cpp:61-72) -> 270-byte message
//     (block.cpp:79-88) -> SHA-256 (picosha2.h:88-136, 5 chunks) ->
//     leading-zero-bit test (block.cpp:91-96, trap T3) for every counter of a
//     range.  MODE 0 = sweep (record every solution), 1 = mine (lowest
//     solving counter, early exit).  FULL = difficulty > 32 bits.
// K2  pow_hash_kernel — block_to_hash (block.cpp:74-77) for a batch of blocks;
// K2' pow_hash_one — the same for ONE block at low latency (validation).
//
// Work decomposition of K1 (DESIGN.md "Kernel K1"): counter c = 62*P + j.
//   * one LANE owns a prefix P (nonce chars 0..7, message words W1, W2);
//     the prefix-dependent rounds 1-2 (and all of round 3 but its K+W3 add)
//     and schedule terms are computed once per prefix, then
//   * the lane loops over j = 0..61 (the last nonce char, word W3) — j is
//     wave-uniform, so W3 and every term derived from it are scalar loads.
//   Per trial the lane runs chunk-0 rounds 4..63 and chunks 1-4 (whose K+W
//   are template constants, read from an LDS copy) — no memory traffic.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pow_template.h"
#include "sha256_dev.h"

using namespace powdev;


namespace {

__device__ __forceinline__ uint32_t digit_char(uint32_t d) {
  // block.cpp:61-72: 0-25 'a'+d, 26-51 'A'+d-26, 52-61 '0'+d-52
  return d + (d < 26u ? 97u : (d < 52u ? 39u : 0xFFFFFFFCu));
}

__device__ __forceinline__ unsigned long long uniform64(unsigned long long v) {
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

// Constant-address-space (addrspace 4) pointer: loads through it are known
// read-only, so wave-uniform ones become scalar loads (s_load_dwordx*) into
// SGPRs, which a VOP3 instruction reads as its one scalar operand.
typedef const __attribute__((address_space(4))) uint32_t* cptr;

__device__ __forceinline__ cptr as_const(const uint32_t* p) {
  return (cptr)(const __attribute__((address_space(1))) uint32_t*)p;
}

// Make a uniform constant pointer opaque and data-dependent on `dep`, so the
// scalar loads through it can neither be hoisted out of the j-loop (256 K+W
// words do not fit in SGPRs: hoisting spills them) nor issued before `dep`.
__device__ __forceinline__ cptr pin(cptr p, uint32_t dep) {
  asm volatile("" : "+s"(p) : "v"(dep));
  return p;
}

// 64 rounds of a chunk whose K+W are template constants (chunks 1-4, K1 and
// K1'): the K+W words come from LDS (a per-workgroup copy of C->kw) into
// VGPRs, 4 per ds_read_b128 (every lane reads the same address: a
// broadcast), so the K+W add has two VGPR operands.  A VALU op with an SGPR
// operand issues at half rate on gfx950; moving these 256 adds
// per trial off SGPRs made the sweep 0.7% faster (profiles/r02/ab/).  Chunk
// 0's K and K+W words stay scalar loads: its SGPR operands sit in v_add3
// (half rate anyway), and LDS copies of them measured 0.4-0.6% slower.
//
// ASM (K1): each group of 4 rounds is one asm block of 8-byte instructions
// held 4 bytes past an 8-byte boundary (sha256_dev.h rounds4_asm): 4.1% less
// kernel time than the compiler's mix of 4- and 8-byte encodings, whose phase
// flipped at every 4-byte instruction (profiles/r03/ab/ab8_*).  K1' (one wave
// per SIMD at low d) keeps the compiler's rounds: its time-to-block at d = 13
// went from 0.034 to 0.038 ms with the asm groups.
template <bool ASM>
__device__ __forceinline__ void const_chunk_lds(St& t, const uint32_t* lkw) {
  if (ASM) {
    POW_SB();
    const uint4 v0 = *reinterpret_cast<const uint4*>(lkw);
    POW_SB();
    t = rounds4_asm_from(t, v0.x, v0.y, v0.z, v0.w);
#pragma unroll
    for (int g = 4; g < 64; g += 4) {
      POW_SB();
      const uint4 v = *reinterpret_cast<const uint4*>(lkw + g);
      POW_SB();
      rounds4_asm(t, v.x, v.y, v.z, v.w);
    }
    POW_SB();
  } else {
#pragma unroll
    for (int g = 0; g < 64; g += 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(lkw + g);
      round_kw_o(t, v.x);
      round_kw_o(t, v.y);
      round_kw_o(t, v.z);
      round_kw_o(t, v.w);
    }
  }
}

// Chunks as 14-op asm groups in the one-wave order (sha256_dev.h POW_RX_1W)
// whose K+W reads are issued one group (~56 instructions) ahead of their use
// and waited for explicitly; the first group of each chunk leaves the chunk's
// input state untouched for the feed-forward.  H holds the first chunk's
// input state; afterwards H holds the last chunk's input state and t its
// final state.  Used by K2' (5 chunks, one wave: kernel 10.9 -> 10.0 us with
// the host-side schedule, profiles/r04/ab/ab1_*, ab2_*).  For K1' at 1-2 waves
// per SIMD (chunks 1-4, POW_LAT_PIPE=1) it measured no better than the
// compiler's rounds, whose reads sit ~10 instructions ahead: time-to-block
// d = 9 0.0237 -> 0.0243 ms, d = 13 0.0334 -> 0.0340, d = 17 0.0473 -> 0.0471
// (profiles/r04/ab/ab4_*), so K1' keeps the compiler's form.
#ifndef POW_LAT_PIPE
#define POW_LAT_PIPE 0
#endif
// K2' (one block, one wave) runs its 5 chunks through the same helper (NC = 5).
// The read and its wait are two asm statements: the compiler does not track
// loads issued from inline asm, so nothing stops it from placing a copy of q
// between them.  tests/test_build.py (test_asm_lds_reads_waited_before_use)
// checks on the generated code that no instruction touches an in-flight read's
// registers before its lgkmcnt(0) wait.
template <int NC = 4>
__device__ __forceinline__ void const_chunks_lds_pipelined(uint32_t H[8], St& t, const uint32_t* lk) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint32_t lbase = (uint32_t)(uintptr_t)lk;
  u32x4 q;
  asm volatile("ds_read_b128 %0, %1" : "=v"(q) : "v"(lbase));
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int g = 0; g < 64; g += 4) {
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(q));  // q holds its words from here on
      const u32x4 cur = q;
      if (64 * c + g + 4 < 64 * NC)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(q) : "v"(lbase), "i"(4 * (64 * c + g + 4)));
      if (g == 0)
        t = rounds4_asm_from_v(St{H[0], H[1], H[2], H[3], H[4], H[5], H[6], H[7]}, cur.x, cur.y, cur.z, cur.w);
      else
        rounds4_kwv_asm_v(t, cur.x, cur.y, cur.z, cur.w);
    }
    if (c < NC - 1) {
      H[0] += t.a; H[1] += t.b; H[2] += t.c; H[3] += t.d;
      H[4] += t.e; H[5] += t.f; H[6] += t.g; H[7] += t.h;
    }
  }
}

// Chunks 2-4 (K1): the previous chunk's feed-forward H += t and this chunk's
// first four rounds as one group (rounds4_asm_ff), then 15 groups as above;
// t ends as this chunk's final state.
__device__ __forceinline__ void const_chunk_lds_ff(St& H, St& t, const uint32_t* lkw) {
  POW_SB();
  const uint4 v0 = *reinterpret_cast<const uint4*>(lkw);
  POW_SB();
  rounds4_asm_ff(H, t, v0.x, v0.y, v0.z, v0.w);
#pragma unroll
  for (int g = 4; g < 64; g += 4) {
    POW_SB();
    const uint4 v = *reinterpret_cast<const uint4*>(lkw + g);
    POW_SB();
    rounds4_asm(t, v.x, v.y, v.z, v.w);
  }
  POW_SB();
}

// Append the 32-entry-aligned part of a wave's staged solutions (nst <= 255,
// in LDS) to the global list with one atomic; the remainder (< 32) moves to
// the stage front.  Every reservation is a multiple of 32 entries, so each
// block starts on a 128-byte line of `out` (hipMalloc alignment) and lanes
// write it as whole lines, 16 B per lane: no line is written in parts by two
// waves (with 4-B lanes at arbitrary offsets the memory-side write requests
// were 2.3x the list's bytes, profiles/r01/final/pmc_summary.json).
__device__ __forceinline__ void flush_stage(uint32_t* wst, uint32_t& nst, uint32_t lane, PowResult* res,
                                            uint32_t* out, uint32_t cap) {
  const uint32_t n = nst & ~31u;
  unsigned long long got = 0;
  if (lane == 0) got = atomicAdd(&res->count, (unsigned long long)n);
  const unsigned long long base = uniform64(got);  // 64-bit: 2^32 solutions at d = 0
  const uint32_t i = lane * 4u;  // n <= 224: one pass of <= 56 lanes
  if (i < n) {
    const uint32_t e0 = wst[i], e1 = wst[i + 1u], e2 = wst[i + 2u], e3 = wst[i + 3u];
    const unsigned long long o = base + i;
    if (o + 4u <= cap && ((uintptr_t)out & 15u) == 0) {
      *reinterpret_cast<uint4*>(out + o) = make_uint4(e0, e1, e2, e3);
    } else {
      if (o < cap) out[o] = e0;
      if (o + 1u < cap) out[o + 1u] = e1;
      if (o + 2u < cap) out[o + 2u] = e2;
      if (o + 3u < cap) out[o + 3u] = e3;
    }
  }
  const uint32_t rem = nst - n;  // source [n, n + rem) and target [0, rem) do not overlap (n >= 32 > rem)
  const uint32_t t = lane < rem ? wst[n + lane] : 0u;
  if (lane < rem) wst[lane] = t;
  nst = rem;
}

// A wave's last staged solutions (< 32) go to the side list res->tail_buf; the
// host appends it to the main list after the launch.
__device__ __forceinline__ void flush_tail(const uint32_t* wst, uint32_t nst, uint32_t lane, PowResult* res) {
  uint32_t got = 0;
  if (lane == 0) got = atomicAdd(&res->tail, nst);
  const uint32_t base = __builtin_amdgcn_readfirstlane(got);
  uint32_t* const tail = res->tail_buf;
  const uint32_t tail_cap = res->tail_cap;
  if (lane < nst && base + lane < tail_cap) tail[base + lane] = wst[lane];
}

// Should this wave stop for a reason outside its own launch?  Two sources:
//   * pow_cancel: the caller's epoch (mapped host memory) moved off the
//     launch's epoch;
//   * a bound stop board: a peer (another GPU or context of the same search)
//     published a solution below `lowest_abs`, the lowest absolute counter the
//     wave would still compute (~0 in any-mode: any peer solution stops it).
// Host memory is read by ONE sentinel wave (workgroup 0, wave 0: one PCIe
// read per poll, not one per wave).  It raises device words every wave polls:
// `cancelled`, and `peer_abs` = the lowest peer counter seen.  A memset or
// copy into device memory could not do this: the copy engine's blit kernel
// waits for a free CU, and the mining kernel holds them all.  Wave-uniform.
__device__ __forceinline__ bool poll_stop(const PowWatch& w, unsigned int* cancelled, unsigned long long* peer_abs,
                                          unsigned long long lowest_abs) {
  const uint32_t watch = w.watch_epoch;
  const unsigned long long* const board = w.board;
  if (!watch && !board) return false;
  if (blockIdx.x == 0 && threadIdx.x < 64u) {
    const uint32_t lane = threadIdx.x;
    if (watch) {
      const unsigned int now = __hip_atomic_load(w.host_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((uint32_t)__builtin_amdgcn_readfirstlane(now) != w.launch_epoch && lane == 0)
        __hip_atomic_store(cancelled, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (board) {
      unsigned long long c = ~0ull;
      if (lane < w.board_n && board + lane != w.board_mine) {
        const unsigned long long v = __hip_atomic_load(board + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((uint32_t)(v >> POW_BOARD_SHIFT) == w.board_tag && (v & POW_BOARD_NONE) != POW_BOARD_NONE)
          c = v & POW_BOARD_NONE;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(c, off, 64);
        c = o < c ? o : c;
      }
      if (lane == 0 && c != ~0ull) atomicMin(peer_abs, c);
    }
  }
  if (watch && __builtin_amdgcn_readfirstlane(
                   __hip_atomic_load(cancelled, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0u)
    return true;
  return board && uniform64(__hip_atomic_load(peer_abs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < lowest_abs;
}

// A hit of a mine launch goes to this context's board slot at once (system
// scope, straight into host memory), so the peers' sentinels see it within
// their next poll.  Only a lane whose atomicMin lowered the launch's minimum
// stores (the callers below), so the slot's value only falls, except in the
// rare race of two lowering lanes whose stores land out of order; the host
// posts the call's exact result when it returns.  Any stored value is a real
// solution, and a peer only ever compares against it.
__device__ __forceinline__ void publish_hit(const PowWatch& w, unsigned long long rel) {
  unsigned long long* const mine = w.board_mine;
  if (mine)
    __hip_atomic_store(mine, ((unsigned long long)w.board_tag << POW_BOARD_SHIFT) | (w.abs_start + rel),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Leading zero bits of the 256-bit digest H[0..7] >= d  (d > 32 path only).
__device__ __forceinline__ bool full_test(const uint32_t H[8], uint32_t d) {
  uint32_t lz = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (lz == 32u * i) lz += (H[i] == 0u) ? 32u : (uint32_t)__builtin_clz(H[i]);
  }
  return lz >= d;
}

}  // namespace

#define POW_BATCH 8u  // chunks claimed per global atomic (one workgroup's batch)

// Work distribution: each wave dequeues chunks of 64 consecutive prefixes (one
// per lane) in increasing order, through its workgroup's batches of POW_BATCH
// chunks (one global atomic on res->next per batch).  Any grid
// size and residency gives a tail of at most one chunk per wave (~2 ms), and
// mine mode stays exact: a wave stops only when the lowest solution already
// found is below its next chunk, and every lower chunk is owned by a wave
// that is still running it or still sits in a workgroup's batch (a batch's
// chunks are handed out in increasing order, so a workgroup whose wave saw its
// next chunk above the solution holds no lower one).
// 80 SGPRs: the measured admission rule for 256-thread workgroups on gfx950
// (MI355X_MICROARCH.md "Residency") gives 8 per CU only at <= 80; at the
// compiler's natural ~92 it is 7.
template <int MODE, bool FULL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_sgpr(80), amdgpu_waves_per_eu(8))) void pow_search(
    const PowConsts* __restrict__ C, PowLaunch L, uint32_t* __restrict__ out,
    PowResult* __restrict__ res) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t iters = 0;
  // Sweep mode: solutions are staged per wave in LDS and flushed in 32-entry
  // blocks (one atomic + whole-line stores per >= 192 solutions); the lowest solution
  // is kept per lane and min-reduced once per wave at exit.  One atomic per
  // solution would make every solution a separate memory-side request
  // (~0.68 GB of requests per 2^32 sweep at d = 9 for 34 MB of data).  A
  // 256-entry stage flushed at >= 192 (round 3; was 128 at >= 64) cut the
  // flush atomics ~3x: WRITE_SIZE 42.8 -> 40.0 MB per 2^32 window at equal
  // speed (profiles/r03/ab/ab16_*).
  __shared__ __attribute__((aligned(16))) uint32_t stage[4][256];
  uint32_t* wst = stage[threadIdx.x >> 6];
  uint32_t nst = 0;                     // staged entries (wave-uniform)
  // lowest solution of this lane, 32-bit (a sweep window is <= 2^32 counters,
  // so rel < 2^32): one VGPR, not two (the 64-bit form spilled to scratch once
  // the chunk-0 schedule moved into the asm groups).  0xFFFFFFFF means none; a
  // solution AT rel = 0xFFFFFFFF goes straight to res->min_rel (at most once).
  uint32_t mymin = 0xFFFFFFFFu;
  // chunks 1-4's K+W words, one per thread (blockDim = 256 = 4 x 64)
  __shared__ __attribute__((aligned(16))) uint32_t lkw[4 * 64];
  lkw[threadIdx.x] = (&C->kw[0][0])[threadIdx.x];
  __shared__ uint32_t sibs_done;  // mine modes, workgroup 0: waves 1..3 that have finished (see the exit)
  __shared__ uint32_t wg_tick;                  // dequeue tickets of this workgroup
  __shared__ unsigned long long wg_ring[4];     // (batch + 1) << 32 | base of the batch's first chunk
  __shared__ uint32_t wg_reads[4];              // reads of the batch that holds each ring slot
  if (threadIdx.x == 0) {
    sibs_done = 0;
    wg_tick = 0;
  }
  if (threadIdx.x < 4) {
    wg_ring[threadIdx.x] = 0;
    wg_reads[threadIdx.x] = POW_BATCH - 1u;  // as if a batch -4..-1 had been read in full
  }
  __syncthreads();

  // (test library only: the sentinel idles from the start, pow_template.h)
  const bool sentinel_idle = MODE >= 1 && (L.mode & POW_LAUNCH_SENTINEL_IDLE) && blockIdx.x == 0 && threadIdx.x < 64u;
  for (;;) {
    if (sentinel_idle) break;
    // Dequeue one 64-prefix chunk.  Tickets come from an LDS counter: ticket
    // t is chunk t % POW_BATCH of the workgroup's batch t / POW_BATCH, and the
    // wave holding a batch's first ticket claims the whole batch (POW_BATCH
    // chunks) with ONE global atomic and publishes its base in a 4-slot LDS
    // ring tagged with the batch number; the batch's other waves read it there.
    // A slot is reused by batch b + 4 only after all POW_BATCH - 1 readers of
    // batch b have read it (wg_reads): every drawn ticket is read before its
    // wave can leave, and batch b's leader published before drawing again, so
    // the wait ends (without it, a reader stalled while the other
    // waves drew 25 tickets would have spun forever on an overwritten tag).
    // Chunks are still handed out one per wave in increasing order within a
    // workgroup, and batches in increasing order across the grid.
    // 8 chunks per atomic: WRITE_SIZE 73.2 -> 42.7 MB per 2^32 window (the
    // atomics were ~37 MB of it) at equal speed (profiles/r03/ab/ab4_*).
    uint32_t got = 0;
    if (lane == 0) {
      const uint32_t t = atomicAdd(&wg_tick, 1u);
      const uint32_t b = t / POW_BATCH, slot = t % POW_BATCH;
      unsigned long long* const ring = &wg_ring[b & 3u];
      uint32_t* const reads = &wg_reads[b & 3u];
      if (slot == 0) {
        got = atomicAdd(&res->next, 64u * POW_BATCH);
        while (__hip_atomic_load(reads, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != POW_BATCH - 1u)
          __builtin_amdgcn_s_sleep(1);  // batch b - 4 still has a reader: never in practice
        __hip_atomic_store(reads, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(ring, ((unsigned long long)(b + 1u) << 32) | got, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
        unsigned long long v;
        while ((uint32_t)((v = __hip_atomic_load(ring, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) >> 32) !=
               b + 1u)
          __builtin_amdgcn_s_sleep(1);
        got = (uint32_t)v + 64u * slot;
        __hip_atomic_fetch_add(reads, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    const uint32_t rbase = __builtin_amdgcn_readfirstlane(got);
    if (rbase >= L.n_prefix) break;
    if (MODE >= 1) {
      // Early exit.  MODE 1: every counter of this and later chunks is
      // >= 62*rbase - off0.  MODE 2 (first found): any solution ends the search.
      unsigned long long f =
          __hip_atomic_load(&res->min_rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      f = uniform64(f);
      long long lo = (long long)rbase * 62 - (long long)L.off0;
      if (MODE == 2 && f != ~0ull) break;
      if (lo > 0 && f < (unsigned long long)lo) break;
      if (poll_stop(res->watch, &res->cancelled, &res->peer_abs,
                    MODE == 2 ? ~0ull : res->watch.abs_start + (lo > 0 ? (unsigned long long)lo : 0ull)))
        break;
    }
    const uint32_t r = rbase + lane;

    // ---- per-prefix: nonce digits 0..7 = base digits + r (base 62) ----
    uint32_t dg[8];
    {
      uint32_t x = r, carry = 0;
#pragma unroll
      for (int i = 7; i >= 0; --i) {
        uint32_t q = x / 62u;
        uint32_t s = L.base_digit[i] + (x - q * 62u) + carry;
        x = q;
        carry = s >= 62u ? 1u : 0u;
        dg[i] = carry ? s - 62u : s;
      }
    }
    const uint32_t W1 = (digit_char(dg[0]) << 24) | (digit_char(dg[1]) << 16) |
                        (digit_char(dg[2]) << 8) | digit_char(dg[3]);
    const uint32_t W2 = (digit_char(dg[4]) << 24) | (digit_char(dg[5]) << 16) |
                        (digit_char(dg[6]) << 8) | digit_char(dg[7]);

    // ---- per-prefix: chunk-0 rounds 1, 2 and the prefix schedule terms ----
    St s2{C->st0[0], C->st0[1], C->st0[2], C->st0[3], C->st0[4], C->st0[5], C->st0[6], C->st0[7]};
    round_k_w(s2, K[1], W1);
    round_k_w(s2, K[2], W2);
    const uint32_t W16 = C->u16 + ssig0(W1);
    const uint32_t W17 = C->u17 + ssig0(W2) + W1;
    const uint32_t c18 = ssig1(W16) + W2;
    const uint32_t c19 = ssig1(W17) + C->u19;
    const uint32_t c23 = W16 + C->u23;
    const uint32_t c24 = W17 + C->u24;
    const uint32_t c31 = ssig0(W16) + C->w15;
    const uint32_t c32 = ssig0(W17) + W16;
    // Round 3 adds K[3] + W3(j) to a per-prefix T1 and nothing else depends
    // on j: a4 = A3 + kw3(j), e4 = E3 + kw3(j) (2 adds per trial, not 14 ops).
    const uint32_t P3 = s2.h + bsig1(s2.e) + ch(s2.e, s2.f, s2.g);
    const uint32_t A3 = P3 + bsig0(s2.a) + maj(s2.a, s2.b, s2.c);
    const uint32_t E3 = s2.d + P3;

    bool stop = false;
    for (uint32_t j = 0; j < POW_J; ++j) {
      if (MODE == 1 && j != 0 && (j & 1u) == 0) {
        // Mid-chunk exit: this wave's remaining counters are all >= 62*rbase + j - off0.
        unsigned long long f =
            __hip_atomic_load(&res->min_rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        f = uniform64(f);
        long long lo = (long long)rbase * 62 + j - (long long)L.off0;
        if (lo > 0 && f < (unsigned long long)lo) break;
        // (cancelled, or a peer holds a lower counter: every later chunk is higher still)
        if (poll_stop(res->watch, &res->cancelled, &res->peer_abs,
                      res->watch.abs_start + (lo > 0 ? (unsigned long long)lo : 0ull))) {
          stop = true;
          break;
        }
      }
      if (MODE == 2 && j != 0) {
        unsigned long long f =
            __hip_atomic_load(&res->min_rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (uniform64(f) != ~0ull || poll_stop(res->watch, &res->cancelled, &res->peer_abs, ~0ull)) {
          stop = true;
          break;
        }
      }
      ++iters;
      // ---------------- chunk 0, rounds 4..63 ----------------
      cptr Cb = as_const(reinterpret_cast<const uint32_t*>(C));
      cptr J = pin(Cb, s2.a ^ j);  // per-j words and the chunk-0 uniform terms
      const uint32_t kw3 = J[PC_KW3 + j];
      const St s4{A3 + kw3, s2.a, s2.b, s2.c, E3 + kw3, s2.e, s2.f, s2.g};
      // Code placement: the trial block runs ~1.1% faster when it starts on an
      // 8-byte boundary than 4 bytes past one (same instructions; A/B in one
      // process, profiles/r03/ab/ab3_code_placement.log: 498.3 vs 504.0 ms per
      // 2^32 window).  The alignment pins that phase whatever code precedes the
      // loop; it costs at most one s_nop per trial (tests/test_build.py).
      asm volatile(".p2align 3");
      // Every round and schedule word of the trial is hand-written asm, four
      // rounds per group, each group at the pinned code phase (sha256_dev.h;
      // DESIGN.md §4 "Code placement"), the rounds in round_ordered's issue
      // order; each schedule word is computed just before its round
      // (computing it one round earlier measured 0.9% slower, profiles/r02/ab/ab8).
      POW_SB();
      St s = rounds4_kws_asm_from(s4, J[PC_KW0 + 4], J[PC_KW0 + 5], J[PC_KW0 + 6], J[PC_KW0 + 7]);
#pragma unroll
      for (int i = 8; i < 16; i += 4) {
        POW_SB();
        rounds4_kws_asm(s, J[PC_KW0 + i], J[PC_KW0 + i + 1], J[PC_KW0 + i + 2], J[PC_KW0 + i + 3]);
      }
      uint32_t w[64];
      w[16] = W16;
      w[17] = W17;
      // rounds i..i+3 with their four schedule words, as one asm group at the
      // pinned phase (template-uniform and per-prefix terms folded)
      auto rnd4 = [&](int i, cptr Kx) {
        if (i >= 36) {  // generic schedule words: computed inside the group
          POW_SB();
          uint32_t q[4] = {w[i - 16], w[i - 15], w[i - 14], w[i - 13]};
          rounds4_sched_asm(s, Kx[i], Kx[i + 1], Kx[i + 2], Kx[i + 3], q, w[i - 12], &w[i - 7], w[i - 2], w[i - 1]);
          w[i] = q[0];
          w[i + 1] = q[1];
          w[i + 2] = q[2];
          w[i + 3] = q[3];
          return;
        }
        // rounds 16-35: the folded schedule words inside the groups
        POW_SB();
        if (i == 16)
          rounds4_w_asm<0>(s, Kx[16], Kx[17], Kx[18], Kx[19], w, J[PC_U18 + j], J[PC_W3 + j], 0u, c18, c19);
        else if (i == 20)
          rounds4_w_asm<1>(s, Kx[20], Kx[21], Kx[22], Kx[23], w, J[PC_U20], J[PC_U20 + 1], J[PC_U20 + 2], c23, 0u);
        else if (i == 24)
          rounds4_w_asm<2>(s, Kx[24], Kx[25], Kx[26], Kx[27], w, J[PC_U25], J[PC_U25 + 1], J[PC_U25 + 2], c24, 0u);
        else if (i == 28)
          rounds4_w_asm<3>(s, Kx[28], Kx[29], Kx[30], Kx[31], w, J[PC_U25 + 3], J[PC_U25 + 4], J[PC_U25 + 5], c31,
                           0u);
        else
          rounds4_w_asm<4>(s, Kx[32], Kx[33], Kx[34], Kx[35], w, 0u, 0u, 0u, c32, 0u);
      };
      {
        cptr Kp = pin(Cb + PC_K, s.e);  // K[16..63], streamed like the K+W words
#pragma unroll
        for (int i = 16; i < 32; i += 4) rnd4(i, Kp);
      }
      {
        cptr K2 = pin(Cb + PC_K, s.e);
#pragma unroll
        for (int i = 32; i < 48; i += 4) rnd4(i, K2);
      }
      {
        cptr K3 = pin(Cb + PC_K, s.e);
#pragma unroll
        for (int i = 48; i < 64; i += 4) rnd4(i, K3);
      }
      uint32_t H[8] = {IV[0] + s.a, IV[1] + s.b, IV[2] + s.c, IV[3] + s.d,
                       IV[4] + s.e, IV[5] + s.f, IV[6] + s.g, IV[7] + s.h};

      // ---------------- chunks 1..4: constant schedule ----------------
      // Chunk c's feed-forward (H += t) opens chunk c + 1's first asm group
      // (8-byte adds at the pinned phase, sha256_dev.h rounds4_asm_ff).
      St Hs{H[0], H[1], H[2], H[3], H[4], H[5], H[6], H[7]};
      St t = Hs;
      const_chunk_lds<true>(t, lkw);
      // (chunk 4's last round still computes e' although H0 needs only a':
      // skipping it measured 469.40 vs 469.36 ms per window, profiles/r04/ab/ab5_*)
#pragma unroll
      for (int c = 1; c < 4; ++c) const_chunk_lds_ff(Hs, t, lkw + 64 * c);
      // ---------------- chunk 4 (last): only what the test needs ----------------
      const uint32_t h0 = Hs.a + t.a;

      bool hit = h0 <= L.thr;
      if (FULL && hit) {
        uint32_t D[8] = {h0, Hs.b + t.b, Hs.c + t.c, Hs.d + t.d,
                         Hs.e + t.e, Hs.f + t.f, Hs.g + t.g, Hs.h + t.h};
        hit = full_test(D, L.diff);
      }
      if (MODE != 0) {
        if (__builtin_expect(hit, 0)) {
          const unsigned long long rel = (unsigned long long)r * 62ull + j - L.off0;
          // rel < count also rejects j < off0 at r = 0 (wraps) and lanes past the end
          if (rel < L.count && rel < atomicMin(&res->min_rel, rel)) publish_hit(res->watch, rel);
        }
      } else {
        bool ok = false;
        uint32_t relv = 0;
        if (__builtin_expect(hit, 0)) {
          const unsigned long long rel = (unsigned long long)r * 62ull + j - L.off0;
          ok = rel < L.count;
          relv = (uint32_t)rel;
          if (ok && relv < mymin) mymin = relv;
          if (ok && relv == 0xFFFFFFFFu) atomicMin(&res->min_rel, rel);
        }
        const unsigned long long m = __ballot(ok);
        if (m) {  // wave-uniform
          const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          if (ok) wst[nst + rank] = relv;
          nst += (uint32_t)__popcll(m);
          if (nst >= 192) flush_stage(wst, nst, lane, res, out, L.cap);
        }
      }
    }
    if (MODE >= 1 && stop) break;
  }
  if (MODE == 0) {
    if (nst >= 32) flush_stage(wst, nst, lane, res, out, L.cap);
    if (nst) flush_tail(wst, nst, lane, res);
    // wave min of the per-lane minima, one atomic per wave
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint32_t o = __shfl_xor(mymin, off, 64);
      mymin = o < mymin ? o : mymin;
    }
    if (lane == 0 && mymin != 0xFFFFFFFFu) atomicMin(&res->min_rel, (unsigned long long)mymin);
  }
  if (MODE >= 1) {
    // The sentinel (workgroup 0, wave 0) is the only reader of host memory
    // (poll_stop).  It must outlive every other wave of the launch: once it
    // leaves, the waves still finishing their last chunks would miss a
    // pow_cancel or a peer's hit (up to ~1 chunk, ~4 ms).  So it keeps
    // polling, with s_sleep between polls, until its three siblings are done
    // and every other workgroup has counted its exit.  Every other wave has
    // finite work (and a workgroup that starts late finds the queue empty),
    // so the wait ends.
    if (blockIdx.x == 0) {
      if (threadIdx.x >= 64u) {
        if (lane == 0) __hip_atomic_fetch_add(&sibs_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if (res->watch.watch_epoch || res->watch.board) {
        for (;;) {
          const uint32_t sd = __hip_atomic_load(&sibs_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const uint32_t ex = __hip_atomic_load(&res->wg_exits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (__builtin_amdgcn_readfirstlane(sd) >= (blockDim.x >> 6) - 1u &&
              __builtin_amdgcn_readfirstlane(ex) >= gridDim.x - 1u)
            break;
          (void)poll_stop(res->watch, &res->cancelled, &res->peer_abs, ~0ull);
          __builtin_amdgcn_s_sleep(32);
        }
      }
    }
    // Trials computed (lanes of a wave run the same iterations), summed per
    // workgroup first: after a hit in MODE 2 all ~8,000 waves exit within one
    // step, and one atomic each on the same address would queue for tens of us.
    __shared__ uint32_t wave_iters[4];
    if ((threadIdx.x & 63u) == 0) wave_iters[threadIdx.x >> 6] = iters;
    __syncthreads();
    if (threadIdx.x == 0) {
      atomicAdd(&res->hashes,
                (unsigned long long)(wave_iters[0] + wave_iters[1] + wave_iters[2] + wave_iters[3]) * 64ull);
      if (blockIdx.x != 0) atomicAdd(&res->wg_exits, 1u);
    }
  }
}

template __global__ void pow_search<0, false>(const PowConsts*, PowLaunch, uint32_t*, PowResult*);
template __global__ void pow_search<0, true>(const PowConsts*, PowLaunch, uint32_t*, PowResult*);
template __global__ void pow_search<1, false>(const PowConsts*, PowLaunch, uint32_t*, PowResult*);
template __global__ void pow_search<1, true>(const PowConsts*, PowLaunch, uint32_t*, PowResult*);
template __global__ void pow_search<2, false>(const PowConsts*, PowLaunch, uint32_t*, PowResult*);
template __global__ void pow_search<2, true>(const PowConsts*, PowLaunch, uint32_t*, PowResult*);

// K1' pow_search_lat<FULL> — latency form of the mining loop for short
// ranges (the first sub-rounds of pow_mine).  One counter per lane; in
// iteration k, wave w of W takes the 64 CONSECUTIVE counters starting at
// 64*(k*W + w), so the grid sweeps the range in increasing order and the
// search can stop one wave-iteration after the first solution (the lowest
// counter is final once every lower iteration has finished).  The assignment
// is static: with thousands of waves a shared atomic queue head (~88 dequeues
// per us) would itself bound the rate.  K1 instead keeps the lowest
// prefixes' wave busy for all 62 values of the last digit (~0.6 ms on an idle
// SIMD).  Costs ~5% more VALU per trial than K1 (no j-uniform terms).
//
// Launch overhead matters at this size (~17 us of kernel at d = 9), so the
// constants travel as a by-value kernel argument (kernarg segment, read by
// scalar loads like any constant; chunks 1-4's K+W by one vector load per
// thread into LDS) instead of a separate H2D copy, the device result words
// `res` reset themselves (the last wave to exit re-initialises them), and that
// last wave also copies them to `hout`, mapped host memory: a launch is one
// dispatch and no copy kernels.
template <bool FULL, bool ANY, bool ASM>
__global__ __launch_bounds__(256) void pow_search_lat(
    const PowConstsLat C0, PowLaunchLat L, PowResult* __restrict__ res, PowResult* __restrict__ hout) {
  (void)C0;
  // C0 is the first kernel argument, at offset 0 of the kernarg segment: read
  // it through that (constant address space) pointer.  Taking C0's address
  // would make the compiler copy 1.4 KB into private memory per lane.  Every
  // grid reads the kernarg copy: since chunks 1-4's K+W moved to one vector
  // load per thread (LDS copy), 256-1024 workgroups fetch it faster than an
  // H2D copy (a blit kernel and a second dispatch) takes: time-to-block
  // d = 13 0.0447 -> 0.0408 ms, d = 17 0.0578 -> 0.0544 ms (profiles/r02/ab/ab15).
  const cptr Cb = (cptr)__builtin_amdgcn_kernarg_segment_ptr();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
  const uint32_t nwaves = L.nwg * 4u;  // L.nwg == gridDim.x (no implicit kernel argument needed)
  uint32_t iters = 0;
  bool wrote_hit = false;  // this wave wrote a hit record (wave-uniform after each step)
  __shared__ uint32_t wg_iters;  // wave-iterations of this workgroup
  if (threadIdx.x == 0) wg_iters = 0;
  // The launch's duration is measured on the GPU (constant-rate realtime
  // counter): the host returns when `done` is published, not at the kernel's
  // completion signal, so it records no HIP events around the launch.
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    __hip_atomic_store(&res->t_start, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // into host memory, not waited for: the host's watchdog tells a launch
    // that never ran from one that ran and did not finish
    __hip_atomic_store(&hout->started, L.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // chunks 1-4's K+W words (PowConsts::kw), one per thread, as in K1
  __shared__ __attribute__((aligned(16))) uint32_t lkw[4 * 64];
  lkw[threadIdx.x] = Cb[threadIdx.x];
  __syncthreads();
  for (unsigned long long qq = (unsigned long long)wave * 64u; qq < L.count;
       qq += (unsigned long long)nwaves * 64u) {
    const uint32_t q = (uint32_t)qq;
    // The stop checks wait for device (and, for the sentinel wave, host)
    // memory before the trial can start: skipped in a wave's first iteration,
    // where no hit of this launch can exist yet and a cancel or a peer's hit
    // is seen one trial later.  At d <= 13 most launches are that one
    // iteration, and those round trips were on the time-to-block's path.
    if (iters != 0) {
      unsigned long long f =
          __hip_atomic_load(&res->min_rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      f = uniform64(f);
      if (ANY ? f != ~0ull : f < (unsigned long long)q) break;
      if (poll_stop(L.watch, &res->cancelled, &res->peer_abs, ANY ? ~0ull : L.watch.abs_start + q)) break;
    }
    ++iters;
    const uint32_t rel = q + lane;
    uint32_t dg[9];
    {
      uint32_t x = rel, carry = 0;
#pragma unroll
      for (int i = 8; i >= 0; --i) {
        uint32_t quo = x / 62u;
        uint32_t sm = L.base_digit[i] + (x - quo * 62u) + carry;
        x = quo;
        carry = sm >= 62u ? 1u : 0u;
        dg[i] = carry ? sm - 62u : sm;
      }
    }
    cptr P = pin(Cb, rel);
    uint32_t w[64];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = P[LC_WRAW + i];
    w[1] = (digit_char(dg[0]) << 24) | (digit_char(dg[1]) << 16) | (digit_char(dg[2]) << 8) | digit_char(dg[3]);
    w[2] = (digit_char(dg[4]) << 24) | (digit_char(dg[5]) << 16) | (digit_char(dg[6]) << 8) | digit_char(dg[7]);
    w[3] |= digit_char(dg[8]) << 24;  // [nonce[8], NUL, prev0, prev1]
    St s{P[LC_ST0 + 0], P[LC_ST0 + 1], P[LC_ST0 + 2], P[LC_ST0 + 3],
         P[LC_ST0 + 4], P[LC_ST0 + 5], P[LC_ST0 + 6], P[LC_ST0 + 7]};  // after round 0
    round_k_w_o(s, P[LC_K + 1], w[1]);
    round_k_w_o(s, P[LC_K + 2], w[2]);
    round_k_w_o(s, P[LC_K + 3], w[3]);
#pragma unroll
    for (int i = 4; i < 16; ++i) round_kw_o(s, P[LC_KW0 + i]);
    cptr Kp = pin(Cb + LC_K, s.e);
#pragma unroll
    for (int i = 16; i < 40; ++i) {
      w[i] = ssig1(w[i - 2]) + w[i - 7] + ssig0(w[i - 15]) + w[i - 16];
      round_k_w_o(s, Kp[i], w[i]);
    }
    cptr K2 = pin(Cb + LC_K, s.e);
#pragma unroll
    for (int i = 40; i < 64; ++i) {
      w[i] = ssig1(w[i - 2]) + w[i - 7] + ssig0(w[i - 15]) + w[i - 16];
      round_k_w_o(s, K2[i], w[i]);
    }
    uint32_t H[8] = {IV[0] + s.a, IV[1] + s.b, IV[2] + s.c, IV[3] + s.d,
                     IV[4] + s.e, IV[5] + s.f, IV[6] + s.g, IV[7] + s.h};
    // an opaque offset (always 0) keeps the 256 LDS reads inside the loop:
    // hoisted out of it, they would take 256 VGPRs
    uint32_t lo = 0;
    asm volatile("" : "+v"(lo) : "v"(s.a));
    const uint32_t* lk = lkw + lo;
    St t;
    if (!ASM && POW_LAT_PIPE) {
      const_chunks_lds_pipelined(H, t, lk);
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        t = St{H[0], H[1], H[2], H[3], H[4], H[5], H[6], H[7]};
        const_chunk_lds<ASM>(t, lk + 64 * c);
        H[0] += t.a; H[1] += t.b; H[2] += t.c; H[3] += t.d;
        H[4] += t.e; H[5] += t.f; H[6] += t.g; H[7] += t.h;
      }
      t = St{H[0], H[1], H[2], H[3], H[4], H[5], H[6], H[7]};
      const_chunk_lds<ASM>(t, lk + 64 * 3);
    }
    // The whole digest stays live here (this kernel runs at <= 4 waves/SIMD,
    // so the 7 extra VGPRs cost no residency): a hit records it, and the
    // winner's block_hash needs no K2 launch (one serial SHA-256 of 5 chunks
    // in one lane is ~15 us, as long as this whole kernel at low d).
    const uint32_t D[8] = {H[0] + t.a, H[1] + t.b, H[2] + t.c, H[3] + t.d,
                           H[4] + t.e, H[5] + t.f, H[6] + t.g, H[7] + t.h};
    bool hit = D[0] <= L.thr;
    if (FULL && hit) hit = full_test(D, L.diff);
    if (__builtin_expect(hit, 0) && (unsigned long long)rel < L.count) {
      if ((unsigned long long)rel < atomicMin(&res->min_rel, (unsigned long long)rel)) publish_hit(L.watch, rel);
      const uint32_t slot = atomicAdd(&res->nhit, 1u);
      if (slot < POW_HITS) {
        res->hit[slot].rel = rel;
#pragma unroll
        for (int k = 0; k < 8; ++k) res->hit[slot].digest[k] = D[k];
      }
      wrote_hit = true;
    }
    wrote_hit = __builtin_amdgcn_readfirstlane(__ballot(wrote_hit) != 0ull);
  }
  // Last workgroup out: publish the result to host memory and reset `res`
  // for the next launch.  One 64-bit atomic per WORKGROUP (its 4 waves sum
  // their iterations in LDS first) counts both the workgroups that have
  // exited (low 32 bits) and the wave-iterations done (high 32 bits): at
  // thousands of waves per launch, per-wave atomics on one address cost tens
  // of microseconds.  Only waves that wrote hit records release them (an
  // agent-scope release writes back L2); min_rel and nhit are atomics.  The
  // last workgroup acquires.
  if (wrote_hit || blockIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  if (lane == 0) atomicAdd(&wg_iters, iters);
  __syncthreads();
  if (threadIdx.x < 64u) {
    unsigned long long old = 0;
    if (lane == 0)
      old = __hip_atomic_fetch_add(&res->hashes, ((unsigned long long)wg_iters << 32) | 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    old = uniform64(old);
    if ((uint32_t)old == L.nwg - 1u) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const uint32_t nh = res->nhit < POW_HITS ? res->nhit : POW_HITS;
      if (lane < nh) {  // one lane per recorded hit
        hout->hit[lane].rel = res->hit[lane].rel;
#pragma unroll
        for (int k = 0; k < 8; ++k) hout->hit[lane].digest[k] = res->hit[lane].digest[k];
      }
      if (lane == 0) {
        hout->min_rel = res->min_rel;
        hout->hashes = ((old >> 32) + wg_iters) * 64ull;
        hout->nhit = res->nhit;
        hout->cancelled = res->cancelled;
        hout->ticks = __builtin_amdgcn_s_memrealtime() -
                      __hip_atomic_load(&res->t_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        res->min_rel = ~0ull;
        res->hashes = 0;
        res->nhit = 0;
        res->cancelled = 0;
        res->peer_abs = ~0ull;
      }
      // Release at system scope, then `done`: the result words above (host
      // memory) and the reset of `res` are visible before the host sees this
      // launch's seq.  A release fence, not __threadfence_system: its acquire
      // half invalidated the whole L2 again at the end of every launch.
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      if (lane == 0) __hip_atomic_store(&hout->done, L.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template __global__ void pow_search_lat<false, false, false>(const PowConstsLat, PowLaunchLat, PowResult*, PowResult*);
template __global__ void pow_search_lat<true, false, false>(const PowConstsLat, PowLaunchLat, PowResult*, PowResult*);
template __global__ void pow_search_lat<false, true, false>(const PowConstsLat, PowLaunchLat, PowResult*, PowResult*);
template __global__ void pow_search_lat<true, true, false>(const PowConstsLat, PowLaunchLat, PowResult*, PowResult*);
template __global__ void pow_search_lat<false, false, true>(const PowConstsLat, PowLaunchLat, PowResult*, PowResult*);
template __global__ void pow_search_lat<true, false, true>(const PowConstsLat, PowLaunchLat, PowResult*, PowResult*);
template __global__ void pow_search_lat<false, true, true>(const PowConstsLat, PowLaunchLat, PowResult*, PowResult*);
template __global__ void pow_search_lat<true, true, true>(const PowConstsLat, PowLaunchLat, PowResult*, PowResult*);

// K2: block_to_hash for n blocks; `msgs` holds each block's 270-byte message
// already padded on the host to 320 bytes (80 big-endian words).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8))) void pow_hash_kernel(const uint32_t* __restrict__ msgs, uint32_t n,
                                                      uint32_t* __restrict__ digests) {
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  if (i >= n) return;
  uint32_t h[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = IV[k];
  const uint32_t* m = msgs + (size_t)i * 80u;
#pragma unroll 1
  for (int c = 0; c < 5; ++c) {
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = m[c * 16 + k];
    compress(h, w);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) digests[(size_t)i * 8u + k] = h[k];
}

// K2': block_to_hash (block.cpp:74-77) of ONE block, for validation
// (pow_hash_block).  A received block is checked one at a time
// (validate_block_for_chain, node.cpp:199-253), so the latency of one hash is
// what counts.  One wave; the host expands the five chunks' message schedules
// (K folded in, as pow_build_consts does for K1's chunks 1-4) and passes the
// 320 K+W words by value in the kernarg segment, which the wave copies into
// LDS (one vector load per lane, then a barrier) and reads back 16 B at a time
// one round group ahead of use: no H2D copy, only the 320 compression rounds
// (the digest's chained part) on the GPU.  The
// digest, its duration and a done word go into mapped host memory (no D2H
// copy, no completion-signal wait).  One wave alone issues a VALU instruction
// every ~4 cycles whether it is full or half rate (MI355X_MICROARCH.md,
// vector-instruction issue cost), so the kernel time is the instruction
// count: 320 rounds x 14 in asm groups with the K+W word in the v_add3 (the
// compiler's form takes 16: six separate adds), 4,520 in all (round 3's form,
// which also ran the schedule on the device: 5,100 instructions, 10.9 us).  <= 64 VGPRs: it must fit the
// workgroup slot a running K1 leaves free.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8))) void pow_hash_one(
    const PowMsg M, PowHashOut* __restrict__ hout, uint32_t seq) {
  (void)M;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0)  // the watchdog's "did it run" word (host memory, not waited for)
    __hip_atomic_store(&hout->started, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // M is the first kernel argument: read it through the kernarg pointer (its
  // address would make a private copy); uniform indices -> scalar loads.
  const uint32_t* const kw = (const uint32_t*)__builtin_amdgcn_kernarg_segment_ptr();
  __shared__ __attribute__((aligned(16))) uint32_t lkw[320];
  {
    const uint32_t lane = threadIdx.x;
    uint32_t v[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) v[k] = kw[lane + 64u * k];
#pragma unroll
    for (int k = 0; k < 5; ++k) lkw[lane + 64u * k] = v[k];
  }
  __syncthreads();
  // K+W four words at a time, each read issued one group (4 rounds, ~220
  // cycles) before its use (const_chunks_lds_pipelined, as K1' at one wave
  // per SIMD); the first group of each chunk leaves the chunk's input state
  // untouched for the feed-forward.
  uint32_t H[8] = {IV[0], IV[1], IV[2], IV[3], IV[4], IV[5], IV[6], IV[7]};
  St t;
  const_chunks_lds_pipelined<5>(H, t, lkw);
  const St h{H[0] + t.a, H[1] + t.b, H[2] + t.c, H[3] + t.d, H[4] + t.e, H[5] + t.f, H[6] + t.g, H[7] + t.h};
  if (threadIdx.x == 0) {
    const uint32_t d[8] = {h.a, h.b, h.c, h.d, h.e, h.f, h.g, h.h};
#pragma unroll
    for (int k = 0; k < 8; ++k) __hip_atomic_store(&hout->digest[k], d[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&hout->ticks, __builtin_amdgcn_s_memrealtime() - t0, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&hout->done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- host-side launch wrappers (called from pow_api.cpp) ----
extern "C++" hipError_t pow_launch_search(int mode, bool full, unsigned grid, hipStream_t stream,
                                          const PowConsts* C, const PowLaunch& L, uint32_t* out,
                                          PowResult* res) {
  dim3 g(grid), b(256);
  if (mode == 0 && !full) hipLaunchKernelGGL((pow_search<0, false>), g, b, 0, stream, C, L, out, res);
  else if (mode == 0) hipLaunchKernelGGL((pow_search<0, true>), g, b, 0, stream, C, L, out, res);
  else if (mode == 1 && !full) hipLaunchKernelGGL((pow_search<1, false>), g, b, 0, stream, C, L, out, res);
  else if (mode == 1) hipLaunchKernelGGL((pow_search<1, true>), g, b, 0, stream, C, L, out, res);
  else if (!full) hipLaunchKernelGGL((pow_search<2, false>), g, b, 0, stream, C, L, out, res);
  else hipLaunchKernelGGL((pow_search<2, true>), g, b, 0, stream, C, L, out, res);
  return hipGetLastError();
}

extern "C++" hipError_t pow_launch_search_lat(bool full, bool any, bool asm_groups, unsigned grid,
                                              hipStream_t stream, const PowConstsLat& C, const PowLaunchLat& L,
                                              PowResult* res, PowResult* hout) {
  dim3 g(grid), b(256);
#define POW_LAT(F, A, G) hipLaunchKernelGGL((pow_search_lat<F, A, G>), g, b, 0, stream, C, L, res, hout)
  if (asm_groups) {
    if (!full && !any) POW_LAT(false, false, true);
    else if (!any) POW_LAT(true, false, true);
    else if (!full) POW_LAT(false, true, true);
    else POW_LAT(true, true, true);
  } else {
    if (!full && !any) POW_LAT(false, false, false);
    else if (!any) POW_LAT(true, false, false);
    else if (!full) POW_LAT(false, true, false);
    else POW_LAT(true, true, false);
  }
#undef POW_LAT
  return hipGetLastError();
}

extern "C++" hipError_t pow_launch_hash_one(hipStream_t stream, const PowMsg& M, PowHashOut* hout, uint32_t seq) {
  hipLaunchKernelGGL(pow_hash_one, dim3(1), dim3(64), 0, stream, M, hout, seq);
  return hipGetLastError();
}

extern "C++" hipError_t pow_launch_hash(uint32_t n, hipStream_t stream, const uint32_t* msgs,
                                        uint32_t* digests) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(pow_hash_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, msgs, n, digests);
  return hipGetLastError();
}
