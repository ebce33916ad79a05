// Per-template constants of the gfx950 mining kernel (host precompute).
//
// The reference hashes, per trial, the 270-byte message of block_to_str
// (block.cpp:79-88): [idx&ff, owner&ff, diff&ff, created_at&ff] nonce[0..9]
// prev[0..255], padded by picosha2 (picosha2.h:201-218) to 320 bytes = five
// 64-byte chunks.  With counter nonces (include/pow_gpu.h) the words are
//
//   chunk 0:  W0      = header bytes                         uniform
//             W1, W2  = nonce[0..3], nonce[4..7]             per lane: the counter's
//                                                            "prefix" c / 62
//             W3      = [nonce[8], nonce[9]=0, prev0, prev1] per inner-loop step j = c % 62,
//                                                            wave-uniform
//             W4..W15 = prev[2..49]                          uniform
//   chunks 1-4: prev[50..255] + 0x80 + zeros + bit length 2160   uniform
//
// so chunks 1-4 have a template-constant message schedule: their K[i]+W[i]
// (4 x 64 words) are folded on the host and streamed to the kernel through
// scalar loads; round 0 of chunk 0 is uniform and precomputed; the chunk-0
// schedule terms that do not depend on the lane's W1/W2 or on j are folded
// here too (u16.. below).  See DESIGN.md "Kernel K1".
#pragma once
#include <stdint.h>

#define POW_J 62 /* inner-loop steps per prefix: the last base-62 nonce digit */

struct PowConsts {
  uint32_t kw[4][64];   // chunks 1..4: K[i] + W[i]                        (1024 B)
  uint32_t st0[8];      // chunk-0 working variables after round 0
  uint32_t kw0[16];     // chunk 0: K[i] + W[i] for i = 4..15 (0..3 unused)
  uint32_t w0, w1_unused, w2_unused, w3lo;  // W0; low 24 bits of W3 (nonce[9], prev0, prev1)
  // Uniform partial sums of the chunk-0 schedule (sigma terms of uniform words):
  uint32_t u16;  // s1(W14) + W9 + W0            -> W16 = u16 + s0(W1)
  uint32_t u17;  // s1(W15) + W10                -> W17 = u17 + s0(W2) + W1
  uint32_t u19;  // W12 + s0(W4)                 -> W19 = s1(W17) + u19 + W3
  uint32_t u20, u21, u22;        // W_{i-7} + s0(W_{i-15}) + W_{i-16}, i = 20..22
  uint32_t u23, u24;             // s0(W_{i-15}) + W_{i-16}, i = 23, 24 (W16/W17 added per lane)
  uint32_t u25[6];               // s0(W_{i-15}) + W_{i-16}, i = 25..30
  uint32_t w15;                  // W15 (for W31 = s1(W29) + W24 + s0(W16) + W15)
  uint32_t pad[3];
  // Per inner step j (the nonce's last char), wave-uniform:
  uint32_t kw3[POW_J];   // K[3] + W3(j)
  uint32_t u18[POW_J];   // s0(W3(j)) + W11          -> W18 = s1(W16) + W2 + u18[j]
  uint32_t w3[POW_J];    // W3(j)                      -> W19
  uint32_t k[64];        // K[0..63] (streamed from memory: VOP3 takes no literal)
  uint32_t w0raw[16];    // chunk-0 words as hashed (W1..W3 = 0 placeholders; latency kernel)
};

// The part of PowConsts the latency kernel K1' reads, passed by value as its
// kernel argument (1.4 KB of kernarg instead of 2.7 KB: the j-uniform tables
// and schedule partial sums are K1's alone).
struct PowConstsLat {
  uint32_t kw[4][64];   // = PowConsts::kw
  uint32_t st0[8];      // = PowConsts::st0
  uint32_t kw0[16];     // = PowConsts::kw0
  uint32_t k[64];       // = PowConsts::k
  uint32_t w0raw[16];   // = PowConsts::w0raw
};
#define LC_ST0 256
#define LC_KW0 (LC_ST0 + 8)
#define LC_K (LC_KW0 + 16)
#define LC_WRAW (LC_K + 64)

// Word offsets into PowConsts for the kernel's constant-address-space loads.
#define PC_ST0 256
#define PC_KW0 (PC_ST0 + 8)
#define PC_U20 (PC_KW0 + 16 + 4 + 3)
#define PC_U25 (PC_U20 + 5)
#define PC_KW3 (PC_U25 + 6 + 4)
#define PC_U18 (PC_KW3 + POW_J)
#define PC_W3 (PC_U18 + POW_J)
#define PC_K (PC_W3 + POW_J)
#define PC_WRAW (PC_K + 64)

// Stop board slots (include/pow_gpu.h "cross-GPU stop board"): one u64 per
// rank in host memory every GPU of the node maps; bits 63..54 hold the
// search tag, bits 53..0 an absolute counter (62^9 < 2^54), all ones = none.
#define POW_BOARD_SHIFT 54
#define POW_BOARD_NONE ((1ull << POW_BOARD_SHIFT) - 1)

// What a mine launch watches besides its own result words (both kernels):
//   * the caller's cancel epoch (pow_cancel), in mapped host memory;
//   * the peers' slots of a bound stop board, and it publishes its own hits
//     to its slot.  Only one sentinel wave per launch reads host memory; it
//     raises device words (`cancelled`, `peer_abs` of the result) that every
//     wave polls.
struct PowWatch {
  const unsigned int* host_epoch;     // pow_cancel's word (device address of mapped host memory)
  const unsigned long long* board;    // null: no board bound
  unsigned long long* board_mine;     // this ctx's slot (a hit is stored here at system scope)
  unsigned long long abs_start;       // absolute counter of relative counter 0
  uint32_t watch_epoch;               // pow_cancel armed: watch host_epoch against launch_epoch
  uint32_t launch_epoch;
  uint32_t board_n;                   // slots (<= 64: one lane each)
  uint32_t board_tag;                 // search tag of the bound search (1..1023)
};

// Launch parameters of the latency kernel (one counter per lane).
struct PowLaunchLat {
  uint32_t base_digit[9];  // base-62 digits of ctr_start (nonce[0..8])
  uint32_t thr;            // as PowLaunch
  uint32_t diff;
  uint32_t seq;            // launch sequence number, published last (PowResult::done)
  uint64_t count;          // counters [ctr_start, ctr_start + count), count <= 2^31
  PowWatch watch;
  uint32_t nwg;            // workgroups of the launch (= gridDim.x): passed explicitly so the
  uint32_t pad;            // kernel reads no implicit argument (direct AQL dispatch, pow_aql.cpp)
};

struct PowLaunch {
  uint32_t base_digit[8];  // base-62 digits of the first prefix P0 (nonce[0..7])
  uint32_t n_prefix;       // prefixes P0 .. P0 + n_prefix - 1
  uint32_t off0;           // ctr_start - 62*P0   (0..61)
  uint64_t count;          // counters requested (relative range [0, count))
  uint32_t thr;            // d <= 32: solution iff H0 <= thr;  d > 32: thr = 0
  uint32_t diff;           // difficulty in bits
  uint32_t cap;            // sweep output capacity
  uint32_t mode;           // 0 = sweep (record all), 1 = mine (lowest + early exit); flags below
};
// Set only by the test library (POW_TEST_HOOKS): in the mine modes the sentinel
// wave (workgroup 0, wave 0) takes no chunk and goes straight to its exit wait,
// so a test can cancel while the sentinel's own work is done and the rest of
// the grid still runs (the path that keeps cancellation alive in the tail).
#define POW_LAUNCH_SENTINEL_IDLE 0x100u

// A solution recorded with its digest by the latency kernel, so the winner's
// block_hash needs no second hashing launch.
#define POW_HITS 8
struct PowHit {
  unsigned long long rel;  // counter - ctr_start
  uint32_t digest[8];      // H0..H7
};

// Device-side result words of one launch (zeroed / ~0 before each launch).
struct PowResult {
  unsigned long long min_rel;  // lowest solving (counter - ctr_start); ~0 = none
  unsigned long long hashes;   // mine mode: trials actually computed
  unsigned long long count;    // sweep: solutions in the main list (32-entry blocks); 64-bit, since
                               // at d = 0 a 2^32 window has 2^32 solutions
  unsigned int next;           // next prefix chunk to hand out (dynamic work queue)
  unsigned int wg_exits;       // K1 mine modes: workgroups other than 0 that have exited (the
                               // sentinel wave of workgroup 0 polls host memory until all have)
  unsigned int tail;           // sweep: solutions in tail_buf (< 32 per wave)
  unsigned int tail_cap;       // entries of tail_buf
  unsigned int* tail_buf;      // sweep: each wave's last < 32 solutions (appended by the host);
                               // read from here at wave exit, not held in SGPRs all kernel long
  unsigned int nhit;           // latency kernel: solutions found (the first POW_HITS are in hit[])
  unsigned int cancelled;      // set once a sentinel wave saw host_epoch != launch_epoch
  unsigned long long peer_abs; // lowest counter a peer published on the board (sentinel wave), ~0 = none
  PowWatch watch;              // K1 mine modes (K1' takes it in its launch parameters)
  unsigned long long t_start;  // K1': s_memrealtime at workgroup 0's start ...
  unsigned long long ticks;    // ... and the last workgroup's exit minus it (published)
  unsigned int done;           // K1': the launch's seq, stored last (system scope): the host
                               //      polls it instead of waiting for the completion signal
  unsigned int started;        // K1': the launch's seq, stored by workgroup 0 as it starts (the
                               //      watchdog's diagnostic: did a stuck launch ever run?)
  PowHit hit[POW_HITS];
};

// K2' (pow_hash_block's one-block path): the five chunks' K[i] + W[i] words of
// the padded 320-byte message (the message schedule, expanded on the host as
// pow_build_consts does for K1's chunks 1-4), passed by value (kernarg: no H2D
// copy; the wave copies it into LDS with one vector load per lane and a
// barrier, then reads it 16 B at a time ahead of each round group) ...
struct PowMsg {
  uint32_t kw[5][64];
};
// ... and its result, written by the kernel into mapped host memory (no D2H
// copy): the digest, the kernel's duration in realtime ticks, and `done` = the
// launch's seq, stored last (system scope) for the host to poll.
struct PowHashOut {
  uint32_t digest[8];
  unsigned long long ticks;
  unsigned int done;
  unsigned int started;  // the launch's seq, stored as the wave starts (the watchdog's diagnostic)
};

// Constants and result words of a context, contiguous so that one H2D copy
// from a pinned staging twin refreshes both before a launch.
struct PowBlob {
  PowConsts consts;
  alignas(256) PowResult res;
};

#ifdef __cplusplus
extern "C++" {
struct pow_block;
struct pow_ctx;
// Fill PowConsts from a template block (nonce field ignored).
void pow_build_consts(const struct pow_block* tmpl, PowConsts* out);
// Library-internal accessors of a context (used by pow_group.cpp).
int pow_ctx_device(const struct pow_ctx* ctx);
void* pow_ctx_stream(const struct pow_ctx* ctx);  // the ctx's hipStream_t
// A watchdog of the ctx fired: a launch may still be queued (never reuse the
// stream, never free what it may write).
bool pow_ctx_wedged(const struct pow_ctx* ctx);
// Bounded wait for everything queued on the ctx's stream (the watchdog):
// POW_OK, or POW_EHIP naming `what` once `budget_ns` past the base deadline
// has gone by without the stream draining.
int pow_ctx_stream_wait(struct pow_ctx* ctx, const char* what, uint64_t budget_ns);
// Record `msg` for pow_last_error(); returns `code`.
int pow_set_error(int code, const char* msg);
// True once another thread moved the caller's cancel word off `epoch` (acquire load).
bool cancel_moved(const volatile uint32_t* cancel_word, uint32_t epoch);
// Sum of per-call statistics kept across several calls (pow_group rounds).
struct pow_stats;
void pow_ctx_set_stats(struct pow_ctx* ctx, const struct pow_stats& s);
// Stop board internals (pow_board.cpp).
struct pow_board;
uint64_t* pow_board_host_slots(const struct pow_board* b);
int pow_board_nslots(const struct pow_board* b);
int pow_board_register(struct pow_board* b);  // hipHostRegister once (first bind)
}
#endif
