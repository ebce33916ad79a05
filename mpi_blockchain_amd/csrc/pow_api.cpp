// C ABI of the gfx950 miner (include/pow_gpu.h): context, per-template
// precompute, launch sizing, result read-back.
//
// Replaces the inner loop of proof_of_work (node.cpp:292-308) and
// block_to_hash (block.cpp:74-77); see include/pow_gpu.h for the mapping of
// each entry point to the reference function it replaces.
#include <hip/hip_runtime.h>
#include <sys/prctl.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/pow_gpu.h"
#include "pow_template.h"
#ifdef POW_TEST_HOOKS
#include "pow_aql.h"  // direct dispatch: test library only (POW_AQL=1)
#endif

#ifndef POW_WAIT_POLL_US
#define POW_WAIT_POLL_US 50  // long launches: host poll period (us) of the completion event
#endif

static_assert(sizeof(pow_block) == 552, "pow_block must match block.h:17-25 (LP64)");
static_assert(offsetof(pow_block, created_at) == 16, "layout");
static_assert(offsetof(pow_block, nonce) == 24, "layout");
static_assert(offsetof(pow_block, previous_block_hash) == 34, "layout");
static_assert(offsetof(pow_block, block_hash) == 290, "layout");
static_assert(sizeof(PowConsts) % 4 == 0 && sizeof(PowConsts) < 4096, "consts");
static_assert(offsetof(PowConsts, kw0) == 4 * PC_KW0, "PC_KW0");
static_assert(offsetof(PowConsts, u20) == 4 * PC_U20, "PC_U20");
static_assert(offsetof(PowConsts, u21) == 4 * (PC_U20 + 1), "PC_U21");
static_assert(offsetof(PowConsts, u22) == 4 * (PC_U20 + 2), "PC_U22");
static_assert(offsetof(PowConsts, u25) == 4 * PC_U25, "PC_U25");
static_assert(offsetof(PowConsts, kw3) == 4 * PC_KW3, "PC_KW3");
static_assert(offsetof(PowConsts, u18) == 4 * PC_U18, "PC_U18");
static_assert(offsetof(PowConsts, w3) == 4 * PC_W3, "PC_W3");
static_assert(offsetof(PowConsts, k) == 4 * PC_K, "PC_K");
static_assert(offsetof(PowConsts, st0) == 4 * PC_ST0, "PC_ST0");
static_assert(offsetof(PowConsts, w0raw) == 4 * PC_WRAW, "PC_WRAW");
static_assert(offsetof(PowConstsLat, st0) == 4 * LC_ST0 && offsetof(PowConstsLat, kw0) == 4 * LC_KW0 &&
                  offsetof(PowConstsLat, k) == 4 * LC_K && offsetof(PowConstsLat, w0raw) == 4 * LC_WRAW,
              "LC_*");

hipError_t pow_launch_search(int mode, bool full, unsigned grid, hipStream_t stream, const PowConsts* C,
                             const PowLaunch& L, uint32_t* out, PowResult* res);
hipError_t pow_launch_hash(uint32_t n, hipStream_t stream, const uint32_t* msgs, uint32_t* digests);
hipError_t pow_launch_hash_one(hipStream_t stream, const PowMsg& M, PowHashOut* hout, uint32_t seq);
hipError_t pow_sort_u32(void* temp, size_t* temp_bytes, uint32_t* keys, uint32_t* alt, uint32_t n,
                        uint32_t** sorted, hipStream_t stream);
hipError_t pow_launch_search_lat(bool full, bool any, bool asm_groups, unsigned grid, hipStream_t stream,
                                 const PowConstsLat& C, const PowLaunchLat& L, PowResult* res, PowResult* hout);
#ifdef POW_TEST_HOOKS
hipError_t pow_launch_test_stall(hipStream_t stream, unsigned us, int realtime_khz);  // pow_test_kernels.hip
#endif

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

uint64_t mono_ns() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

#define HIP_OK(expr)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail(POW_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                  __LINE__);                                                               \
  } while (0)

// ---------------- host SHA-256 pieces for the template precompute ----------------
// (FIPS 180-4 / picosha2.h:46-136; only the parts needed to fold constants)
const uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
const uint32_t kIV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                         0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
inline uint32_t ssig0(uint32_t x) { return rotr(x, 7) ^ rotr(x, 18) ^ (x >> 3); }
inline uint32_t ssig1(uint32_t x) { return rotr(x, 17) ^ rotr(x, 19) ^ (x >> 10); }
inline uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// block.cpp:61-72 alphabet.
inline char digit_char(unsigned d) {
  return d < 26 ? (char)('a' + d) : d < 52 ? (char)('A' + d - 26) : (char)('0' + d - 52);
}

// block.cpp:79-88 + picosha2.h:201-218: the padded 320-byte message.
void padded_message(const pow_block* b, uint8_t m[320]) {
  memset(m, 0, 320);
  pow_block_to_bytes(b, m);
  m[POW_MSG_BYTES] = 0x80;
  const uint64_t bits = (uint64_t)POW_MSG_BYTES * 8;  // 2160
  for (int i = 0; i < 8; ++i) m[319 - i] = (uint8_t)(bits >> (8 * i));
}

void expand(uint32_t w[64], const uint8_t* chunk) {
  for (int i = 0; i < 16; ++i) w[i] = be32(chunk + 4 * i);
  for (int i = 16; i < 64; ++i) w[i] = ssig1(w[i - 2]) + w[i - 7] + ssig0(w[i - 15]) + w[i - 16];
}

}  // namespace

void pow_build_consts(const pow_block* tmpl, PowConsts* C) {
  memset(C, 0, sizeof *C);
  pow_block b = *tmpl;
  memset(b.nonce, 0, sizeof b.nonce);  // nonce bytes are per trial; nonce[9] stays NUL
  uint8_t m[320];
  padded_message(&b, m);
  for (int c = 1; c < 5; ++c) {
    uint32_t w[64];
    expand(w, m + 64 * c);
    for (int i = 0; i < 64; ++i) C->kw[c - 1][i] = kK[i] + w[i];
  }
  uint32_t W[16];
  for (int i = 0; i < 16; ++i) W[i] = be32(m + 4 * i);
  C->w0 = W[0];
  C->w3lo = W[3] & 0x00FFFFFFu;  // [nonce[9]=0, prev[0], prev[1]]
  for (int i = 4; i < 16; ++i) C->kw0[i] = kK[i] + W[i];
  // round 0 of chunk 0 (uniform)
  uint32_t a = kIV[0], bb = kIV[1], c = kIV[2], d = kIV[3], e = kIV[4], f = kIV[5], g = kIV[6], h = kIV[7];
  {
    uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    uint32_t chv = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + chv + kK[0] + W[0];
    uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    uint32_t mj = (a & bb) ^ (a & c) ^ (bb & c);
    h = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + S0 + mj;
  }
  const uint32_t st[8] = {a, bb, c, d, e, f, g, h};
  memcpy(C->st0, st, sizeof st);
  C->u16 = ssig1(W[14]) + W[9] + W[0];
  C->u17 = ssig1(W[15]) + W[10];
  C->u19 = W[12] + ssig0(W[4]);
  C->u20 = W[13] + ssig0(W[5]) + W[4];
  C->u21 = W[14] + ssig0(W[6]) + W[5];
  C->u22 = W[15] + ssig0(W[7]) + W[6];
  C->u23 = ssig0(W[8]) + W[7];
  C->u24 = ssig0(W[9]) + W[8];
  for (int k = 0; k < 6; ++k) C->u25[k] = ssig0(W[10 + k]) + W[9 + k];
  C->w15 = W[15];
  memcpy(C->k, kK, sizeof kK);
  memcpy(C->w0raw, W, sizeof W);  // nonce words zero: W1 = W2 = 0, W3 = w3lo
  for (unsigned j = 0; j < POW_J; ++j) {
    const uint32_t w3 = ((uint32_t)(uint8_t)digit_char(j) << 24) | C->w3lo;
    C->w3[j] = w3;
    C->kw3[j] = kK[3] + w3;
    C->u18[j] = ssig0(w3) + W[11];
  }
}

struct pow_ctx {
  int device = 0;
  int cu_count = 0;
  int clock_khz = 0;
  int realtime_khz = 100000;  // s_memrealtime rate (hipDeviceAttributeWallClockRate)
  uint32_t lat_seq = 0;       // K1' launches so far (PowLaunchLat::seq)
  PowConstsLat lat_consts{};  // K1''s kernel argument (the subset of h_blob->consts it reads)
  char name[256] = {0};
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t ev_block = nullptr;  // polled with sleeps during long launches
  PowBlob* d_blob = nullptr;   // per-template constants + result words, one allocation
  PowBlob* h_blob = nullptr;   // pinned staging copy: uploaded with one H2D per launch
  bool consts_dirty = false;   // h_blob->consts not yet on the device
  PowResult* d_lat = nullptr;           // latency kernel: self-resetting device result words ...
  PowResult* h_lat = nullptr;           // ... published by its last wave here (mapped host memory)
  PowHashOut* h_one = nullptr;          // K2' (pow_hash_block): digest + done word (mapped host memory)
  PowHashOut* d_one = nullptr;          // device address of h_one
  uint32_t one_seq = 0;                 // K2' launches so far (the done word's value)
  PowResult* d_lat_host = nullptr;      // device address of h_lat
  unsigned int* h_epoch = nullptr;      // pow_cancel's word: mapped, coherent host memory ...
  unsigned int* d_epoch = nullptr;      // ... and its device address
  std::atomic<bool> armed{false};       // pow_cancel has published an epoch
  uint32_t launch_epoch = 0;            // mine calls: the caller's epoch ...
  bool watch_epoch = false;             // ... watched on the GPU when armed
  pow_board* board = nullptr;           // bound stop board (pow_board_bind) ...
  const unsigned long long* board_dev = nullptr;  // ... its slots, device address
  int board_slot = -1;
  uint32_t board_tag = 0;
  bool board_off = false;               // winner re-hash: not part of the search
  PowConsts* d_consts = nullptr;  // = &d_blob->consts
  PowResult* d_res = nullptr;     // = &d_blob->res
  PowResult* h_res = nullptr;  // pinned read-back of d_res
  uint32_t* d_tail = nullptr;  // sweep: per-wave remainders (< 32 each), appended after the launch
  uint32_t tail_cap = 0;
  uint32_t* d_out = nullptr;   // pow_sweep's device list and its radix-sort twin
  uint32_t* d_alt = nullptr;
  void* d_sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  size_t out_cap = 0;
  uint32_t* d_msgs = nullptr;
  uint32_t* d_dig = nullptr;
  size_t hash_cap = 0;
  unsigned grid_full = 0;  // workgroups that fill the chip (8 per CU)
  // Set only by the test library's hooks (POW_TEST_HOOKS, pow_init):
  bool force_full = false;        // use the d > 32 kernel for every d
  bool fault_mine = false;        // every pow_mine[_any] call fails (failure-propagation tests)
  uint64_t lat_max = 1ull << 24;  // first-sub-round cap for K1' (0 = K1 only)
  unsigned lat_wps = 0;           // K1' waves per SIMD at every d (0 = the plan)
  bool sentinel_idle = false;     // K1 mine launches: the sentinel wave takes no chunk (POW_LAUNCH_SENTINEL_IDLE)
  unsigned test_stall_us = 0;     // POW_TEST_STALL_US: a bounded stall kernel in front of every HIP launch (watchdog tests)
#ifdef POW_TEST_HOOKS
  // K1' and K2' launches as AQL packets (pow_aql.cpp) instead of
  // hipLaunchKernel: test library only, with POW_AQL=1; null = the HIP launch
  // path, the only one the shipped library has.
  pow_aql* aql = nullptr;
  std::string aql_why;            // why aql is null, if it is
#endif
  // Watchdog (every host wait on a launch is bounded): base deadline of a
  // latency launch, and of a throughput launch on top of its per-counter share.
  uint64_t watchdog_ns = 10ull * 1000000000ull;
  // A watchdog fired (or a direct dispatch was refused after its packet slot
  // was reserved): a launch of this context may still be queued.  pow_group_*
  // then do not queue a collective behind it; pow_destroy frees only what a
  // bounded wait shows drained.
  bool wedged = false;
#ifdef POW_TEST_HOOKS
  bool aql_lost = false;  // the direct dispatcher was closed with a packet still in flight
#endif
  pow_stats stats{};
};

namespace {

int stage_result(pow_ctx* ctx, bool with_tail, uint64_t abs_start);
void digest_out(const uint32_t* h, uint8_t* digest, char* hex);

// What a mine launch watches: the caller's epoch (pow_cancel) and the bound
// stop board.  abs_start = absolute counter of the launch's relative 0.
void fill_watch(const pow_ctx* ctx, PowWatch& w, uint64_t abs_start) {
  memset(&w, 0, sizeof w);
  w.watch_epoch = ctx->watch_epoch && ctx->armed.load(std::memory_order_acquire) ? 1u : 0u;
  w.host_epoch = ctx->d_epoch;
  w.launch_epoch = ctx->launch_epoch;
  w.abs_start = abs_start;
  if (ctx->board && !ctx->board_off) {
    w.board = ctx->board_dev;
    w.board_mine = const_cast<unsigned long long*>(ctx->board_dev) + ctx->board_slot;
    w.board_n = (uint32_t)pow_board_nslots(ctx->board);
    w.board_tag = ctx->board_tag;
  }
}

// Lowest counter a peer published for the bound search (host view).
uint64_t board_peer_min(const pow_ctx* ctx) {
  uint64_t m = UINT64_MAX;
  if (ctx->board && !ctx->board_off) pow_board_peek(ctx->board, ctx->board_slot, ctx->board_tag, &m);
  return m;
}

int set_dev(const pow_ctx* ctx) {
  HIP_OK(hipSetDevice(ctx->device));
  return POW_OK;
}

// Every host wait on the context's stream goes through here (the watchdog):
// an event recorded behind the queued work is polled until it completes or
// `deadline_ns` (CLOCK_MONOTONIC) passes.  nap = long waits: 50 us sleeps
// between polls instead of a spinning core (a protocol rank
// should not burn a core while its GPU mines; hipEventSynchronize spins,
// blocking-sync event or not), at most 50 us late on a >= 8 ms launch, with
// the calling thread's timer slack lowered to 1 us meanwhile (a 50 us sleep
// otherwise lasts ~100 us: the end of a pow_mine_any launch that found a block
// at d = 25 was seen 50-75 us late, rocprofv3 HIP trace of tools/ttb_c 25).
// Past the deadline: POW_EHIP naming `what`, and the context must not be
// reused (its work may still be queued).  On success a final
// hipStreamSynchronize returns at once and reports any error of the work.
int stream_wait(pow_ctx* ctx, const char* what, uint64_t t0, uint64_t deadline_ns, bool nap) {
  HIP_OK(hipEventRecord(ctx->ev_block, ctx->stream));
  const int slack = nap ? prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0) : 0;
  if (slack > 1000) prctl(PR_SET_TIMERSLACK, 1000ul, 0, 0, 0);
  hipError_t q;
  bool late = false;
  for (uint32_t n = 1; (q = hipEventQuery(ctx->ev_block)) == hipErrorNotReady; ++n) {
    if (nap) std::this_thread::sleep_for(std::chrono::microseconds(POW_WAIT_POLL_US));
    if ((nap || (n & 255u) == 0) && mono_ns() > deadline_ns) {
      late = true;
      break;
    }
  }
  if (slack > 1000) prctl(PR_SET_TIMERSLACK, (unsigned long)slack, 0, 0, 0);
  if (late) {
    ctx->wedged = true;
    return fail(POW_EHIP, "%s: watchdog: not complete after %.3f s (deadline %.3f s; hipStreamQuery: %s); "
                "the context must not be reused",
                what, (mono_ns() - t0) * 1e-9, (deadline_ns - t0) * 1e-9, hipGetErrorString(hipStreamQuery(ctx->stream)));
  }
  HIP_OK(q);
  HIP_OK(hipStreamSynchronize(ctx->stream));
  return POW_OK;
}

// The common case: `what` must be done within the base deadline plus `extra_ns`.
int stream_wait_for(pow_ctx* ctx, const char* what, uint64_t extra_ns) {
  const uint64_t t0 = mono_ns();
  return stream_wait(ctx, what, t0, t0 + ctx->watchdog_ns + extra_ns, false);
}

// Split [start, start+count) (count <= 2^32) into the kernel's prefix form.
int make_launch(uint64_t start, uint64_t count, unsigned diff, uint32_t cap, uint32_t mode,
                PowLaunch* L) {
  memset(L, 0, sizeof *L);
  const uint64_t P0 = start / POW_J;
  L->off0 = (uint32_t)(start - P0 * POW_J);
  const uint64_t np = (L->off0 + count + POW_J - 1) / POW_J;
  if (np > 0xFFFFFFFFull - (1u << 26)) return fail(POW_EINVAL, "launch too large");
  L->n_prefix = (uint32_t)np;
  uint64_t p = P0;
  for (int i = 7; i >= 0; --i) {
    L->base_digit[i] = (uint32_t)(p % 62);
    p /= 62;
  }
  L->count = count;
  L->diff = diff;
  L->thr = diff >= 32 ? 0u : (0xFFFFFFFFu >> diff);
  L->cap = cap;
  L->mode = mode;
  return POW_OK;
}

unsigned grid_for(const pow_ctx* ctx, uint32_t n_prefix) {
  // one lane per prefix per chunk; no more workgroups than there are chunks
  const uint64_t want = ((uint64_t)n_prefix + 255) / 256;
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, ctx->grid_full));
}

int check_range(const pow_block* tmpl, uint64_t start, uint64_t count, unsigned diff) {
  if (!tmpl) return fail(POW_EINVAL, "null template");
  if (diff > 256) return fail(POW_EINVAL, "difficulty %u > 256 bits", diff);
  if (start >= POW_COUNTER_LIMIT || count > POW_COUNTER_LIMIT - start)
    return fail(POW_EINVAL, "counter range past 62^9");
  return POW_OK;
}

// One timed launch of K1 over [start, start+count) (count <= 2^32) with the
// consts already resident; leaves the result in ctx->h_res.
int run_search(pow_ctx* ctx, uint64_t start, uint64_t count, unsigned diff, uint32_t mode,
               uint32_t* dev_out, uint32_t cap) {
  PowLaunch L;
  int rc = make_launch(start, count, diff, cap, mode, &L);
  if (rc) return rc;
#ifdef POW_TEST_HOOKS
  if (ctx->sentinel_idle && mode >= 1) L.mode |= POW_LAUNCH_SENTINEL_IDLE;
#endif
  if (int rc2 = stage_result(ctx, true, start)) return rc2;
  const unsigned grid = grid_for(ctx, L.n_prefix);
#ifdef POW_TEST_HOOKS
  if (ctx->test_stall_us) HIP_OK(pow_launch_test_stall(ctx->stream, ctx->test_stall_us, ctx->realtime_khz));
#endif
  HIP_OK(hipEventRecord(ctx->ev0, ctx->stream));
  HIP_OK(pow_launch_search((int)mode, diff > 32 || ctx->force_full, grid, ctx->stream, ctx->d_consts, L, dev_out,
                           ctx->d_res));
  HIP_OK(hipEventRecord(ctx->ev1, ctx->stream));
  HIP_OK(hipMemcpyAsync(ctx->h_res, ctx->d_res, sizeof(PowResult), hipMemcpyDeviceToHost, ctx->stream));
  // Bounded wait (watchdog): the base deadline plus 2 ns per counter, i.e. a
  // launch slower than 0.5 G trials/s (1/18 of the chip's rate, e.g. one GPU
  // shared by many processes) is reported as stuck instead of waited for
  // forever.  Long launches (>= 2^26 counters, >= 8 ms) sleep between polls;
  // short ones spin: their latency is the whole time-to-block at low
  // difficulty.
  {
    char what[160];
    snprintf(what, sizeof what, "search kernel (mode %u, %llu counters from %llu, d = %u)", mode,
             (unsigned long long)count, (unsigned long long)start, diff);
    const uint64_t t0 = mono_ns();
    if (int rc2 = stream_wait(ctx, what, t0, t0 + ctx->watchdog_ns + 2ull * count, count >= (1ull << 26)))
      return rc2;
  }
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  ctx->stats.kernel_ms += ms;
  ctx->stats.launches += 1;
  ctx->stats.hashes += mode >= 1 ? ctx->h_res->hashes : (uint64_t)L.n_prefix * POW_J;
  return POW_OK;
}

#ifdef POW_TEST_HOOKS
// The explicit kernel arguments of a direct dispatch (pow_aql.cpp): the
// parameters in declaration order, each at its natural alignment.
struct ArgPack {
  alignas(8) uint8_t b[2048];
  uint32_t n = 0;
  template <class T>
  void put(const T& v) {
    n = (n + (uint32_t)alignof(T) - 1) & ~((uint32_t)alignof(T) - 1);
    memcpy(b + n, &v, sizeof v);
    n += (uint32_t)sizeof v;
  }
};
#endif

// Wait for a latency-bound launch to publish `seq` into its done word (mapped
// host memory): return as soon as it shows, without waiting for the kernel's
// completion signal (~5 us later; rocprofv3 trace of tools/ttb_c, DESIGN.md
// §4).  A launch that ends without publishing (a fault, a queue error) is
// caught by a completion check every 65536 polls (~60 us), and one that does
// not end by `deadline_ns` (CLOCK_MONOTONIC) by the watchdog: POW_EHIP with
// the launch's sequence number, the done word and the launch path's state
// (HIP: the stream's status; direct dispatch: the completion signal, the
// queue's indices and the header in the packet's slot).  The context must not
// be reused after a watchdog error: its launch may still be queued.
int wait_published(pow_ctx* ctx, const volatile uint32_t* done, const volatile uint32_t* started, uint32_t seq,
                   const char* what, uint64_t t0, uint64_t deadline_ns) {
  for (uint32_t n = 1; __atomic_load_n(const_cast<const uint32_t*>(done), __ATOMIC_ACQUIRE) != seq; ++n) {
    if ((n & 0xFFFFu) != 0) continue;
    int st;  // 1 = running, 0 = ended, < 0 = error
    hipError_t q = hipSuccess;
#ifdef POW_TEST_HOOKS
    if (ctx->aql) {
      st = pow_aql_status(ctx->aql);
    } else
#endif
    {
      q = hipStreamQuery(ctx->stream);
      st = q == hipErrorNotReady ? 1 : q == hipSuccess ? 0 : -1;
    }
    if (st == 1) {
      if (mono_ns() <= deadline_ns) continue;
      const uint32_t seen = __atomic_load_n(const_cast<const uint32_t*>(done), __ATOMIC_ACQUIRE);
      if (seen == seq) break;
      std::string path = "launch path hip, hipStreamQuery: not ready";
#ifdef POW_TEST_HOOKS
      if (ctx->aql) path = "launch path direct, " + pow_aql_diag(ctx->aql);
#endif
      const uint32_t st_word = __atomic_load_n(const_cast<const uint32_t*>(started), __ATOMIC_ACQUIRE);
      ctx->wedged = true;
      return fail(POW_EHIP,
                  "%s: watchdog: no result after %.3f s (seq %u, done word %u; the kernel %s (started word %u); %s); "
                  "the context must not be reused",
                  what, (mono_ns() - t0) * 1e-9, seq, seen,
                  st_word == seq ? "started: its first workgroup ran" : "never started", st_word, path.c_str());
    }
    if (__atomic_load_n(const_cast<const uint32_t*>(done), __ATOMIC_ACQUIRE) == seq) break;
#ifdef POW_TEST_HOOKS
    if (st < 0 && ctx->aql) return fail(POW_EHIP, "%s: the dispatch queue reported HSA status 0x%x", what, -st);
#endif
    HIP_OK(q);
    return fail(POW_EHIP, "%s ended without publishing its result (seq %u, done word %u)", what, seq,
                __atomic_load_n(const_cast<const uint32_t*>(done), __ATOMIC_ACQUIRE));
  }
  return POW_OK;
}

#ifdef POW_TEST_HOOKS
// A context whose direct-dispatch queue has reported an error goes back to
// the HIP launch path for good (pow_launch_path then says so).
bool aql_usable(pow_ctx* ctx) {
  if (!ctx->aql) return false;
  if (pow_aql_status(ctx->aql) >= 0) return true;
  ctx->aql_why = "the dispatch queue reported an error; back on the HIP launch path";
  if (!pow_aql_close(ctx->aql)) ctx->wedged = ctx->aql_lost = true;  // a packet may still be in flight
  ctx->aql = nullptr;
  return false;
}
#endif

int launch_hash_one(pow_ctx* ctx, const PowMsg& M, uint32_t seq, uint64_t deadline_ns) {
#ifdef POW_TEST_HOOKS
  if (aql_usable(ctx)) {
    ArgPack a;
    a.put(M);
    a.put(ctx->d_one);
    a.put(seq);
    std::string why;
    if (pow_aql_dispatch(ctx->aql, POW_AQL_HASH_ONE, 1, 64, a.b, a.n, deadline_ns, &why)) {
      ctx->wedged = true;  // a refused packet may have left its reserved slot behind (pow_aql_dispatch)
      return fail(POW_EHIP, "dispatch of pow_hash_one failed: %s (%s)", why.c_str(), pow_aql_diag(ctx->aql).c_str());
    }
    return POW_OK;
  }
#endif
  (void)deadline_ns;
#ifdef POW_TEST_HOOKS
  if (ctx->test_stall_us) HIP_OK(pow_launch_test_stall(ctx->stream, ctx->test_stall_us, ctx->realtime_khz));
#endif
  HIP_OK(pow_launch_hash_one(ctx->stream, M, ctx->d_one, seq));
  return POW_OK;
}

int launch_search_lat(pow_ctx* ctx, bool full, bool any, bool asm_groups, unsigned grid, const PowLaunchLat& L,
                      uint64_t deadline_ns) {
#ifdef POW_TEST_HOOKS
  if (aql_usable(ctx)) {
    ArgPack a;
    a.put(ctx->lat_consts);
    a.put(L);
    a.put(ctx->d_lat);
    a.put(ctx->d_lat_host);
    const int k = POW_AQL_LAT0 + (full ? 1 : 0) + (any ? 2 : 0) + (asm_groups ? 4 : 0);
    std::string why;
    if (pow_aql_dispatch(ctx->aql, k, grid, 256, a.b, a.n, deadline_ns, &why)) {
      ctx->wedged = true;
      return fail(POW_EHIP, "dispatch of pow_search_lat failed: %s (%s)", why.c_str(), pow_aql_diag(ctx->aql).c_str());
    }
    return POW_OK;
  }
#endif
  (void)deadline_ns;
#ifdef POW_TEST_HOOKS
  if (ctx->test_stall_us) HIP_OK(pow_launch_test_stall(ctx->stream, ctx->test_stall_us, ctx->realtime_khz));
#endif
  HIP_OK(pow_launch_search_lat(full, any, asm_groups, grid, ctx->stream, ctx->lat_consts, L, ctx->d_lat,
                               ctx->d_lat_host));
  return POW_OK;
}

// One timed launch of the latency kernel K1' over [start, start+count), count <= 2^31.
int run_search_lat(pow_ctx* ctx, uint64_t start, uint64_t count, unsigned diff, bool any,
                   unsigned waves_per_simd) {
  PowLaunchLat L;
  memset(&L, 0, sizeof L);
  uint64_t p = start;
  for (int i = 8; i >= 0; --i) {
    L.base_digit[i] = (uint32_t)(p % 62);
    p /= 62;
  }
  L.count = count;
  L.diff = diff;
  L.thr = diff >= 32 ? 0u : (0xFFFFFFFFu >> diff);
  fill_watch(ctx, L.watch, start);
  // A 256-thread workgroup puts one wave on each SIMD of its CU.
  const uint64_t wg_cap = (uint64_t)ctx->cu_count * std::max(1u, std::min(8u, waves_per_simd));
  const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((count + 255) / 256, wg_cap));
  L.nwg = grid;
  if (++ctx->lat_seq == 0) ctx->lat_seq = 1;  // never 0: warm-up launches publish 0
  L.seq = ctx->lat_seq;
  // One dispatch: constants by value (kernarg), result published by the
  // kernel's last wave into mapped host memory (no copy kernels), `done` last.
  // At 4+ waves per SIMD (d = 20, 21) chunks 1-4 run as K1's asm groups
  // (8-byte encodings at the pinned phase): K1' at d = 21 7.79 -> 7.93 G
  // trials/s, time-to-block 0.2136 -> 0.2125 ms (profiles/r03/ab/ab14_*).  At 1-2 waves per SIMD the kernel is latency-bound and the
  // compiler's interleaving of independent ops serves it better (d = 13:
  // 0.034 -> 0.038 ms with the groups; profiles/r03/ab/ab8_*).
  // Watchdog: the base deadline plus 2 ns per counter (count <= 2^31).
  const uint64_t t0 = mono_ns(), deadline = t0 + ctx->watchdog_ns + 2ull * count;
  if (int rc = launch_search_lat(ctx, diff > 32 || ctx->force_full, any, waves_per_simd >= 4, grid, L, deadline))
    return rc;
  if (int rc = wait_published(ctx, &ctx->h_lat->done, &ctx->h_lat->started, L.seq, "latency kernel", t0, deadline))
    return rc;
  memcpy(ctx->h_res, (const void*)ctx->h_lat, sizeof(PowResult));
  const double ms = (double)ctx->h_res->ticks / ctx->realtime_khz;
  ctx->stats.kernel_ms += ms;
  ctx->stats.launches += 1;
  ctx->stats.hashes += ctx->h_res->hashes;
  return POW_OK;
}

// The template's constants go into the pinned staging blob; the next launch
// uploads them together with its result words (one H2D copy).
int upload_consts(pow_ctx* ctx, const pow_block* tmpl) {
  pow_build_consts(tmpl, &ctx->h_blob->consts);
  const PowConsts& C = ctx->h_blob->consts;
  PowConstsLat& Q = ctx->lat_consts;
  memcpy(Q.kw, C.kw, sizeof Q.kw);
  memcpy(Q.st0, C.st0, sizeof Q.st0);
  memcpy(Q.kw0, C.kw0, sizeof Q.kw0);
  memcpy(Q.k, C.k, sizeof Q.k);
  memcpy(Q.w0raw, C.w0raw, sizeof Q.w0raw);
  ctx->consts_dirty = true;
  return POW_OK;
}

// Reset the device result words (and upload pending constants) before a launch.
int stage_result(pow_ctx* ctx, bool with_tail, uint64_t abs_start) {
  PowResult& r = ctx->h_blob->res;
  memset(&r, 0, sizeof r);
  r.min_rel = ~0ull;
  r.peer_abs = ~0ull;
  fill_watch(ctx, r.watch, abs_start);
  if (with_tail) {
    r.tail_buf = ctx->d_tail;
    r.tail_cap = ctx->tail_cap;
  }
  const size_t off = ctx->consts_dirty ? 0 : offsetof(PowBlob, res);
  HIP_OK(hipMemcpyAsync((char*)ctx->d_blob + off, (const char*)ctx->h_blob + off, sizeof(PowBlob) - off,
                        hipMemcpyHostToDevice, ctx->stream));
  ctx->consts_dirty = false;
  return POW_OK;
}

// picosha2's output_hex (picosha2.h:141-150): big-endian digest bytes, lowercase hex.
void digest_out(const uint32_t* h, uint8_t* digest, char* hex) {
  static const char hexd[] = "0123456789abcdef";
  uint8_t d[32];
  for (int k = 0; k < 8; ++k) {
    d[4 * k] = (uint8_t)(h[k] >> 24);
    d[4 * k + 1] = (uint8_t)(h[k] >> 16);
    d[4 * k + 2] = (uint8_t)(h[k] >> 8);
    d[4 * k + 3] = (uint8_t)h[k];
  }
  if (digest) memcpy(digest, d, 32);
  if (hex) {
    for (int k = 0; k < 32; ++k) {
      hex[2 * k] = hexd[d[k] >> 4];
      hex[2 * k + 1] = hexd[d[k] & 15];
    }
    hex[64] = 0;
  }
}

}  // namespace

// The caller's cancel word is written by another thread (the receive loop):
// read it with an acquire load, not a plain volatile read.
bool cancel_moved(const volatile uint32_t* cancel_word, uint32_t epoch) {
  return cancel_word && __atomic_load_n(const_cast<const uint32_t*>(cancel_word), __ATOMIC_ACQUIRE) != epoch;
}

int pow_ctx_device(const pow_ctx* ctx) { return ctx->device; }
bool pow_ctx_wedged(const pow_ctx* ctx) { return ctx->wedged; }
void pow_ctx_set_stats(pow_ctx* ctx, const pow_stats& s) { ctx->stats = s; }
void* pow_ctx_stream(const pow_ctx* ctx) { return (void*)ctx->stream; }
int pow_ctx_stream_wait(pow_ctx* ctx, const char* what, uint64_t budget_ns) {
  return stream_wait_for(ctx, what, budget_ns);
}
int pow_set_error(int code, const char* msg) { return fail(code, "%s", msg); }

extern "C" {

const char* pow_last_error(void) { return g_err.c_str(); }

int pow_device_count(int* n) {
  if (!n) return fail(POW_EINVAL, "null");
  *n = 0;
  HIP_OK(hipGetDeviceCount(n));
  return POW_OK;
}

int pow_init(int device, pow_ctx** out) {
  if (!out) return fail(POW_EINVAL, "null out");
  *out = nullptr;
  int n = 0;
  HIP_OK(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(POW_ENODEV, "device %d of %d", device, n);
  HIP_OK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(POW_ENODEV, "device %d is %s; this library is built for gfx950 only", device,
                prop.gcnArchName);
  pow_ctx* ctx = new pow_ctx;
  ctx->device = device;
  ctx->cu_count = prop.multiProcessorCount;
  {
    int rt = 0;
    if (hipDeviceGetAttribute(&rt, hipDeviceAttributeWallClockRate, device) == hipSuccess && rt > 0)
      ctx->realtime_khz = rt;
  }
  ctx->clock_khz = prop.clockRate;
  snprintf(ctx->name, sizeof ctx->name, "%s", prop.name);
  // 8 x 256-thread WGs = 32 waves/CU fill the chip; one slot stays free so
  // that a K2 launch (block validation on another stream/context, 40 VGPRs)
  // can run beside a K1 launch instead of waiting up to its whole ~0.13 s.
  ctx->grid_full = (unsigned)prop.multiProcessorCount * 8u - 1u;
#ifdef POW_TEST_HOOKS
  // Test and tuning switches: compiled only into libpow_gpu_test.so
  // (mpi_blockchain_amd/build.py), never into the shipped libpow_gpu.so.
  if (const char* ff = getenv("POW_FORCE_FULL")) ctx->force_full = ff[0] == '1';
  if (const char* fi = getenv("POW_FAULT_INJECT")) ctx->fault_mine = std::strcmp(fi, "mine") == 0;
  if (const char* lm = getenv("POW_LAT_MAX")) ctx->lat_max = std::min<uint64_t>(strtoull(lm, nullptr, 0), 1ull << 31);
  if (const char* lw = getenv("POW_LAT_WPS")) ctx->lat_wps = (unsigned)std::min(8ul, strtoul(lw, nullptr, 0));
  if (const char* si = getenv("POW_TEST_SENTINEL_IDLE")) ctx->sentinel_idle = si[0] == '1';
  if (const char* ts = getenv("POW_TEST_STALL_US")) ctx->test_stall_us = (unsigned)strtoul(ts, nullptr, 0);
  if (const char* g = getenv("POW_GRID_PER_CU")) {  // launch-geometry experiments
    const int per = atoi(g);
    if (per > 0 && per <= 64) ctx->grid_full = (unsigned)prop.multiProcessorCount * (unsigned)per;
  }
  // POW_AQL=1: K1'/K2' as AQL packets (pow_aql.cpp; dispatch A/B and the
  // multi-producer ordering test), POW_AQL_EXP its experiment flags.
  const char* use_aql = getenv("POW_AQL");
  const unsigned aql_flags = getenv("POW_AQL_EXP") ? (unsigned)strtoul(getenv("POW_AQL_EXP"), nullptr, 0) : 0u;
  // POW_WATCHDOG_MS: the watchdog's base deadline (tests of the watchdog itself)
  if (const char* wd = getenv("POW_WATCHDOG_MS")) ctx->watchdog_ns = std::max(1ull, strtoull(wd, nullptr, 0)) * 1000000ull;
#endif
  int rc = POW_OK;
  auto chk = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && rc == POW_OK) rc = fail(POW_EHIP, "%s: %s", what, hipGetErrorString(e));
  };
  chk(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking), "hipStreamCreate");
  chk(hipEventCreate(&ctx->ev0), "hipEventCreate");
  chk(hipEventCreate(&ctx->ev1), "hipEventCreate");
  chk(hipEventCreateWithFlags(&ctx->ev_block, hipEventDisableTiming), "hipEventCreate");
  // Every copy and fill goes on the context's own stream, never on HIP's null
  // stream: a process that never touches the null stream holds one hardware
  // queue per context (HIP creates queues as streams first use them), and the
  // GPU has 24 compute queue slots for every process on it.  Beyond them the
  // scheduler time-slices queues and a launch can wait seconds for its queue
  // to be mapped ("Queue pressure").
  chk(hipMalloc(&ctx->d_blob, sizeof(PowBlob)), "hipMalloc consts/result");
  if (ctx->d_blob) chk(hipMemsetAsync(ctx->d_blob, 0, sizeof(PowBlob), ctx->stream), "hipMemsetAsync");
  chk(hipMalloc(&ctx->d_lat, sizeof(PowResult)), "hipMalloc latency result");
  chk(hipHostMalloc(&ctx->h_lat, sizeof(PowResult), hipHostMallocMapped | hipHostMallocCoherent),
      "hipHostMalloc latency result");
  if (ctx->d_lat && ctx->h_lat) {
    PowResult* init = ctx->h_lat;  // mapped host memory: the copy's source, read before the stream drains
    memset(init, 0, sizeof *init);
    init->min_rel = ~0ull;
    init->peer_abs = ~0ull;
    chk(hipMemcpyAsync(ctx->d_lat, init, sizeof *init, hipMemcpyHostToDevice, ctx->stream), "hipMemcpyAsync");
    if (rc == POW_OK) rc = stream_wait_for(ctx, "pow_init copies", 0);
    chk(hipHostGetDevicePointer((void**)&ctx->d_lat_host, ctx->h_lat, 0), "hipHostGetDevicePointer");
  }
  chk(hipHostMalloc(&ctx->h_one, sizeof(PowHashOut), hipHostMallocMapped | hipHostMallocCoherent),
      "hipHostMalloc hash result");
  if (ctx->h_one) {
    memset(ctx->h_one, 0, sizeof(PowHashOut));
    chk(hipHostGetDevicePointer((void**)&ctx->d_one, ctx->h_one, 0), "hipHostGetDevicePointer");
  }
  chk(hipHostMalloc(&ctx->h_epoch, 64, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc epoch");
  if (ctx->h_epoch) {
    *ctx->h_epoch = 0;
    chk(hipHostGetDevicePointer((void**)&ctx->d_epoch, ctx->h_epoch, 0), "hipHostGetDevicePointer");
  }
  chk(hipHostMalloc(&ctx->h_blob, sizeof(PowBlob), hipHostMallocDefault), "hipHostMalloc staging");
  if (ctx->d_blob) {
    ctx->d_consts = &ctx->d_blob->consts;
    ctx->d_res = &ctx->d_blob->res;
  }
  chk(hipHostMalloc(&ctx->h_res, sizeof(PowResult), hipHostMallocDefault), "hipHostMalloc");
  ctx->tail_cap = ctx->grid_full * 4u * 32u;  // < 32 per wave, 4 waves per workgroup
  chk(hipMalloc(&ctx->d_tail, (size_t)ctx->tail_cap * sizeof(uint32_t)), "hipMalloc sweep tail");
#ifdef POW_TEST_HOOKS
  if (rc == POW_OK && use_aql && use_aql[0] == '1' && pow_aql_open(device, aql_flags, &ctx->aql, &ctx->aql_why) != 0)
    ctx->aql = nullptr;  // the HIP launch path
#endif
  if (rc != POW_OK) {
    pow_destroy(ctx);
    return rc;
  }
  *out = ctx;
  return POW_OK;
}

void pow_destroy(pow_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  // A context whose launch has not completed (after a watchdog error) is left
  // allocated rather than freed under a kernel that may still write it.  Each
  // launch path has its own bounded wait: the stream (the base deadline +
  // 10 s; a launch the watchdog only stopped waiting for usually ends within
  // it, and its stream, and with it the hardware queue, are then released:
  // leaking every wedged context's stream instead put 4 more queues on the
  // test process and starved an 8-rank network), and for
  // direct-dispatch packets, which the stream does not see, the dispatcher's
  // completion signal (pow_aql_close).  (No event: pow_init failed before any
  // launch, nothing is queued.)
  if (ctx->stream && ctx->ev_block && stream_wait_for(ctx, "pow_destroy", 10ull * 1000000000ull) != POW_OK) return;
#ifdef POW_TEST_HOOKS
  if (ctx->aql_lost || !pow_aql_close(ctx->aql)) return;  // a packet may still write: keep what it writes
#endif
  (void)hipFree(ctx->d_blob);
  if (ctx->h_blob) (void)hipHostFree(ctx->h_blob);
  (void)hipFree(ctx->d_tail);
  (void)hipFree(ctx->d_out);
  (void)hipFree(ctx->d_alt);
  (void)hipFree(ctx->d_sort_tmp);
  (void)hipFree(ctx->d_msgs);
  (void)hipFree(ctx->d_dig);
  if (ctx->h_res) (void)hipHostFree(ctx->h_res);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->ev_block) (void)hipEventDestroy(ctx->ev_block);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->h_epoch) (void)hipHostFree(ctx->h_epoch);
  (void)hipFree(ctx->d_lat);
  if (ctx->h_lat) (void)hipHostFree(ctx->h_lat);
  if (ctx->h_one) (void)hipHostFree(ctx->h_one);
  delete ctx;
}

int pow_warmup(pow_ctx* ctx) {
  if (!ctx) return fail(POW_EINVAL, "null");
  if (int rc = set_dev(ctx)) return rc;
  PowLaunch L;
  memset(&L, 0, sizeof L);  // n_prefix = 0: every wave exits at its first dequeue
  PowLaunchLat LL;
  memset(&LL, 0, sizeof LL);  // count = 0
  LL.nwg = 1;                 // one workgroup: it is the last one out, publishes done = 0 and resets
  for (int mode = 0; mode < 3; ++mode)
    for (int full = 0; full < 2; ++full)
      HIP_OK(pow_launch_search(mode, full != 0, 1, ctx->stream, ctx->d_consts, L, nullptr, ctx->d_res));
  for (int any = 0; any < 2; ++any)
    for (int full = 0; full < 2; ++full)
      for (int grp = 0; grp < 2; ++grp)
        HIP_OK(pow_launch_search_lat(full != 0, any != 0, grp != 0, 1, ctx->stream, ctx->lat_consts, LL,
                                     ctx->d_lat, ctx->d_lat_host));
  HIP_OK(pow_launch_hash(0, ctx->stream, nullptr, nullptr));
  PowMsg M;
  memset(&M, 0, sizeof M);
  HIP_OK(pow_launch_hash_one(ctx->stream, M, ctx->d_one, 0));  // publishes done = 0: never a live seq
  if (int rc = stream_wait_for(ctx, "warm-up launches", 0)) return rc;
#ifdef POW_TEST_HOOKS
  if (ctx->aql) {  // the same launches once through the direct-dispatch queue (its first packets)
    for (int k = 0; k < 9; ++k) {
      const uint64_t deadline = mono_ns() + ctx->watchdog_ns;
      if (int rc = k < 8 ? launch_search_lat(ctx, k & 1, k & 2, k & 4, 1, LL, deadline)
                         : launch_hash_one(ctx, M, 0, deadline))
        return rc;
      for (int st, n = 0; (st = pow_aql_status(ctx->aql)) != 0; ++n) {
        if (st < 0) return fail(POW_EHIP, "warm-up dispatch: queue error 0x%x", -st);
        if (n > 20000) break;  // POW_AQL_EXP_NO_SIGNAL: no completion to wait for; ~20 ms
        std::this_thread::sleep_for(std::chrono::microseconds(1));
      }
    }
  }
#endif
  pow_block b;
  memset(&b, 0, sizeof b);
  return pow_hash_blocks(ctx, &b, 1, nullptr, nullptr);
}

int pow_launch_path(const pow_ctx* ctx) {
  if (!ctx) return fail(POW_EINVAL, "null");
#ifdef POW_TEST_HOOKS
  if (ctx->aql) return POW_LAUNCH_DIRECT;
#endif
  return POW_LAUNCH_HIP;
}

int pow_get_stats(const pow_ctx* ctx, pow_stats* out) {
  if (!ctx || !out) return fail(POW_EINVAL, "null");
  *out = ctx->stats;
  return POW_OK;
}

int pow_device_info(const pow_ctx* ctx, int* cu_count, int* clock_khz, char* name, size_t name_cap) {
  if (!ctx) return fail(POW_EINVAL, "null");
  if (cu_count) *cu_count = ctx->cu_count;
  if (clock_khz) *clock_khz = ctx->clock_khz;
  if (name && name_cap) snprintf(name, name_cap, "%s", ctx->name);
  return POW_OK;
}

int pow_device_pci_bus_id(const pow_ctx* ctx, char* out, size_t cap) {
  if (!ctx || !out || cap < 2) return fail(POW_EINVAL, "null");
  out[0] = 0;
  HIP_OK(hipDeviceGetPCIBusId(out, (int)std::min<size_t>(cap, 1024), ctx->device));
  return POW_OK;
}

int pow_nonce_from_counter(uint64_t ctr, char nonce[POW_NONCE_SIZE]) {
  if (!nonce) return fail(POW_EINVAL, "null nonce");
  if (ctr >= POW_COUNTER_LIMIT) return fail(POW_EINVAL, "counter >= 62^9");
  for (int i = POW_NONCE_SIZE - 2; i >= 0; --i) {
    nonce[i] = digit_char((unsigned)(ctr % 62));
    ctr /= 62;
  }
  nonce[POW_NONCE_SIZE - 1] = 0;  // block.cpp:71
  return POW_OK;
}

int pow_block_to_bytes(const pow_block* b, uint8_t out[POW_MSG_BYTES]) {
  if (!b || !out) return fail(POW_EINVAL, "null");
  // block.cpp:81-84: std::string::operator+=(char) keeps the low byte (trap T1)
  out[0] = (uint8_t)b->index;
  out[1] = (uint8_t)b->node_owner_number;
  out[2] = (uint8_t)b->difficulty;
  out[3] = (uint8_t)b->created_at;
  memcpy(out + 4, b->nonce, POW_NONCE_SIZE);                        // block.cpp:85
  memcpy(out + 4 + POW_NONCE_SIZE, b->previous_block_hash, POW_HASH_SIZE);  // block.cpp:86
  return POW_OK;
}

int pow_solves_problem(const char* hex, unsigned diff_bits) {
  if (!hex) return 0;
  // block.cpp:28-58, 91-96: binary expansion of the hex string (toupper;
  // non-hex chars count as "1111"), first diff_bits chars must be '0'.
  const size_t len = strlen(hex);
  if ((size_t)diff_bits > 4 * len) return 0;
  for (unsigned i = 0; i < diff_bits; ++i) {
    char c = hex[i / 4];
    unsigned v;
    if (c >= '0' && c <= '9') v = (unsigned)(c - '0');
    else if ((c >= 'a' && c <= 'e') || (c >= 'A' && c <= 'E')) v = 10u + (unsigned)((c | 0x20) - 'a');
    else v = 15;
    if ((v >> (3 - i % 4)) & 1u) return 0;
  }
  return 1;
}

namespace {
// One block through K2' (pow_hash_one): the message by value, the digest from
// mapped host memory once the kernel's done word shows this launch's seq.
int hash_one(pow_ctx* ctx, const pow_block* b, uint8_t* digest, char* hex) {
  PowMsg M;
  uint8_t m[320];
  padded_message(b, m);
  for (int c = 0; c < 5; ++c) {  // the message schedules, K folded in (the rounds run on the GPU)
    uint32_t w[64];
    expand(w, m + 64 * c);
    for (int i = 0; i < 64; ++i) M.kw[c][i] = kK[i] + w[i];
  }
  if (++ctx->one_seq == 0) ctx->one_seq = 1;  // never 0: the warm-up launch publishes 0
  const uint32_t seq = ctx->one_seq;
  const uint64_t t0 = mono_ns(), deadline = t0 + ctx->watchdog_ns;
  if (int rc = launch_hash_one(ctx, M, seq, deadline)) return rc;
  if (int rc = wait_published(ctx, &ctx->h_one->done, &ctx->h_one->started, seq, "hash kernel", t0, deadline))
    return rc;
  uint32_t dg[8];
  for (int k = 0; k < 8; ++k) dg[k] = __atomic_load_n(&ctx->h_one->digest[k], __ATOMIC_RELAXED);
  ctx->stats = pow_stats{(double)ctx->h_one->ticks / ctx->realtime_khz, 1u, 1u};
  digest_out(dg, digest, hex);
  return POW_OK;
}
}  // namespace

int pow_hash_blocks(pow_ctx* ctx, const pow_block* blocks, size_t n, uint8_t* digests, char* hex) {
  if (!ctx || (!blocks && n)) return fail(POW_EINVAL, "null");
  if (n == 0) return POW_OK;
  if (n > (1u << 24)) return fail(POW_EINVAL, "batch too large");
  if (int rc = set_dev(ctx)) return rc;
  if (n == 1) return hash_one(ctx, blocks, digests, hex);  // validation: one block, lowest latency
  if (n > ctx->hash_cap) {
    (void)hipFree(ctx->d_msgs);
    (void)hipFree(ctx->d_dig);
    ctx->d_msgs = nullptr;
    ctx->d_dig = nullptr;
    ctx->hash_cap = 0;
    HIP_OK(hipMalloc(&ctx->d_msgs, n * 320));
    HIP_OK(hipMalloc(&ctx->d_dig, n * 32));
    ctx->hash_cap = n;
  }
  std::vector<uint32_t> words(n * 80);
  for (size_t i = 0; i < n; ++i) {
    uint8_t m[320];
    padded_message(&blocks[i], m);
    for (int k = 0; k < 80; ++k) words[i * 80 + k] = be32(m + 4 * k);
  }
  HIP_OK(hipMemcpyAsync(ctx->d_msgs, words.data(), n * 320, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipEventRecord(ctx->ev0, ctx->stream));
  HIP_OK(pow_launch_hash((uint32_t)n, ctx->stream, ctx->d_msgs, ctx->d_dig));
  HIP_OK(hipEventRecord(ctx->ev1, ctx->stream));
  std::vector<uint32_t> dg(n * 8);
  HIP_OK(hipMemcpyAsync(dg.data(), ctx->d_dig, n * 32, hipMemcpyDeviceToHost, ctx->stream));
  if (int rc = stream_wait_for(ctx, "batch hash kernel", 100ull * n)) return rc;  // + 100 ns per block
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  ctx->stats = pow_stats{ms, 1u, (uint64_t)n};
  for (size_t i = 0; i < n; ++i)
    digest_out(&dg[i * 8], digests ? digests + 32 * i : nullptr, hex ? hex + 65 * i : nullptr);
  return POW_OK;
}

int pow_hash_block(pow_ctx* ctx, const pow_block* b, uint8_t digest[32], char hex[65]) {
  return pow_hash_blocks(ctx, b, 1, digest, hex);
}



int pow_sweep_device(pow_ctx* ctx, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
                     unsigned diff_bits, uint32_t* dev_out, size_t cap, size_t* n_found,
                     uint64_t* min_ctr) {
  if (!ctx) return fail(POW_EINVAL, "null ctx");
  if (int rc = check_range(tmpl, ctr_start, ctr_count, diff_bits)) return rc;
  if (ctr_count > (1ull << 32)) return fail(POW_EINVAL, "sweep count > 2^32");
  if (cap && !dev_out) return fail(POW_EINVAL, "cap without buffer");
  if (int rc = set_dev(ctx)) return rc;
  ctx->stats = pow_stats{};
  if (n_found) *n_found = 0;
  if (min_ctr) *min_ctr = ~0ull;
  if (ctr_count == 0) return POW_OK;
  if (int rc = upload_consts(ctx, tmpl)) return rc;
  const uint32_t cap32 = (uint32_t)std::min<size_t>(cap, 0xFFFFFFFFu);
  if (int rc = run_search(ctx, ctr_start, ctr_count, diff_bits, 0, dev_out, cap32)) return rc;
  // The kernel writes 32-entry blocks to dev_out and each wave's last < 32
  // solutions to ctx->d_tail: append those behind the blocks.
  const uint64_t nblk = ctx->h_res->count, ntail = ctx->h_res->tail;  // count is 64-bit: d = 0 fills 2^32
  if (ntail > ctx->tail_cap) return fail(POW_EHIP, "sweep tail overflow (%llu)", (unsigned long long)ntail);
  if (ntail && nblk < cap32) {
    const uint64_t k = std::min<uint64_t>(ntail, cap32 - nblk);
    HIP_OK(hipMemcpyAsync(dev_out + nblk, ctx->d_tail, k * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                          ctx->stream));
    if (int rc = stream_wait_for(ctx, "sweep tail copy", 0)) return rc;
  }
  if (n_found) *n_found = nblk + ntail;
  if (min_ctr && ctx->h_res->min_rel != ~0ull) *min_ctr = ctr_start + ctx->h_res->min_rel;
  return POW_OK;
}

int pow_sweep(pow_ctx* ctx, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
              unsigned diff_bits, uint32_t* out_ctrs, size_t cap, size_t* n_found) {
  // The device radix sort takes a signed 32-bit item count (hipCUB).
  if (cap > 0x7FFFFFFFu) return fail(POW_EINVAL, "cap %zu > 2^31-1 (the host-list form sorts on the device)", cap);
  if (!ctx || !n_found) return fail(POW_EINVAL, "null");
  if (cap && !out_ctrs) return fail(POW_EINVAL, "cap without buffer");
  if (int rc = set_dev(ctx)) return rc;
  if (cap > ctx->out_cap) {
    (void)hipFree(ctx->d_out);
    (void)hipFree(ctx->d_alt);
    (void)hipFree(ctx->d_sort_tmp);
    ctx->d_out = ctx->d_alt = nullptr;
    ctx->d_sort_tmp = nullptr;
    ctx->out_cap = ctx->sort_tmp_bytes = 0;
    HIP_OK(hipMalloc(&ctx->d_out, cap * sizeof(uint32_t)));
    HIP_OK(hipMalloc(&ctx->d_alt, cap * sizeof(uint32_t)));
    size_t tb = 0;
    HIP_OK(pow_sort_u32(nullptr, &tb, ctx->d_out, ctx->d_alt, (uint32_t)cap, nullptr, ctx->stream));
    HIP_OK(hipMalloc(&ctx->d_sort_tmp, tb ? tb : 1));
    ctx->sort_tmp_bytes = tb;
    ctx->out_cap = cap;
  }
  size_t n = 0;
  uint64_t mn = 0;
  int rc = pow_sweep_device(ctx, tmpl, ctr_start, ctr_count, diff_bits, cap ? ctx->d_out : nullptr,
                            cap, &n, &mn);
  if (rc) return rc;
  *n_found = n;
  const size_t got = std::min(n, cap);
  if (got) {
    // ascending order: device radix sort (the kernel appends in completion order)
    uint32_t* sorted = ctx->d_out;
    size_t tb = ctx->sort_tmp_bytes;
    HIP_OK(pow_sort_u32(ctx->d_sort_tmp, &tb, ctx->d_out, ctx->d_alt, (uint32_t)got, &sorted, ctx->stream));
    HIP_OK(hipMemcpyAsync(out_ctrs, sorted, got * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
    if (int rc = stream_wait_for(ctx, "sweep sort and copy", 4ull * got)) return rc;  // + 1 ns per byte
  }
  return n > cap ? fail(POW_ENOSPC, "%zu solutions > cap %zu", n, cap) : POW_OK;
}

// pow_mine (any = false: lowest solving counter, deterministic) and
// pow_mine_any (any = true: the first solution any wave finds; the whole grid
// stops at its next step — the reference's random-nonce miner has no order
// either, node.cpp:302).
static int mine_impl(pow_ctx* ctx, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
                     unsigned diff_bits, const volatile uint32_t* cancel_word, uint32_t epoch,
                     pow_block* out, uint64_t* found_ctr, uint64_t* hashes_done, bool any) {
  if (!ctx || !out) return fail(POW_EINVAL, "null");
  if (int rc = check_range(tmpl, ctr_start, ctr_count, diff_bits)) return rc;
  if (int rc = set_dev(ctx)) return rc;
  ctx->stats = pow_stats{};
  if (hashes_done) *hashes_done = 0;
#ifdef POW_TEST_HOOKS
  if (ctx->fault_mine) return fail(POW_EHIP, "injected fault (POW_FAULT_INJECT=mine)");
#endif
  if (int rc = upload_consts(ctx, tmpl)) return rc;
  ctx->launch_epoch = epoch;
  ctx->watch_epoch = cancel_word != nullptr;
  struct Unwatch {  // sweeps and later calls start unwatched
    pow_ctx* c;
    ~Unwatch() { c->watch_epoch = false; }
  } unwatch{ctx};
  // Sub-round plan.
  //  * d <= 21 (expected trials <= 2M): sub-round 1 on the latency kernel K1'
  //    over 16x the expected trials, capped at ctx->lat_max.  Few waves per
  //    SIMD: a wave-iteration (64 trials per lane-set) then takes ~10 us
  //    instead of ~66 us at 8 waves/SIMD, which sets the time to first hit.
  //  * then the throughput kernel K1.  pow_mine_any: single 2^30-counter
  //    launches (~0.13 s, the cancel-poll granularity); every wave stops
  //    within one j-step of the first hit.  pow_mine (lowest counter): waves
  //    holding lower counters must finish, so sub-rounds start near the
  //    expected trials and grow 4x.
  const unsigned dcap = diff_bits > 40 ? 40 : diff_bits;
  const bool use_lat = ctx->lat_max > 0 && diff_bits <= 21;
  const unsigned lat_wps = ctx->lat_wps ? ctx->lat_wps : diff_bits <= 17 ? 1 : diff_bits <= 19 ? 2 : 4;
  uint64_t step = use_lat ? std::max<uint64_t>(1ull << 12, 1ull << (dcap + 4))
                          : (any ? 1ull << 30 : std::max<uint64_t>(1ull << 12, 1ull << std::min(dcap + 2, 30u)));
  // Bound stop board: a peer's solution makes the rest of the range moot —
  // any peer solution in any-mode, one below `next` in lowest mode.
  auto preempted = [&](uint64_t next) {
    const uint64_t m = board_peer_min(ctx);
    return any ? m != UINT64_MAX : m < next;
  };
  uint64_t done = 0;
  bool first = true;
  while (done < ctr_count) {
    if (cancel_moved(cancel_word, epoch) || preempted(ctr_start + done)) break;
    const bool lat = first && use_lat;
    const uint64_t cap = lat ? ctx->lat_max : (uint64_t)1 << 30;
    const uint64_t n = std::min<uint64_t>(std::min<uint64_t>(step, cap), ctr_count - done);
    const uint64_t s0 = ctr_start + done;
    if (int rc = lat ? run_search_lat(ctx, s0, n, diff_bits, any, lat_wps)
                     : run_search(ctx, s0, n, diff_bits, any ? 2 : 1, nullptr, 0))
      return rc;
    first = false;
    done += n;
    // cancelled while the launch ran (pow_cancel stops it early; its result,
    // if any, belongs to a stale template and, in lowest mode, may not be final)
    if (cancel_moved(cancel_word, epoch) || ctx->h_res->cancelled) break;
    if (ctx->h_res->min_rel != ~0ull) {
      const PowResult& r = *ctx->h_res;
      // The latency kernel records its first POW_HITS hits with their digests.
      // pow_mine needs the lowest hit (min_rel); pow_mine_any takes the lowest
      // RECORDED hit, so at low d (more hits per launch than slots) it still
      // needs no K2 launch.  Otherwise K2 hashes the winner.
      const PowHit* h = nullptr;
      for (uint32_t k = 0; lat && k < std::min<uint32_t>(r.nhit, POW_HITS); ++k) {
        const PowHit* c = &r.hit[k];
        if (any ? (!h || c->rel < h->rel) : c->rel == r.min_rel) h = c;
      }
      const uint64_t ctr = s0 + (h ? h->rel : r.min_rel);
      // Lowest mode with a bound board: a peer already holds a lower counter,
      // so this one is not the search's answer (and, since waves between the
      // peer's counter and this one may have stopped early, not necessarily
      // the lowest of this call's range either): the peer's result wins.
      if (!any && board_peer_min(ctx) < ctr) break;
      *out = *tmpl;
      pow_nonce_from_counter(ctr, out->nonce);
      char hx[65];
      if (h) {
        digest_out(h->digest, nullptr, hx);
      } else {
        // Hash the winner with a one-counter K1' launch (difficulty 0: it
        // records its digest): one dispatch with the constants as kernel
        // argument, about half the latency of K2's copy-in / hash / copy-out.
        const pow_stats keep = ctx->stats;
        ctx->watch_epoch = false;  // the winner is hashed even if the epoch moves now ...
        ctx->board_off = true;     // ... or a peer has published a solution
        const int rc = run_search_lat(ctx, ctr, 1, 0, true, 1);
        ctx->board_off = false;
        if (rc) return rc;
        ctx->stats = keep;
        const PowResult& w = *ctx->h_res;
        if (w.nhit < 1 || w.hit[0].rel != 0) return fail(POW_EHIP, "winner re-hash recorded no digest");
        digest_out(w.hit[0].digest, nullptr, hx);
      }
      memcpy(out->block_hash, hx, 65);  // strcpy semantics (node.cpp:318)
      if (found_ctr) *found_ctr = ctr;
      if (hashes_done) *hashes_done = ctx->stats.hashes;
      // The kernel already stored its hits; this is the exact result.
      if (ctx->board) pow_board_post(ctx->board, ctx->board_slot, ctx->board_tag, ctr);
      return 1;
    }
    if (preempted(ctr_start + done)) break;
    step = any ? 1ull << 30 : std::min<uint64_t>(n * 4, 1ull << 30);
  }
  if (hashes_done) *hashes_done = ctx->stats.hashes;
  return 0;
}

int pow_mine(pow_ctx* ctx, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
             unsigned diff_bits, const volatile uint32_t* cancel_word, uint32_t epoch,
             pow_block* out, uint64_t* found_ctr, uint64_t* hashes_done) {
  return mine_impl(ctx, tmpl, ctr_start, ctr_count, diff_bits, cancel_word, epoch, out, found_ctr,
                   hashes_done, false);
}

int pow_mine_any(pow_ctx* ctx, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
                 unsigned diff_bits, const volatile uint32_t* cancel_word, uint32_t epoch,
                 pow_block* out, uint64_t* found_ctr, uint64_t* hashes_done) {
  return mine_impl(ctx, tmpl, ctr_start, ctr_count, diff_bits, cancel_word, epoch, out, found_ctr,
                   hashes_done, true);
}

int pow_cancel(pow_ctx* ctx, uint32_t epoch) {
  if (!ctx) return fail(POW_EINVAL, "null");
  // A plain store into mapped host memory: no HIP call, no stream; the
  // kernel's sentinel wave reads it over PCIe at its next poll.
  __atomic_store_n(ctx->h_epoch, epoch, __ATOMIC_SEQ_CST);
  ctx->armed.store(true, std::memory_order_release);
  return POW_OK;
}

int pow_board_bind(pow_ctx* ctx, pow_board* b, int slot, uint32_t tag) {
  if (!ctx) return fail(POW_EINVAL, "null ctx");
  if (!b) {
    ctx->board = nullptr;
    ctx->board_dev = nullptr;
    ctx->board_slot = -1;
    ctx->board_tag = 0;
    return POW_OK;
  }
  if (slot < 0 || slot >= pow_board_nslots(b)) return fail(POW_EINVAL, "slot %d of %d", slot, pow_board_nslots(b));
  if (tag < 1 || tag > POW_BOARD_MAX_TAG) return fail(POW_EINVAL, "tag must be 1..1023");
  if (int rc = set_dev(ctx)) return rc;
  if (int rc = pow_board_register(b)) return rc;
  void* d = nullptr;
  HIP_OK(hipHostGetDevicePointer(&d, pow_board_host_slots(b), 0));
  ctx->board = b;
  ctx->board_dev = (const unsigned long long*)d;
  ctx->board_slot = slot;
  ctx->board_tag = tag;
  return pow_board_post(b, slot, tag, UINT64_MAX);  // nothing found yet in this search
}

int pow_dev_alloc(pow_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !out) return fail(POW_EINVAL, "null");
  *out = nullptr;
  if (int rc = set_dev(ctx)) return rc;
  HIP_OK(hipMalloc(out, bytes ? bytes : 1));
  return POW_OK;
}

int pow_dev_free(pow_ctx* ctx, void* p) {
  if (!ctx) return fail(POW_EINVAL, "null");
  if (int rc = set_dev(ctx)) return rc;
  HIP_OK(hipFree(p));
  return POW_OK;
}

int pow_dev_read(pow_ctx* ctx, const void* dev, void* host, size_t bytes) {
  if (!ctx || (bytes && (!dev || !host))) return fail(POW_EINVAL, "null");
  if (int rc = set_dev(ctx)) return rc;
  HIP_OK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
  return stream_wait_for(ctx, "device read", bytes);  // + 1 ns per byte
}

}  // extern "C"
