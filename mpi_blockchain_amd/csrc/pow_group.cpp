// Sharded multi-GPU search over RCCL (BASELINE config 4).
//
// One pow_ctx per GPU, one process (or host thread) per GPU.  A search of
// [start, start + count) runs in rounds of `round_size` counters.  Each round
// is cut into `nranks` contiguous static shards (pow_group_partition, the same
// split as mpi_blockchain_amd/shard.py); every rank runs pow_mine (lowest
// solving counter) on its shard, then ONE ncclAllReduce(ncclUint64, ncclMin)
// of three words {lowest counter, go, ok} picks the winner, carries
// cancellation and reports a failed peer.  Every rank returns the same
// counter: the one a single GPU (or the CPU oracle) finds first.
//
// The reference has no mining-side collective: each MPI rank mines its own
// template with its own rand() stream (node.cpp:302, 386) and talks only on
// success (send_block_to_everyone, node.cpp:260-273).  This is the
// cooperative form of that search: one template, several GPUs.
//
// Inside a round, the ranks of one node also share a stop board
// (pow_board.cpp), named after the RCCL id: a rank's hit reaches the other
// GPUs' running kernels within one inner step, so they stop mining instead of
// finishing their shards (any-mode: every peer stops; lowest mode: peers stop
// the counters above the hit).  The round's all-reduce then only agrees on a
// winner the ranks already know of.
//
// RCCL is opened with dlopen at first use, so libpow_gpu.so has no link-time
// dependency on it and the single-GPU entry points never load it.  A group
// made by pow_group_init_custom runs the same rounds over the caller's
// reduction instead (MPI_Allreduce, torch.distributed, or several test ranks
// sharing one GPU, which RCCL refuses).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <link.h>
#include <rccl/rccl.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>

#include "../../include/pow_gpu.h"
#include "pow_template.h"

namespace {

// The RCCL entry points used here (rccl.h:187, 204, 260, 271, 339, 362, 378, 389, 611).
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRankConfig) comm_init_rank_config = nullptr;
  decltype(&ncclCommGetAsyncError) get_async_error = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclCommCount) comm_count = nullptr;
  decltype(&ncclCommCuDevice) comm_cu_device = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;
  char why[256] = {0};   // non-empty: RCCL is unusable
  char path[512] = {0};  // the file the entry points come from
};

// An RCCL the process has already loaded (torch's libtorch_hip pulls in its
// own torch/lib/librccl.so at import): its path, or "" if none.
int find_loaded_rccl(struct dl_phdr_info* info, size_t, void* data) {
  const char* name = info->dlpi_name;
  if (!name || !*name) return 0;
  const char* base = strrchr(name, '/');
  base = base ? base + 1 : name;
  if (strncmp(base, "librccl.so", 10) != 0) return 0;
  snprintf(static_cast<char*>(data), 512, "%s", name);
  return 1;
}

const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = nullptr;
#ifdef POW_TEST_HOOKS
    // Test library only: a stand-in RCCL (tests/stub_rccl) that reduces over
    // POSIX shared memory, so pow_group_init's RCCL leg runs with several
    // ranks on the one GPU of a test box (RCCL refuses two ranks per GPU).
    if (const char* p = getenv("POW_TEST_RCCL_LIB")) {
      if (!(h = dlopen(p, RTLD_NOW | RTLD_LOCAL))) {
        snprintf(x.why, sizeof x.why, "cannot load POW_TEST_RCCL_LIB %s: %s", p, dlerror());
        return x;
      }
    }
#endif
    // One RCCL runtime per process: if one is loaded already (torch's, in
    // bench.py's ranks), bind to that very copy (RTLD_NOLOAD: no second
    // load) instead of resolving librccl.so.1 on our own, which could map
    // /opt/rocm's copy beside torch's and run two RCCL runtimes side by side.
    char loaded[512] = {0};
    if (!h && dl_iterate_phdr(find_loaded_rccl, loaded) && loaded[0])
      h = dlopen(loaded, RTLD_NOW | RTLD_NOLOAD | RTLD_LOCAL);
    for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if (h || (h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
    if (!h) {
      snprintf(x.why, sizeof x.why, "cannot load RCCL: %s", dlerror());
      return x;
    }
    x.get_unique_id = (decltype(x.get_unique_id))dlsym(h, "ncclGetUniqueId");
    x.comm_init_rank_config = (decltype(x.comm_init_rank_config))dlsym(h, "ncclCommInitRankConfig");
    x.get_async_error = (decltype(x.get_async_error))dlsym(h, "ncclCommGetAsyncError");
    x.comm_destroy = (decltype(x.comm_destroy))dlsym(h, "ncclCommDestroy");
    x.all_reduce = (decltype(x.all_reduce))dlsym(h, "ncclAllReduce");
    x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
    x.comm_count = (decltype(x.comm_count))dlsym(h, "ncclCommCount");
    x.comm_cu_device = (decltype(x.comm_cu_device))dlsym(h, "ncclCommCuDevice");
    x.comm_abort = (decltype(x.comm_abort))dlsym(h, "ncclCommAbort");
    if (!x.get_unique_id || !x.comm_init_rank_config || !x.get_async_error || !x.comm_destroy || !x.all_reduce || !x.error_string ||
        !x.comm_count || !x.comm_cu_device || !x.comm_abort)
      snprintf(x.why, sizeof x.why, "RCCL lacks an entry point");
    Dl_info info;
    if (x.all_reduce && dladdr((const void*)x.all_reduce, &info) && info.dli_fname) {
      // dladdr names the object as it was loaded; resolve it to a canonical path
      char* real = realpath(info.dli_fname, nullptr);
      snprintf(x.path, sizeof x.path, "%s", real ? real : info.dli_fname);
      free(real);
    }
    return x;
  }();
  return r;
}

int comm_fail(const char* what, ncclResult_t r) {
  char buf[320];
  snprintf(buf, sizeof buf, "%s: %s", what, rccl().error_string ? rccl().error_string(r) : "?");
  return pow_set_error(POW_ECOMM, buf);
}

int hip_fail(const char* what, hipError_t e) {
  char buf[320];
  snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
  return pow_set_error(POW_EHIP, buf);
}

constexpr size_t kMaxWords = 8;

uint64_t now_ns() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

// pow_group_init's deadline for every rank to join the communicator.
constexpr unsigned kInitTimeoutMs = 60000;

// The communicator is non-blocking (config.blocking = 0): RCCL calls on it may
// return ncclInProgress while their work goes on in the background (joining
// the peers at init, connecting to them at the first collective), and the
// next call on the communicator or its stream must wait until the state
// leaves ncclInProgress.  That wait is polled here against `deadline_ns`
// (CLOCK_MONOTONIC); *late = true if it ran out first (the state is then
// still ncclInProgress and the communicator must be aborted).
ncclResult_t comm_settle(ncclComm_t c, uint64_t deadline_ns, bool* late) {
  *late = false;
  for (;;) {
    ncclResult_t st = ncclInProgress;
    const ncclResult_t r = rccl().get_async_error(c, &st);
    if (r != ncclSuccess) return r;
    if (st != ncclInProgress) return st;
    if (now_ns() > deadline_ns) {
      *late = true;
      return ncclInProgress;
    }
    const timespec nap{0, 200000};  // 0.2 ms: a peer that is late by seconds costs no spinning core
    nanosleep(&nap, nullptr);
  }
}

// ncclCommAbort with a bound, for a communicator whose collective failed or
// ran out of time (a peer that never joined it).  RCCL's abort waits for its
// own threads (the init thread, the proxy), and one of them may be waiting for
// that peer: on the MI355X box RCCL 2.27.7's init thread spun in the
// bootstrap for as long as the missing peer stayed away
// (profiles/r06/verify/rccl_abort_probe).  So the abort runs on a detached
// thread and is given `grace_ms`; past that the communicator (and the thread)
// are left behind, and the caller, whose rank has already failed, goes on.
// true = the abort returned in time.
bool abort_bounded(ncclComm_t c, unsigned grace_ms) {
  auto done = std::make_shared<std::atomic<bool>>(false);
  std::thread([c, done] {
    (void)rccl().comm_abort(c);
    done->store(true, std::memory_order_release);
  }).detach();
  const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(grace_ms);
  while (!done->load(std::memory_order_acquire) && std::chrono::steady_clock::now() < until)
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  return done->load(std::memory_order_acquire);
}

constexpr unsigned kAbortGraceMs = 5000;

// One ncclCommInitRankConfig call, run on a helper thread so that the caller
// can stop waiting for it.  RCCL 2.27.7 does not return from the call until
// the communicator is complete even with config.blocking = 0 (1 rank: 5.5 s,
// ncclSuccess; 2 ranks with the peer missing: no return in 40 s; its own init
// thread does the work while the calling thread sleeps in a wait loop,
// profiles/r06/verify/rccl_abort_probe).  An RCCL that honours the
// non-blocking config returns ncclInProgress at once; the helper then polls
// ncclCommGetAsyncError itself until the communicator is ready, so the init
// completes on the thread that started it (RCCL may keep a pending init in
// that thread's state).  A failed init is aborted on the helper too.  A caller
// that gives up marks the job abandoned; the helper then aborts whatever it
// gets.  The caller only reads the published result.
struct InitJob {
  std::atomic<int> state{0};  // 0 running, 1 published, 2 abandoned by the caller
  ncclComm_t comm = nullptr;  // published: a ready communicator, or null
  ncclResult_t r = ncclInternalError;
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  ncclUniqueId id{};
  int nranks = 0, rank = 0, device = 0;
};

void run_init(std::shared_ptr<InitJob> job) {
  ncclComm_t c = nullptr;
  ncclResult_t r = ncclUnhandledCudaError;
  if (hipSetDevice(job->device) == hipSuccess)  // RCCL binds the communicator to the calling thread's device
    r = rccl().comm_init_rank_config(&c, job->nranks, job->id, job->rank, &job->cfg);
  while (r == ncclInProgress && c && job->state.load(std::memory_order_acquire) == 0) {
    ncclResult_t st = ncclInProgress;
    if (rccl().get_async_error(c, &st) != ncclSuccess) st = ncclInternalError;
    r = st;
    if (r == ncclInProgress) std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  const bool ok = r == ncclSuccess && c;
  job->comm = ok ? c : nullptr;
  job->r = ok ? ncclSuccess : (r == ncclSuccess ? ncclInternalError : r);
  int running = 0;
  const bool published = job->state.compare_exchange_strong(running, 1, std::memory_order_acq_rel);
  if (c && (!ok || !published)) (void)rccl().comm_abort(c);  // failed, or nobody will use it
}

}  // namespace

struct pow_group {
  pow_ctx* ctx = nullptr;     // null: a group that only carries collectives (pow_group_init_custom)
  int nranks = 1, rank = 0;
  ncclComm_t comm = nullptr;  // RCCL communicator (pow_group_init) ...
  pow_group_reduce_fn reduce = nullptr;  // ... or the caller's reduction (pow_group_init_custom)
  void* reduce_user = nullptr;
  uint64_t* d_buf = nullptr;  // kMaxWords device words: the all-reduce operand
  uint64_t* h_buf = nullptr;  // pinned host mirror
  pow_board* board = nullptr; // the node's stop board (null: more than 64 ranks, or none available)
  uint32_t searches = 0;      // searches so far: every rank counts the same (the calls are collective)
  uint64_t shard_budget = 0;  // counters of the current round's largest shard (the all-reduce's watchdog budget)
  // A collective failed or passed its deadline (or this rank left a round
  // without joining its all-reduce): the ranks are out of step, so every later
  // collective is refused, and destroy aborts the communicator (ncclCommAbort,
  // not ncclCommDestroy) and frees the buffers only once the stream drained.
  bool broken = false;
  pow_group_search_info last{};  // the last pow_group_mine[_any] call (pow_group_last_search)
};

namespace {

// In-place all-reduce of n <= kMaxWords u64 (op = POW_REDUCE_*): RCCL on the
// ctx's stream, or the caller's reduction of a custom group.
int group_allreduce(pow_group* g, uint64_t* v, size_t n, int op) {
  if (g->broken)
    return pow_set_error(POW_ECOMM, "the group is broken (an earlier collective failed or ran out of time, or a rank "
                                    "left a round without it): destroy it");
  if (g->reduce) {
    if (g->reduce(g->reduce_user, v, n, op) != 0) {
      g->broken = true;
      return pow_set_error(POW_ECOMM, "custom reduction failed");
    }
    return POW_OK;
  }
  const ncclRedOp_t o = op == POW_REDUCE_MIN ? ncclMin : op == POW_REDUCE_MAX ? ncclMax : ncclSum;
  hipError_t e = hipSetDevice(pow_ctx_device(g->ctx));
  if (e != hipSuccess) return hip_fail("hipSetDevice", e);
  hipStream_t st = (hipStream_t)pow_ctx_stream(g->ctx);
  memcpy(g->h_buf, v, n * sizeof(uint64_t));
  if ((e = hipMemcpyAsync(g->d_buf, g->h_buf, n * 8, hipMemcpyHostToDevice, st)) != hipSuccess) {
    g->broken = true;
    return hip_fail("hipMemcpyAsync", e);
  }
  // Bounded (the watchdog): a peer that never joins this all-reduce (dead, or
  // stuck in its own launch) fails the call instead of hanging every rank.  A
  // peer still mining its shard of the round is waited for: the budget grows
  // with the round's shard (2 ns per counter, as the launch watchdog).
  const uint64_t t0 = now_ns(), budget = 10ull * 1000000000ull + 2ull * g->shard_budget;
  ncclResult_t r = rccl().all_reduce(g->d_buf, g->d_buf, n, ncclUint64, o, g->comm, st);
  bool late = false;
  if (r == ncclInProgress) r = comm_settle(g->comm, t0 + budget, &late);  // enqueued in the background
  if (r != ncclSuccess) {
    g->broken = true;
    if (!late) return comm_fail("ncclAllReduce", r);
    char buf[256];
    snprintf(buf, sizeof buf, "ncclAllReduce: not enqueued within %.3f s (the communicator stayed in progress)",
             (now_ns() - t0) * 1e-9);
    return pow_set_error(POW_ECOMM, buf);
  }
  if ((e = hipMemcpyAsync(g->h_buf, g->d_buf, n * 8, hipMemcpyDeviceToHost, st)) != hipSuccess) {
    g->broken = true;
    return hip_fail("hipMemcpyAsync", e);
  }
  if (pow_ctx_stream_wait(g->ctx, "ncclAllReduce", 2ull * g->shard_budget) != POW_OK) {
    g->broken = true;  // the communicator has an operation in flight: destroy aborts it
    char buf[512];
    snprintf(buf, sizeof buf, "%s", pow_last_error());
    return pow_set_error(POW_ECOMM, buf);
  }
  memcpy(v, g->h_buf, n * sizeof(uint64_t));
  return POW_OK;
}

// The board's shared-memory name: from the RCCL id, the same on every rank.
void board_name(const uint8_t id[POW_GROUP_ID_BYTES], char name[40]) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a
  for (int i = 0; i < POW_GROUP_ID_BYTES; ++i) h = (h ^ id[i]) * 1099511628211ull;
  snprintf(name, 40, "/pow_board_%016llx", (unsigned long long)h);
}

// Search tag of the next search (1..1023, the same on every rank).
uint32_t next_tag(pow_group* g) { return 1u + (g->searches++ % POW_BOARD_MAX_TAG); }

// Statistics of a multi-call search (pow_mine resets the ctx's per call).
struct StatSum {
  pow_stats s{};
  void add(const pow_ctx* ctx) {
    pow_stats t{};
    pow_get_stats(ctx, &t);
    s.kernel_ms += t.kernel_ms;
    s.launches += t.launches;
    s.hashes += t.hashes;
  }
};

// The winner's digest travels from the rank that found it: its 64-char hex
// (pow_mine's block_hash) as 4 big-endian words.  false = not 64 hex digits.
bool digest_words(const char* hex, uint64_t w[4]) {
  for (int i = 0; i < 4; ++i) {
    uint64_t x = 0;
    for (int j = 0; j < 16; ++j) {
      const char ch = hex[16 * i + j];
      const int d = ch >= '0' && ch <= '9' ? ch - '0' : ch >= 'a' && ch <= 'f' ? ch - 'a' + 10 : -1;
      if (d < 0) return false;
      x = x << 4 | (uint64_t)d;
    }
    w[i] = x;
  }
  return true;
}

// The block every rank returns: *tmpl with the winning counter's nonce and the
// finder's digest as 64 hex chars + NUL (pow_mine's strcpy semantics,
// node.cpp:318: bytes 65..255 keep the template's).
void winner_block(const pow_block* tmpl, uint64_t ctr, const uint64_t w[4], pow_block* out) {
  static const char hexd[] = "0123456789abcdef";
  *out = *tmpl;
  pow_nonce_from_counter(ctr, out->nonce);
  for (int i = 0; i < 64; ++i) out->block_hash[i] = hexd[(w[i / 16] >> (4 * (15 - i % 16))) & 15];
  out->block_hash[64] = 0;
}

// Rounds of a collective search (both modes): every rank mines its static
// shard of each round (with the board bound), then one all-reduce(min) of
// {counter found, go, ok} picks the winner, spreads cancellation and failure.
int group_search(pow_group* g, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count, uint64_t round_size,
                 bool adaptive, unsigned diff_bits, const volatile uint32_t* cancel_word, uint32_t epoch,
                 pow_block* out, uint64_t* found_ctr, uint64_t* hashes_done, bool any) {
  const uint64_t big = (uint64_t)g->nranks << 30;
  const uint32_t tag = next_tag(g);
  pow_group_search_info& info = g->last;
  info = pow_group_search_info{};
  info.board_open = g->board != nullptr;
  if (g->broken) return group_allreduce(g, nullptr, 0, POW_REDUCE_MIN);  // refused: says why
  if (g->board) {
    if (int rc = pow_board_bind(g->ctx, g->board, g->rank, tag)) return rc;
    info.board_bound = 1;
  }
  struct Unbind {
    pow_group* g;
    ~Unbind() { pow_board_bind(g->ctx, nullptr, 0, 0); }
  } unbind{g};
  StatSum st;
  if (hashes_done) *hashes_done = 0;
  for (uint64_t done = 0; done < ctr_count;) {
    const uint64_t n = std::min(round_size, ctr_count - done);
    uint64_t s = 0, k = 0;
    pow_group_partition(ctr_start + done, n, g->rank, g->nranks, &s, &k);
    g->shard_budget = n / (uint64_t)g->nranks + 1;  // the largest shard of the round
    // {counter found by this rank (any: its first; lowest: its shard's lowest), go (0 = cancelled), ok (0 = failed)}
    uint64_t v[3] = {UINT64_MAX, 1, 1};
    int local_rc = POW_OK;
    char local_err[512] = {0};
    pow_block mine_blk;  // this rank's own solution of the round (local_rc == 1)
    uint64_t c = UINT64_MAX;
    ++info.rounds;
    info.local_found = 0;
    if (k) {
      const uint64_t m0 = now_ns();
      local_rc = any ? pow_mine_any(g->ctx, tmpl, s, k, diff_bits, cancel_word, epoch, &mine_blk, &c, nullptr)
                     : pow_mine(g->ctx, tmpl, s, k, diff_bits, cancel_word, epoch, &mine_blk, &c, nullptr);
      info.mine_end_ns = now_ns();
      info.mine_ms += (info.mine_end_ns - m0) * 1e-6;
      st.add(g->ctx);
      if (local_rc == 1) {
        v[0] = c;
        info.local_found = 1;
      }
      if (local_rc < 0) {
        v[2] = 0;
        snprintf(local_err, sizeof local_err, "%s", pow_last_error());
      }
    }
    if (local_rc < 0 && pow_ctx_wedged(g->ctx)) {
      // This rank's launch is stuck on the ctx's stream (its watchdog fired):
      // an all-reduce queued behind it would never run.  Leave at once with
      // the real cause; the peers' all-reduce of this round fails at its own
      // deadline, and the group is unusable from here on.
      g->broken = true;
      g->shard_budget = 0;
      char buf[700];
      snprintf(buf, sizeof buf, "%s; rank %d did not join the round's all-reduce (its stream holds the stuck launch)",
               local_err, g->rank);
      return pow_set_error(local_rc, buf);
    }
    if (cancel_moved(cancel_word, epoch)) v[1] = 0;
    const uint64_t a0 = now_ns();
    const int arc = group_allreduce(g, v, 3, POW_REDUCE_MIN);
    info.allreduce_ms += (now_ns() - a0) * 1e-6;
    g->shard_budget = 0;
    if (arc) {
      if (local_rc >= 0) return arc;
      // Both failed: the rank's own error is the cause, the collective's the consequence.
      char buf[900];
      snprintf(buf, sizeof buf, "%s (and the round's all-reduce failed: %s)", local_err, pow_last_error());
      return pow_set_error(local_rc, buf);
    }
    if (hashes_done) *hashes_done = st.s.hashes;
    pow_ctx_set_stats(g->ctx, st.s);
    if (v[2] == 0)  // every rank leaves the search together
      return local_rc < 0 ? pow_set_error(local_rc, local_err) : pow_set_error(POW_ECOMM, "a peer rank failed");
    if (v[1] == 0) return 0;  // cancelled on some rank
    if (v[0] != UINT64_MAX) {
      // The winner: the rank whose own solution it is contributes its digest
      // (4 words + a presence word; zeros elsewhere) to one all-reduce(max), and
      // every rank writes the same block from it.  No rank re-hashes the winner,
      // so no rank can fail alone after the ranks agreed (round 5 re-hashed it
      // with a one-counter launch on every rank, whose failure on one rank left
      // that rank with an error and the others with the block).
      uint64_t w[5] = {0, 0, 0, 0, 0};
      if (local_rc == 1 && c == v[0] && digest_words(mine_blk.block_hash, w)) w[4] = 1;
      const uint64_t a1 = now_ns();
      const int drc = group_allreduce(g, w, 5, POW_REDUCE_MAX);
      info.allreduce_ms += (now_ns() - a1) * 1e-6;
      if (drc) return drc;
      if (w[4] != 1) return pow_set_error(POW_ECOMM, "the winner's digest did not arrive");
      winner_block(tmpl, v[0], w, out);
      if (found_ctr) *found_ctr = v[0];
      return 1;
    }
    done += n;
    if (adaptive) round_size = std::min<uint64_t>(big, round_size * 4);
  }
  return 0;
}

int check_args(const pow_group* g, const pow_block* tmpl, const pow_block* out, uint64_t ctr_start,
               uint64_t ctr_count, unsigned diff_bits) {
  if (!g || !tmpl || !out) return pow_set_error(POW_EINVAL, "null");
  if (!g->ctx) return pow_set_error(POW_EINVAL, "group has no context (collectives only)");
  if (ctr_start >= POW_COUNTER_LIMIT || ctr_count > POW_COUNTER_LIMIT - ctr_start)
    return pow_set_error(POW_EINVAL, "counter range past 62^9");
  if (diff_bits > 256) return pow_set_error(POW_EINVAL, "difficulty > 256 bits");
  return POW_OK;
}

}  // namespace

extern "C" {

void pow_group_partition(uint64_t start, uint64_t count, int rank, int nranks, uint64_t* shard_start,
                         uint64_t* shard_count) {
  if (nranks < 1) nranks = 1;
  const uint64_t base = count / (uint64_t)nranks, extra = count % (uint64_t)nranks;
  const uint64_t r = (uint64_t)std::max(0, std::min(rank, nranks - 1));
  if (shard_start) *shard_start = start + r * base + std::min(r, extra);
  if (shard_count) *shard_count = base + (r < extra ? 1 : 0);
}

int pow_group_unique_id(uint8_t id[POW_GROUP_ID_BYTES]) {
  if (!id) return pow_set_error(POW_EINVAL, "null id");
  const Rccl& R = rccl();
  if (R.why[0]) return pow_set_error(POW_ECOMM, R.why);
  ncclUniqueId u;
  static_assert(sizeof(u) == POW_GROUP_ID_BYTES, "ncclUniqueId size");
  ncclResult_t r = R.get_unique_id(&u);
  if (r != ncclSuccess) return comm_fail("ncclGetUniqueId", r);
  memcpy(id, &u, sizeof u);
  return POW_OK;
}

int pow_group_init(pow_ctx* ctx, int nranks, int rank, const uint8_t id[POW_GROUP_ID_BYTES],
                   pow_group** out) {
  return pow_group_init_within(ctx, nranks, rank, id, kInitTimeoutMs, out);
}

int pow_group_init_within(pow_ctx* ctx, int nranks, int rank, const uint8_t id[POW_GROUP_ID_BYTES],
                          unsigned timeout_ms, pow_group** out) {
  if (!out) return pow_set_error(POW_EINVAL, "null out");
  *out = nullptr;
  if (!ctx || !id) return pow_set_error(POW_EINVAL, "null ctx/id");
  if (nranks < 1 || rank < 0 || rank >= nranks) return pow_set_error(POW_EINVAL, "bad rank/nranks");
  if (timeout_ms == 0) return pow_set_error(POW_EINVAL, "timeout_ms = 0");
  const Rccl& R = rccl();
  if (R.why[0]) return pow_set_error(POW_ECOMM, R.why);
  hipError_t e = hipSetDevice(pow_ctx_device(ctx));
  if (e != hipSuccess) return hip_fail("hipSetDevice", e);
  pow_group* g = new pow_group;
  g->ctx = ctx;
  g->nranks = nranks;
  g->rank = rank;
  if ((e = hipMalloc(&g->d_buf, kMaxWords * 8)) != hipSuccess ||
      (e = hipHostMalloc(&g->h_buf, kMaxWords * 8, hipHostMallocDefault)) != hipSuccess) {
    pow_group_destroy(g);
    return hip_fail("group buffers", e);
  }
  // The node's stop board: opened before the communicator, so that once
  // the communicator is up (every rank joined) every rank has it mapped and
  // its name can go.  Without one (> 64 ranks, no shared memory) the ranks
  // still stop together at the end of each round.
  char name[40];
  board_name(id, name);
  if (nranks <= POW_BOARD_MAX_SLOTS && pow_board_open(name, nranks, &g->board) != POW_OK) g->board = nullptr;
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  // Init under a deadline: ncclCommInitRank would wait for every rank with
  // no bound, so one rank that fails before it joins (a GPU set-up error, a
  // wrong device map, an exception) would hang the other N - 1 forever.  Here
  // they give up after timeout_ms and report who waited for how long.  The
  // init runs on a helper thread (InitJob: RCCL may block in the call whatever
  // the config says), with a non-blocking config.
  auto job = std::make_shared<InitJob>();
  job->cfg.blocking = 0;
  job->id = u;
  job->nranks = nranks;
  job->rank = rank;
  job->device = pow_ctx_device(ctx);
  const uint64_t t0 = now_ns(), budget = (uint64_t)timeout_ms * 1000000ull;
  std::thread(run_init, job).detach();
  bool late = false;
  while (job->state.load(std::memory_order_acquire) == 0 && !late) {
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    late = now_ns() > t0 + budget;
  }
  int running = 0;
  if (late && job->state.compare_exchange_strong(running, 2, std::memory_order_acq_rel)) {
    pow_board_unlink(name);
    char buf[480];
    snprintf(buf, sizeof buf,
             "ncclCommInitRankConfig: rank %d of %d on HIP device %d: not every rank joined within %.3f s "
             "(elapsed %.3f s); the call is left to a helper thread, which aborts the communicator if it ever "
             "returns",
             rank, nranks, pow_ctx_device(ctx), budget * 1e-9, (now_ns() - t0) * 1e-9);
    pow_group_destroy(g);
    return pow_set_error(POW_ECOMM, buf);
  }
  g->comm = job->comm;
  const ncclResult_t r = job->r;
  pow_board_unlink(name);
  if (r != ncclSuccess) {
    char buf[480];
    snprintf(buf, sizeof buf,
             "ncclCommInitRankConfig: rank %d of %d on HIP device %d: %s (after %.3f s); communicator aborted", rank,
             nranks, pow_ctx_device(ctx), R.error_string(r), (now_ns() - t0) * 1e-9);
    g->comm = nullptr;
    pow_group_destroy(g);
    return pow_set_error(POW_ECOMM, buf);
  }
  *out = g;
  return POW_OK;
}

int pow_group_init_custom(pow_ctx* ctx, int nranks, int rank, pow_group_reduce_fn reduce, void* user,
                          const char* board_name, pow_group** out) {
  if (!out) return pow_set_error(POW_EINVAL, "null out");
  *out = nullptr;
  if (!reduce) return pow_set_error(POW_EINVAL, "null reduction");
  if (nranks < 1 || rank < 0 || rank >= nranks) return pow_set_error(POW_EINVAL, "bad rank/nranks");
  pow_group* g = new pow_group;
  g->ctx = ctx;
  g->nranks = nranks;
  g->rank = rank;
  g->reduce = reduce;
  g->reduce_user = user;
  // As pow_group_init: every rank opens the board before the first
  // collective, which doubles as the barrier after which the name can go.
  if (board_name && ctx && nranks <= POW_BOARD_MAX_SLOTS && pow_board_open(board_name, nranks, &g->board) != POW_OK)
    g->board = nullptr;
  uint64_t joined = 1;
  const int rc = group_allreduce(g, &joined, 1, POW_REDUCE_SUM);
  if (board_name && ctx) pow_board_unlink(board_name);
  if (rc != POW_OK || joined != (uint64_t)nranks) {
    pow_group_destroy(g);
    if (rc != POW_OK) return rc;
    char msg[128];
    snprintf(msg, sizeof msg, "%llu ranks joined a group of %d", (unsigned long long)joined, nranks);
    return pow_set_error(POW_ECOMM, msg);
  }
  *out = g;
  return POW_OK;
}

void pow_group_destroy(pow_group* g) {
  if (!g) return;
  if (g->ctx) {
    (void)hipSetDevice(pow_ctx_device(g->ctx));
    pow_board_bind(g->ctx, nullptr, 0, 0);
  }
  if (g->comm) {
    if (g->broken)
      (void)abort_bounded(g->comm, kAbortGraceMs);
    else
      (void)rccl().comm_destroy(g->comm);
  }
  pow_board_close(g->board);
  // hipFree waits for the whole device: after a failed collective (or a stuck
  // launch of the ctx) free the staging buffers only once a bounded wait saw
  // the ctx's stream drain, and leak them otherwise, as pow_destroy does.
  bool drained = true;
  if (g->ctx && (g->d_buf || g->h_buf) && (g->broken || pow_ctx_wedged(g->ctx)))
    drained = pow_ctx_stream_wait(g->ctx, "pow_group_destroy", 0) == POW_OK;
  if (drained) {
    if (g->d_buf) (void)hipFree(g->d_buf);
    if (g->h_buf) (void)hipHostFree(g->h_buf);
  }
  delete g;
}

int pow_group_rccl_path(char* path, size_t cap) {
  if (!path || !cap) return pow_set_error(POW_EINVAL, "null path");
  path[0] = 0;
  const Rccl& R = rccl();
  if (R.why[0]) return pow_set_error(POW_ECOMM, R.why);
  snprintf(path, cap, "%s", R.path);
  return POW_OK;
}

int pow_group_info(const pow_group* g, int* comm_count, int* comm_device) {
  if (!g) return pow_set_error(POW_EINVAL, "null group");
  int n = g->nranks, dev = g->ctx ? pow_ctx_device(g->ctx) : -1;
  if (g->comm) {  // RCCL's own view of the communicator
    ncclResult_t r = rccl().comm_count(g->comm, &n);
    if (r != ncclSuccess) return comm_fail("ncclCommCount", r);
    if ((r = rccl().comm_cu_device(g->comm, &dev)) != ncclSuccess) return comm_fail("ncclCommCuDevice", r);
  }
  if (comm_count) *comm_count = n;
  if (comm_device) *comm_device = dev;
  return POW_OK;
}

int pow_group_last_search(const pow_group* g, pow_group_search_info* out) {
  if (!g || !out) return pow_set_error(POW_EINVAL, "null");
  *out = g->last;
  out->board_open = g->board != nullptr;
  return POW_OK;
}

int pow_group_allreduce_u64(pow_group* g, uint64_t* vals, size_t n, int op) {
  if (!g || (n && !vals)) return pow_set_error(POW_EINVAL, "null");
  if (n > kMaxWords) return pow_set_error(POW_EINVAL, "at most 8 words per all-reduce");
  if (op != POW_REDUCE_MIN && op != POW_REDUCE_MAX && op != POW_REDUCE_SUM)
    return pow_set_error(POW_EINVAL, "unknown reduction");
  if (n == 0) return POW_OK;
  return group_allreduce(g, vals, n, op);
}

int pow_group_mine(pow_group* g, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
                   uint64_t round_size, unsigned diff_bits, const volatile uint32_t* cancel_word,
                   uint32_t epoch, pow_block* out, uint64_t* found_ctr, uint64_t* hashes_done) {
  if (int rc = check_args(g, tmpl, out, ctr_start, ctr_count, diff_bits)) return rc;
  // Default (round_size = 0): adaptive rounds, as pow_mine's sub-rounds.  The
  // first round covers ~4x the expected trials (2^(d+2) counters, at least
  // 2^16 per GPU), later ones grow 4x up to 2^30 counters per GPU (~0.13 s at
  // 8 G/s, where the one all-reduce per round costs well under 1%).  A fixed
  // 2^30 per GPU would make every search take ~0.13 s per round even when the
  // lowest solution sits in the first milliseconds of rank 0's shard.
  const uint64_t big = (uint64_t)g->nranks << 30;
  const bool adaptive = round_size == 0;
  if (adaptive) {
    const unsigned dcap = diff_bits > 40 ? 40 : diff_bits;
    round_size = std::min<uint64_t>(big, std::max<uint64_t>((uint64_t)g->nranks << 16, 1ull << (dcap + 2)));
  }
  return group_search(g, tmpl, ctr_start, ctr_count, round_size, adaptive, diff_bits, cancel_word, epoch, out,
                      found_ctr, hashes_done, false);
}

int pow_group_mine_any(pow_group* g, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
                       uint64_t round_size, unsigned diff_bits, const volatile uint32_t* cancel_word,
                       uint32_t epoch, pow_block* out, uint64_t* found_ctr, uint64_t* hashes_done) {
  if (int rc = check_args(g, tmpl, out, ctr_start, ctr_count, diff_bits)) return rc;
  // Any-mode needs no growing rounds: pow_mine_any starts each shard with its
  // latency kernel and a hit anywhere on the node stops every GPU through the
  // board.  2^32 counters per rank per round (~0.5 s) keep the all-reduce,
  // which also carries cancellation across nodes, rare.
  if (round_size == 0) round_size = (uint64_t)g->nranks << 32;
  return group_search(g, tmpl, ctr_start, ctr_count, round_size, false, diff_bits, cancel_word, epoch, out,
                      found_ctr, hashes_done, true);
}

}  // extern "C"
