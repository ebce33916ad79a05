/*
 * pow_gpu.h — C ABI of the MI355X (gfx950) proof-of-work miner.
 *
 * Drop-in for the mining hot path of MPI_blockchain (reference at
 * /root/reference): the inner loop of proof_of_work (node.cpp:292-308),
 *     gen_random_nonce (block.cpp:61-72)
 *  -> block_to_hash    (block.cpp:74-88, picosha2::hash256_hex_string)
 *  -> solves_problem   (block.cpp:91-96)
 * moves behind these entry points.  Everything else (node.cpp's MPI protocol,
 * the success tail node.cpp:311-327) stays host C/C++.
 *
 * The reference has no FFI for this path; its de-facto boundary is the
 * free-function set declared in block.h:27-30 and called from the pthread
 * entry `void* proof_of_work(void*)` (node.h:15).  Each entry point below says
 * which of those it replaces.
 *
 * Conventions
 *   - Plain C: pointers and sizes only, no exceptions across the ABI.
 *   - Return codes: >= 0 success (meaning per function), < 0 error, one of
 *     POW_E* below (HIP failures are reported as POW_EHIP; pow_last_error()
 *     gives the text).
 *   - A pow_ctx is bound to one GPU and is NOT thread-safe: exactly one
 *     thread (that rank's mining thread) drives it.  The only cross-thread
 *     inputs are the cancel word passed to pow_mine, which any thread may
 *     bump, and pow_cancel (one other thread).
 *   - The caller owns every pow_block and output array; the library owns the
 *     device buffers, the HIP stream and the per-template constants.
 *
 * Counter nonces.  The reference draws 9 chars with rand()%62 (block.cpp:61-72).
 * The GPU path replaces the RNG by a deterministic counter: counter c maps to
 * the 9 base-62 digits of c, most significant first, through the reference's
 * alphabet (0-25 -> 'a'..'z', 26-51 -> 'A'..'Z', 52-61 -> '0'..'9'), followed
 * by NUL.  The counter space is [0, 62^9).  Any nonce the reference can draw
 * is reachable, with the same probability of solving per trial.
 */
#ifndef POW_GPU_H
#define POW_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define POW_HASH_SIZE 256  /* block.h:4 HASH_SIZE  */
#define POW_NONCE_SIZE 10  /* block.h:5 NONCE_SIZE */
#define POW_MSG_BYTES 270  /* 4 header bytes + nonce[10] + prev[256] (block.cpp:79-88) */
#define POW_COUNTER_LIMIT 13537086546263552ULL /* 62^9 */

/* Byte-identical to the reference's `struct Block` (block.h:17-25) on LP64:
 * sizeof 552; offsets index 0, node_owner_number 4, difficulty 8,
 * created_at 16, nonce 24, previous_block_hash 34, block_hash 290.
 * A reference Block* may be passed wherever a pow_block* is expected. */
typedef struct pow_block {
  uint32_t index;
  uint32_t node_owner_number;
  uint32_t difficulty;
  uint64_t created_at; /* `unsigned long int` in block.h:21 */
  char nonce[POW_NONCE_SIZE];
  char previous_block_hash[POW_HASH_SIZE];
  char block_hash[POW_HASH_SIZE];
} pow_block;

typedef struct pow_ctx pow_ctx;

enum {
  POW_OK = 0,
  POW_EINVAL = -1,    /* bad argument (null pointer, range past 62^9, d > 256, ...) */
  POW_ENOSPC = -2,    /* pow_sweep: more solutions than `cap` */
  POW_EHIP = -3,      /* a HIP runtime call failed; see pow_last_error() */
  POW_ENODEV = -4,    /* no such GPU */
  POW_ECOMM = -5,     /* RCCL unavailable or a collective failed (pow_group_*) */
};

/* Per-call statistics of the last pow_mine / pow_sweep / pow_hash_blocks. */
typedef struct pow_stats {
  double kernel_ms;      /* sum of kernel durations on the ctx stream: HIP events around the
                            sweep/mine kernels; the latency kernel (first sub-round of
                            pow_mine[_any] at d <= 21) times itself with the GPU's realtime
                            counter, from workgroup 0's start to the last workgroup's exit */
  uint32_t launches;     /* kernels launched by the call */
  uint64_t hashes;       /* trials issued to the GPU (incl. edge lanes masked out) */
} pow_stats;

/* ---- context --------------------------------------------------------- */
/* Number of visible GPUs (HIP devices). */
int pow_device_count(int* n);
int pow_init(int device, pow_ctx** out);
void pow_destroy(pow_ctx* ctx);
/* Launch every kernel once with empty work so the code objects are loaded and
 * the first real call pays no start-up cost (HIP loads them lazily). */
int pow_warmup(pow_ctx* ctx);
const char* pow_last_error(void);
int pow_get_stats(const pow_ctx* ctx, pow_stats* out);
/* How the context launches its latency-bound kernels (the one-block hash of
 * pow_hash_block and the first sub-round of pow_mine[_any]):
 * POW_LAUNCH_HIP = hipLaunchKernel on the context's stream, the shipped
 * library's only path; POW_LAUNCH_DIRECT = AQL packets into the process's
 * shared per-device queue (no barrier bit; the test library with POW_AQL=1,
 * for the dispatch A/B and the ordering tests).  Same kernels, same results.
 * Every host wait on a launch is bounded (watchdog): a launch that has not
 * published its result by its deadline (10 s for the latency launches,
 * 10 s + 2 ns per counter for a throughput launch) fails the call with
 * POW_EHIP and a diagnostic in pow_last_error(); the context must then not be
 * reused.  < 0 = error. */
enum { POW_LAUNCH_HIP = 0, POW_LAUNCH_DIRECT = 1 };
int pow_launch_path(const pow_ctx* ctx);
/* Device properties the roofline uses: CU count and peak engine clock (kHz). */
int pow_device_info(const pow_ctx* ctx, int* cu_count, int* clock_khz, char* name, size_t name_cap);
/* The ctx's GPU as "domain:bus:device.function" (hipDeviceGetPCIBusId): the
 * N > 1 bench's check that its ranks run on N distinct devices (partitions of
 * one GPU differ in the function). */
int pow_device_pci_bus_id(const pow_ctx* ctx, char* out, size_t cap);

/* ---- host helpers (no GPU work) ---------------------------------------- */
/* Counter -> nonce[10] (9 base-62 chars MSB first + NUL).
 * Replaces gen_random_nonce (block.cpp:61-72) with a deterministic mapping.
 * Returns POW_EINVAL if ctr >= 62^9. */
int pow_nonce_from_counter(uint64_t ctr, char nonce[POW_NONCE_SIZE]);
/* Exact 270-byte message the reference hashes (block_to_str, block.cpp:79-88):
 * low byte of index, owner, difficulty, created_at; nonce[0..9]; prev[0..255]. */
int pow_block_to_bytes(const pow_block* b, uint8_t out[POW_MSG_BYTES]);
/* solves_problem (block.cpp:91-96) with a run-time difficulty: the first
 * `diff_bits` binary digits of the 64-char hex digest are all '0'. */
int pow_solves_problem(const char* hex, unsigned diff_bits);

/* ---- GPU entry points -------------------------------------------------- */
/* block_to_hash (block.cpp:74-77) for a batch of blocks on the GPU.
 * digests: n*32 bytes (may be NULL); hex: n*65 chars, 64 lowercase hex + NUL
 * each (may be NULL).  Returns POW_OK. */
int pow_hash_blocks(pow_ctx* ctx, const pow_block* blocks, size_t n,
                    uint8_t* digests, char* hex);
/* Single-block form of the above (validation of a received block: valid_new_block,
 * block.cpp:13-25).  One block (also pow_hash_blocks with n = 1) takes the
 * low-latency path: the message travels as a kernel argument and the digest comes
 * back through mapped host memory, no copies (~24 us per call on an MI355X). */
int pow_hash_block(pow_ctx* ctx, const pow_block* b, uint8_t digest[32], char hex[65]);

/* Mining round: replaces node.cpp:302-308 (nonce -> hash -> test) for every
 * counter in [ctr_start, ctr_start + ctr_count).  The header fields and the
 * 256-byte previous_block_hash are taken from `tmpl` as they are (the caller
 * does the template refresh of node.cpp:292-299).
 *   diff_bits     leading zero BITS required (T3), 0..256.
 *   cancel_word   optional; polled between GPU sub-rounds; if it differs from
 *                 `epoch` the call stops early and returns 0.
 * On success returns 1 and fills *out = *tmpl with out->nonce = the nonce of
 * the LOWEST solving counter in range and out->block_hash = its 64-char hex
 * digest + NUL (strcpy semantics of node.cpp:318: bytes 65..255 keep tmpl's);
 * *found_ctr = that counter.  Returns 0 if the range holds no solution or the
 * call was cancelled.  *hashes_done (optional) = trials issued.
 * pow_mine and pow_mine_any return as soon as the GPU has published the
 * result; the ctx's stream may still be retiring the launch's last
 * workgroup for a few microseconds (nothing it does then touches the result,
 * the cancel word or a board, so unbinding or closing a board right away is
 * safe).  The next launch on the ctx and pow_destroy are ordered behind it. */
int pow_mine(pow_ctx* ctx, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
             unsigned diff_bits, const volatile uint32_t* cancel_word, uint32_t epoch,
             pow_block* out, uint64_t* found_ctr, uint64_t* hashes_done);

/* In-flight cancellation (the reference re-checks its chain only after a
 * trial, node.cpp:315).  Publishes `epoch`, the caller's current value of the
 * cancel word, to the GPU: a pow_mine / pow_mine_any launch of this ctx whose
 * `epoch` argument differs stops at its next poll (one inner step, ~60 us)
 * instead of at its sub-round boundary (up to ~0.13 s), and the call returns 0.
 * Call it after bumping the cancel word, with its new value, from one thread
 * at a time.  It is a store into host memory the GPU reads (no HIP call), so
 * the thread driving the ctx may be inside pow_mine meanwhile.  The first
 * call arms the GPU-side check for the ctx.  Returns POW_OK. */
int pow_cancel(pow_ctx* ctx, uint32_t epoch);

/* Lowest-latency form of pow_mine: returns (1) SOME solving counter of the
 * range — the first one the GPU finds; every wave stops at its next step —
 * instead of the lowest.  Same arguments, outputs and return codes.  Not
 * deterministic (like the reference's rand() nonces, node.cpp:302); use it
 * where only time-to-block matters (the protocol node, the difficulty ladder). */
int pow_mine_any(pow_ctx* ctx, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
                 unsigned diff_bits, const volatile uint32_t* cancel_word, uint32_t epoch,
                 pow_block* out, uint64_t* found_ctr, uint64_t* hashes_done);

/* Deterministic parity / throughput mode: every solving counter of
 * [ctr_start, ctr_start + ctr_count) (ctr_count <= 2^32), written to out_ctrs
 * as (counter - ctr_start), ascending.  *n_found = number of solutions
 * (also when it exceeds cap, in which case POW_ENOSPC is returned and the
 * first `cap` entries are an unspecified subset).  out_ctrs may be NULL when
 * cap == 0 (count only).  cap <= 2^31 - 1 (the list is sorted on the device;
 * POW_EINVAL above).  Returns POW_OK. */
int pow_sweep(pow_ctx* ctx, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
              unsigned diff_bits, uint32_t* out_ctrs, size_t cap, size_t* n_found);

/* Sweep variant that leaves the (unsorted) solution list on the device and
 * returns only the count and the lowest solving counter (UINT64_MAX if none):
 * the shape a sharded multi-GPU round needs (the 8-byte min goes to an RCCL
 * all-reduce).  dev_out may be NULL (count + min only). */
int pow_sweep_device(pow_ctx* ctx, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
                     unsigned diff_bits, uint32_t* dev_out, size_t cap, size_t* n_found,
                     uint64_t* min_ctr);

/* Device memory on the ctx's GPU (for pow_sweep_device's dev_out). */
int pow_dev_alloc(pow_ctx* ctx, size_t bytes, void** out);
int pow_dev_free(pow_ctx* ctx, void* p);
/* Copy `bytes` from a device pointer to host memory (synchronous). */
int pow_dev_read(pow_ctx* ctx, const void* dev, void* host, size_t bytes);

/* ---- cross-GPU stop board (one node) ------------------------------------ */
/* The reference's ranks hear of a rival's block only through MPI, between
 * trials (node.cpp:315, 404).  When several GPUs search ONE template together
 * (pow_group_*, BASELINE config 4), the finder must stop the others inside
 * their running launches: a collective only runs between kernels.  A board is
 * a page of host memory every GPU of the node maps, one 64-bit slot per rank.
 * A context bound to slot s of a board, for the search tagged `tag`:
 *   - stores every hit of its pow_mine / pow_mine_any launches into slot s,
 *     from the kernel itself (system-scope store over PCIe);
 *   - stops, within one inner step, as soon as another slot holds a solution
 *     of the same tag that makes its remaining counters moot: in
 *     pow_mine_any any peer solution; in pow_mine a peer solution below the
 *     counters it would still compute (the lowest-counter result stays exact:
 *     counters below the peer's are always finished).
 * Such a call then returns 0 (the peer's result wins the caller's
 * reduction).  In pow_mine that includes a call that found a solution while a
 * peer already holds a lower one: the call's own counter is then not the
 * search's answer, and not necessarily the lowest of its own range (its waves
 * above the peer's counter may have stopped), so it is not reported.  A 1 from
 * a bound pow_mine is the lowest solution of its range; the search's answer is
 * the minimum over the ranks' results (pow_group_* reduce it for you).
 * pow_group_* use a board automatically; these entry points are for callers
 * that drive several contexts themselves. */
#define POW_BOARD_MAX_SLOTS 64
#define POW_BOARD_MAX_TAG 1023
typedef struct pow_board pow_board;
/* name NULL: memory private to this process (contexts of one process, one
 * host thread per GPU).  name "/x": POSIX shared memory shared by every
 * process of the node that opens the same name (one process per GPU); it is
 * created zeroed if absent.  nslots 1..64.  Opening, posting and peeking
 * need no GPU; the first pow_board_bind maps the page for the GPUs. */
int pow_board_open(const char* name, int nslots, pow_board** out);
/* Remove a named board's name (processes that opened it keep their mapping). */
int pow_board_unlink(const char* name);
/* Unbind every context from the board first. */
void pow_board_close(pow_board* b);
/* Bind ctx to `slot` for the search tagged `tag` (1..1023; use a new tag per
 * search so stale slots are ignored) and mark the slot "nothing found yet";
 * b = NULL unbinds.  The ctx's launches watch and feed the board until
 * unbound. */
int pow_board_bind(pow_ctx* ctx, pow_board* b, int slot, uint32_t tag);
/* Host-side view: publish `ctr` in `slot` for `tag`; lowest counter any other
 * slot holds for `tag` (UINT64_MAX = none). */
int pow_board_post(pow_board* b, int slot, uint32_t tag, uint64_t ctr);
int pow_board_peek(const pow_board* b, int except_slot, uint32_t tag, uint64_t* min_ctr);

/* ---- sharded search over several GPUs (RCCL) --------------------------- */
/* One template mined cooperatively by `nranks` GPUs, one pow_ctx each (one
 * process or host thread per GPU).  The reference has no such mode: its ranks
 * compete, each on its own template (node.cpp:302, 386).  These calls are
 * collective: every rank makes them with the same arguments.  RCCL is loaded
 * on first use (dlopen); without it they return POW_ECOMM. */
#define POW_GROUP_ID_BYTES 128 /* sizeof(ncclUniqueId) */
enum { POW_REDUCE_MIN = 0, POW_REDUCE_MAX = 1, POW_REDUCE_SUM = 2 };
typedef struct pow_group pow_group;

/* Rank `rank`'s contiguous static shard of [start, start + count): shards of
 * ranks 0..nranks-1 are consecutive and differ in size by at most one. */
void pow_group_partition(uint64_t start, uint64_t count, int rank, int nranks,
                         uint64_t* shard_start, uint64_t* shard_count);
/* Rank 0 makes the id; the caller hands it to every rank (MPI_Bcast, a file,
 * torch.distributed ...) before pow_group_init. */
int pow_group_unique_id(uint8_t id[POW_GROUP_ID_BYTES]);
/* Joins the RCCL communicator on ctx's GPU; returns once all ranks joined.
 * Bounded: the communicator is made non-blocking (ncclCommInitRankConfig,
 * config.blocking = 0) and polled (ncclCommGetAsyncError) until every rank
 * joined or 60 s passed; then it is aborted (ncclCommAbort) and POW_ECOMM
 * names the rank, nranks, device and elapsed time.  (The reference's ranks
 * block in MPI_Recv with no bound, node.cpp:155-161.) */
int pow_group_init(pow_ctx* ctx, int nranks, int rank, const uint8_t id[POW_GROUP_ID_BYTES],
                   pow_group** out);
/* pow_group_init with the caller's deadline for every rank to join (ms, > 0). */
int pow_group_init_within(pow_ctx* ctx, int nranks, int rank, const uint8_t id[POW_GROUP_ID_BYTES],
                          unsigned timeout_ms, pow_group** out);
/* The same group over a reduction the caller supplies instead of RCCL: the
 * rounds, the stop board and the {counter, go, ok} consensus of
 * pow_group_mine[_any] are unchanged, only the one all-reduce per round goes
 * through `reduce`.  For ranks that already share a transport (MPI_Allreduce
 * in an MPI job, torch.distributed gloo), and for several ranks on ONE GPU,
 * which RCCL refuses (the multi-process GPU tests).  RCCL stays the
 * collective of one process per GPU (pow_group_init).
 *   reduce(user, vals, n, op): in place over every rank's n <= 8 words with
 *       op = POW_REDUCE_*, collective (every rank calls it in the same order);
 *       returns 0 on success.  Called from the thread that calls pow_group_*.
 *   board_name: "/name" opens that node-local stop board (the same name on
 *       every rank; fresh per group; unlinked once every rank has joined), or
 *       NULL for none.
 *   ctx may be NULL: the group then carries only pow_group_allreduce_u64.
 * Collective: the first reduction (a barrier that also checks nranks) runs
 * inside this call. */
typedef int (*pow_group_reduce_fn)(void* user, uint64_t* vals, size_t n, int op);
int pow_group_init_custom(pow_ctx* ctx, int nranks, int rank, pow_group_reduce_fn reduce, void* user,
                          const char* board_name, pow_group** out);
void pow_group_destroy(pow_group* g);
/* The group as its transport sees it: *comm_count = the ranks in RCCL's
 * communicator (ncclCommCount) and *comm_device = its HIP device
 * (ncclCommCuDevice); for a custom group, nranks (every rank joined) and the
 * ctx's device (-1 without one).  Either pointer may be NULL.  The scaling
 * bench records both per rank to show that N distinct GPUs took part. */
int pow_group_info(const pow_group* g, int* comm_count, int* comm_device);
/* The file of the RCCL library pow_group_* use (loaded at the first call of
 * any pow_group_* that needs RCCL; no GPU work): the copy another library of
 * the process had already loaded (torch's librccl.so) if there is one, else
 * librccl.so.1 from the library search path.  POW_ECOMM if RCCL cannot be
 * loaded. */
int pow_group_rccl_path(char* path, size_t cap);
/* In-place all-reduce of n <= 8 uint64 words (POW_REDUCE_*), on ctx's stream.
 * A collective that fails or passes its deadline leaves the group broken:
 * every later collective of it returns POW_ECOMM at once (destroy it). */
int pow_group_allreduce_u64(pow_group* g, uint64_t* vals, size_t n, int op);
/* What this rank did in the group's last pow_group_mine[_any] call (no GPU
 * work, no collective): the N > 1 bench's record of whether the stop board
 * worked (a missing board shows as peers that run out their shards: a large
 * spread between the finder's and the last peer's mine_end_ns). */
typedef struct pow_group_search_info {
  int board_open;        /* the group has the node's stop board (pow_group_init opened it) */
  int board_bound;       /* the last search ran with this rank's context bound to it */
  uint32_t rounds;       /* rounds of the last search (one all-reduce each) */
  int local_found;       /* this rank's own launch found a solution in the last round */
  uint64_t mine_end_ns;  /* CLOCK_MONOTONIC when that launch returned (0: none ran) */
  double mine_ms;        /* wall ms in this rank's own launches, all rounds */
  double allreduce_ms;   /* wall ms in the rounds' all-reduces, waiting for peers included */
} pow_group_search_info;
int pow_group_last_search(const pow_group* g, pow_group_search_info* out);
/* On one node the ranks also share a stop board (named after the id, opened
 * by pow_group_init): a rank's hit stops the other GPUs inside their running
 * launches, not only at the round's all-reduce.
 * pow_mine over all ranks: rounds of `round_size` counters (0 = adaptive:
 * ~4x the expected trials first, then 4x larger up to 2^30 per rank), each
 * split into static shards; each rank mines the lowest solving
 * counter of its shard, then one 24-byte ncclAllReduce(ncclMin) per round
 * picks the winner, spreads cancellation (any rank whose cancel word moved
 * stops every rank: returns 0) and failures (every rank returns < 0).  On 1 the
 * result equals pow_mine's over the whole range on one GPU, on every rank:
 * *out / *found_ctr as pow_mine; *hashes_done = this rank's trials. */
int pow_group_mine(pow_group* g, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
                   uint64_t round_size, unsigned diff_bits, const volatile uint32_t* cancel_word,
                   uint32_t epoch, pow_block* out, uint64_t* found_ctr, uint64_t* hashes_done);
/* pow_mine_any over all ranks (time-to-block: the first solution any GPU
 * finds ends the search on every GPU).  Rounds of `round_size` counters (0 =
 * 2^32 per rank), static shards; the first hit stops the node's other GPUs
 * through the board, and one 24-byte all-reduce(min) per round agrees on the
 * winner: the lowest counter among the solutions the ranks found.  Same
 * outputs and return codes as pow_group_mine, the same result on every rank. */
int pow_group_mine_any(pow_group* g, const pow_block* tmpl, uint64_t ctr_start, uint64_t ctr_count,
                       uint64_t round_size, unsigned diff_bits, const volatile uint32_t* cancel_word,
                       uint32_t epoch, pow_block* out, uint64_t* found_ctr, uint64_t* hashes_done);

#ifdef __cplusplus
}
#endif

#endif /* POW_GPU_H */
