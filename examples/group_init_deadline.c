/*
 * The N > 1 start-up failure, from C: this process is rank 0 of a 2-rank
 * group whose rank 1 never calls pow_group_init (a rank that died during GPU
 * set-up, say).  The reference would wait forever, as its ranks do in
 * MPI_Recv (node.cpp:155-161); pow_group_init must instead return POW_ECOMM
 * once its deadline passes (pow_group_init_within's timeout), with the rank, the
 * group size, the device and the time waited in pow_last_error(), and leave
 * the context usable: a one-rank group on it then forms, all-reduces and mines
 * S0 at d = 21 to its lowest solving counter, 2392323
 * (tests/golden/fingerprints_2p32.json).
 *
 *   group_init_deadline [timeout_ms]     (default 3000)
 *
 * Linked against libpow_gpu.so it exercises RCCL itself (ncclCommInitRankConfig
 * in non-blocking mode, ncclCommAbort of a communicator still initialising);
 * against libpow_gpu_test.so with POW_TEST_RCCL_LIB the stand-in of
 * tests/stub_rccl.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pow_gpu.h"

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static int fail(const char* what) {
  fprintf(stderr, "FAIL %s: %s\n", what, pow_last_error());
  return 1;
}

int main(int argc, char** argv) {
  const long ms = argc > 1 ? atol(argv[1]) : 3000;
  setvbuf(stdout, NULL, _IONBF, 0);  /* every line out at once: a run killed by its time limit still shows its stage */
  pow_ctx* ctx = NULL;
  if (pow_init(0, &ctx) != POW_OK) return fail("pow_init");
  printf("stage: joining a 2-rank group alone (deadline %ld ms)\n", ms);

  uint8_t id[POW_GROUP_ID_BYTES];
  if (pow_group_unique_id(id) != POW_OK) return fail("pow_group_unique_id");
  pow_group* g = NULL;
  const double t0 = now_s();
  const int rc = pow_group_init_within(ctx, 2, 0, id, (unsigned)ms, &g);
  const double dt = now_s() - t0;
  printf("lonely rank 0 of 2: rc %d after %.3f s: %s\n", rc, dt, pow_last_error());
  if (rc != POW_ECOMM || g != NULL) return fail("expected POW_ECOMM and no group");
  if (dt < 0.9 * ms / 1e3 || dt > ms / 1e3 + 10.0) return fail("returned outside its deadline");
  if (!strstr(pow_last_error(), "rank 0 of 2") || !strstr(pow_last_error(), "not every rank joined"))
    return fail("error text");

  /* the context is still good: a one-rank group forms, all-reduces and mines */
  printf("stage: one-rank group\n");
  if (pow_group_unique_id(id) != POW_OK) return fail("pow_group_unique_id (2)");
  if (pow_group_init(ctx, 1, 0, id, &g) != POW_OK) return fail("pow_group_init (1 rank)");
  uint64_t v[2] = {5, 7};
  if (pow_group_allreduce_u64(g, v, 2, POW_REDUCE_MIN) != POW_OK || v[0] != 5 || v[1] != 7)
    return fail("pow_group_allreduce_u64");
  pow_block t, out;
  memset(&t, 0, sizeof t);
  t.index = 1;
  t.difficulty = 9;
  t.created_at = 1700000000u;
  uint64_t ctr = 0, hashes = 0;
  if (pow_group_mine(g, &t, 0, 1ull << 32, 0, 21, NULL, 0, &out, &ctr, &hashes) != 1 || ctr != 2392323u)
    return fail("pow_group_mine");
  pow_group_search_info info;
  if (pow_group_last_search(g, &info) != POW_OK || info.rounds < 1 || !info.local_found || !info.mine_end_ns)
    return fail("pow_group_last_search");
  printf("one-rank group: counter %llu, %u rounds, board %d/%d, mine %.3f ms, all-reduce %.3f ms\n",
         (unsigned long long)ctr, info.rounds, info.board_open, info.board_bound, info.mine_ms, info.allreduce_ms);
  printf("stage: destroy\n");
  pow_group_destroy(g);
  pow_destroy(ctx);
  printf("ok\n");
  return 0;
}
