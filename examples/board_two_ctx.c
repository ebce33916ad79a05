/* Two GPU contexts of one search, stopped by the cross-GPU stop board
 * (include/pow_gpu.h, pow_board_*), from plain C with one host thread per
 * context — the shape of a single-process multi-GPU miner.
 *
 * Thread B mines a range with no solution (difficulty 64); once its kernel
 * runs, thread A mines S0 at difficulty 9 from counter 0 and finds one within
 * microseconds.  A's kernel stores the hit into its board slot, B's running
 * kernel sees it at its next poll and B's call returns 0.  Prints how long B
 * ran after A returned.  Exit status 0 iff B stopped early and A's block
 * solves.  Used by tools/host_sanitize.sh (ASan/UBSan and TSan runs).
 *
 * On one GPU the two contexts share the chip, so the test run links the test
 * build (libpow_gpu_test.so), whose POW_GRID_PER_CU switch sizes B's grid to
 * half the workgroup slots; across two GPUs the shipped library needs none:
 *   cc -I include examples/board_two_ctx.c -L mpi_blockchain_amd -lpow_gpu_test -lpthread
 *   POW_GRID_PER_CU=4 ./a.out
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pow_gpu.h"

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

struct job {
  pow_ctx* ctx;
  pow_block tmpl;
  uint64_t start, count;
  unsigned diff;
  int rc;
  uint64_t ctr, hashes;
  double t_end;
  pow_block out;
};

static void* run(void* p) {
  struct job* j = (struct job*)p;
  j->rc = pow_mine_any(j->ctx, &j->tmpl, j->start, j->count, j->diff, NULL, 0, &j->out, &j->ctr, &j->hashes);
  j->t_end = now_s();
  return NULL;
}

int main(void) {
  pow_block s0;
  memset(&s0, 0, sizeof s0);
  s0.index = 1;
  s0.difficulty = 9;
  s0.created_at = 1700000000ull;
  pow_board* board = NULL;
  pow_ctx *a = NULL, *b = NULL;
  if (pow_board_open(NULL, 2, &board) != POW_OK || pow_init(0, &a) != POW_OK || pow_init(0, &b) != POW_OK ||
      pow_warmup(a) != POW_OK || pow_warmup(b) != POW_OK || pow_board_bind(a, board, 0, 5) != POW_OK ||
      pow_board_bind(b, board, 1, 5) != POW_OK) {
    fprintf(stderr, "set-up: %s\n", pow_last_error());
    return 1;
  }
  struct job jb = {b, s0, 1ull << 33, 1ull << 32, 64, 0, 0, 0, 0.0, {0}};
  struct job ja = {a, s0, 0, 1u << 20, 9, 0, 0, 0, 0.0, {0}};
  pthread_t tb, ta;
  const double t0 = now_s();
  pthread_create(&tb, NULL, run, &jb);
  struct timespec nap = {0, 150 * 1000 * 1000};  /* B's kernel is running */
  nanosleep(&nap, NULL);
  pthread_create(&ta, NULL, run, &ja);
  pthread_join(ta, NULL);
  pthread_join(tb, NULL);
  char hex[65];
  memcpy(hex, ja.out.block_hash, 64);
  hex[64] = 0;
  const int solves = ja.rc == 1 && pow_solves_problem(hex, 9);
  uint64_t seen = 0;
  pow_board_peek(board, 1, 5, &seen);
  printf("A: rc %d counter %llu hash %s; B: rc %d after %.3f s, stopped %.3f ms after A returned, %llu trials;"
         " board slot 0 = %llu\n",
         ja.rc, (unsigned long long)ja.ctr, hex, jb.rc, jb.t_end - t0, 1e3 * (jb.t_end - ja.t_end),
         (unsigned long long)jb.hashes, (unsigned long long)seen);
  pow_board_bind(a, NULL, 0, 0);
  pow_board_bind(b, NULL, 0, 0);
  pow_destroy(a);
  pow_destroy(b);
  pow_board_close(board);
  return solves && jb.rc == 0 && jb.t_end - ja.t_end < 0.005 ? 0 : 1;
}
