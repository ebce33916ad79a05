/* Time-to-block through the C ABI (what pow_node sees): pow_mine_any over
 * 201 random templates at difficulty d, median and 10th/90th percentile.
 *   gcc -O2 -I include tools/ttb_c.c -L mpi_blockchain_amd -lpow_gpu -o tools/ttb_c && tools/ttb_c 9 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pow_gpu.h"

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}
static int cmp(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char** argv) {
  const unsigned d = argc > 1 ? (unsigned)atoi(argv[1]) : 9;
  pow_ctx* ctx;
  if (pow_init(0, &ctx) || pow_warmup(ctx)) {
    fprintf(stderr, "%s\n", pow_last_error());
    return 1;
  }
  srand(1);
  double t[201];
  for (int k = 0; k < 201; ++k) {
    pow_block b, out;
    memset(&b, 0, sizeof b);
    b.index = 1 + rand() % 65535;
    b.difficulty = 9;
    b.created_at = 1700000000 + rand() % 256;
    for (int i = 0; i < 64; ++i) b.previous_block_hash[i] = "0123456789abcdef"[rand() % 16];
    uint64_t ctr = 0;
    const double t0 = now();
    const int rc = pow_mine_any(ctx, &b, 0, 1ull << 42, d, NULL, 0, &out, &ctr, NULL);
    t[k] = now() - t0;
    if (rc != 1) {
      fprintf(stderr, "rc %d\n", rc);
      return 1;
    }
  }
  qsort(t, 201, sizeof(double), cmp);
  printf("{\"d\": %u, \"ttb_ms_median\": %.4f, \"p10\": %.4f, \"p90\": %.4f}\n", d, 1e3 * t[100], 1e3 * t[20],
         1e3 * t[180]);
  pow_destroy(ctx);
  return 0;
}
