/* K2 latency through the C ABI: median kernel time (pow_get_stats) and call
 * time of pow_hash_block over 200 calls.
 *   gcc -O2 -I include tools/k2_c.c -L mpi_blockchain_amd -lpow_gpu -o tools/k2_c */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pow_gpu.h"

static int cmp(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}
int main(void) {
  pow_ctx* ctx;
  if (pow_init(0, &ctx) || pow_warmup(ctx)) return 1;
  pow_block b;
  memset(&b, 0, sizeof b);
  b.index = 3;
  b.difficulty = 9;
  b.created_at = 1700000000;
  double k[200], w[200];
  for (int i = 0; i < 200; ++i) {
    struct timespec t0, t1;
    char hex[65];
    clock_gettime(CLOCK_MONOTONIC, &t0);
    if (pow_hash_block(ctx, &b, NULL, hex)) return 1;
    clock_gettime(CLOCK_MONOTONIC, &t1);
    pow_stats st;
    pow_get_stats(ctx, &st);
    k[i] = st.kernel_ms * 1e3;
    w[i] = (t1.tv_sec - t0.tv_sec) * 1e6 + (t1.tv_nsec - t0.tv_nsec) * 1e-3;
  }
  qsort(k, 200, sizeof(double), cmp);
  qsort(w, 200, sizeof(double), cmp);
  printf("{\"k2_kernel_us_median\": %.2f, \"call_us_median\": %.2f}\n", k[100], w[100]);
  return 0;
}
