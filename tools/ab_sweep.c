/* A/B timing of kernel variants: each argument is a build of libpow_gpu.so;
 * the libraries are loaded side by side (RTLD_LOCAL) and take turns sweeping
 * S0's first 2^32 counters at d = 9 (BASELINE config 2), `reps` rounds, so
 * clock drift and box-to-box variation hit every variant alike.  Prints one
 * JSON line per variant: median / best kernel ms and G trials/s, and the
 * solution count (must equal 8,393,539 for every variant).
 *
 *   gcc -O2 -I include tools/ab_sweep.c -ldl -o tools/ab_sweep
 *   tools/ab_sweep 5 a/libpow_gpu.so b/libpow_gpu.so
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pow_gpu.h"

typedef int (*init_fn)(int, pow_ctx**);
typedef int (*warm_fn)(pow_ctx*);
typedef int (*sweepd_fn)(pow_ctx*, const pow_block*, uint64_t, uint64_t, unsigned, uint32_t*, size_t, size_t*,
                         uint64_t*);
typedef int (*stats_fn)(const pow_ctx*, pow_stats*);
typedef int (*alloc_fn)(pow_ctx*, size_t, void**);

static int cmp(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s reps lib.so [lib.so ...]\n", argv[0]);
    return 2;
  }
  const int reps = atoi(argv[1]), nv = argc - 2;
  if (reps < 1 || reps > 50 || nv > 8) return 2;
  pow_ctx* ctx[8];
  sweepd_fn sweep[8];
  stats_fn stats[8];
  uint32_t* buf[8];
  double ms[8][50];
  size_t found[8];
  pow_block b;
  memset(&b, 0, sizeof b);
  b.index = 1;
  b.node_owner_number = 0;
  b.difficulty = 9;
  b.created_at = 1700000000;
  const size_t cap = 12000000;
  for (int v = 0; v < nv; ++v) {
    void* h = dlopen(argv[2 + v], RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      fprintf(stderr, "%s\n", dlerror());
      return 1;
    }
    init_fn init = (init_fn)dlsym(h, "pow_init");
    warm_fn warm = (warm_fn)dlsym(h, "pow_warmup");
    alloc_fn alloc = (alloc_fn)dlsym(h, "pow_dev_alloc");
    sweep[v] = (sweepd_fn)dlsym(h, "pow_sweep_device");
    stats[v] = (stats_fn)dlsym(h, "pow_get_stats");
    if (init(0, &ctx[v]) || warm(ctx[v]) || alloc(ctx[v], 4 * cap, (void**)&buf[v])) {
      fprintf(stderr, "init failed for %s\n", argv[2 + v]);
      return 1;
    }
  }
  for (int r = -1; r < reps; ++r) {  /* r = -1: untimed warm-up round */
    for (int v = 0; v < nv; ++v) {
      uint64_t mn = 0;
      if (sweep[v](ctx[v], &b, 0, 1ull << 32, 9, buf[v], cap, &found[v], &mn)) {
        fprintf(stderr, "sweep failed (%s)\n", argv[2 + v]);
        return 1;
      }
      pow_stats st;
      stats[v](ctx[v], &st);
      if (r >= 0) ms[v][r] = st.kernel_ms;
    }
    fprintf(stderr, "round %d done\n", r);
  }
  for (int v = 0; v < nv; ++v) {
    qsort(ms[v], reps, sizeof(double), cmp);
    const double med = ms[v][reps / 2], best = ms[v][0];
    printf("{\"lib\": \"%s\", \"reps\": %d, \"kernel_ms_median\": %.3f, \"kernel_ms_best\": %.3f, "
           "\"gtrials_per_s_median\": %.4f, \"solutions\": %zu, \"count_ok\": %s}\n",
           argv[2 + v], reps, med, best, 4294967296.0 / med / 1e6, found[v],
           found[v] == 8393539 ? "true" : "false");
  }
  return 0;
}
