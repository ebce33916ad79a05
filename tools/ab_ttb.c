/* A/B of time-to-block between builds of libpow_gpu.so (the latency path,
 * kernel K1', for d <= 21): the libraries are loaded side by side and take
 * turns on the same random templates, so box and clock variation hit them
 * alike.  Per library: median / p90 wall time of pow_mine_any, and the kernel
 * rate (sum of trials / sum of HIP-event kernel time over all calls).
 *
 *   gcc -O2 -I include tools/ab_ttb.c -ldl -o tools/ab_ttb
 *   [AB_TTB_LOWEST=1] tools/ab_ttb <d> <templates> a/libpow_gpu.so b/libpow_gpu.so ...  */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pow_gpu.h"

typedef int (*init_fn)(int, pow_ctx**);
typedef int (*warm_fn)(pow_ctx*);
typedef int (*any_fn)(pow_ctx*, const pow_block*, uint64_t, uint64_t, unsigned, volatile const uint32_t*, uint32_t,
                      pow_block*, uint64_t*, uint64_t*);
typedef int (*stats_fn)(const pow_ctx*, pow_stats*);

/* A library argument may carry environment settings for its pow_init:
 * "path@VAR=VAL,VAR=VAL" (the test library's switches).  Sets them;
 * env_clear() unsets them after the context exists. */
static char env_names[8][64];
static int env_n = 0;
static void env_apply(const char* spec) {
  static char buf[512];
  snprintf(buf, sizeof buf, "%s", spec);
  char* at = strchr(buf, '@');
  env_n = 0;
  if (!at) return;
  for (char* kv = strtok(at + 1, ","); kv && env_n < 8; kv = strtok(NULL, ",")) {
    char* eq = strchr(kv, '=');
    if (!eq) continue;
    *eq = 0;
    snprintf(env_names[env_n++], 64, "%s", kv);
    setenv(kv, eq + 1, 1);
  }
}
static void env_clear(void) {
  for (int i = 0; i < env_n; ++i) unsetenv(env_names[i]);
  env_n = 0;
}

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
  if (argc < 4) {
    fprintf(stderr, "usage: %s d templates lib.so [lib.so ...]\n", argv[0]);
    return 2;
  }
  const unsigned d = (unsigned)atoi(argv[1]);
  const int nt = atoi(argv[2]), nv = argc - 3;
  if (nt < 1 || nt > 1001 || nv > 8 || d > 40) return 2;
  pow_ctx* ctx[8];
  any_fn mine[8];
  stats_fn stats[8];
  static double wall[8][1001];
  double kms[8] = {0}, hashes[8] = {0};
  for (int v = 0; v < nv; ++v) {
    char path[512];
    snprintf(path, sizeof path, "%s", argv[3 + v]);
    char* at = strchr(path, '@');
    env_apply(argv[3 + v]);
    if (at) *at = 0;
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      fprintf(stderr, "%s\n", dlerror());
      return 1;
    }
    init_fn init = (init_fn)dlsym(h, "pow_init");
    warm_fn warm = (warm_fn)dlsym(h, "pow_warmup");
    /* AB_TTB_LOWEST=1: pow_mine (lowest solving counter: the same work on
     * every library, so the wall times pair up exactly) */
    const char* lo = getenv("AB_TTB_LOWEST");
    mine[v] = (any_fn)dlsym(h, lo && lo[0] == '1' ? "pow_mine" : "pow_mine_any");
    stats[v] = (stats_fn)dlsym(h, "pow_get_stats");
    if (!init || !warm || !mine[v] || !stats[v] || init(0, &ctx[v]) || warm(ctx[v])) {
      fprintf(stderr, "init failed for %s\n", argv[3 + v]);
      return 1;
    }
    env_clear();
  }
  srand(1);
  for (int k = -5; k < nt; ++k) { /* k < 0: untimed warm-up templates */
    pow_block b;
    memset(&b, 0, sizeof b);
    b.index = 1 + rand() % 65535;
    b.difficulty = 9;
    b.created_at = 1700000000 + rand() % 256;
    for (int i = 0; i < 64; ++i) b.previous_block_hash[i] = "0123456789abcdef"[rand() % 16];
    for (int v = 0; v < nv; ++v) {
      pow_block out;
      uint64_t ctr = 0;
      const double t0 = now();
      const int rc = mine[v](ctx[v], &b, 0, 1ull << 42, d, NULL, 0, &out, &ctr, NULL);
      const double t1 = now() - t0;
      if (rc != 1) {
        fprintf(stderr, "rc %d (%s)\n", rc, argv[3 + v]);
        return 1;
      }
      if (k < 0) continue;
      pow_stats st;
      stats[v](ctx[v], &st);
      wall[v][k] = t1;
      kms[v] += st.kernel_ms;
      hashes[v] += (double)st.hashes;
    }
  }
  for (int v = 0; v < nv; ++v) {
    qsort(wall[v], nt, sizeof(double), cmp);
    printf("{\"lib\": \"%s\", \"d\": %u, \"templates\": %d, \"ttb_ms_median\": %.4f, \"ttb_ms_p90\": %.4f, "
           "\"kernel_ms_sum\": %.3f, \"kernel_gtrials_per_s\": %.4f}\n",
           argv[3 + v], d, nt, 1e3 * wall[v][nt / 2], 1e3 * wall[v][(nt * 9) / 10], kms[v],
           hashes[v] / kms[v] / 1e6);
  }
  return 0;
}
