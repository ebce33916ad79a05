/* A/B of pow_hash_block (K2', one block: the validation of a received block)
 * between builds of libpow_gpu.so: the libraries are loaded side by side
 * (RTLD_LOCAL) and take turns, `reps` rounds of 200 calls each on 200
 * different blocks, so box and clock variation hit them alike.  Per library:
 * median call time (what validate_block_for_chain waits) and median kernel
 * time (pow_get_stats); every digest is compared across the libraries.
 *   gcc -O2 -I include tools/ab_k2.c -ldl -o tools/ab_k2
 *   tools/ab_k2 <reps> a/libpow_gpu.so b/libpow_gpu.so ...            */
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pow_gpu.h"

typedef int (*init_fn)(int, pow_ctx**);
typedef int (*warm_fn)(pow_ctx*);
typedef int (*hash_fn)(pow_ctx*, const pow_block*, uint8_t*, char*);
typedef int (*stats_fn)(const pow_ctx*, pow_stats*);

#define N 200
#define MAXL 8

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

static int cmp(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: ab_k2 <reps> lib...\n");
    return 2;
  }
  const int reps = atoi(argv[1]), nl = argc - 2;
  if (nl > MAXL) return 2;
  hash_fn hash[MAXL];
  stats_fn stats[MAXL];
  pow_ctx* ctx[MAXL];
  static pow_block blk[N];
  for (int i = 0; i < N; ++i) {
    memset(&blk[i], 0, sizeof blk[i]);
    blk[i].index = 3 + i;
    blk[i].node_owner_number = i % 7;
    blk[i].difficulty = 9;
    blk[i].created_at = 1700000000 + i;
    for (int k = 0; k < 9; ++k) blk[i].nonce[k] = 'a' + (i * 7 + k) % 26;
    for (int k = 0; k < 64; ++k) blk[i].previous_block_hash[k] = "0123456789abcdef"[(i + k * 5) % 16];
  }
  for (int l = 0; l < nl; ++l) {
    char path[512];
    snprintf(path, sizeof path, "%s", argv[2 + l]);
    char* at = strchr(path, '@');
    env_apply(argv[2 + l]);
    if (at) *at = 0;
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      fprintf(stderr, "%s\n", dlerror());
      return 1;
    }
    init_fn init = (init_fn)dlsym(h, "pow_init");
    warm_fn warm = (warm_fn)dlsym(h, "pow_warmup");
    hash[l] = (hash_fn)dlsym(h, "pow_hash_block");
    stats[l] = (stats_fn)dlsym(h, "pow_get_stats");
    if (init(0, &ctx[l]) || warm(ctx[l])) return 1;
    env_clear();
    /* AB_K2_IDLE_CTX=n: n more contexts of this library that never hash (their streams exist) */
    const char* e = getenv("AB_K2_IDLE_CTX");
    for (int k = 0; e && k < atoi(e); ++k) {
      pow_ctx* idle;
      if (init(0, &idle) || warm(idle)) return 1;
    }
  }
  static double call[MAXL][4096], kern[MAXL][4096];
  static char hex0[N][65];
  int nc = 0;
  for (int r = 0; r < reps; ++r)
    for (int l = 0; l < nl; ++l)
      for (int i = 0; i < N; ++i) {
        struct timespec t0, t1;
        char hex[65];
        clock_gettime(CLOCK_MONOTONIC, &t0);
        if (hash[l](ctx[l], &blk[i], NULL, hex)) return 1;
        clock_gettime(CLOCK_MONOTONIC, &t1);
        pow_stats st;
        stats[l](ctx[l], &st);
        const int k = r * N + i;
        if (k < 4096) {
          call[l][k] = (t1.tv_sec - t0.tv_sec) * 1e6 + (t1.tv_nsec - t0.tv_nsec) * 1e-3;
          kern[l][k] = st.kernel_ms * 1e3;
        }
        if (r == 0 && l == 0) memcpy(hex0[i], hex, 65);
        else if (memcmp(hex0[i], hex, 65) != 0) {
          fprintf(stderr, "digest mismatch: lib %d block %d\n", l, i);
          return 3;
        }
        nc = k + 1 < 4096 ? k + 1 : 4096;
      }
  for (int l = 0; l < nl; ++l) {
    qsort(call[l], nc, sizeof(double), cmp);
    qsort(kern[l], nc, sizeof(double), cmp);
    printf("{\"lib\": \"%s\", \"calls\": %d, \"call_us_median\": %.2f, \"call_us_p10\": %.2f, \"call_us_p90\": %.2f, "
           "\"kernel_us_median\": %.2f}\n",
           argv[2 + l], nc, call[l][nc / 2], call[l][nc / 10], call[l][nc * 9 / 10], kern[l][nc / 2]);
  }
  return 0;
}
