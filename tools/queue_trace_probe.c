/* How many hardware queues does a process of this library hold?  Run under
 * `rocprofv3 --hsa-trace` (tools/queue_trace.sh), which records every
 * hsa_queue_create / hsa_queue_destroy the HIP runtime makes; no GPU counters.
 * Modes (argv[1]):
 *   rank    - a pow_node rank's GPU side: two contexts (mining, validation),
 *             warm-up, a mine on one and a block validation on the other
 *   valu    - the same, plus pow_valu_rate (a stream of its own, destroyed)
 *   valu_ctx - the same, plus pow_valu_rate_ctx on context a's stream (what
 *             bench rank 0 runs for its roofline peaks)
 *   one     - a single context (the C consumer, bench's sweep tool)
 */
#include <stdio.h>
#include <string.h>

#include "pow_gpu.h"
#include "pow_tools.h"

static int die(const char* w) {
  fprintf(stderr, "%s: %s\n", w, pow_last_error());
  return 1;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "rank";
  pow_ctx *a = NULL, *b = NULL;
  if (pow_init(0, &a) != POW_OK || pow_warmup(a) != POW_OK) return die("ctx a");
  if (strcmp(mode, "one") != 0 && (pow_init(0, &b) != POW_OK || pow_warmup(b) != POW_OK)) return die("ctx b");
  pow_block t, out;
  memset(&t, 0, sizeof t);
  t.index = 1;
  t.difficulty = 9;
  t.created_at = 1700000000u;
  uint64_t ctr = 0;
  if (pow_mine_any(a, &t, 0, 1ull << 32, 21, NULL, 0, &out, &ctr, NULL) != 1) return die("mine");
  if (b) {
    char hex[65];
    if (pow_hash_block(b, &out, NULL, hex) != POW_OK) return die("hash");
  }
  if (strcmp(mode, "valu") == 0) {
    pow_valu_result r;
    if (pow_valu_rate(0, POW_VALU_FULL, &r) != POW_OK) return die("valu");
  }
  if (strcmp(mode, "valu_ctx") == 0) {
    pow_valu_result r;
    if (pow_valu_rate_ctx(a, POW_VALU_FULL, &r) != POW_OK) return die("valu_ctx");
  }
  printf("mode %s: mined counter %llu\n", mode, (unsigned long long)ctr);
  pow_destroy(a);
  pow_destroy(b);
  return 0;
}
