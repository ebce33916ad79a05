/*
 * mine_chain.c — a plain-C consumer of include/pow_gpu.h.
 *
 * Does what the reference's mining thread does (node.cpp:285-327) for one
 * rank without MPI: start from a genesis block whose hash is zeroed
 * (node.cpp:361-372), refresh the template (node.cpp:292-299), mine with the
 * GPU, strcpy the hex into the block (node.cpp:318), and re-validate every
 * block the way a receiver would (valid_new_block, block.cpp:13-25: the
 * recomputed hash equals the stored one; here also prev == parent's hash and
 * the leading-zero test of solves_problem, block.cpp:91-96).
 *
 *   cc -std=c11 -I include examples/mine_chain.c -L mpi_blockchain_amd -lpow_gpu \
 *      -Wl,-rpath,$PWD/mpi_blockchain_amd -o mine_chain && ./mine_chain [blocks] [difficulty]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pow_gpu.h"

#define CHECK(x)                                                                   \
  do {                                                                             \
    int rc_ = (x);                                                                 \
    if (rc_ < 0) {                                                                 \
      fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, pow_last_error());          \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 10;
  const unsigned diff = argc > 2 ? (unsigned)atoi(argv[2]) : 9;
  pow_ctx* ctx = NULL;
  CHECK(pow_init(0, &ctx));
  CHECK(pow_warmup(ctx));

  pow_block* chain = calloc((size_t)blocks + 1, sizeof(pow_block));
  chain[0].difficulty = diff;  /* genesis: index 0, block_hash all zero */
  chain[0].created_at = (uint64_t)time(NULL);
  for (int i = 1; i <= blocks; ++i) {
    pow_block tmpl = chain[i - 1];             /* node.cpp:292 */
    tmpl.index += 1;                           /* node.cpp:295-299 */
    tmpl.node_owner_number = 0;
    tmpl.difficulty = diff;
    tmpl.created_at = (uint64_t)time(NULL);
    memcpy(tmpl.previous_block_hash, tmpl.block_hash, POW_HASH_SIZE);
    uint64_t ctr = 0, hashes = 0;
    int rc = pow_mine_any(ctx, &tmpl, (uint64_t)i << 36, 1ull << 36, diff, NULL, 0, &chain[i], &ctr, &hashes);
    CHECK(rc);
    if (rc != 1) {
      fprintf(stderr, "no solution for block %d\n", i);
      return 1;
    }
    printf("block %d nonce %.9s hash %s (%llu trials)\n", i, chain[i].nonce, chain[i].block_hash,
           (unsigned long long)hashes);
  }
  /* receiver-side validation of the whole chain */
  for (int i = 1; i <= blocks; ++i) {
    char hex[65];
    CHECK(pow_hash_block(ctx, &chain[i], NULL, hex));
    if (strcmp(hex, chain[i].block_hash) != 0) return fprintf(stderr, "hash mismatch at %d\n", i), 1;
    if (memcmp(chain[i].previous_block_hash, chain[i - 1].block_hash, POW_HASH_SIZE) != 0)
      return fprintf(stderr, "broken link at %d\n", i), 1;
    if (!pow_solves_problem(hex, diff)) return fprintf(stderr, "difficulty not met at %d\n", i), 1;
  }
  printf("chain of %d blocks at difficulty %u: valid\n", blocks, diff);
  free(chain);
  pow_destroy(ctx);
  return 0;
}
