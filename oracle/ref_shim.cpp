// ORACLE — TEST INFRASTRUCTURE ONLY (never part of the product path).
//
// Thin extern "C" driver around the UNMODIFIED reference sources
// /root/reference/block.cpp + picosha2.h, compiled by oracle/Makefile into
// oracle/_ref/ (git-ignored).  It lets the tests and the golden-vector script
// call the reference's own block_to_str / block_to_hash / solves_problem /
// gen_random_nonce, and lets bench.py time the reference's mining loop body
// (node.cpp:292-308) on the host cores ("reference" cpu_baseline).
//
// Nothing here re-implements the reference: every hash and test below is the
// reference's own function.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "block.h"  // /root/reference/block.h (via -I)

#define REF_API extern "C" __attribute__((visibility("default")))

REF_API unsigned ref_sizeof_block() { return (unsigned)sizeof(Block); }
REF_API unsigned ref_default_difficulty() { return DEFAULT_DIFFICULTY; }

// block.cpp:79-88
REF_API int ref_block_to_str(const Block* b, unsigned char* out, int cap) {
  std::string s = block_to_str(b);
  int n = (int)s.size();
  if (n > cap) return -n;
  memcpy(out, s.data(), (size_t)n);
  return n;
}

// block.cpp:74-77 -> 64 lowercase hex chars + NUL
REF_API int ref_block_to_hash(const Block* b, char* hex65) {
  std::string s;
  block_to_hash(b, s);
  if (s.size() != 64) return -1;
  memcpy(hex65, s.c_str(), 65);
  return 64;
}

// block.cpp:91-96 (difficulty = the compile-time DEFAULT_DIFFICULTY, 9)
REF_API int ref_solves_problem(const char* hex) { return solves_problem(std::string(hex)) ? 1 : 0; }

// block.cpp:61-72
REF_API void ref_srand(unsigned seed) { srand(seed); }
REF_API void ref_gen_random_nonce(char* nonce10) { gen_random_nonce(nonce10); }

// Counter -> nonce, the deterministic stand-in for rand() used by the GPU
// path (same alphabet and order as block.cpp:61-72).  Local to this shim so
// the reference driver below has no dependency on the product library.
static void nonce_from_counter(uint64_t c, char* nonce) {
  for (int i = NONCE_SIZE - 2; i >= 0; --i) {
    unsigned d = (unsigned)(c % 62);
    c /= 62;
    nonce[i] = d < 26 ? (char)('a' + d) : d < 52 ? (char)('A' + d - 26) : (char)('0' + d - 52);
  }
  nonce[NONCE_SIZE - 1] = 0;
}

// Deterministic counter sweep through the reference's own block_to_hash and
// solves_problem (difficulty fixed at DEFAULT_DIFFICULTY = 9 by block.h:6).
// Writes (counter - start) of every solving counter, ascending.
REF_API long ref_sweep(const Block* tmpl, uint64_t start, uint64_t count, uint32_t* out, long cap) {
  Block b = *tmpl;
  std::string h;
  long n = 0;
  for (uint64_t i = 0; i < count; ++i) {
    nonce_from_counter(start + i, b.nonce);
    block_to_hash(&b, h);
    if (solves_problem(h)) {
      if (n < cap) out[n] = (uint32_t)i;
      ++n;
    }
  }
  return n;
}

// The reference's mining loop body, node.cpp:292-308, verbatim in behaviour:
// copy the last block, refresh the header (index+1, owner, DEFAULT_DIFFICULTY,
// time(NULL), memcpy prev <- last.block_hash), gen_random_nonce, block_to_hash,
// solves_problem.  Runs `trials` iterations; returns the number of solutions.
REF_API uint64_t ref_mine_loop(const Block* last, int rank, uint64_t trials) {
  std::string hash_hex_str;
  Block block;
  uint64_t hits = 0;
  for (uint64_t t = 0; t < trials; ++t) {
    block = *last;
    block.index += 1;
    block.node_owner_number = rank;
    block.difficulty = DEFAULT_DIFFICULTY;
    block.created_at = static_cast<unsigned long int>(time(NULL));
    memcpy(block.previous_block_hash, block.block_hash, HASH_SIZE);
    gen_random_nonce(block.nonce);
    block_to_hash(&block, hash_hex_str);
    if (solves_problem(hash_hex_str)) ++hits;
  }
  return hits;
}

// The validation hash of a received block (valid_new_block, block.cpp:13-25:
// block_to_hash, block.cpp:74-77), timed in-process: `n` calls on `n` blocks
// that differ in their nonce; returns the median call time in nanoseconds
// (bench.py's protocol block, beside pow_hash_block's call median).
REF_API double ref_block_to_hash_median_ns(const Block* tmpl, int n) {
  std::vector<double> t((size_t)(n > 0 ? n : 1));
  Block b = *tmpl;
  std::string h;
  for (int i = 0; i < n; ++i) {
    nonce_from_counter((uint64_t)i * 7919u, b.nonce);
    timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    block_to_hash(&b, h);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    t[(size_t)i] = (double)(t1.tv_sec - t0.tv_sec) * 1e9 + (double)(t1.tv_nsec - t0.tv_nsec);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}
