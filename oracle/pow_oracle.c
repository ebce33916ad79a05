/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, called by, or
 * shipped with the product path (mpi_blockchain_amd/, include/).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it,
 * and only as the checker.
 *
 * Plain-C restatement of the reference's mining hot path
 * (/root/reference, CatOfTheCannals/MPI_blockchain):
 *   - Block layout                 block.h:17-25
 *   - block_to_str (270 B message) block.cpp:79-88   (traps T1, T2, T5)
 *   - gen_random_nonce alphabet    block.cpp:61-72   (T6; RNG replaced by a counter)
 *   - SHA-256 (picosha2)           picosha2.h:46-61 (K, IV), 88-136 (block),
 *                                  190-228 (streaming + padding), 141-150 (hex)
 *   - solves_problem               block.cpp:28-58, 91-96 (T3: leading zero BITS)
 *
 * Pinning: checked in tests/test_oracle.py against golden vectors produced by
 * the reference's own block_to_hash / solves_problem compiled from
 * /root/reference (oracle/_ref, tests/golden/gen_golden.py) and against
 * Python hashlib.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define HASH_SIZE 256   /* block.h:4 */
#define NONCE_SIZE 10   /* block.h:5 */
#define MSG_BYTES 270

typedef struct {          /* block.h:17-25 */
  unsigned int index;
  unsigned int node_owner_number;
  unsigned int difficulty;
  unsigned long created_at;
  char nonce[NONCE_SIZE];
  char previous_block_hash[HASH_SIZE];
  char block_hash[HASH_SIZE];
} oracle_block;

/* picosha2.h:46-57 — the 64 round constants. */
static const uint32_t K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

/* picosha2.h:59-61 — initial hash value. */
static const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                               0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

/* picosha2.h:88-136 hash256_block: one 64-byte chunk, big-endian words. */
static void compress(uint32_t h[8], const uint8_t* chunk) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = ((uint32_t)chunk[4 * i] << 24) | ((uint32_t)chunk[4 * i + 1] << 16) |
           ((uint32_t)chunk[4 * i + 2] << 8) | (uint32_t)chunk[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = s1 + w[i - 7] + s0 + w[i - 16];
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = hh + S1 + ch + K[i] + w[i];
    uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

/* picosha2.h:178-228: stream the message in 64-byte chunks, then pad with
 * 0x80, zeros and the 64-bit big-endian bit length; digest big-endian. */
void oracle_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  uint32_t h[8];
  memcpy(h, IV, sizeof h);
  size_t off = 0;
  for (; off + 64 <= len; off += 64) compress(h, msg + off);
  uint8_t tail[128];
  size_t rem = len - off;
  memset(tail, 0, sizeof tail);
  memcpy(tail, msg + off, rem);
  tail[rem] = 0x80;
  size_t tl = (rem + 1 + 8 <= 64) ? 64 : 128;
  uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
  compress(h, tail);
  if (tl == 128) compress(h, tail + 64);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(h[i] >> 8);
    out[4 * i + 3] = (uint8_t)h[i];
  }
}

/* picosha2.h:141-150 output_hex: lowercase, two chars per byte. */
void oracle_hex(const uint8_t d[32], char hex[65]) {
  static const char digits[] = "0123456789abcdef";
  for (int i = 0; i < 32; ++i) {
    hex[2 * i] = digits[d[i] >> 4];
    hex[2 * i + 1] = digits[d[i] & 15];
  }
  hex[64] = 0;
}

/* block.cpp:79-88 block_to_str.  `str += block->index` appends ONE char: the
 * low byte of each integer field (T1).  Then nonce[0..9] including its NUL and
 * all 256 bytes of previous_block_hash (T2, T5). */
size_t oracle_block_to_str(const oracle_block* b, uint8_t out[MSG_BYTES]) {
  out[0] = (uint8_t)b->index;
  out[1] = (uint8_t)b->node_owner_number;
  out[2] = (uint8_t)b->difficulty;
  out[3] = (uint8_t)b->created_at;
  memcpy(out + 4, b->nonce, NONCE_SIZE);
  memcpy(out + 4 + NONCE_SIZE, b->previous_block_hash, HASH_SIZE);
  return MSG_BYTES;
}

/* block.cpp:74-77 block_to_hash. */
void oracle_block_to_hash(const oracle_block* b, uint8_t digest[32], char hex[65]) {
  uint8_t msg[MSG_BYTES];
  oracle_block_to_str(b, msg);
  uint8_t d[32];
  oracle_sha256(msg, MSG_BYTES, d);
  if (digest) memcpy(digest, d, 32);
  if (hex) oracle_hex(d, hex);
}

/* block.cpp:61-72 alphabet: 0-25 'a'.., 26-51 'A'.., 52-61 '0'..  The RNG
 * (rand()%62 per char) is replaced by the base-62 digits of a counter, most
 * significant first; nonce[9] = 0 (block.cpp:71). */
static char digit_char(unsigned d) {
  if (d < 26) return (char)('a' + d);
  if (d < 52) return (char)('A' + d - 26);
  return (char)('0' + d - 52);
}

int oracle_nonce_from_counter(uint64_t c, char nonce[NONCE_SIZE]) {
  for (int i = NONCE_SIZE - 2; i >= 0; --i) {
    nonce[i] = digit_char((unsigned)(c % 62));
    c /= 62;
  }
  nonce[NONCE_SIZE - 1] = 0;
  return c == 0 ? 0 : -1; /* -1: counter >= 62^9 */
}

/* block.cpp:28-49 hex_char_to_bin: toupper(c) -> 4 binary chars; anything
 * that is not 0-9/A-E falls to "1111". */
static const char* hex_char_to_bin(char c) {
  static const char* tab[16] = {"0000", "0001", "0010", "0011", "0100", "0101", "0110", "0111",
                                "1000", "1001", "1010", "1011", "1100", "1101", "1110", "1111"};
  if (c >= '0' && c <= '9') return tab[c - '0'];
  if (c >= 'a' && c <= 'z') c = (char)(c - 'a' + 'A');
  if (c >= 'A' && c <= 'E') return tab[10 + c - 'A'];
  return tab[15];
}

/* block.cpp:91-96 solves_problem, with the compile-time DEFAULT_DIFFICULTY
 * (block.h:6) made a run-time argument: the first `d` chars of the binary
 * expansion (block.cpp:52-58) must all be '0'.  string::compare(0, d, start)
 * on a shorter string compares only what exists, so d > 4*len can never match
 * ("0"*d is longer) — reproduced by requiring d <= 4*len. */
int oracle_solves_problem(const char* hex, unsigned d) {
  size_t len = strlen(hex);
  if (d > 4 * len) return 0;
  for (unsigned i = 0; i < d; ++i)
    if (hex_char_to_bin(hex[i / 4])[i % 4] != '0') return 0;
  return 1;
}

/* Bit test on the raw digest: the first d bits are zero (equivalent to the
 * above for a valid 64-char digest; T3). */
static int digest_has_zero_bits(const uint8_t dg[32], unsigned d) {
  if (d > 256) return 0;
  for (unsigned i = 0; i < d; ++i)
    if (dg[i / 8] & (0x80u >> (i % 8))) return 0;
  return 1;
}

/* ---- deterministic counter sweep (the GPU path's parity target) --------- */
typedef struct {
  const oracle_block* tmpl;
  uint64_t start, count;
  unsigned d;
  uint32_t* out; /* per-thread buffer */
  uint8_t* lz;   /* optional: leading zero bits of each solution's digest */
  size_t cap, n;
} sweep_job;

static unsigned leading_zero_bits(const uint8_t dg[32]) {
  unsigned n = 0;
  for (int i = 0; i < 32; ++i) {
    if (dg[i] == 0) { n += 8; continue; }
    for (unsigned m = 0x80; m && !(dg[i] & m); m >>= 1) ++n;
    break;
  }
  return n;
}

static void* sweep_worker(void* p) {
  sweep_job* j = (sweep_job*)p;
  oracle_block b = *j->tmpl;
  uint8_t msg[MSG_BYTES], dg[32];
  j->n = 0;
  for (uint64_t i = 0; i < j->count; ++i) {
    oracle_nonce_from_counter(j->start + i, b.nonce);
    oracle_block_to_str(&b, msg);
    oracle_sha256(msg, MSG_BYTES, dg);
    if (digest_has_zero_bits(dg, j->d)) {
      if (j->n < j->cap) {
        j->out[j->n] = (uint32_t)i;
        if (j->lz) j->lz[j->n] = (uint8_t)leading_zero_bits(dg);
      }
      j->n++;
    }
  }
  return NULL;
}

/* Every solving counter in [start, start+count) (count <= 2^32), as
 * (counter - start), ascending.  Returns the number found (which may exceed
 * cap; then only the first cap are stored).  nthreads <= 64. */
size_t oracle_sweep_lz(const oracle_block* tmpl, uint64_t start, uint64_t count, unsigned d,
                       uint32_t* out, uint8_t* lz, size_t cap, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  if ((uint64_t)nthreads > count) nthreads = count ? (int)count : 1;
  sweep_job jobs[64];
  pthread_t th[64];
  uint64_t per = count / (uint64_t)nthreads, extra = count % (uint64_t)nthreads, at = 0;
  for (int t = 0; t < nthreads; ++t) {
    jobs[t].tmpl = tmpl;
    jobs[t].start = start + at;
    jobs[t].count = per + ((uint64_t)t < extra ? 1 : 0);
    jobs[t].d = d;
    jobs[t].cap = cap;
    jobs[t].out = cap ? (uint32_t*)malloc(cap * sizeof(uint32_t)) : NULL;
    jobs[t].lz = (cap && lz) ? (uint8_t*)malloc(cap) : NULL;
    at += jobs[t].count;
    pthread_create(&th[t], NULL, sweep_worker, &jobs[t]);
  }
  size_t total = 0;
  uint64_t off = 0;
  for (int t = 0; t < nthreads; ++t) {
    pthread_join(th[t], NULL);
    for (size_t i = 0; i < jobs[t].n && i < jobs[t].cap && total + i < cap; ++i) {
      out[total + i] = (uint32_t)(jobs[t].out[i] + off);
      if (lz) lz[total + i] = jobs[t].lz[i];
    }
    total += jobs[t].n;
    off += jobs[t].count;
    free(jobs[t].out);
    free(jobs[t].lz);
  }
  return total; /* thread ranges are contiguous and ascending: output is sorted */
}

size_t oracle_sweep(const oracle_block* tmpl, uint64_t start, uint64_t count, unsigned d,
                    uint32_t* out, size_t cap, int nthreads) {
  return oracle_sweep_lz(tmpl, start, count, d, out, NULL, cap, nthreads);
}

/* Lowest solving counter in [start, start+count), or UINT64_MAX. */
uint64_t oracle_mine(const oracle_block* tmpl, uint64_t start, uint64_t count, unsigned d) {
  oracle_block b = *tmpl;
  uint8_t msg[MSG_BYTES], dg[32];
  for (uint64_t i = 0; i < count; ++i) {
    oracle_nonce_from_counter(start + i, b.nonce);
    oracle_block_to_str(&b, msg);
    oracle_sha256(msg, MSG_BYTES, dg);
    if (digest_has_zero_bits(dg, d)) return start + i;
  }
  return UINT64_MAX;
}

/* Trials/s of this restatement on one core over `n` counters (cpu_baseline
 * "port" kind). Returns the number of solutions so the loop is not elided. */
uint64_t oracle_bench(const oracle_block* tmpl, uint64_t start, uint64_t n, unsigned d) {
  oracle_block b = *tmpl;
  uint8_t msg[MSG_BYTES], dg[32];
  uint64_t hits = 0;
  for (uint64_t i = 0; i < n; ++i) {
    oracle_nonce_from_counter(start + i, b.nonce);
    oracle_block_to_str(&b, msg);
    oracle_sha256(msg, MSG_BYTES, dg);
    hits += (uint64_t)digest_has_zero_bits(dg, d);
  }
  return hits;
}

unsigned oracle_sizeof_block(void) { return (unsigned)sizeof(oracle_block); }
