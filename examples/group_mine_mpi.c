/*
 * Cooperative mining of one block over every MPI rank, one GPU per rank,
 * through the sharded-search calls of include/pow_gpu.h (pow_group_*).
 *
 * Rank 0 makes the RCCL id, MPI_Bcast hands it to the other ranks (the
 * reference's processes already share MPI_COMM_WORLD, blockchain.cpp:15),
 * then every rank calls pow_group_mine on the same template: each mines its
 * static shard of every round on its GPU and one RCCL all-reduce(min) per
 * round picks the lowest solving counter, identical on every rank.
 *
 *   mpiexec -np N group_mine_mpi [difficulty_bits] [log2_counters]
 *
 * The template is the synthetic block S0 (tests/golden): index 1, owner 0,
 * difficulty 9, created_at 1700000000, previous hash all zero.
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pow_gpu.h"

static void die(int rank, const char* what) {
  fprintf(stderr, "[%d] %s: %s\n", rank, what, pow_last_error());
  MPI_Abort(MPI_COMM_WORLD, 1);
}

int main(int argc, char** argv) {
  const unsigned diff = argc > 1 ? (unsigned)atoi(argv[1]) : 21;
  const int lg = argc > 2 ? atoi(argv[2]) : 32;
  MPI_Init(&argc, &argv);
  int rank = 0, size = 1, ndev = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  if (pow_device_count(&ndev) != POW_OK || ndev < 1) die(rank, "no GPU");
  pow_ctx* ctx = NULL;
  if (pow_init(rank % ndev, &ctx) != POW_OK) die(rank, "pow_init");

  uint8_t id[POW_GROUP_ID_BYTES];
  if (rank == 0 && pow_group_unique_id(id) != POW_OK) die(rank, "pow_group_unique_id");
  MPI_Bcast(id, POW_GROUP_ID_BYTES, MPI_BYTE, 0, MPI_COMM_WORLD);
  pow_group* g = NULL;
  if (pow_group_init(ctx, size, rank, id, &g) != POW_OK) die(rank, "pow_group_init");

  pow_block t;
  memset(&t, 0, sizeof t);
  t.index = 1;
  t.difficulty = 9;
  t.created_at = 1700000000u;
  pow_block out;
  uint64_t ctr = 0, hashes = 0;
  const double t0 = MPI_Wtime();
  const int rc = pow_group_mine(g, &t, 0, 1ull << lg, 0, diff, NULL, 0, &out, &ctr, &hashes);
  const double dt = MPI_Wtime() - t0;
  if (rc < 0) die(rank, "pow_group_mine");

  /* every rank must hold the same winner, and it must validate */
  int ok = rc == 1;
  if (ok) {
    char hex[65];
    if (pow_hash_block(ctx, &out, NULL, hex) != POW_OK) die(rank, "pow_hash_block");
    ok = strcmp(hex, out.block_hash) == 0 && pow_solves_problem(hex, diff);
  }
  unsigned long long lo = rc == 1 ? ctr : ~0ull, hi = lo, mn = 0, mx = 0, sum = 0;
  MPI_Allreduce(&lo, &mn, 1, MPI_UNSIGNED_LONG_LONG, MPI_MIN, MPI_COMM_WORLD);
  MPI_Allreduce(&hi, &mx, 1, MPI_UNSIGNED_LONG_LONG, MPI_MAX, MPI_COMM_WORLD);
  unsigned long long h = hashes;
  MPI_Allreduce(&h, &sum, 1, MPI_UNSIGNED_LONG_LONG, MPI_SUM, MPI_COMM_WORLD);
  int all_ok = 0;
  MPI_Allreduce(&ok, &all_ok, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
  if (rank == 0)
    printf("%d ranks: counter %llu nonce %.9s hash %s; %s; %llu trials in %.3f s\n", size, mn, out.nonce,
           rc == 1 ? out.block_hash : "-", all_ok && mn == mx ? "agreed and valid" : "MISMATCH", sum, dt);
  pow_group_destroy(g);
  pow_destroy(ctx);
  MPI_Finalize();
  return all_ok && mn == mx ? 0 : 2;
}
