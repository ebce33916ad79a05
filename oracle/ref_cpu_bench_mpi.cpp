// ORACLE — TEST INFRASTRUCTURE ONLY: the "reference" cpu_baseline of bench.py,
// run the way the reference itself runs: one MPI rank per host core
// (`mpiexec -np N ./blockchain`, Makefile:24; README.md:8-13).
//
// Every rank times the reference's mining loop body (node.cpp:292-308:
// template refresh, gen_random_nonce, picosha2 block_to_hash, solves_problem —
// the reference's own functions, linked from /root/reference/block.cpp by
// oracle/Makefile) for the same wall-clock window, after a common barrier;
// rank 0 sums the ranks' trial rates and prints one JSON line:
//   {"ranks":N,"seconds":S,"trials":T,"trials_per_s":R,"per_rank":R/N,
//    "per_rank_min":..,"per_rank_max":..,"hits":H}
//
//   mpiexec -np N ref_cpu_bench_mpi <seconds>
#include <mpi.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>

#include "block.h"

extern "C" uint64_t ref_mine_loop(const Block* last, int rank, uint64_t trials);

// Wait for a non-blocking collective without spinning: MPICH's blocking
// collectives busy-poll, and with more ranks than CPUs (or a CPU quota) the
// waiting ranks would take CPU time from the ones still computing.
static void wait_quietly(MPI_Request* req) {
  int done = 0;
  for (;;) {
    MPI_Test(req, &done, MPI_STATUS_IGNORE);
    if (done) return;
    usleep(1000);
  }
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank = 0, size = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  const double seconds = argc > 1 ? atof(argv[1]) : 2.0;
  srand((unsigned)time(NULL) + (unsigned)rank);  // node.cpp:386
  // Genesis-like last block (node.cpp:361-372): index 0, block_hash zeroed.
  Block last;
  memset(&last, 0, sizeof last);
  last.difficulty = DEFAULT_DIFFICULTY;
  last.created_at = (unsigned long)time(NULL);
  MPI_Request req;
  MPI_Ibarrier(MPI_COMM_WORLD, &req);  // one start line, as MPI_Init is for the reference's ranks
  wait_quietly(&req);
  const auto t0 = std::chrono::steady_clock::now();
  uint64_t trials = 0, hits = 0;
  const uint64_t batch = 256;
  double el = 0;
  while (el < seconds) {
    hits += ref_mine_loop(&last, rank, batch);
    trials += batch;
    el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  double rate = (double)trials / el;
  double r3[3] = {rate, rate, rate}, sum = 0, mn = 0, mx = 0;
  unsigned long long th[2] = {trials, hits}, th_sum[2] = {0, 0};
  MPI_Request rq[4];
  MPI_Ireduce(&r3[0], &sum, 1, MPI_DOUBLE, MPI_SUM, 0, MPI_COMM_WORLD, &rq[0]);
  MPI_Ireduce(&r3[1], &mn, 1, MPI_DOUBLE, MPI_MIN, 0, MPI_COMM_WORLD, &rq[1]);
  MPI_Ireduce(&r3[2], &mx, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD, &rq[2]);
  MPI_Ireduce(th, th_sum, 2, MPI_UNSIGNED_LONG_LONG, MPI_SUM, 0, MPI_COMM_WORLD, &rq[3]);
  for (auto& r : rq) wait_quietly(&r);
  const unsigned long long tr_sum = th_sum[0], h_sum = th_sum[1];
  if (rank == 0)
    printf("{\"ranks\": %d, \"seconds\": %.3f, \"trials\": %llu, \"trials_per_s\": %.1f, \"per_rank\": %.1f, "
           "\"per_rank_min\": %.1f, \"per_rank_max\": %.1f, \"hits\": %llu}\n",
           size, seconds, tr_sum, sum, sum / size, mn, mx, h_sum);
  MPI_Finalize();
  return 0;
}
