// ORACLE — TEST INFRASTRUCTURE ONLY: the "reference" cpu_baseline of bench.py.
//
// Times the reference's mining loop body (node.cpp:292-308: template refresh,
// gen_random_nonce, picosha2 block_to_hash, solves_problem — the reference's
// own functions, linked from /root/reference/block.cpp by oracle/Makefile) on
// P host cores, one forked process per core, like one MPI rank per core.
//
//   ref_cpu_bench <procs> <seconds>
// prints one JSON line: {"procs":P,"seconds":S,"trials":T,"trials_per_s":R,
//                        "per_core":R/P,"hits":H}
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>

#include "block.h"

extern "C" uint64_t ref_mine_loop(const Block* last, int rank, uint64_t trials);

int main(int argc, char** argv) {
  int procs = argc > 1 ? atoi(argv[1]) : 1;
  double seconds = argc > 2 ? atof(argv[2]) : 2.0;
  if (procs < 1) procs = 1;
  struct Res { uint64_t trials, hits; double secs; };
  Res* res = (Res*)mmap(nullptr, sizeof(Res) * (size_t)procs, PROT_READ | PROT_WRITE,
                        MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (res == MAP_FAILED) return 1;
  memset(res, 0, sizeof(Res) * (size_t)procs);
  // Genesis-like last block (node.cpp:361-372): index 0, block_hash zeroed.
  Block last;
  memset(&last, 0, sizeof last);
  last.difficulty = DEFAULT_DIFFICULTY;
  last.created_at = (unsigned long)time(NULL);
  for (int p = 0; p < procs; ++p) {
    pid_t pid = fork();
    if (pid == 0) {
      srand((unsigned)time(NULL) + (unsigned)p);  // node.cpp:386
      auto t0 = std::chrono::steady_clock::now();
      uint64_t trials = 0, hits = 0, batch = 256;
      double el = 0;
      while (el < seconds) {
        hits += ref_mine_loop(&last, p, batch);
        trials += batch;
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      }
      res[p].trials = trials;
      res[p].hits = hits;
      res[p].secs = el;
      _exit(0);
    }
  }
  for (int p = 0; p < procs; ++p) wait(nullptr);
  uint64_t trials = 0, hits = 0;
  double rate = 0;
  for (int p = 0; p < procs; ++p) {
    trials += res[p].trials;
    hits += res[p].hits;
    if (res[p].secs > 0) rate += (double)res[p].trials / res[p].secs;
  }
  printf("{\"procs\": %d, \"seconds\": %.3f, \"trials\": %llu, \"trials_per_s\": %.1f, "
         "\"per_core\": %.1f, \"hits\": %llu}\n",
         procs, seconds, (unsigned long long)trials, rate, rate / procs, (unsigned long long)hits);
  return 0;
}
