// pow_node — one MPI rank of the MPI_blockchain protocol with the gfx950 miner.
//
// Rebuilds the reference's node (node.cpp / blockchain.cpp) around the C ABI of
// include/pow_gpu.h.  The protocol is kept as the reference defines it:
//   * wire format: the MPI_BLOCK datatype of block.cpp:99-120 ({3 x MPI_INT @0,
//     1 x MPI_UNSIGNED_LONG @16, 522 x MPI_UNSIGNED_CHAR @24}), tags 10/21/22
//     (node.h:7-9) — reference CPU ranks and GPU ranks interoperate in one
//     mpiexec (tests/test_node_gpu.py);
//   * validation: valid_new_block (block.cpp:13-25) with the hash recomputed
//     by the GPU (pow_hash_block) instead of picosha2;
//   * fork resolution: the six cases of validate_block_for_chain
//     (node.cpp:194-257), chain migration (node.cpp:152-191), chain service
//     (node.cpp:334-359), broadcast in rotated order (node.cpp:260-273);
//   * logging: the same stdout lines and <rank>.out chain dump (node.cpp:28-68);
//   * termination: the first rank whose chain reaches BLOCKS_TO_MINE logs and
//     calls MPI_Abort (node.cpp:286-290, 330).
// What changes:
//   * mining (node.cpp:292-308): each round refreshes the template exactly as
//     node.cpp:292-299 and runs pow_mine over a counter range on this rank's
//     GPU; the receive thread bumps a cancel epoch whenever the chain moves
//     and publishes it with pow_cancel, which stops the running launch within
//     ~0.4 ms;
//   * hardening: while waiting for a TAG_CHAIN_RESPONSE
//     the receive thread keeps serving TAG_CHAIN_HASH requests and defers
//     TAG_NEW_BLOCK messages, so two ranks asking each other cannot deadlock
//     (node.cpp:161 blocks inside the mutex); the miner copies the last block
//     under the mutex (node.cpp:292 reads it unlocked); a missing ancestor
//     ends send_blockchain's walk instead of throwing (node.cpp:348); the
//     receive loop polls with a backoff instead of MPICH's spinning probe
//     (T12: the reference burns a core per rank there).
//
// Start line.  The reference's ranks start mining as soon as MPI_Init returns
// (blockchain.cpp:15 -> node.cpp:396), and MPI_Init synchronises the job.
// Here GPU set-up (160-220 ms per process) runs beside MPI_Init, so ranks
// would leave it at different times: an MPI_Barrier after both puts them back
// on one start line before any miner starts.  In a job that mixes in
// reference ranks (which never join a barrier) pass --serial-init 1: GPU
// set-up then runs BEFORE MPI_Init, and MPI_Init is the start line, as in the
// reference.
//
//   pow_node [--difficulty D] [--blocks N] [--device G] [--round LOG2] [--serial-init 0|1]
//
// Test knobs.  bin/pow_node behaves only as node.cpp does.  The race-shaping
// switches the protocol tests need are compiled only into bin/pow_node_test
// (-DPOW_NODE_TEST_KNOBS, mpi_blockchain_amd/build.py):
//            [--pause-ms MS | --pause-us US] [--winner-pause-us US] [--hold-first 0|1]
//            [--idle-below K] [--private-lead K [--lead-barrier 0|1]
//             [--recv-delay-rank R --recv-delay-us US]]
#include <mpi.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <deque>
#include <fstream>
#include <iostream>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "pow_gpu.h"

namespace {

// block.h:6-9, node.h:7-9
constexpr int kValidationMinutes = 1;
constexpr int kValidationBlocks = 5;
constexpr int kTagNewBlock = 10;
constexpr int kTagChainHash = 21;
constexpr int kTagChainResponse = 22;

#ifdef POW_NODE_TEST_KNOBS
// Race shaping for the protocol tests (bin/pow_node_test only).
struct TestKnobs {
  unsigned winner_pause_us = 0;  // sleep after mining a block (GPU blocks take ~35 us, so the last
                                 // finder would otherwise start every race first)
  unsigned pause_us = 0;         // sleep a random 0..pause_us us before each round (lets slower CPU
                                 // ranks compete, and decorrelates GPU ranks so forks happen)
  bool hold_first = false;       // every rank mines block 1, then all publish it after one
                                 // MPI_Barrier, so every rank receives a rival block 1 (a certain fork)
  unsigned idle_below = 0;       // do not mine while the chain is below this index (the blocks
                                 // before it come from other ranks, e.g. the reference's CPU ranks)
  bool lead_barrier = true;      // --private-lead: the miners' barrier after every migration (0 = round 4's shape)
  int recv_delay_rank = -1;      // this rank's receive thread sleeps recv_delay_us after the tips'
  unsigned recv_delay_us = 0;    // barrier, before its first validation (the termination-race reproduction)
  unsigned private_lead = 0;     // K >= 2: every rank mines blocks 1..K on a private branch, then all
                                 // publish their tips after one barrier: each receiver is K behind
                                 // and asks the tip's owner for its chain while that owner asks it
                                 // (the mutual request node.cpp:155-161, 404-405 deadlocks on)
};
#endif

struct Options {
  unsigned difficulty = 9;  // DEFAULT_DIFFICULTY (block.h:6)
  unsigned blocks = 10;     // BLOCKS_TO_MINE (block.h:7)
  int device = -1;          // -1: local rank modulo visible GPUs
  unsigned round_log2 = 32; // counters per pow_mine call
  bool serial_init = false; // --serial-init 1: GPU set-up before MPI_Init instead of beside it
                            // (and no start barrier: mixed jobs with reference ranks)
#ifdef POW_NODE_TEST_KNOBS
  TestKnobs t;
#endif
};

// MPI_Probe that sleeps between polls instead of spinning.  MPICH's blocking
// probe/receive busy-polls, so every reference rank burns a core in its
// receive loop on top of its mining thread (node.cpp:404).
// Here the GPU does the mining, so the receive thread should not take a core:
// it polls with MPI_Iprobe and backs off from 5 us to 50 us while idle (the
// first polls after a message stay fast, so a burst is served at full speed).
void probe_any(MPI_Status* st) {
  int flag = 0;
  unsigned nap_us = 5;
  for (;;) {
    MPI_Iprobe(MPI_ANY_SOURCE, MPI_ANY_TAG, MPI_COMM_WORLD, &flag, st);
    if (flag) return;
    std::this_thread::sleep_for(std::chrono::microseconds(nap_us));
    nap_us = std::min(50u, nap_us * 2);
  }
}

// Bounded: a peer's block need not hold a NUL inside its 256-byte fields.
std::string hash_of(const pow_block& b) { return std::string(b.block_hash, strnlen(b.block_hash, POW_HASH_SIZE)); }
std::string prev_of(const pow_block& b) {
  return std::string(b.previous_block_hash, strnlen(b.previous_block_hash, POW_HASH_SIZE));
}

class Node {
 public:
  Node(const Options& o) : opt_(o) {}

  int init_gpu();
  void report_device();
  int run();
#ifdef POW_NODE_TEST_KNOBS
  // --log-chain-stdin <rank> (test build): no MPI, no GPU.  Load a chain from
  // stdin (one block per line, tip first: index, owner, previous_block_hash,
  // block_hash, tab-separated) and write the termination dump exactly as
  // proof_of_work does (node.cpp:286-289), so tests can compare this node's
  // log_msg + log_chain with the reference's (oracle/_ref/ref_log_chain).
  int dump_from_stdin(int rank) {
    rank_ = rank;
    std::string line, tip;
    while (std::getline(std::cin, line)) {
      std::vector<std::string> f;
      size_t a = 0;
      for (size_t t; (t = line.find('\t', a)) != std::string::npos; a = t + 1) f.push_back(line.substr(a, t - a));
      f.push_back(line.substr(a));
      if (f.size() != 4 || f[2].size() >= POW_HASH_SIZE || f[3].size() >= POW_HASH_SIZE) continue;
      pow_block b{};
      b.index = (uint32_t)std::stoul(f[0]);
      b.node_owner_number = (uint32_t)std::stoul(f[1]);
      memcpy(b.previous_block_hash, f[2].data(), f[2].size());
      memcpy(b.block_hash, f[3].data(), f[3].size());
      blocks_[f[3]] = b;
      if (tip.empty()) tip = f[3];
    }
    if (tip.empty()) return 2;
    last_ = &blocks_.at(tip);
    log_msg("Terminé con la siguiente cadena");
    log_chain("");
    return 0;
  }
#endif

 private:
  // ---- state (node.cpp:19-26) ----
  Options opt_;
  int rank_ = 0, size_ = 1;
  std::map<std::string, pow_block> blocks_;  // node_blocks
  const pow_block* last_ = nullptr;          // last_block_in_chain
  pow_block genesis_{};
  std::mutex mu_;                            // _sendMutex
  uint32_t epoch_ = 0;                       // bumped whenever last_ moves
  MPI_Datatype block_type_{};
  pow_ctx* mine_ctx_ = nullptr;              // used only by the mining thread
  pow_ctx* recv_ctx_ = nullptr;              // used only by the receive thread
  int device_ = -1, visible_gpus_ = 0, local_rank_ = 0;
  const char* local_rank_from_ = nullptr;    // the launcher variable the device came from (null: none)
  std::deque<std::pair<pow_block, MPI_Status>> deferred_;
#ifdef POW_NODE_TEST_KNOBS
  std::atomic<int> rivals1_{0};  // --hold-first: peers' blocks 1 this rank has processed
  MPI_Comm test_comm_ = MPI_COMM_NULL;  // --private-lead: the receive thread's own barrier
  MPI_Comm lead_comm_ = MPI_COMM_NULL;  // --private-lead: the miners' barrier after every migration
  bool tip_seen_ = false;               // --private-lead: a peer's private tip has arrived
#endif

  // The chain moved: a running pow_mine_any on the old template stops at its
  // next GPU poll (pow_cancel), not at its next sub-round (up to ~0.13 s).
  void bump_epoch() {
    const uint32_t e = __atomic_add_fetch(&epoch_, 1u, __ATOMIC_SEQ_CST);
    if (mine_ctx_) pow_cancel(mine_ctx_, e);
  }
  void set_last(const pow_block* b) {
    last_ = b;
    bump_epoch();
  }

  // block.cpp:99-120
  void define_block_type() {
    MPI_Aint disp[3] = {offsetof(pow_block, index), offsetof(pow_block, created_at),
                        offsetof(pow_block, nonce)};
    int len[3] = {3, 1, POW_NONCE_SIZE + POW_HASH_SIZE + POW_HASH_SIZE};
    MPI_Datatype types[3] = {MPI_INT, MPI_UNSIGNED_LONG, MPI_UNSIGNED_CHAR};
    if (MPI_Type_create_struct(3, len, disp, types, &block_type_) != MPI_SUCCESS ||
        MPI_Type_commit(&block_type_) != MPI_SUCCESS) {
      fprintf(stderr, "Error al crear el tipo\n");
      MPI_Abort(MPI_COMM_WORLD, 1);
    }
  }

  // block.cpp:74-77 through the GPU (K2) on the receive thread's context.
  std::string gpu_hash(const pow_block& b) {
    char hex[65];
    if (pow_hash_block(recv_ctx_, &b, nullptr, hex) != POW_OK) {
      fprintf(stderr, "[%d] pow_hash_block: %s\n", rank_, pow_last_error());
      MPI_Abort(MPI_COMM_WORLD, 1);
    }
    return std::string(hex);
  }

  // block.cpp:13-25
  bool valid_new_block(const pow_block& b) {
    const unsigned long now = (unsigned long)time(nullptr);
    bool valid = b.created_at + 60ul * kValidationMinutes >= now;
    return valid && gpu_hash(b) == hash_of(b);
  }

  // node.cpp:111-115
  bool check_first(const pow_block* chain, const pow_block& r) {
    const std::string h = gpu_hash(chain[0]);
    return chain[0].index == r.index && hash_of(chain[0]) == hash_of(r) && hash_of(chain[0]) == h;
  }
  // node.cpp:117-125
  static bool check_chain(const pow_block* chain) {
    bool ok = true;
    for (int i = 0; i < kValidationBlocks - 1; ++i) {
      if (prev_of(chain[i]).empty()) break;
      ok = prev_of(chain[i]) == hash_of(chain[i + 1]) && chain[i].index - 1 == chain[i + 1].index && ok;
    }
    return ok;
  }
  // node.cpp:127-129
  static bool equal(const pow_block& a, const pow_block& b) {
    return a.index == b.index && a.node_owner_number == b.node_owner_number &&
           a.difficulty == b.difficulty && a.created_at == b.created_at &&
           std::string(a.nonce, strnlen(a.nonce, POW_NONCE_SIZE)) ==
               std::string(b.nonce, strnlen(b.nonce, POW_NONCE_SIZE)) &&
           prev_of(a) == prev_of(b) && hash_of(a) == hash_of(b);
  }
  // node.cpp:131-139: is `b` on my current chain?
  bool look_for_block(const pow_block& b) {
    const pow_block* cur = last_;
    while (cur) {
      if (equal(*cur, b)) return true;
      const std::string p = prev_of(*cur);
      if (p.empty()) break;
      auto it = blocks_.find(p);
      cur = it == blocks_.end() ? nullptr : &it->second;
    }
    return false;
  }
  // node.cpp:141-148
  int find_block(const pow_block* chain) {
    for (int i = 0; i < kValidationBlocks; ++i)
      if (look_for_block(chain[i]) || chain[i].index == 1) return i;
    return -1;
  }

  // node.cpp:334-359: up to VALIDATION_BLOCKS blocks back from the requested one.
  void send_blockchain(pow_block from, int asker) {
    std::vector<pow_block> chain(kValidationBlocks);
    for (int i = 0; i < kValidationBlocks; ++i) {
      chain[i] = from;
      const std::string p = prev_of(from);
      if (p.empty()) break;
      auto it = blocks_.find(p);
      if (it == blocks_.end()) break;  // the reference throws std::out_of_range here
      from = it->second;
    }
    int rc = MPI_Send(chain.data(), kValidationBlocks, block_type_, asker, kTagChainResponse, MPI_COMM_WORLD);
    if (rc != MPI_SUCCESS) printf("[%d] send to node %d failed with error code %d \n", rank_, asker, rc);
  }

  // node.cpp:152-191, with the wait made deadlock-free (see header).
  bool verificar_y_migrar_cadena(const pow_block& r) {
    const int owner = (int)r.node_owner_number;
    MPI_Send(&r, 1, block_type_, owner, kTagChainHash, MPI_COMM_WORLD);
    std::vector<pow_block> chain(kValidationBlocks);
    for (;;) {
      MPI_Status st;
      probe_any(&st);
      if (st.MPI_TAG == kTagChainResponse && st.MPI_SOURCE == owner) {
        MPI_Recv(chain.data(), kValidationBlocks, block_type_, owner, kTagChainResponse, MPI_COMM_WORLD, &st);
        break;
      }
      if (st.MPI_TAG == kTagChainResponse) {  // stale response from another rank: drop
        std::vector<pow_block> junk(kValidationBlocks);
        MPI_Recv(junk.data(), kValidationBlocks, block_type_, st.MPI_SOURCE, st.MPI_TAG, MPI_COMM_WORLD, &st);
        continue;
      }
      pow_block buf;
      MPI_Recv(&buf, 1, block_type_, st.MPI_SOURCE, st.MPI_TAG, MPI_COMM_WORLD, &st);
      if (st.MPI_TAG == kTagChainHash) {
        printf("[%u] TAG_CHAIN_HASH \n", rank_);
#ifdef POW_NODE_TEST_KNOBS
        // the case the hardening is for: a chain request served while this
        // rank itself waits for a TAG_CHAIN_RESPONSE (the reference blocks in
        // MPI_Recv here, holding the mutex its receive loop needs)
        printf("[%d] TAG_CHAIN_HASH de %d atendido mientras espero la cadena de %d \n", rank_, st.MPI_SOURCE, owner);
#endif
        send_blockchain(buf, st.MPI_SOURCE);
      } else if (st.MPI_TAG == kTagNewBlock) {
        deferred_.emplace_back(buf, st);
      }
    }
    const bool checks = check_first(chain.data(), r) && check_chain(chain.data());
    const int i = find_block(chain.data());
    printf("[%d]: find = %d | received_blockchain_checks = %d\n", rank_, i, checks ? 1 : 0);
    if (checks && i > -1) {
      for (int j = 0; j < i + 1; ++j) blocks_.insert({hash_of(chain[j]), chain[j]});
      set_last(&blocks_.at(hash_of(chain[0])));
      return true;
    }
    return false;
  }

  // node.cpp:194-257
  bool validate_block_for_chain(const pow_block& r, const MPI_Status& st) {
    if (valid_new_block(r)) {
      blocks_.insert({hash_of(r), r});
      const pow_block& last = *last_;
      if (r.index == 1 && last.index == 0) {
        set_last(&blocks_.at(hash_of(r)));
        printf("[%d] Agregado a la lista bloque con index %u enviado por %d \n", rank_, r.index, st.MPI_SOURCE);
        return true;
      }
      if (r.index == last.index + 1 && prev_of(r) == hash_of(last)) {
        set_last(&blocks_.at(hash_of(r)));
        printf("[%d] Agregado a la lista bloque con index %u enviado por %d \n", rank_, r.index, st.MPI_SOURCE);
        return true;
      }
      if (r.index == last.index + 1 && prev_of(r) != hash_of(last)) {
        printf("[%d] Perdí la carrera por uno (%d) contra %d \n", rank_, r.index, st.MPI_SOURCE);
        return verificar_y_migrar_cadena(r);
      }
      if (r.index == last.index) {
        printf("[%d] Conflicto suave: Conflicto de branch (%d) contra %d \n", rank_, r.index, st.MPI_SOURCE);
        return false;
      }
      if (r.index < last.index) {
        printf("[%d] Conflicto suave: Descarto el bloque (%d vs %d) contra %d \n", rank_, r.index, last.index,
               st.MPI_SOURCE);
        return false;
      }
      if (r.index > last.index + 1) {
        printf("[%d] Perdí la carrera por varios contra %d \n", rank_, st.MPI_SOURCE);
        return verificar_y_migrar_cadena(r);
      }
    }
    printf("[%d] Error duro: Descarto el bloque recibido de %d porque no es válido \n", rank_, st.MPI_SOURCE);
    return false;
  }

  // node.cpp:260-273
  void send_block_to_everyone(const pow_block& b) {
    for (int i = 1; i < size_; ++i) {
      const int to = (rank_ + i) % size_;
      int rc = MPI_Send(&b, 1, block_type_, to, kTagNewBlock, MPI_COMM_WORLD);
      if (rc != MPI_SUCCESS) printf("[%d] send to node %d failed with error code %d \n", rank_, to, rc);
    }
  }

  // node.cpp:40-68
  void log_msg(const std::string& msg) {
    std::ofstream out(std::to_string((unsigned long)rank_) + ".out", std::ios::app);
    out << msg << "\n--------------------\n";
  }
  void log_chain(const std::string& info) {
    std::ofstream out(std::to_string((unsigned long)rank_) + ".out", std::ios::app);
    pow_block cur = *last_;
    out << "Mi blockchain es la siguiente en " + info << "\n";
    for (;;) {
      out << "--------------------\n"
          << "Block number: " << cur.index << "\n"
          << "Owner: " << cur.node_owner_number << "\n"
          << "Previous block hash: " << prev_of(cur) << "\n"
          << "Block hash: " << hash_of(cur) << "\n"
          << "--------------------\n";
      const std::string p = prev_of(cur);
      if (p.empty()) break;
      auto it = blocks_.find(p);
      if (it == blocks_.end()) break;
      cur = it->second;
    }
  }

  // node.cpp:278-332 with node.cpp:302-308 on the GPU.
#ifdef POW_NODE_TEST_KNOBS
  // --private-lead K: mine blocks 1..K on a private branch (inserted into
  // node_blocks so send_blockchain can serve them, but never adopted as
  // last_block_in_chain), then publish only the tip after one barrier, outside
  // the mutex, so every rank's tip goes out at once.  Each receiver is K
  // behind ("Perdí la carrera por varios", node.cpp:249-253) and asks the
  // tip's owner for its chain while that owner asks it.  Then wait (bounded)
  // until this rank has migrated, so no block 1 is mined on genesis meanwhile,
  // and then for every other rank's miner to have done the same (lead_comm_):
  // without that, the first ranks to migrate mine blocks 4..10 in a few ms and
  // the finisher's MPI_Abort (node.cpp:330) can end the job before a slower
  // rank has logged its own migration (the test then sees a rank that "logged
  // nothing" after its tip: a termination race, not a hang).  The bound (30 s)
  // is longer than the launch watchdog (10 s), so a launch that never
  // completes aborts the job with its diagnostic before the bound expires.
  void private_lead(std::mt19937_64& rng, uint64_t round) {
    pow_block prev;
    {
      std::lock_guard<std::mutex> g(mu_);
      prev = *last_;
    }
    for (unsigned k = 0; k < opt_.t.private_lead;) {
      pow_block tmpl = prev, solved;
      tmpl.index += 1;
      tmpl.node_owner_number = (uint32_t)rank_;
      tmpl.difficulty = opt_.difficulty;
      tmpl.created_at = (uint64_t)time(nullptr);
      memcpy(tmpl.previous_block_hash, prev.block_hash, POW_HASH_SIZE);
      uint64_t ctr = 0;
      const int rc = pow_mine_any(mine_ctx_, &tmpl, rng() % (POW_COUNTER_LIMIT - round), round, opt_.difficulty,
                                  nullptr, 0, &solved, &ctr, nullptr);
      if (rc < 0) {
        fprintf(stderr, "[%d] pow_mine_any: %s\n", rank_, pow_last_error());
        MPI_Abort(MPI_COMM_WORLD, 1);
      }
      if (rc != 1) continue;
      {
        std::lock_guard<std::mutex> g(mu_);
        blocks_.insert({hash_of(solved), solved});
      }
      printf("[%d] Bloque privado con index %u \n", rank_, solved.index);
      prev = solved;
      ++k;
    }
    MPI_Barrier(MPI_COMM_WORLD);
    send_block_to_everyone(prev);
    const auto t0 = std::chrono::steady_clock::now();
    for (bool migrated = false; !migrated;) {
      {
        std::lock_guard<std::mutex> g(mu_);
        migrated = last_->index >= opt_.t.private_lead;
      }
      if (!migrated && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
        printf("[%d] private-lead: no migration after 30 s\n", rank_);
        break;
      }
      if (!migrated) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    if (opt_.t.lead_barrier) MPI_Barrier(lead_comm_);
  }
#endif

  void proof_of_work() {
    std::mt19937_64 rng((uint64_t)time(nullptr) + (uint64_t)rank_);  // node.cpp:386
    const uint64_t round = 1ull << opt_.round_log2;
#ifdef POW_NODE_TEST_KNOBS
    if (opt_.t.private_lead >= 2) private_lead(rng, round);
#endif
    for (;;) {
      pow_block tmpl;
      uint32_t ep;
      {
        std::lock_guard<std::mutex> g(mu_);
        if (last_->index >= opt_.blocks) {  // node.cpp:286-290
          log_msg("Terminé con la siguiente cadena");
          log_chain("");
          break;
        }
        tmpl = *last_;
        ep = __atomic_load_n(&epoch_, __ATOMIC_SEQ_CST);
      }
#ifdef POW_NODE_TEST_KNOBS
      if (tmpl.index < opt_.t.idle_below) {  // --idle-below: only receive for now
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        continue;
      }
#endif
      // node.cpp:295-299
      tmpl.index += 1;
      tmpl.node_owner_number = (uint32_t)rank_;
      tmpl.difficulty = opt_.difficulty;
      tmpl.created_at = (uint64_t)time(nullptr);
      memcpy(tmpl.previous_block_hash, tmpl.block_hash, POW_HASH_SIZE);
#ifdef POW_NODE_TEST_KNOBS
      if (opt_.t.pause_us) std::this_thread::sleep_for(std::chrono::microseconds(rng() % (opt_.t.pause_us + 1ull)));
#endif
      const uint64_t start = rng() % (POW_COUNTER_LIMIT - round);
      pow_block solved;
      uint64_t ctr = 0;
      // first solution found in the range: the reference's random nonces have no order either
      int rc = pow_mine_any(mine_ctx_, &tmpl, start, round, opt_.difficulty, &epoch_, ep, &solved, &ctr, nullptr);
      if (rc < 0) {
        fprintf(stderr, "[%d] pow_mine_any: %s\n", rank_, pow_last_error());
        MPI_Abort(MPI_COMM_WORLD, 1);
      }
#ifdef POW_NODE_TEST_KNOBS
      if (rc == 1 && opt_.t.hold_first && solved.index == 1) {
        // --hold-first: adopt block 1, wait until every rank has mined its
        // own block 1, then publish.  Each rank then receives rival blocks 1
        // while its chain is at index 1: "Conflicto de branch" (node.cpp:235)
        // on every rank, deterministically.
        bool adopted = false;
        {
          std::lock_guard<std::mutex> g(mu_);
          if (last_->index < solved.index) {
            const std::string h = hash_of(solved);
            blocks_.insert({h, solved});
            set_last(&blocks_.at(h));
            printf("[%d] Agregué un producido con index %u \n", rank_, last_->index);
            adopted = true;
          }
        }
        MPI_Barrier(MPI_COMM_WORLD);  // nobody sends before this, so our block 1 stands
        if (adopted) {
          std::lock_guard<std::mutex> g(mu_);
          send_block_to_everyone(blocks_.at(hash_of(solved)));
        }
        // ... and mine block 2 only once every peer's block 1 has been through
        // validate_block_for_chain here: otherwise, with blocks taking ~20 us
        // at d = 5, a fast rank can finish the chain (MPI_Abort) before a slow
        // receive thread has handled (and logged) its rival block 1.  Bounded
        // wait: a peer whose block 1 never comes (it adopted ours first) does
        // not hold the network up past 2 s.
        for (int w = 0; w < 40000 && rivals1_.load(std::memory_order_acquire) < size_ - 1; ++w)
          std::this_thread::sleep_for(std::chrono::microseconds(50));
        continue;
      }
#endif
      if (rc == 1) {  // node.cpp:311-327
        std::lock_guard<std::mutex> g(mu_);
        if (last_->index < solved.index) {
          const std::string h = hash_of(solved);
          blocks_.insert({h, solved});
          set_last(&blocks_.at(h));
          printf("[%d] Agregué un producido con index %u \n", rank_, last_->index);
          send_block_to_everyone(*last_);
        }
      }
#ifdef POW_NODE_TEST_KNOBS
      // Tests: let the other ranks receive this block before racing on the next.
      if (rc == 1 && opt_.t.winner_pause_us)
        std::this_thread::sleep_for(std::chrono::microseconds(opt_.t.winner_pause_us));
#endif
    }
    MPI_Abort(MPI_COMM_WORLD, 0);  // node.cpp:330
  }
};

// GPU set-up (HIP start-up, 160-220 ms per process, two contexts, kernel
// warm-up) runs on a thread beside MPI_Init, which itself waits for every
// process of the job, so a rank's start-up costs the longer of the two rather
// than their sum.  The miner starts only once both are done and every rank
// has passed the start barrier in main().  (--serial-init 1
// runs it before MPI_Init instead: then no reference rank of a mixed job can
// start mining while a GPU rank is still initialising.)  The device is the
// node-local rank (from the launcher's environment) modulo the visible GPUs;
// report_device says which one it was and where the choice came from.
int Node::init_gpu() {
  int ndev = 0, local = 0;
  if (pow_device_count(&ndev) != POW_OK || ndev < 1) {
    fprintf(stderr, "no GPU: %s\n", pow_last_error());
    return 1;
  }
  for (const char* k : {"MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", "LOCAL_RANK", "PMI_RANK"})
    if (const char* e = getenv(k)) {
      local = atoi(e);
      local_rank_from_ = k;
      break;
    }
  const int dev = opt_.device >= 0 ? opt_.device : local % ndev;
  device_ = dev;
  visible_gpus_ = ndev;
  local_rank_ = local;
  if (pow_init(dev, &mine_ctx_) != POW_OK || pow_init(dev, &recv_ctx_) != POW_OK ||
      pow_warmup(mine_ctx_) != POW_OK || pow_warmup(recv_ctx_) != POW_OK) {
    fprintf(stderr, "pow_init(%d): %s\n", dev, pow_last_error());
    return 1;
  }
  return 0;
}

// One stderr line per rank at start-up, after MPI_Init: the GPU this rank
// mines on (HIP index and PCI address) and where the choice came from, so a
// job's placement can be checked (bench.py's config-5 block requires one rank
// per distinct GPU at N > 1).  The reference runs one process per node
// (node.cpp:379-396) and has no device to choose.  A job of several ranks
// whose launcher set no node-local rank would put every rank on GPU 0: that
// is said on stderr rather than done silently.
void Node::report_device() {
  int rank = 0, size = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  char pci[64] = "?";
  if (pow_device_pci_bus_id(mine_ctx_, pci, sizeof pci) != POW_OK) snprintf(pci, sizeof pci, "?");
  char host[128] = "?";
  if (gethostname(host, sizeof host) != 0) snprintf(host, sizeof host, "?");
  host[sizeof host - 1] = 0;
  const char* from = opt_.device >= 0 ? "--device" : local_rank_from_ ? local_rank_from_ : "none";
  fprintf(stderr,
          "pow_node device {\"rank\": %d, \"size\": %d, \"device\": %d, \"pci\": \"%s\", \"host\": \"%s\", "
          "\"pid\": %d, \"local_rank\": %d, \"local_rank_from\": \"%s\", \"visible_gpus\": %d}\n",
          rank, size, device_, pci, host, (int)getpid(), local_rank_, from, visible_gpus_);
  if (opt_.device < 0 && !local_rank_from_ && size > 1)
    fprintf(stderr,
            "pow_node: rank %d of %d: no node-local rank in the environment (MPI_LOCALRANKID, "
            "OMPI_COMM_WORLD_LOCAL_RANK, LOCAL_RANK, PMI_RANK): mining on GPU %d like every other such rank; "
            "launch with mpiexec or pass --device\n",
            rank, size, device_);
}

int Node::run() {
  MPI_Comm_size(MPI_COMM_WORLD, &size_);
  MPI_Comm_rank(MPI_COMM_WORLD, &rank_);
  define_block_type();
#ifdef POW_NODE_TEST_KNOBS
  if (opt_.t.private_lead >= 2) {
    MPI_Comm_dup(MPI_COMM_WORLD, &test_comm_);
    MPI_Comm_dup(MPI_COMM_WORLD, &lead_comm_);
  }
#endif
  printf("[MPI] Lanzando proceso %u\n", rank_);
  std::remove((std::to_string(rank_) + ".out").c_str());  // blockchain.cpp:31 does `rm *.out`

  // node.cpp:361-372
  memset(&genesis_, 0, sizeof genesis_);
  genesis_.index = 0;
  genesis_.node_owner_number = (uint32_t)rank_;
  genesis_.difficulty = opt_.difficulty;
  genesis_.created_at = (uint64_t)time(nullptr);
  last_ = &genesis_;

  pow_cancel(mine_ctx_, epoch_);  // arm the GPU-side epoch check
  std::thread miner([this] {
    pthread_setname_np(pthread_self(), "pow_miner");
    proof_of_work();
  });
  for (;;) {  // node.cpp:398-420
    pow_block buf;
    MPI_Status st;
    if (!deferred_.empty()) {
      buf = deferred_.front().first;
      st = deferred_.front().second;
      deferred_.pop_front();
    } else {
      probe_any(&st);
      if (st.MPI_TAG == kTagChainResponse) {  // not waiting for one: drop it
        std::vector<pow_block> junk(kValidationBlocks);
        MPI_Recv(junk.data(), kValidationBlocks, block_type_, st.MPI_SOURCE, st.MPI_TAG, MPI_COMM_WORLD, &st);
        continue;
      }
      MPI_Recv(&buf, 1, block_type_, st.MPI_SOURCE, st.MPI_TAG, MPI_COMM_WORLD, &st);
    }
#ifdef POW_NODE_TEST_KNOBS
    // --private-lead: every receive thread holds its first peer tip until all
    // have one, so all ranks enter verificar_y_migrar_cadena together and each
    // one's TAG_CHAIN_HASH reaches a rank that is itself waiting for a chain.
    if (opt_.t.private_lead >= 2 && !tip_seen_ && st.MPI_TAG == kTagNewBlock && buf.index == opt_.t.private_lead) {
      tip_seen_ = true;
      MPI_Barrier(test_comm_);
      if (rank_ == opt_.t.recv_delay_rank && opt_.t.recv_delay_us)  // a slow receive thread, on purpose
        std::this_thread::sleep_for(std::chrono::microseconds(opt_.t.recv_delay_us));
    }
#endif
    std::lock_guard<std::mutex> g(mu_);
    if (st.MPI_TAG == kTagNewBlock) {
      validate_block_for_chain(buf, st);
#ifdef POW_NODE_TEST_KNOBS
      if (buf.index == 1) rivals1_.fetch_add(1, std::memory_order_release);
#endif
    } else if (st.MPI_TAG == kTagChainHash) {
      printf("[%u] TAG_CHAIN_HASH \n", rank_);
      send_blockchain(buf, st.MPI_SOURCE);
    }
  }
  miner.join();
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
#ifdef POW_NODE_TEST_KNOBS
  if (argc == 3 && std::string(argv[1]) == "--log-chain-stdin") return Node(o).dump_from_stdin(atoi(argv[2]));
#endif
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string k = argv[i];
    const long v = strtol(argv[i + 1], nullptr, 10);
    if (k == "--difficulty") o.difficulty = (unsigned)v;
    else if (k == "--blocks") o.blocks = (unsigned)v;
    else if (k == "--device") o.device = (int)v;
    else if (k == "--round") o.round_log2 = (unsigned)std::min(40l, std::max(12l, v));
    else if (k == "--serial-init") o.serial_init = v != 0;
#ifdef POW_NODE_TEST_KNOBS
    else if (k == "--pause-ms") o.t.pause_us = (unsigned)v * 1000u;
    else if (k == "--pause-us") o.t.pause_us = (unsigned)v;
    else if (k == "--winner-pause-us") o.t.winner_pause_us = (unsigned)v;
    else if (k == "--hold-first") o.t.hold_first = v != 0;
    else if (k == "--idle-below") o.t.idle_below = (unsigned)std::max(0l, v);
    else if (k == "--private-lead") o.t.private_lead = (unsigned)std::min(5l, std::max(0l, v));  // <= VALIDATION_BLOCKS
    else if (k == "--lead-barrier") o.t.lead_barrier = v != 0;
    else if (k == "--recv-delay-rank") o.t.recv_delay_rank = (int)v;
    else if (k == "--recv-delay-us") o.t.recv_delay_us = (unsigned)std::max(0l, v);
#endif
    else {
      fprintf(stderr, "pow_node: unknown option %s (race-shaping test knobs are in pow_node_test)\n", k.c_str());
      return 2;
    }
  }
  Node n(o);
  int gpu_rc = 0;
  std::thread gpu_init;
  using clk = std::chrono::steady_clock;
  const auto t_start = clk::now();
  double gpu_ms = 0;
  auto timed_init = [&] {
    const auto t = clk::now();
    gpu_rc = n.init_gpu();
    gpu_ms = std::chrono::duration<double, std::milli>(clk::now() - t).count();
  };
  if (o.serial_init) {
    timed_init();
    if (gpu_rc != 0) return 1;
  } else {
    gpu_init = std::thread(timed_init);
  }
  int provided = 0;
  const int mpi_rc = MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided);
  const double mpi_ms = std::chrono::duration<double, std::milli>(clk::now() - t_start).count();
  if (gpu_init.joinable()) gpu_init.join();
  if (mpi_rc != MPI_SUCCESS) {
    fprintf(stderr, "Error de MPI al inicializar.\n");
    return 1;
  }
  if (gpu_rc != 0) MPI_Abort(MPI_COMM_WORLD, 1);
  if (provided < MPI_THREAD_MULTIPLE) {  // blockchain.cpp:15 never checks this
    fprintf(stderr, "MPI_THREAD_MULTIPLE not provided (%d)\n", provided);
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  setbuf(stdout, nullptr);  // blockchain.cpp:27-28
  setbuf(stderr, nullptr);
  // One start line for every rank (see the header): GPU set-up ended at a
  // different time on each rank.  With --serial-init, MPI_Init was it.
  if (!o.serial_init) MPI_Barrier(MPI_COMM_WORLD);
  n.report_device();
#ifdef POW_NODE_TEST_KNOBS
  // Start-up split (test build only, stderr): where a slow network's first
  // second goes (GPU set-up: HIP runtime + two contexts + warm-up; MPI_Init).
  {
    int r = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &r);
    fprintf(stderr, "[%d] start-up: gpu set-up %.1f ms, MPI_Init %.1f ms, start line at %.1f ms\n", r, gpu_ms, mpi_ms,
            std::chrono::duration<double, std::milli>(clk::now() - t_start).count());
  }
#else
  (void)gpu_ms;
  (void)mpi_ms;
#endif
  n.run();
  MPI_Finalize();
  return 0;
}
