// ORACLE — test infrastructure only.
//
// Writes a chain dump with the REFERENCE's own logging code: this driver is
// linked with /root/reference/node.cpp + block.cpp (compiled in place by
// oracle/Makefile, target _ref/ref_log_chain) and calls node.cpp's log_msg
// and log_chain (node.cpp:40-68) exactly as proof_of_work's termination does
// (node.cpp:286-289).  The chain comes from stdin, one block per line, tip
// first, as tab-separated fields: index, owner, previous_block_hash,
// block_hash (the fields log_chain prints; the genesis link is an empty
// previous_block_hash).  The dump lands in <rank>.out in the current
// directory, so tests/test_node_gpu.py can compare a pow_node dump with it
// byte for byte.
//
//   ref_log_chain <rank> < chain.tsv
//
// No MPI call is made (node.cpp references MPI only in functions not called
// here); libmpi.so is linked only to resolve node.cpp's symbols.
#include <cstdio>
#include <cstring>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "block.h"

// node.cpp:19-21 (its globals) and node.cpp:40, 60 (not declared in node.h)
extern int mpi_rank;
extern Block* last_block_in_chain;
extern std::map<std::string, Block> node_blocks;
void log_chain(std::string log_info);
void log_msg(std::string msg);
// blockchain.cpp:9 defines it beside main(); node.cpp's send paths use it, never called here
MPI_Datatype* MPI_BLOCK = nullptr;

int main(int argc, char** argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: ref_log_chain <rank> < chain.tsv\n");
    return 2;
  }
  mpi_rank = atoi(argv[1]);
  std::string line, tip;
  while (std::getline(std::cin, line)) {
    if (line.empty()) continue;
    std::vector<std::string> f;
    std::stringstream ss(line);
    std::string x;
    while (std::getline(ss, x, '\t')) f.push_back(x);
    if (line.back() == '\t') f.push_back("");
    if (f.size() != 4 || f[2].size() >= HASH_SIZE || f[3].size() >= HASH_SIZE) {
      fprintf(stderr, "bad line: %s\n", line.c_str());
      return 2;
    }
    Block b;
    memset(&b, 0, sizeof b);
    b.index = (unsigned)std::stoul(f[0]);
    b.node_owner_number = (unsigned)std::stoul(f[1]);
    strcpy(b.previous_block_hash, f[2].c_str());
    strcpy(b.block_hash, f[3].c_str());
    node_blocks[f[3]] = b;
    if (tip.empty()) tip = f[3];
  }
  if (tip.empty()) {
    fprintf(stderr, "empty chain\n");
    return 2;
  }
  last_block_in_chain = &node_blocks.at(tip);
  log_msg("Terminé con la siguiente cadena");  // node.cpp:287
  log_chain("");                               // node.cpp:288
  return 0;
}
