// Direct AQL dispatch of the latency-bound kernels (pow_aql.cpp).  Compiled
// into the TEST library only (libpow_gpu_test.so, -DPOW_TEST_HOOKS, opt-in
// with POW_AQL=1): the shipped libpow_gpu.so launches every kernel through
// hipLaunchKernel ("Direct dispatch, round 5").  Not part of the
// C ABI.
#pragma once
#include <stdint.h>

#include <string>

struct pow_aql;

enum {
  POW_AQL_HASH_ONE = 0,  // K2' pow_hash_one(PowMsg, PowHashOut*, uint32_t)
  POW_AQL_LAT0 = 1,      // K1' pow_search_lat<FULL, ANY, ASM>: POW_AQL_LAT0 + (FULL | ANY << 1 | ASM << 2)
  POW_AQL_NKERNELS = 9
};

// A dispatcher for one context on `device` (the kernels and the queue are
// shared by the process's contexts on the device).  0 = ready; -1 = not
// available here (*why says why; the caller keeps the HIP launch path).
int pow_aql_open(int device, unsigned flags, pow_aql** out, std::string* why);
// Dispatch experiments (flags of pow_aql_open, from POW_AQL_EXP).
enum {
  POW_AQL_EXP_NO_SIGNAL = 1,    // no completion signal (a launch that ends unpublished is then seen only by the watchdog)
  POW_AQL_EXP_NO_FLUSH = 2,     // no HDP flush / read-back after writing the arguments
  POW_AQL_EXP_NO_READBACK = 4,  // HDP flush, no read-back
  POW_AQL_EXP_HOST_ARGS = 8,    // arguments in coherent host memory instead of device memory
  POW_AQL_EXP_OWN_QUEUE = 16,   // a queue of the context's own (packets with the barrier bit)
  POW_AQL_EXP_READBACK_ONLY = 32,  // no HDP flush: re-store the last word, mfence, read it back
  POW_AQL_EXP_FINE_ARGS = 64,   // arguments in fine-grained device memory (cached in L2)
  POW_AQL_EXP_ACQUIRE_SYSTEM = 128,  // packet acquire fence at system scope (L2 invalidate)
  POW_AQL_EXP_RELEASE_AGENT = 256,   // packet release fence at agent scope (no L2 write-back)
  // The ordering test's hook: after reserving its packet index and writing
  // the packet body, this context sleeps POW_AQL_STALL_US (default 200 ms)
  // before it stores the header and rings the doorbell, so another producer's
  // later packet (and doorbell) overtakes it (tests/test_gpu_parity.py).
  POW_AQL_EXP_STALL_HEADER = 512,
};
// Closes the dispatcher once its last packet has completed (a bounded wait,
// ~1 s).  true = closed (null is); false = the wait ran out or the queue is
// dead with a packet still counted in flight: nothing is freed or destroyed
// (a pending packet may still read its argument slot and write the caller's
// buffers), so the caller must keep what those packets may write.
bool pow_aql_close(pow_aql* a);
// 0 = the last launch completed, 1 = still running, < 0 = the queue reported
// an error (minus the HSA status).
int pow_aql_status(const pow_aql* a);
// One packet: `workgroups` x `wg_size` work-items of `kernel`, its explicit
// arguments `args` (exactly the kernel's kernarg size).  0 = dispatched;
// -1 = refused or failed (*why, if given, says why: a bad argument, a queue
// error, or no free packet slot before `deadline_ns` on CLOCK_MONOTONIC).  A
// failure after the packet's index was reserved leaves that slot INVALID on
// the shared queue, which the packet processor cannot get past: the queue is
// then marked dead (kQueueDead), so every context on it goes back to the HIP
// launch path instead of timing out one by one.
int pow_aql_dispatch(pow_aql* a, int kernel, uint32_t workgroups, uint32_t wg_size, const void* args,
                     uint32_t nbytes, uint64_t deadline_ns, std::string* why);
// The watchdog's view of the context's last packet: completion-signal value,
// the queue's read and write index, the packet's index and the header now in
// its slot, the queue's error state.
std::string pow_aql_diag(const pow_aql* a);
