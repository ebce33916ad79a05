// TEST INFRASTRUCTURE ONLY: a stand-in for the RCCL entry points that
// mpi_blockchain_amd/csrc/pow_group.cpp dlopens (rccl.h:187, 204, 220, 260,
// 271, 339, 362, 378, 389, 611), reducing over POSIX shared memory instead of
// xGMI.
//
// RCCL refuses two ranks on one GPU, and a test box has one GPU, so
// pow_group_init's RCCL leg (the board opened before ncclCommInitRank and
// unlinked after it, the d_buf/h_buf staging around ncclAllReduce, the
// {counter, go, ok} consensus) could only run at world size 1.  With this
// library selected by the TEST build's hook (libpow_gpu_test.so,
// POW_TEST_RCCL_LIB) the very same pow_group code runs with 2 and 4 processes
// sharing the GPU (tests/test_shard_gpu.py).  Built by build.build_test_stub();
// never loaded by the shipped libpow_gpu.so, which has no such hook.
//
// Semantics kept from RCCL: ncclCommInitRank blocks until all nranks joined;
// ncclCommInitRankConfig with config->blocking = 0 returns ncclInProgress at
// once and ncclCommGetAsyncError reports ncclInProgress until every rank has
// joined (then ncclSuccess); ncclCommAbort tears down a communicator in any
// state;
// ncclAllReduce takes device buffers and is ordered on the caller's stream
// (the stub synchronises the stream, reduces on the host, and writes the
// result back on the same stream).  Only what pow_group uses is supported:
// ncclUint64, min/max/sum, at most 8 words per call.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace {

constexpr int kMaxRanks = 64;
constexpr size_t kMaxWords = 8;
constexpr char kMagic[8] = {'p', 'o', 'w', 's', 't', 'u', 'b', '1'};
// A rank that never arrives fails the call, it does not hang the test: after
// 120 s, or POW_STUB_TIMEOUT_S (the broken-group tests shorten it; RCCL itself
// has no such bound, pow_group's own deadlines stand in for it).
double timeout_s() {
  static const double t = [] {
    const char* e = getenv("POW_STUB_TIMEOUT_S");
    const double v = e ? atof(e) : 0.0;
    return v > 0 ? v : 120.0;
  }();
  return t;
}

struct Shared {
  std::atomic<uint32_t> joined;
  std::atomic<uint32_t> arrive;  // central barrier: arrivals of the current phase ...
  std::atomic<uint32_t> phase;   // ... and the phase number (bumped by the last arrival)
  uint64_t slot[kMaxRanks][kMaxWords];
};

std::atomic<uint64_t> g_allreduce_calls{0};
std::atomic<uint64_t> g_aborts{0};

double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

void pause_us(long us) {
  timespec t{0, us * 1000};
  nanosleep(&t, nullptr);
}

void shm_name(const ncclUniqueId& id, char out[48]) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a of the id
  for (int i = 0; i < NCCL_UNIQUE_ID_BYTES; ++i) h = (h ^ (uint8_t)id.internal[i]) * 1099511628211ull;
  snprintf(out, 48, "/pow_stub_rccl_%016llx", (unsigned long long)h);
}

}  // namespace

struct ncclComm {
  Shared* sh = nullptr;
  int nranks = 0, rank = 0;
  int device = -1;  // the HIP device current at ncclCommInitRank (as RCCL binds it)
  bool ready = false;  // every rank joined (a non-blocking init is in progress until then)
  char name[48] = {0};
};

namespace {

bool barrier(ncclComm* c) {
  Shared* s = c->sh;
  const uint32_t ph = s->phase.load(std::memory_order_acquire);
  if (s->arrive.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)c->nranks) {
    s->arrive.store(0, std::memory_order_relaxed);
    s->phase.fetch_add(1, std::memory_order_acq_rel);
    return true;
  }
  const double t0 = now_s();
  while (s->phase.load(std::memory_order_acquire) == ph) {
    if (now_s() - t0 > timeout_s()) return false;
    pause_us(20);
  }
  return true;
}

}  // namespace

extern "C" {

// How many all-reduces this process ran through the stub (tests check that the
// stub, not RCCL, carried the group's collectives).
uint64_t pow_stub_rccl_allreduce_calls(void) { return g_allreduce_calls.load(); }
// How many communicators this process aborted (the init-deadline test).
uint64_t pow_stub_rccl_aborts(void) { return g_aborts.load(); }

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  const int fd = open("/dev/urandom", O_RDONLY);
  if (fd < 0) return ncclSystemError;
  const ssize_t n = read(fd, id->internal, sizeof id->internal);
  close(fd);
  if (n != (ssize_t)sizeof id->internal) return ncclSystemError;
  memcpy(id->internal, kMagic, sizeof kMagic);
  return ncclSuccess;
}

namespace {

// Map the id's segment and count this rank in; *out = the communicator, not yet ready.
ncclResult_t comm_join(ncclComm_t* comm, int nranks, const ncclUniqueId& id, int rank) {
  if (!comm || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  if (memcmp(id.internal, kMagic, sizeof kMagic) != 0) return ncclInvalidArgument;  // not a stub id
  *comm = nullptr;
  char name[48];
  shm_name(id, name);
  const int fd = shm_open(name, O_RDWR | O_CREAT, 0600);
  if (fd < 0) return ncclSystemError;
  struct stat st;
  if (fstat(fd, &st) != 0 || (st.st_size < (off_t)sizeof(Shared) && ftruncate(fd, sizeof(Shared)) != 0)) {
    close(fd);
    return ncclSystemError;
  }
  void* p = mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return ncclSystemError;
  ncclComm* c = new ncclComm;
  c->sh = (Shared*)p;  // a fresh object is zero-filled: all counters 0
  c->nranks = nranks;
  c->rank = rank;
  snprintf(c->name, sizeof c->name, "%s", name);
  if (hipGetDevice(&c->device) != hipSuccess) c->device = -1;
  c->sh->joined.fetch_add(1, std::memory_order_acq_rel);
  *comm = c;
  return ncclSuccess;
}

// Every rank has joined: the communicator is ready, and the name can go.
bool comm_ready(ncclComm* c) {
  if (!c->ready && c->sh->joined.load(std::memory_order_acquire) >= (uint32_t)c->nranks) {
    c->ready = true;
    shm_unlink(c->name);  // every rank has it mapped; nothing is left in /dev/shm
  }
  return c->ready;
}

}  // namespace

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  ncclResult_t r = comm_join(comm, nranks, id, rank);
  if (r != ncclSuccess) return r;
  ncclComm* c = *comm;
  // As RCCL: return once every rank has joined.
  const double t0 = now_s();
  while (!comm_ready(c)) {
    if (now_s() - t0 > timeout_s()) {
      munmap(c->sh, sizeof(Shared));
      delete c;
      *comm = nullptr;
      return ncclSystemError;
    }
    pause_us(50);
  }
  return ncclSuccess;
}

ncclResult_t ncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank, ncclConfig_t* config) {
  if (config && config->magic != 0xcafebeef) return ncclInvalidArgument;
  if (!config || config->blocking != 0) return ncclCommInitRank(comm, nranks, id, rank);
  ncclResult_t r = comm_join(comm, nranks, id, rank);
  if (r != ncclSuccess) return r;
  return comm_ready(*comm) ? ncclSuccess : ncclInProgress;
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError) {
  if (!comm || !asyncError) return ncclInvalidArgument;
  *asyncError = comm_ready(comm) ? ncclSuccess : ncclInProgress;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  if (!comm->ready) return ncclInvalidUsage;  // RCCL: an initialising communicator is aborted, not destroyed
  munmap(comm->sh, sizeof(Shared));
  delete comm;
  return ncclSuccess;
}

// As RCCL's: tear the communicator down without waiting for operations in
// flight (the stub has none once a call returns), also one whose non-blocking
// init never completed (its segment's name is removed: nobody else will).
ncclResult_t ncclCommAbort(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  if (!comm->ready) shm_unlink(comm->name);
  munmap(comm->sh, sizeof(Shared));
  delete comm;
  g_aborts.fetch_add(1);
  return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  if (!comm || !count) return ncclInvalidArgument;
  *count = comm->nranks;
  return ncclSuccess;
}

ncclResult_t ncclCommCuDevice(const ncclComm_t comm, int* device) {
  if (!comm || !device) return ncclInvalidArgument;
  *device = comm->device;
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error (stub RCCL)";
    case ncclInvalidArgument: return "invalid argument (stub RCCL)";
    case ncclSystemError: return "system error or timeout (stub RCCL)";
    case ncclUnhandledCudaError: return "HIP error (stub RCCL)";
    default: return "unsupported (stub RCCL)";
  }
}

ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                           ncclRedOp_t op, ncclComm_t comm, hipStream_t stream) {
  if (!comm || datatype != ncclUint64 || count > kMaxWords) return ncclInvalidArgument;
  if (!comm->ready) return ncclInvalidUsage;
  if (op != ncclMin && op != ncclMax && op != ncclSum) return ncclInvalidArgument;
  uint64_t v[kMaxWords] = {0};
  // The operand was staged on `stream` (pow_group: hipMemcpyAsync H2D): read it
  // back on the same stream.  (Never HIP's null stream: that would give every
  // rank of a rehearsal one hardware queue more, and the GPU has 24 for all of
  // them; DESIGN.md §7, "Queue pressure".)
  if (count && hipMemcpyAsync(v, sendbuff, count * 8, hipMemcpyDeviceToHost, stream) != hipSuccess)
    return ncclUnhandledCudaError;
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  Shared* s = comm->sh;
  memcpy(s->slot[comm->rank], v, count * 8);
  if (!barrier(comm)) return ncclSystemError;  // every rank's words are in
  uint64_t r[kMaxWords];
  memcpy(r, s->slot[0], count * 8);
  for (int k = 1; k < comm->nranks; ++k)
    for (size_t i = 0; i < count; ++i) {
      const uint64_t x = s->slot[k][i];
      r[i] = op == ncclMin ? (x < r[i] ? x : r[i]) : op == ncclMax ? (x > r[i] ? x : r[i]) : r[i] + x;
    }
  if (!barrier(comm)) return ncclSystemError;  // every rank has read them: the slots may be reused
  if (count && hipMemcpyAsync(recvbuff, r, count * 8, hipMemcpyHostToDevice, stream) != hipSuccess)
    return ncclUnhandledCudaError;
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  g_allreduce_calls.fetch_add(1);
  return ncclSuccess;
}

}  // extern "C"
