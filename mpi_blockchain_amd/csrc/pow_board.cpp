// Cross-GPU stop board (include/pow_gpu.h): a page of host memory every GPU of
// the node maps, one 64-bit slot per rank of a search.
//
// The reference's ranks each mine their own template and learn of a rival's
// block only through MPI (node.cpp:260-273, 404); a cooperative search over
// several GPUs (BASELINE config 4) needs more: when one GPU finds the winner,
// the others should stop within one inner step, not at the end of their
// launch.  RCCL cannot do that — a collective runs only between kernels — so
// the running kernels poll this page instead: one sentinel wave per launch
// reads the peers' slots over PCIe (pow_kernels.hip: poll_stop), and a hit is
// stored into the finder's own slot from the kernel itself (publish_hit).
//
// Slot encoding: bits 63..54 = the search tag (1..1023, so a slot left over
// from an earlier search is ignored), bits 53..0 = absolute counter
// (62^9 < 2^54), all ones = nothing found yet.
//
//  * name == NULL: a page of this process's memory, shared by its contexts
//    (one host thread per GPU, or tests with several contexts on one GPU);
//  * name != NULL: a POSIX shared-memory page (shm_open + mmap), shared by
//    every process of the node that opens the same name (one process per
//    GPU).  Processes on other nodes open their own page of that name: their
//    cancellation crosses nodes only at round ends (pow_group's all-reduce).
// Either way the page is registered with HIP (hipHostRegister, mapped and
// portable: every GPU of the process gets a device address for it) when the
// first context binds to it, so opening, posting and peeking need no GPU.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "../../include/pow_gpu.h"
#include "pow_template.h"

struct pow_board {
  uint64_t* slots = nullptr;  // host address
  int nslots = 0;
  bool shm = false;           // mmap'ed shared memory (else aligned_alloc)
  std::mutex mu;              // guards `registered` (contexts bind from their own threads)
  bool registered = false;    // hipHostRegister'ed
};

namespace {
constexpr size_t kBoardBytes = 4096;  // one page: 64 slots used
}

uint64_t* pow_board_host_slots(const pow_board* b) { return b ? b->slots : nullptr; }
int pow_board_nslots(const pow_board* b) { return b ? b->nslots : 0; }

// Map the page for the GPUs (once per board; called by pow_board_bind).
int pow_board_register(pow_board* b) {
  std::lock_guard<std::mutex> g(b->mu);
  if (b->registered) return POW_OK;
  hipError_t e = hipHostRegister(b->slots, kBoardBytes, hipHostRegisterMapped | hipHostRegisterPortable);
  if (e != hipSuccess) {
    char msg[320];
    snprintf(msg, sizeof msg, "hipHostRegister board: %s", hipGetErrorString(e));
    return pow_set_error(POW_EHIP, msg);
  }
  b->registered = true;
  return POW_OK;
}

extern "C" {

int pow_board_open(const char* name, int nslots, pow_board** out) {
  if (!out) return pow_set_error(POW_EINVAL, "null out");
  *out = nullptr;
  if (nslots < 1 || nslots > POW_BOARD_MAX_SLOTS) return pow_set_error(POW_EINVAL, "nslots must be 1..64");
  pow_board* b = new pow_board;
  b->nslots = nslots;
  char msg[320];
  if (!name) {
    void* p = aligned_alloc(kBoardBytes, kBoardBytes);
    if (!p) {
      delete b;
      return pow_set_error(POW_EINVAL, "out of memory");
    }
    memset(p, 0, kBoardBytes);
    b->slots = (uint64_t*)p;
    *out = b;
    return POW_OK;
  }
  if (name[0] != '/' || strchr(name + 1, '/') || strlen(name) > 200) {
    delete b;
    return pow_set_error(POW_EINVAL, "board name must look like \"/name\"");
  }
  const int fd = shm_open(name, O_RDWR | O_CREAT, 0600);
  if (fd < 0) {
    delete b;
    snprintf(msg, sizeof msg, "shm_open(%s): %s", name, strerror(errno));
    return pow_set_error(POW_EINVAL, msg);
  }
  struct stat st;
  // A fresh object is 0 bytes and grows to a zero-filled page; an existing one is kept.
  if (fstat(fd, &st) != 0 || (st.st_size < (off_t)kBoardBytes && ftruncate(fd, (off_t)kBoardBytes) != 0)) {
    snprintf(msg, sizeof msg, "sizing %s: %s", name, strerror(errno));
    close(fd);
    delete b;
    return pow_set_error(POW_EINVAL, msg);
  }
  void* p = mmap(nullptr, kBoardBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    delete b;
    snprintf(msg, sizeof msg, "mmap(%s): %s", name, strerror(errno));
    return pow_set_error(POW_EINVAL, msg);
  }
  b->slots = (uint64_t*)p;
  b->shm = true;
  *out = b;
  return POW_OK;
}

int pow_board_unlink(const char* name) {
  if (!name) return pow_set_error(POW_EINVAL, "null name");
  if (shm_unlink(name) != 0 && errno != ENOENT) {
    char msg[320];
    snprintf(msg, sizeof msg, "shm_unlink(%s): %s", name, strerror(errno));
    return pow_set_error(POW_EINVAL, msg);
  }
  return POW_OK;
}

void pow_board_close(pow_board* b) {
  if (!b) return;
  if (b->registered) (void)hipHostUnregister(b->slots);
  if (b->shm) munmap(b->slots, kBoardBytes);
  else free(b->slots);
  delete b;
}

int pow_board_post(pow_board* b, int slot, uint32_t tag, uint64_t ctr) {
  if (!b || slot < 0 || slot >= b->nslots) return pow_set_error(POW_EINVAL, "bad board/slot");
  if (tag < 1 || tag > POW_BOARD_MAX_TAG) return pow_set_error(POW_EINVAL, "tag must be 1..1023");
  const uint64_t v = ((uint64_t)tag << POW_BOARD_SHIFT) | (ctr < POW_BOARD_NONE ? ctr : POW_BOARD_NONE);
  __atomic_store_n(&b->slots[slot], v, __ATOMIC_SEQ_CST);
  return POW_OK;
}

int pow_board_peek(const pow_board* b, int except_slot, uint32_t tag, uint64_t* min_ctr) {
  if (!b || !min_ctr) return pow_set_error(POW_EINVAL, "null");
  uint64_t m = UINT64_MAX;
  for (int i = 0; i < b->nslots; ++i) {
    if (i == except_slot) continue;
    const uint64_t v = __atomic_load_n(&b->slots[i], __ATOMIC_ACQUIRE);
    if ((uint32_t)(v >> POW_BOARD_SHIFT) != tag) continue;
    const uint64_t c = v & POW_BOARD_NONE;
    if (c != POW_BOARD_NONE && c < m) m = c;
  }
  *min_ctr = m;
  return POW_OK;
}

}  // extern "C"
