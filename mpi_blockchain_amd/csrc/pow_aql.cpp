// Direct AQL dispatch of the one-block and latency kernels (K2' pow_hash_one,
// K1' pow_search_lat): an AQL kernel-dispatch packet written into an HSA queue
// of the library's own and its doorbell rung, instead of hipLaunchKernel.
//
// TEST LIBRARY ONLY since round 5 (libpow_gpu_test.so, opt-in with POW_AQL=1).
// It saved 1-2 us per launch at d <= 13 and nothing above (DESIGN.md §4 K2'),
// and the one unexplained protocol failure of round 4 happened under it, so
// the shipped libpow_gpu.so launches every kernel through hipLaunchKernel.  It
// stays here for the dispatch A/B (tools/abttb_sweep.sh) and for the
// multi-producer ordering test (POW_AQL_EXP_STALL_HEADER below).
//
// What is dispatched is the library's own code: the gfx950 code object is
// copied out of the offload bundle embedded in this shared library's file (the
// bundle hipcc linked in, so it cannot be stale), loaded once per device into
// an HSA executable and looked up by symbol.  Every kernel dispatched here
// reads only explicit arguments (no hidden ones: K1' takes its workgroup count
// in PowLaunchLat::nwg), and the loader checks each symbol's kernarg size
// against the argument structs before anything is dispatched.
//
// Memory protocol of a dispatch:
//  * arguments: a ring of device memory, uncached on the GPU side, written by
//    the host through the BAR (pow_aql_open checks the host can reach it);
//    then an HDP flush and a read-back of the last word, so they are in HBM
//    before the doorbell;
//  * acquire fence at AGENT scope: no L2 invalidate at the start of every
//    launch (at system scope K1' at d = 9 ran 17 us instead of 15: its code
//    and tables came from HBM again);
//  * release fence at system scope, and a completion signal per context that
//    counts its launches in flight, so a launch that ends without publishing
//    its result is still seen;
//  * one queue per device and process (pow_aql_open), HSA_QUEUE_TYPE_MULTI,
//    packets without the barrier bit: each context orders its own launches by
//    waiting for each one's result.
// Multi-producer ordering ("the ordering argument"): a producer
// reserves its index (atomic add on the write index), waits for the slot to be
// free (read index > idx - size), writes the body, stores the 32-bit
// header+setup word with release semantics, then rings the doorbell with idx.
// It relies on three statements of hsa.h (ROCm 7.2): every slot starts
// INVALID (hsa.h:2368-2371) and a processed slot is INVALID again ("processed
// in the past, but not reassigned", hsa.h:2815-2818); a packet processor must
// not process an INVALID packet (hsa.h:2818-2819); and on a MULTI queue the
// doorbell "can be updated with any value" (hsa.h:2343-2346), i.e. out of
// order.  tests/test_gpu_parity.py::test_direct_dispatch_stalled_producer
// forces the case that matters (a later producer's header and doorbell before
// an earlier producer's header).
// Any failure to set this up leaves the caller on the HIP launch path (the
// same kernels).
#include <dlfcn.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "pow_aql.h"
#include "pow_template.h"

namespace {

constexpr uint32_t kQueueSize = 64;         // argument slots per context (and packets of an own queue)
constexpr uint32_t kSharedQueueSize = 256;  // packets of the device's shared queue
constexpr uint32_t kSlotBytes = 2048;       // kernel-argument slot (largest: K1', 1,568 B)
constexpr int kMaxDevices = 64;

const char* kNames[POW_AQL_NKERNELS] = {
    "_Z12pow_hash_one6PowMsgP10PowHashOutj.kd",
    "_Z14pow_search_latILb0ELb0ELb0EEv12PowConstsLat12PowLaunchLatP9PowResultS3_.kd",
    "_Z14pow_search_latILb1ELb0ELb0EEv12PowConstsLat12PowLaunchLatP9PowResultS3_.kd",
    "_Z14pow_search_latILb0ELb1ELb0EEv12PowConstsLat12PowLaunchLatP9PowResultS3_.kd",
    "_Z14pow_search_latILb1ELb1ELb0EEv12PowConstsLat12PowLaunchLatP9PowResultS3_.kd",
    "_Z14pow_search_latILb0ELb0ELb1EEv12PowConstsLat12PowLaunchLatP9PowResultS3_.kd",
    "_Z14pow_search_latILb1ELb0ELb1EEv12PowConstsLat12PowLaunchLatP9PowResultS3_.kd",
    "_Z14pow_search_latILb0ELb1ELb1EEv12PowConstsLat12PowLaunchLatP9PowResultS3_.kd",
    "_Z14pow_search_latILb1ELb1ELb1EEv12PowConstsLat12PowLaunchLatP9PowResultS3_.kd",
};

// Explicit argument bytes of each kernel: its parameters in declaration
// order, each at its natural alignment (the structs are multiples of 8).
constexpr uint32_t kHashArgs = (uint32_t)(sizeof(PowMsg) + 8 + 4);  // M, hout, seq
constexpr uint32_t kLatArgs = (uint32_t)(sizeof(PowConstsLat) + sizeof(PowLaunchLat) + 8 + 8);  // C, L, res, hout
static_assert(sizeof(PowMsg) % 8 == 0 && sizeof(PowConstsLat) % 8 == 0 && sizeof(PowLaunchLat) % 8 == 0,
              "argument offsets");
static_assert(kLatArgs <= kSlotBytes && kHashArgs <= kSlotBytes, "slot size");

// The kernels of one device, loaded once per process and released at its
// exit (release_all), before the HIP runtime's own teardown.
struct DeviceKernels {
  bool tried = false, ok = false;
  std::string why;
  hsa_agent_t agent{};
  uint32_t* hdp_flush = nullptr;  // HDP_MEM_FLUSH_CNTL: the host's device-memory writes become visible
  struct Kern {
    uint64_t object = 0;
    uint32_t kernarg = 0, group = 0, priv = 0;
  } k[POW_AQL_NKERNELS];
  // The device's dispatch queue, shared by every context of the process
  // (created at the first pow_aql_open, destroyed by release_all at exit)
  hsa_queue_t* queue = nullptr;
  int queue_users = 0;  // open contexts on it: the last to close destroys it (it holds one of the GPU's 24 queue slots)
  std::atomic<int> queue_error{0};
  bool hsa_up = false, reader_up = false, exe_up = false;
  hsa_code_object_reader_t reader{};
  hsa_executable_t exe{};
  std::vector<char> code;  // the code object the reader was made from
};

std::mutex g_mu;
DeviceKernels g_dev[kMaxDevices];
bool g_atexit = false;

// At process exit: the shared queues, the executables and this library's
// reference on the HSA runtime (hsa_init is reference-counted), so the
// runtime's own teardown (HIP's, registered before this one, so it runs after
// it) finds nothing of ours and joins its threads.  Contexts still open at
// exit have no launch in flight (every launch is host-waited).
void release_all() {
  std::lock_guard<std::mutex> g(g_mu);
  for (DeviceKernels& D : g_dev) {
    if (D.queue) hsa_queue_destroy(D.queue);
    if (D.exe_up) hsa_executable_destroy(D.exe);
    if (D.reader_up) hsa_code_object_reader_destroy(D.reader);
    if (D.hsa_up) hsa_shut_down();
    D.queue = nullptr;
    D.ok = D.exe_up = D.reader_up = D.hsa_up = false;
  }
}

// The HSA agent of HIP device `device` (the current device): the owner of a
// probe allocation made on it.  Matching on PCI bus/device/domain is not
// enough: in a partition mode (CPX, DPX) several agents share them and differ
// only in the function bits.  Without the pointer query, a BDF match is used
// only when it is unique.
struct AgentSearch {
  uint32_t bdf, domain;
  hsa_agent_t found{};
  int matches = 0;
};

hsa_status_t match_agent(hsa_agent_t a, void* p) {
  AgentSearch* s = static_cast<AgentSearch*>(p);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0, dom = 0;
  hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
  hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
  if ((bdf & 0xFFF8u) == (s->bdf & 0xFFF8u) && dom == s->domain) {
    if (s->matches++ == 0) s->found = a;
  }
  return HSA_STATUS_SUCCESS;
}

bool device_agent(int device, const hipDeviceProp_t& prop, hsa_agent_t* out, std::string& why) {
  void* probe = nullptr;
  if (hipSetDevice(device) == hipSuccess && hipMalloc(&probe, 64) == hipSuccess) {
    hsa_amd_pointer_info_t info{};
    info.size = sizeof info;
    const bool ok = hsa_amd_pointer_info(probe, &info, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
                    info.type == HSA_EXT_POINTER_TYPE_HSA && info.agentOwner.handle != 0;
    (void)hipFree(probe);
    if (ok) {
      *out = info.agentOwner;
      return true;
    }
  }
  AgentSearch s{((uint32_t)prop.pciBusID << 8) | ((uint32_t)prop.pciDeviceID << 3), (uint32_t)prop.pciDomainID};
  if (hsa_iterate_agents(match_agent, &s) != HSA_STATUS_SUCCESS || s.matches != 1) {
    why = s.matches > 1 ? "several HSA agents share the device's PCI address (partition mode)" : "no HSA agent for the device";
    return false;
  }
  *out = s.found;
  return true;
}

// The gfx950 code object holding the kernels, out of the offload bundles that
// hipcc embedded in this library's file (one bundle per translation unit with
// device code; the one naming pow_hash_one is pow_kernels.hip's).
bool own_code_object(std::vector<char>& out, std::string& why) {
  Dl_info info;
  if (!dladdr((const void*)&pow_aql_open, &info) || !info.dli_fname) {
    why = "dladdr failed";
    return false;
  }
  const int fd = open(info.dli_fname, O_RDONLY);
  if (fd < 0) {
    why = std::string("cannot open ") + info.dli_fname;
    return false;
  }
  struct stat st;
  std::vector<char> file;
  if (fstat(fd, &st) == 0 && st.st_size > 0) {
    file.resize((size_t)st.st_size);
    size_t got = 0;
    while (got < file.size()) {
      const ssize_t n = read(fd, file.data() + got, file.size() - got);
      if (n <= 0) break;
      got += (size_t)n;
    }
    file.resize(got);
  }
  close(fd);
  static const char kMagic[] = "__CLANG_OFFLOAD_BUNDLE__";
  static const char kTriple[] = "hipv4-amdgcn-amd-amdhsa--gfx950";
  static const char kNeedle[] = "_Z12pow_hash_one";
  const char* base = file.data();
  const size_t n = file.size();
  for (size_t i = 0; i + 32 <= n; ++i) {
    if (memcmp(base + i, kMagic, 24) != 0) continue;
    uint64_t entries = 0;
    memcpy(&entries, base + i + 24, 8);
    size_t off = i + 32;
    for (uint64_t e = 0; e < entries && e < 16 && off + 24 <= n; ++e) {
      uint64_t o = 0, sz = 0, tl = 0;
      memcpy(&o, base + off, 8);
      memcpy(&sz, base + off + 8, 8);
      memcpy(&tl, base + off + 16, 8);
      off += 24;
      if (tl > 256 || off + tl > n) break;
      const std::string triple(base + off, (size_t)tl);
      off += tl;
      if (triple != kTriple || sz == 0 || o > n - i || sz > n - i - o) continue;
      const char* co = base + i + o;
      if (std::search(co, co + sz, kNeedle, kNeedle + sizeof kNeedle - 1) == co + sz) continue;
      out.assign(co, co + sz);
      return true;
    }
  }
  why = "no gfx950 code object with the kernels in the library's offload bundles";
  return false;
}

// Load (once) the kernels for `device`; the caller holds g_mu.
DeviceKernels* device_kernels(int device) {
  DeviceKernels& D = g_dev[device];
  if (D.tried) return &D;
  D.tried = true;
  auto bail = [&](const std::string& why) {
    D.why = why;
    return &D;
  };
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return bail("hipGetDeviceProperties");
  if (hsa_init() != HSA_STATUS_SUCCESS) return bail("hsa_init");  // reference-counted; the HIP runtime holds one
  D.hsa_up = true;
  if (!g_atexit) g_atexit = atexit(release_all) == 0;
  if (!device_agent(device, prop, &D.agent, D.why)) return bail(D.why);
  if (!own_code_object(D.code, D.why)) return bail(D.why);
  if (hsa_code_object_reader_create_from_memory(D.code.data(), D.code.size(), &D.reader) != HSA_STATUS_SUCCESS)
    return bail("hsa_code_object_reader_create_from_memory");
  D.reader_up = true;
  if (hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &D.exe) !=
      HSA_STATUS_SUCCESS)
    return bail("hsa_executable_create_alt");
  D.exe_up = true;
  if (hsa_executable_load_agent_code_object(D.exe, D.agent, D.reader, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
      hsa_executable_freeze(D.exe, nullptr) != HSA_STATUS_SUCCESS)
    return bail("loading the code object");
  for (int i = 0; i < POW_AQL_NKERNELS; ++i) {
    hsa_executable_symbol_t sym;
    DeviceKernels::Kern& K = D.k[i];
    if (hsa_executable_get_symbol_by_name(D.exe, kNames[i], &D.agent, &sym) != HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &K.object) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &K.kernarg) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &K.group) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &K.priv) !=
            HSA_STATUS_SUCCESS)
      return bail(std::string("symbol ") + kNames[i]);
    // The bytes the host writes must be exactly what the kernel reads: explicit
    // arguments only (a kernel with hidden arguments has a larger segment).
    if (K.kernarg != (i == POW_AQL_HASH_ONE ? kHashArgs : kLatArgs))
      return bail(std::string("kernarg size of ") + kNames[i] + " is " + std::to_string(K.kernarg));
  }
  hsa_amd_hdp_flush_t hdp{};
  if (hsa_agent_get_info(D.agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &hdp) != HSA_STATUS_SUCCESS ||
      !hdp.HDP_MEM_FLUSH_CNTL)
    return bail("no HDP flush register");
  D.hdp_flush = hdp.HDP_MEM_FLUSH_CNTL;
  D.ok = true;
  return &D;
}

}  // namespace

struct pow_aql {
  const DeviceKernels* dk = nullptr;
  unsigned flags = 0;        // POW_AQL_EXP_* (test library experiments)
  hsa_queue_t* q = nullptr;  // the device's shared queue, or (POW_AQL_EXP_OWN_QUEUE) this context's own
  bool own_q = false;
  std::atomic<int> own_error{0};
  std::atomic<int>* queue_error = nullptr;  // set by the queue's error callback
  hsa_signal_t done{};       // completion signal: this context's launches in flight
  bool signal_up = false;
  uint8_t* ring = nullptr;   // kernel-argument slots: device memory the host writes
  int ring_kind = 0;         // 1 host memory, 2 device memory
  uint32_t next_slot = 0;    // this context's launches so far (ring slot = next_slot % kQueueSize)
  uint64_t last_idx = ~0ull; // packet index of this context's last dispatch (the watchdog's diagnostic)
  unsigned stall_us = 0;     // POW_AQL_EXP_STALL_HEADER: sleep between body and header
};

namespace {
// The value the host stores into a queue's error word when it abandons a
// reserved packet slot (not an HSA status): the queue is dead from then on.
constexpr int kQueueDead = 0x7D0D;

void on_queue_error(hsa_status_t st, hsa_queue_t*, void* data) {
  static_cast<std::atomic<int>*>(data)->store((int)st, std::memory_order_release);
}

uint64_t now_ns() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}
}  // namespace

int pow_aql_open(int device, unsigned flags, pow_aql** out, std::string* why) {
  *out = nullptr;
  if (device < 0 || device >= kMaxDevices) {
    if (why) *why = "device index";
    return -1;
  }
  // One queue per device and process, shared by its contexts: a pow_node rank
  // has two (mining, validation), and a network of ranks on one GPU would
  // otherwise hold two user-mode queues per rank beside HIP's own.  Packets
  // carry no barrier bit, so a validation is not held behind a running
  // latency search of another context: each context orders its own launches
  // by waiting for each one's result.
  DeviceKernels* dk;
  hsa_queue_t* shared = nullptr;
  {
    std::lock_guard<std::mutex> g(g_mu);
    dk = device_kernels(device);
    if (dk->ok && !dk->queue && !(flags & POW_AQL_EXP_OWN_QUEUE)) {
      dk->queue_error.store(0, std::memory_order_relaxed);  // a fresh queue
      if (hsa_queue_create(dk->agent, kSharedQueueSize, HSA_QUEUE_TYPE_MULTI, on_queue_error, &dk->queue_error,
                           UINT32_MAX, UINT32_MAX, &dk->queue) != HSA_STATUS_SUCCESS)
        dk->queue = nullptr;
    }
    shared = dk->queue;
    // A queue that has reported an error is dead: new contexts stay on the
    // HIP launch path (the last context closing destroys it).
    if (shared && !(flags & POW_AQL_EXP_OWN_QUEUE) && dk->queue_error.load(std::memory_order_acquire)) shared = nullptr;
    if (shared && !(flags & POW_AQL_EXP_OWN_QUEUE)) ++dk->queue_users;
  }
  if (!dk->ok) {
    if (why) *why = dk->why;
    return -1;
  }
  if (!shared && !(flags & POW_AQL_EXP_OWN_QUEUE)) {
    if (why) *why = dk->queue ? "the device's dispatch queue reported an error" : "hsa_queue_create";
    return -1;
  }
  pow_aql* a = new pow_aql;
  a->dk = dk;
  a->flags = flags;
  a->q = (flags & POW_AQL_EXP_OWN_QUEUE) ? nullptr : shared;  // (its own queue is made below)
  a->queue_error = &dk->queue_error;
  if (flags & POW_AQL_EXP_STALL_HEADER) {
    const char* e = getenv("POW_AQL_STALL_US");
    a->stall_us = e ? (unsigned)strtoul(e, nullptr, 0) : 200000u;
  }
  auto bail = [&](const char* w) {
    if (why) *why = w;
    pow_aql_close(a);
    return -1;
  };
  const size_t ring_bytes = (size_t)kQueueSize * kSlotBytes;
  if (flags & POW_AQL_EXP_HOST_ARGS) {
    a->ring_kind = 1;
    if (hipHostMalloc((void**)&a->ring, ring_bytes, hipHostMallocCoherent) != hipSuccess)
      return bail("kernel-argument ring");
  } else {
    // Device memory the host writes through the BAR, uncached on the GPU
    // side: no L2 line can hold a slot's previous arguments, so the packets
    // need no L2 invalidate (agent-scope acquire; see pow_aql_dispatch).
    a->ring_kind = 2;
    if (hipExtMallocWithFlags((void**)&a->ring, ring_bytes,
                              (flags & POW_AQL_EXP_FINE_ARGS) ? hipDeviceMallocFinegrained
                                                              : hipDeviceMallocUncached) != hipSuccess)
      return bail("kernel-argument ring");
    // The host writes the ring with plain stores: it must be mapped into the
    // host's address space (large BAR).  Otherwise the first dispatch would
    // fault instead of taking the HIP launch path.
    hsa_amd_pointer_info_t info{};
    info.size = sizeof info;
    if (hsa_amd_pointer_info(a->ring, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS || !info.hostBaseAddress)
      return bail("the kernel-argument ring is not host-accessible (no large BAR)");
  }
  // A signal only the GPU's packet processor writes and the host reads: no
  // interrupt event behind it (the host never sleeps on it).
  if (hsa_amd_signal_create(0, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &a->done) != HSA_STATUS_SUCCESS &&
      hsa_signal_create(0, 0, nullptr, &a->done) != HSA_STATUS_SUCCESS)
    return bail("completion signal");
  a->signal_up = true;
  if (flags & POW_AQL_EXP_OWN_QUEUE) {
    a->queue_error = &a->own_error;
    if (hsa_queue_create(dk->agent, kQueueSize, HSA_QUEUE_TYPE_SINGLE, on_queue_error, &a->own_error, UINT32_MAX,
                         UINT32_MAX, &a->q) != HSA_STATUS_SUCCESS) {
      a->q = nullptr;
      return bail("hsa_queue_create");
    }
    a->own_q = true;
  }
  *out = a;
  return 0;
}

bool pow_aql_close(pow_aql* a) {
  if (!a) return true;
  // Launches are host-waited, so none of this context's is in flight unless
  // one failed mid-flight: wait (bounded, ~1 s) for the last one to complete
  // before its argument ring and signal go.
  const bool sig = a->signal_up && a->q && !(a->flags & POW_AQL_EXP_NO_SIGNAL);
  for (int n = 0; n < 1000000 && sig && hsa_signal_load_scacquire(a->done) != 0 &&
                  !a->queue_error->load(std::memory_order_acquire);
       ++n)
    usleep(1);
  // Still counted in flight (the wait ran out, or the queue died under it):
  // the packet may still run, so its argument slot, its signal, the queue and
  // the caller's buffers stay as they are (leaked, not freed under it).
  if (sig && hsa_signal_load_scacquire(a->done) != 0) return false;
  if (a->own_q) hsa_queue_destroy(a->q);
  if (a->q && !a->own_q) {  // the last context on the shared queue gives its slot back
    std::lock_guard<std::mutex> g(g_mu);
    DeviceKernels* dk = const_cast<DeviceKernels*>(a->dk);
    if (dk->queue == a->q && --dk->queue_users == 0) {
      hsa_queue_destroy(dk->queue);
      dk->queue = nullptr;
    }
  }
  if (a->signal_up) hsa_signal_destroy(a->done);
  if (a->ring) (void)(a->ring_kind == 1 ? hipHostFree(a->ring) : hipFree(a->ring));
  delete a;
  return true;
}

int pow_aql_status(const pow_aql* a) {
  const int e = a->queue_error->load(std::memory_order_acquire);
  if (e) return -e;
  if (a->flags & POW_AQL_EXP_NO_SIGNAL) return 1;
  return hsa_signal_load_scacquire(a->done) == 0 ? 0 : 1;
}

std::string pow_aql_diag(const pow_aql* a) {
  char buf[320];
  const hsa_queue_t* q = a->q;
  const uint64_t rd = hsa_queue_load_read_index_scacquire(q), wr = hsa_queue_load_write_index_scacquire(q);
  uint32_t word = 0;
  if (a->last_idx != ~0ull)
    word = __atomic_load_n((const uint32_t*)((const hsa_kernel_dispatch_packet_t*)q->base_address + (a->last_idx % q->size)),
                           __ATOMIC_ACQUIRE);
  const long long sig = a->signal_up ? (long long)hsa_signal_load_scacquire(a->done) : -1;
  snprintf(buf, sizeof buf,
           "completion signal %lld (launches in flight), queue read index %llu, write index %llu, "
           "this context's last packet index %lld, header at its slot 0x%04x (type %u; 1 = INVALID), queue error 0x%x",
           sig, (unsigned long long)rd, (unsigned long long)wr, a->last_idx == ~0ull ? -1ll : (long long)a->last_idx,
           word & 0xFFFFu, (word >> HSA_PACKET_HEADER_TYPE) & ((1u << HSA_PACKET_HEADER_WIDTH_TYPE) - 1u),
           (unsigned)a->queue_error->load(std::memory_order_acquire));
  return buf;
}

int pow_aql_dispatch(pow_aql* a, int kernel, uint32_t workgroups, uint32_t wg_size, const void* args,
                     uint32_t nbytes, uint64_t deadline_ns, std::string* why) {
  auto refuse = [&](const char* w) {
    if (why) *why = w;
    return -1;
  };
  if (kernel < 0 || kernel >= POW_AQL_NKERNELS || !args || workgroups == 0 || wg_size == 0 || wg_size > 1024 ||
      (uint64_t)workgroups * wg_size > 0xFFFFFFFFull)
    return refuse("bad launch geometry");
  const DeviceKernels::Kern& K = a->dk->k[kernel];
  if (nbytes != K.kernarg) return refuse("argument size");
  if (a->queue_error->load(std::memory_order_acquire)) return refuse("the queue reported an error");
  hsa_queue_t* q = a->q;
  // This context's argument slot: its launches are host-waited, so the slot's
  // previous user (kQueueSize launches ago) has finished reading it.
  uint8_t* arg = a->ring + (size_t)kSlotBytes * (a->next_slot++ % kQueueSize);
  memcpy(arg, args, nbytes);
  // Device memory written over PCIe: drain the write-combining buffers, flush
  // the HDP, and read a word back, so the kernel reads the new arguments.
  __builtin_ia32_sfence();
  if (a->flags & POW_AQL_EXP_READBACK_ONLY) {
    // no HDP flush: store the last word again, full fence, read it back
    memcpy(arg + nbytes - 4, (const uint8_t*)args + nbytes - 4, 4);
    __builtin_ia32_mfence();
    (void)*(volatile uint32_t*)(arg + nbytes - 4);
    __builtin_ia32_lfence();
  } else if (!(a->flags & (POW_AQL_EXP_NO_FLUSH | POW_AQL_EXP_HOST_ARGS))) {
    // (a register every context of the process writes: an atomic store)
    __atomic_store_n((volatile uint32_t*)a->dk->hdp_flush, 1u, __ATOMIC_RELAXED);
    if (!(a->flags & POW_AQL_EXP_NO_READBACK)) (void)*(volatile uint32_t*)(arg + nbytes - 4);
  }
  // The packet slot is free once the packet processor has read past
  // idx - size (at most a few packets are ever outstanding).  A slot that
  // stays busy past the deadline means the packet processor has stopped
  // consuming this queue: the reserved slot is left INVALID (nothing may be
  // written into a slot the processor has not released), and the caller gets
  // the error and the diagnostic.
  // Either way the queue is then marked dead (kQueueDead): the packet
  // processor stops at the INVALID slot, so every later packet of every
  // context on the queue would stall; aql_usable sends them all back to the
  // HIP launch path instead.
  const uint64_t idx = hsa_queue_add_write_index_scacq_screl(q, 1);
  a->last_idx = idx;
  for (uint32_t n = 0; idx - hsa_queue_load_read_index_scacquire(q) >= q->size; ++n) {
    if (a->queue_error->load(std::memory_order_acquire)) {
      int zero = 0;
      a->queue_error->compare_exchange_strong(zero, kQueueDead, std::memory_order_acq_rel);
      return refuse("the queue reported an error");
    }
    if ((n & 1023u) == 1023u && now_ns() > deadline_ns) {
      int zero = 0;
      a->queue_error->compare_exchange_strong(zero, kQueueDead, std::memory_order_acq_rel);
      return refuse("no free packet slot before the deadline; the queue is marked dead");
    }
  }
  // in flight += 1; the packet processor subtracts 1 when the launch
  // completes (which may be after the caller has seen the kernel's done word
  // and started the next launch: a count, not a flag)
  const bool sig = !(a->flags & POW_AQL_EXP_NO_SIGNAL);
  if (sig) hsa_signal_add_scacq_screl(a->done, 1);
  hsa_kernel_dispatch_packet_t* pk = (hsa_kernel_dispatch_packet_t*)q->base_address + (idx % q->size);
  memset((uint8_t*)pk + 4, 0, sizeof *pk - 4);  // everything but header + setup, which go last
  pk->workgroup_size_x = (uint16_t)wg_size;
  pk->workgroup_size_y = 1;
  pk->workgroup_size_z = 1;
  pk->grid_size_x = workgroups * wg_size;
  pk->grid_size_y = 1;
  pk->grid_size_z = 1;
  pk->private_segment_size = K.priv;
  pk->group_segment_size = K.group;
  pk->kernel_object = K.object;
  pk->kernarg_address = arg;
  if (sig) pk->completion_signal = a->done;
  const uint16_t header = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                     (a->own_q ? (1 << HSA_PACKET_HEADER_BARRIER) : 0) |
                                     (((a->flags & POW_AQL_EXP_ACQUIRE_SYSTEM) ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_AGENT)
                                      << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                     (((a->flags & POW_AQL_EXP_RELEASE_AGENT) ? HSA_FENCE_SCOPE_AGENT : HSA_FENCE_SCOPE_SYSTEM)
                                      << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  // The ordering test's hook: a producer descheduled between its reservation
  // and its header store, while other producers' later packets go in.
  if (a->stall_us) usleep(a->stall_us);
  __atomic_store_n((uint32_t*)pk, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
  return 0;
}
