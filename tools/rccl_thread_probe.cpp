// Probe: which ways of making a communicator on a helper thread survive
// ncclAllReduce + ncclCommDestroy on the calling thread, per RCCL build
// (torch's 2.26.6 aborted the test process in round 6's first try).
// Built as tools/librccl_thread_probe.so and called from tools/rccl_thread_probe.py
// after `import torch` (so it runs on torch's HIP runtime, as pow_group does in
// bench.py and the GPU tests): rccl_thread_probe(<librccl path>, <mode>).
// mode A: helper calls the non-blocking init and exits; the caller polls
//         ncclCommGetAsyncError, all-reduces and destroys (the round-6 draft)
// mode B: the helper also polls ncclCommGetAsyncError until the communicator
//         is ready before it exits
// mode C: the helper calls a blocking init
// mode D: no helper: non-blocking init and everything on the calling thread (round 6's first GPU run)
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

static double t0;
static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define SAY(...) (fprintf(stderr, "[%7.3f] ", now() - t0), fprintf(stderr, __VA_ARGS__), fputc('\n', stderr))

extern "C" int rccl_thread_probe(const char* path, char mode) {
  t0 = now();
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return SAY("dlopen: %s", dlerror()), 1;
  auto get_id = (decltype(&ncclGetUniqueId))dlsym(h, "ncclGetUniqueId");
  auto init_cfg = (decltype(&ncclCommInitRankConfig))dlsym(h, "ncclCommInitRankConfig");
  auto async_err = (decltype(&ncclCommGetAsyncError))dlsym(h, "ncclCommGetAsyncError");
  auto destroy = (decltype(&ncclCommDestroy))dlsym(h, "ncclCommDestroy");
  auto allreduce = (decltype(&ncclAllReduce))dlsym(h, "ncclAllReduce");
  auto estr = (decltype(&ncclGetErrorString))dlsym(h, "ncclGetErrorString");
  int ver = 0;
  ((decltype(&ncclGetVersion))dlsym(h, "ncclGetVersion"))(&ver);
  SAY("RCCL %d, mode %c", ver, mode);
  (void)hipSetDevice(0);
  ncclUniqueId id;
  get_id(&id);
  ncclComm_t c = nullptr;
  ncclResult_t r = ncclInternalError;
  auto settle = [&](const char* who) {
    ncclResult_t st = ncclInProgress;
    int n = 0;
    do {
      async_err(c, &st);
      ++n;
      if (st == ncclInProgress) std::this_thread::sleep_for(std::chrono::microseconds(200));
    } while (st == ncclInProgress);
    SAY("%s: settled to %s after %d polls", who, estr(st), n);
    return st;
  };
  auto init = [&](int blocking, bool settle_here) {
    (void)hipSetDevice(0);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = blocking;
    r = init_cfg(&c, 1, id, 0, &cfg);
    SAY("init (blocking %d) returned %s", blocking, estr(r));
    if (settle_here && r == ncclInProgress) r = settle("init thread");
  };
  if (mode == 'D') {
    init(0, true);
  } else {
    std::thread th(init, mode == 'C' ? 1 : 0, mode == 'B');
    th.join();
    SAY("helper thread exited");
  }
  if (r == ncclInProgress) r = settle("caller");
  uint64_t* d = nullptr;
  uint64_t hv = 42;
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  (void)hipMalloc(&d, 8);
  (void)hipMemcpyAsync(d, &hv, 8, hipMemcpyHostToDevice, st);
  r = allreduce(d, d, 1, ncclUint64, ncclMin, c, st);
  SAY("allreduce returned %s", estr(r));
  if (r == ncclInProgress) settle("allreduce");
  (void)hipMemcpyAsync(&hv, d, 8, hipMemcpyDeviceToHost, st);
  (void)hipStreamSynchronize(st);
  SAY("value after allreduce %llu", (unsigned long long)hv);
  r = destroy(c);
  SAY("destroy returned %s", estr(r));
  (void)hipFree(d);
  (void)hipStreamDestroy(st);
  SAY("ok");
  return 0;
}
