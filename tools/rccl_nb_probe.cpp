// Probe: RCCL's non-blocking init and abort, step by step, for a rank whose
// peer never joins (the case pow_group_init's deadline is for).  Prints every
// call and its result with a timestamp, unbuffered, so a hang shows where.
//   tools/rccl_nb_probe [nranks] [poll_s]
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <thread>

static double t0;
static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define SAY(...) (fprintf(stderr, "[%7.3f] ", now() - t0), fprintf(stderr, __VA_ARGS__), fputc('\n', stderr))

int main(int argc, char** argv) {
  t0 = now();
  const int nranks = argc > 1 ? atoi(argv[1]) : 2;
  const double poll_s = argc > 2 ? atof(argv[2]) : 3.0;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) return SAY("dlopen: %s", dlerror()), 1;
  auto get_id = (decltype(&ncclGetUniqueId))dlsym(h, "ncclGetUniqueId");
  auto init_cfg = (decltype(&ncclCommInitRankConfig))dlsym(h, "ncclCommInitRankConfig");
  auto async_err = (decltype(&ncclCommGetAsyncError))dlsym(h, "ncclCommGetAsyncError");
  auto abort_ = (decltype(&ncclCommAbort))dlsym(h, "ncclCommAbort");
  auto estr = (decltype(&ncclGetErrorString))dlsym(h, "ncclGetErrorString");
  SAY("hipSetDevice(0) = %d", (int)hipSetDevice(0));
  ncclUniqueId id;
  SAY("ncclGetUniqueId = %s", estr(get_id(&id)));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t c = nullptr;
  SAY("calling ncclCommInitRankConfig(nranks %d, rank 0, blocking 0)", nranks);
  ncclResult_t r = init_cfg(&c, nranks, id, 0, &cfg);
  SAY("ncclCommInitRankConfig = %s, comm %p", estr(r), (void*)c);
  ncclResult_t st = ncclInProgress;
  int polls = 0;
  while (now() - t0 < poll_s + 1.0) {
    SAY("calling ncclCommGetAsyncError (poll %d)", polls);
    r = async_err(c, &st);
    SAY("ncclCommGetAsyncError = %s, state %s", estr(r), estr(st));
    ++polls;
    if (st != ncclInProgress) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(500));
  }
  auto done = std::make_shared<std::atomic<bool>>(false);
  SAY("calling ncclCommAbort on a detached thread");
  std::thread([&, done] {
    ncclResult_t a = abort_(c);
    SAY("ncclCommAbort = %s", estr(a));
    done->store(true);
  }).detach();
  for (int i = 0; i < 100 && !done->load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  SAY("abort %s; exiting", done->load() ? "returned" : "still running after 10 s");
  fflush(stderr);
  return 0;
}
