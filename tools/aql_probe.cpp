// Probe: dispatch K2' (pow_hash_one) by writing an AQL packet into an HSA queue
// directly, instead of through hipLaunchKernel, and compare the call time and
// the digests with pow_hash_block (the HIP path) in the same process.
//
// The code object is the device-only build of pow_kernels.hip
// (mpi_blockchain_amd/pow_kernels_gfx950.hsaco, built by build.py).  The HSA
// queue is this probe's own; the kernel's result words live in HIP-allocated
// mapped host memory (one address space per process).
//
//   g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I /opt/rocm/include -I include -I mpi_blockchain_amd/csrc \
//       tools/aql_probe.cpp -L mpi_blockchain_amd -lpow_gpu -L /opt/rocm/lib -lhsa-runtime64 -lamdhip64 \
//       -Wl,-rpath,$PWD/mpi_blockchain_amd -Wl,-rpath,/opt/rocm/lib -o tools/aql_probe
//   tools/aql_probe mpi_blockchain_amd/pow_kernels_gfx950.hsaco [kernarg: host|dev]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "pow_gpu.h"
#include "pow_template.h"

#define CK(x)                                                              \
  do {                                                                     \
    hsa_status_t s_ = (x);                                                 \
    if (s_ != HSA_STATUS_SUCCESS) {                                        \
      const char* m_ = nullptr;                                            \
      hsa_status_string(s_, &m_);                                          \
      fprintf(stderr, "%s failed: %s (line %d)\n", #x, m_ ? m_ : "?", __LINE__); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

static const uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

struct Found {
  hsa_agent_t gpu{};
  uint32_t want_bdf = 0;
  bool ok = false;
  hsa_region_t kernarg{};
  bool has_kernarg = false;
};

static hsa_status_t find_gpu(hsa_agent_t a, void* p) {
  Found* f = (Found*)p;
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t != HSA_DEVICE_TYPE_GPU) return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0;
  hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
  if ((bdf >> 3) == (f->want_bdf >> 3) && !f->ok) {
    f->gpu = a;
    f->ok = true;
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_kernarg(hsa_region_t r, void* p) {
  Found* f = (Found*)p;
  hsa_region_segment_t seg;
  hsa_region_get_info(r, HSA_REGION_INFO_SEGMENT, &seg);
  if (seg != HSA_REGION_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_region_get_info(r, HSA_REGION_INFO_GLOBAL_FLAGS, &flags);
  if ((flags & HSA_REGION_GLOBAL_FLAG_KERNARG) && !f->has_kernarg) {
    f->kernarg = r;
    f->has_kernarg = true;
  }
  return HSA_STATUS_SUCCESS;
}

static double now_us() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const bool dev_kernarg = argc > 2 && std::string(argv[2]) == "dev";
  // HIP side: the library context (the reference path) and the mapped result words
  pow_ctx* ctx;
  if (pow_init(0, &ctx) || pow_warmup(ctx)) return 1;
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  PowHashOut* h_out = nullptr;
  hipHostMalloc((void**)&h_out, sizeof(PowHashOut), hipHostMallocMapped | hipHostMallocCoherent);
  memset(h_out, 0, sizeof *h_out);
  PowHashOut* d_out = nullptr;
  hipHostGetDevicePointer((void**)&d_out, h_out, 0);

  CK(hsa_init());
  Found f;
  f.want_bdf = ((uint32_t)prop.pciBusID << 8) | ((uint32_t)prop.pciDeviceID << 3);
  CK(hsa_iterate_agents(find_gpu, &f));
  if (!f.ok) {
    fprintf(stderr, "no HSA agent with BDF %x\n", f.want_bdf);
    return 1;
  }
  CK(hsa_agent_iterate_regions(f.gpu, find_kernarg, &f));
  if (!f.has_kernarg) return 1;
  hsa_file_t fd = open(argv[1], O_RDONLY);
  hsa_code_object_reader_t rd;
  CK(hsa_code_object_reader_create_from_file(fd, &rd));
  hsa_executable_t exe;
  CK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
  CK(hsa_executable_load_agent_code_object(exe, f.gpu, rd, nullptr, nullptr));
  CK(hsa_executable_freeze(exe, nullptr));
  hsa_executable_symbol_t sym;
  CK(hsa_executable_get_symbol_by_name(exe, "_Z12pow_hash_one6PowMsgP10PowHashOutj.kd", &f.gpu, &sym));
  uint64_t kobj = 0;
  uint32_t ka_size = 0, grp = 0, priv = 0;
  CK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj));
  CK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &ka_size));
  CK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &grp));
  CK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &priv));
  printf("kernel object %llx kernarg %u group %u private %u\n", (unsigned long long)kobj, ka_size, grp, priv);
  if (ka_size < 1292 || ka_size > 4096) return 1;
  hsa_queue_t* q;
  CK(hsa_queue_create(f.gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
  const size_t slot = 2048;
  uint8_t* ka = nullptr;
  if (dev_kernarg) {
    // device memory the host writes through the BAR (fine-grained VRAM, CPU access allowed)
    if (hipExtMallocWithFlags((void**)&ka, slot * q->size, hipDeviceMallocFinegrained) != hipSuccess) return 1;
  } else {
    CK(hsa_memory_allocate(f.kernarg, slot * q->size, (void**)&ka));
  }

  // blocks: 200 different ones
  std::vector<pow_block> blk(200);
  for (int i = 0; i < 200; ++i) {
    memset(&blk[i], 0, sizeof blk[i]);
    blk[i].index = 3 + i;
    blk[i].node_owner_number = i % 7;
    blk[i].difficulty = 9;
    blk[i].created_at = 1700000000 + i;
    for (int k = 0; k < 9; ++k) blk[i].nonce[k] = 'a' + (i * 7 + k) % 26;
    for (int k = 0; k < 64; ++k) blk[i].previous_block_hash[k] = "0123456789abcdef"[(i + k * 5) % 16];
  }
  std::vector<double> t_aql, t_hip, k_aql, t_prep, t_wait;
  uint32_t seq = 0;
  int bad = 0;
  for (int rep = 0; rep < 5; ++rep) {
    for (int i = 0; i < 200; ++i) {  // AQL path
      const double t0 = now_us();
      uint8_t m[320];
      memset(m, 0, sizeof m);
      pow_block_to_bytes(&blk[i], m);
      m[270] = 0x80;
      const uint64_t bits = 2160;
      for (int k = 0; k < 8; ++k) m[319 - k] = (uint8_t)(bits >> (8 * k));
      const uint64_t idx = hsa_queue_add_write_index_scacq_screl(q, 1);
      while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
      }
      uint8_t* arg = ka + slot * (idx % q->size);
      uint32_t* kw = (uint32_t*)arg;
      for (int c = 0; c < 5; ++c) {
        uint32_t w[64];
        for (int k = 0; k < 16; ++k) {
          const uint8_t* p = m + 64 * c + 4 * k;
          w[k] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
        }
        for (int k = 16; k < 64; ++k) {
          const uint32_t s0 = rotr(w[k - 15], 7) ^ rotr(w[k - 15], 18) ^ (w[k - 15] >> 3);
          const uint32_t s1 = rotr(w[k - 2], 17) ^ rotr(w[k - 2], 19) ^ (w[k - 2] >> 10);
          w[k] = s1 + w[k - 7] + s0 + w[k - 16];
        }
        for (int k = 0; k < 64; ++k) kw[64 * c + k] = kK[k] + w[k];
      }
      ++seq;
      memcpy(arg + 1280, &d_out, 8);
      memcpy(arg + 1288, &seq, 4);
      hsa_kernel_dispatch_packet_t* pk = (hsa_kernel_dispatch_packet_t*)q->base_address + (idx % q->size);
      memset((uint8_t*)pk + 4, 0, sizeof *pk - 4);
      pk->workgroup_size_x = 64;
      pk->workgroup_size_y = 1;
      pk->workgroup_size_z = 1;
      pk->grid_size_x = 64;
      pk->grid_size_y = 1;
      pk->grid_size_z = 1;
      pk->private_segment_size = priv;
      pk->group_segment_size = grp;
      pk->kernel_object = kobj;
      pk->kernarg_address = arg;
      pk->completion_signal.handle = 0;
      const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                              (1 << HSA_PACKET_HEADER_BARRIER) |
                              (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                              (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
      const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
      __atomic_store_n((uint32_t*)pk, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
      const double td = now_us();
      hsa_signal_store_screlease(q->doorbell_signal, idx);
      const double tw = now_us();
      t_prep.push_back(td - t0);
      while (__atomic_load_n(&h_out->done, __ATOMIC_ACQUIRE) != seq) {
        if (now_us() - tw > 2e6) {
          fprintf(stderr, "AQL dispatch timed out\n");
          return 1;
        }
      }
      const double t1 = now_us();
      t_wait.push_back(t1 - tw);
      char hx[65];
      static const char hexd[] = "0123456789abcdef";
      for (int k = 0; k < 8; ++k)
        for (int b = 0; b < 4; ++b) {
          const uint8_t byte = (uint8_t)(h_out->digest[k] >> (24 - 8 * b));
          hx[8 * k + 2 * b] = hexd[byte >> 4];
          hx[8 * k + 2 * b + 1] = hexd[byte & 15];
        }
      hx[64] = 0;
      t_aql.push_back(t1 - t0);
      k_aql.push_back(h_out->ticks / 100.0);
      // the HIP path, same block
      char hx2[65];
      const double t2 = now_us();
      if (pow_hash_block(ctx, &blk[i], nullptr, hx2)) return 1;
      t_hip.push_back(now_us() - t2);
      if (strcmp(hx, hx2) != 0) ++bad;
    }
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  auto p10 = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 10];
  };
  printf("{\"kernarg\": \"%s\", \"calls\": %zu, \"aql_call_us_median\": %.2f, \"aql_call_us_p10\": %.2f, "
         "\"aql_kernel_us_median\": %.2f, \"hip_call_us_median\": %.2f, \"hip_call_us_p10\": %.2f, "
         "\"digest_mismatches\": %d, \"host_prep_us_median\": %.2f, \"doorbell_to_done_us_median\": %.2f}\n",
         dev_kernarg ? "device" : "host", t_aql.size(), med(t_aql), p10(t_aql), med(k_aql), med(t_hip), p10(t_hip),
         bad, med(t_prep), med(t_wait));
  hsa_queue_destroy(q);
  hsa_executable_destroy(exe);
  hsa_code_object_reader_destroy(rd);
  pow_destroy(ctx);
  return bad ? 3 : 0;
}
