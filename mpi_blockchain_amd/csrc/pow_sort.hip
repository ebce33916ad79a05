// Device radix sort of a sweep's solution list (pow_sweep returns counters in
// ascending order; the kernel appends them in completion order).  hipCUB /
// rocPRIM onesweep radix sort, keys only, on the ctx stream.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>
#include <stdint.h>

// Sorts n keys; *sorted receives whichever of (keys, alt) holds the result.
// temp == nullptr: only writes the needed temp size to *temp_bytes.
extern "C++" hipError_t pow_sort_u32(void* temp, size_t* temp_bytes, uint32_t* keys, uint32_t* alt,
                                     uint32_t n, uint32_t** sorted, hipStream_t stream) {
  hipcub::DoubleBuffer<uint32_t> db(keys, alt);
  hipError_t e = hipcub::DeviceRadixSort::SortKeys(temp, *temp_bytes, db, (int)n, 0, 32, stream);
  if (sorted) *sorted = db.Current();
  return e;
}
