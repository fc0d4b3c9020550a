#include "streams.h"

#include <vector>

#include "common.h"

namespace pr {

hipStream_t make_stream(int device, int kind) {
  hip_check(hipSetDevice(device), "hipSetDevice");
  hipStream_t s = nullptr;
  if (kind == kStreamDedicated) {
    hipDeviceProp_t prop{};
    hip_check(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
    const int n_cu = prop.multiProcessorCount;
    std::vector<uint32_t> mask((size_t)(n_cu + 31) / 32, 0u);
    for (int i = 0; i < n_cu; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
    hip_check(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()), "hipExtStreamCreateWithCUMask");
  } else if (kind == kStreamHighPriority) {
    int lo = 0, hi = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
    hip_check(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi), "hipStreamCreateWithPriority");
  } else {
    check(kind == kStreamShared, "make_stream: unknown stream kind");
    hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  }
  return s;
}

}  // namespace pr
