#include "streams.h"

#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "common.h"

namespace pr {

hipStream_t make_stream(int device, int kind) {
  DeviceGuard dg(device);
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

namespace {
std::mutex& pool_mu() {
  static std::mutex* m = new std::mutex();   // leaked: used by destructors at process exit
  return *m;
}
std::map<std::pair<int, int>, std::vector<hipStream_t>>& pool() {
  static auto* p = new std::map<std::pair<int, int>, std::vector<hipStream_t>>();
  return *p;
}
}  // namespace

hipStream_t acquire_stream(int device, int kind) {
  if (kind != kStreamShared) {
    std::lock_guard<std::mutex> lk(pool_mu());
    auto& v = pool()[{device, kind}];
    if (!v.empty()) {
      hipStream_t s = v.back();
      v.pop_back();
      return s;
    }
  }
  return make_stream(device, kind);
}

static bool& pool_closed() {
  static bool* c = new bool(false);
  return *c;
}

void release_stream(int device, int kind, hipStream_t s) {
  if (s == nullptr) return;
  DeviceGuard dg(device);
  (void)hipStreamSynchronize(s);
  {
    std::lock_guard<std::mutex> lk(pool_mu());
    if (kind != kStreamShared && !pool_closed()) {
      pool()[{device, kind}].push_back(s);
      return;
    }
  }
  (void)hipStreamDestroy(s);
}

void close_stream_pool() {
  std::map<std::pair<int, int>, std::vector<hipStream_t>> all;
  {
    std::lock_guard<std::mutex> lk(pool_mu());
    pool_closed() = true;
    all.swap(pool());
  }
  for (auto& kv : all) {
    DeviceGuard dg(kv.first.first);
    for (hipStream_t s : kv.second) {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    }
  }
}

}  // namespace pr
