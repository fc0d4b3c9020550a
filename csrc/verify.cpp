// Host side of the fabric's end-to-end frame checks (csrc/verify.h).
#include "verify.h"

#include <stdlib.h>
#include <string.h>

namespace pr {

uint64_t frame_checksum_host(const void* p, int64_t bytes) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  uint64_t s = 0;
  const int64_t n16 = bytes / 16;
  for (int64_t q = 0; q < n16; ++q) {
    uint64_t w[2];
    memcpy(w, b + q * 16, 16);
    s += ck_word(w[0], w[1], (uint64_t)q);
  }
  if (bytes % 16) {
    uint64_t w[2] = {0, 0};
    memcpy(w, b + n16 * 16, (size_t)(bytes % 16));
    s += ck_word(w[0], w[1], (uint64_t)n16);
  }
  return s;
}

FrameVerifier::FrameVerifier(int device, int64_t frame_bytes) : device_(device), bytes_(frame_bytes) {
  check(frame_bytes > 0, "FrameVerifier: empty frames");
  // A/B switch only (PSANA_RAY_AMD_FABRIC_ACQUIRE=0): rely on the dispatch packets' acquire alone
  if (const char* e = getenv("PSANA_RAY_AMD_FABRIC_ACQUIRE")) acquire_on_ = atoi(e) != 0;
  if (device_ < 0) return;
  check(frame_bytes % 16 == 0, "FrameVerifier: frame size must be a multiple of 16 B on the GPU");
  DeviceGuard dg(device_);
  const size_t rows = (size_t)kRows * kMaxFrames;
  hip_check(hipMalloc(reinterpret_cast<void**>(&acc_), rows * sizeof(uint64_t)), "hipMalloc (verify scratch)");
  hip_check(hipMalloc(reinterpret_cast<void**>(&cnt_), rows * sizeof(uint32_t)), "hipMalloc (verify tickets)");
  hip_check(hipMalloc(reinterpret_cast<void**>(&counters_), 4 * sizeof(int64_t)), "hipMalloc (verify counters)");
  hip_check(hipMemset(acc_, 0, rows * sizeof(uint64_t)), "hipMemset (verify scratch)");
  hip_check(hipMemset(cnt_, 0, rows * sizeof(uint32_t)), "hipMemset (verify tickets)");
  const int64_t init[4] = {0, 0, -1, 0};
  hip_check(hipMemcpy(counters_, init, sizeof(init), hipMemcpyHostToDevice), "hipMemcpy (verify counters)");
  hip_check(hipHostMalloc(reinterpret_cast<void**>(&results_), kResults * sizeof(int64_t), hipHostMallocDefault),
            "hipHostMalloc (verify results)");
  memset(results_, 0, kResults * sizeof(int64_t));
  hip_check(hipStreamCreateWithFlags(&rd_stream_, hipStreamNonBlocking), "hipStreamCreate (verify)");
}

FrameVerifier::~FrameVerifier() {
  if (device_ < 0) return;
  DeviceGuard dg(device_);
  (void)hipDeviceSynchronize();   // no launch of ours may still use the scratch
  if (rd_stream_) (void)hipStreamDestroy(rd_stream_);
  if (acc_) (void)hipFree(acc_);
  if (cnt_) (void)hipFree(cnt_);
  if (counters_) (void)hipFree(counters_);
  if (results_) (void)hipHostFree(results_);
}

int64_t FrameVerifier::take_row() {
  std::lock_guard<std::mutex> lk(mu_);
  const int64_t r = row_;
  row_ = (row_ + 1) % kRows;
  return r;
}

int64_t FrameVerifier::checksum_async(const std::vector<uint64_t>& ptrs, uint64_t stream) {
  check(device_ >= 0, "FrameVerifier::checksum_async: GPU rings only");
  check(!ptrs.empty() && (int)ptrs.size() <= kMaxFrames, "FrameVerifier::checksum_async: 1..kMaxFrames frames");
  int64_t base;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (res_next_ + (int64_t)ptrs.size() > kResults) res_next_ = 0;
    base = res_next_;
    res_next_ += (int64_t)ptrs.size();
  }
  CkFrames a{};
  for (size_t i = 0; i < ptrs.size(); ++i) a.ptr[i] = ptrs[i];
  const int64_t row = take_row();
  DeviceGuard dg(device_);
  launch_frame_checksums(a, (int)ptrs.size(), bytes_ / 16, reinterpret_cast<uint64_t>(acc_ + row * kMaxFrames),
                         reinterpret_cast<uint64_t>(cnt_ + row * kMaxFrames), false,
                         reinterpret_cast<uint64_t>(results_ + base), 0, stream);
  return base;
}

int64_t FrameVerifier::result(int64_t index) const {
  check(device_ >= 0 && index >= 0 && index < kResults, "FrameVerifier::result: bad index");
  return reinterpret_cast<volatile int64_t*>(results_)[index];
}

void FrameVerifier::verify(const std::vector<uint64_t>& ptrs, const std::vector<int64_t>& expect,
                           const std::vector<int64_t>& gevt, uint64_t stream) {
  check(ptrs.size() == expect.size() && ptrs.size() == gevt.size(), "FrameVerifier::verify: size mismatch");
  if (ptrs.empty()) return;
  if (device_ < 0) {
    for (size_t i = 0; i < ptrs.size(); ++i) {
      const int64_t got = ck_tag(frame_checksum_host(reinterpret_cast<const void*>(ptrs[i]), bytes_));
      if (got == expect[i]) {
        h_ok_.fetch_add(1);
      } else {
        h_bad_.fetch_add(1);
        h_last_bad_.store(gevt[i]);
      }
    }
    return;
  }
  DeviceGuard dg(device_);
  for (size_t a0 = 0; a0 < ptrs.size(); a0 += kMaxFrames) {
    const size_t n = std::min(ptrs.size() - a0, (size_t)kMaxFrames);
    CkFrames a{};
    for (size_t i = 0; i < n; ++i) {
      a.ptr[i] = ptrs[a0 + i];
      a.expect[i] = expect[a0 + i];
      a.gevt[i] = gevt[a0 + i];
    }
    const int64_t row = take_row();
    launch_frame_checksums(a, (int)n, bytes_ / 16, reinterpret_cast<uint64_t>(acc_ + row * kMaxFrames),
                           reinterpret_cast<uint64_t>(cnt_ + row * kMaxFrames), true, 0,
                           reinterpret_cast<uint64_t>(counters_), stream);
  }
}

void FrameVerifier::acquire(uint64_t stream) {
  if (!acquire_on_) return;
  acquires_.fetch_add(1);
  if (device_ < 0) {
    std::atomic_thread_fence(std::memory_order_acquire);
    return;
  }
  DeviceGuard dg(device_);
  launch_acquire_fence(stream);
}

std::array<int64_t, 4> FrameVerifier::counts() const {
  if (device_ < 0) return {h_ok_.load(), h_bad_.load(), h_last_bad_.load(), acquires_.load()};
  DeviceGuard dg(device_);
  int64_t c[4] = {0, 0, -1, 0};
  hip_check(hipMemcpyAsync(c, counters_, 3 * sizeof(int64_t), hipMemcpyDeviceToHost, rd_stream_),
            "hipMemcpyAsync (verify counters)");
  hip_check(hipStreamSynchronize(rd_stream_), "hipStreamSynchronize (verify counters)");
  return {c[0], c[1], c[2], acquires_.load()};
}

}  // namespace pr
