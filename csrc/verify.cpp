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
  const size_t rows = (size_t)kRows * kMaxFrames * kCkPartials;
  hip_check(hipMalloc(reinterpret_cast<void**>(&part_), rows * sizeof(uint64_t)), "hipMalloc (verify scratch)");
  hip_check(hipHostMalloc(reinterpret_cast<void**>(&results_), kResults * sizeof(int64_t), hipHostMallocDefault),
            "hipHostMalloc (verify results)");
  memset(results_, 0, kResults * sizeof(int64_t));
}

FrameVerifier::~FrameVerifier() {
  if (device_ < 0) return;
  DeviceGuard dg(device_);
  for (auto& p : pending_) {
    (void)hipEventSynchronize(p.ev);   // no launch of ours may still use the scratch
    (void)hipEventDestroy(p.ev);
  }
  for (auto e : free_ev_) (void)hipEventDestroy(e);
  (void)hipDeviceSynchronize();
  for (auto e : row_ev_)
    if (e != nullptr) (void)hipEventDestroy(e);
  if (part_) (void)hipFree(part_);
  if (results_) (void)hipHostFree(results_);
}

void FrameVerifier::launch_row(const CkFrames& a, int n, int64_t base, uint64_t stream) {
  const int64_t r = row_;
  row_ = (row_ + 1) % kRows;
  if (row_ev_.empty()) row_ev_.assign(kRows, nullptr);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (row_ev_[(size_t)r] != nullptr) {
    hip_check(hipStreamWaitEvent(s, row_ev_[(size_t)r], 0), "hipStreamWaitEvent (verify row)");
  } else {
    hip_check(hipEventCreateWithFlags(&row_ev_[(size_t)r], hipEventDisableTiming), "hipEventCreate (verify row)");
  }
  launch_frame_checksums(a, n, bytes_ / 16, reinterpret_cast<uint64_t>(part_ + r * kMaxFrames * kCkPartials),
                         reinterpret_cast<uint64_t>(results_ + base), stream);
  hip_check(hipEventRecord(row_ev_[(size_t)r], s), "hipEventRecord (verify row)");
}

int64_t FrameVerifier::take_results(int n) {
  if (res_next_ + n > kResults) res_next_ = 0;
  const int64_t base = res_next_;
  res_next_ += n;
  return base;
}

int64_t FrameVerifier::checksum_async(const std::vector<uint64_t>& ptrs, uint64_t stream) {
  check(device_ >= 0, "FrameVerifier::checksum_async: GPU rings only");
  check(!ptrs.empty() && (int)ptrs.size() <= kMaxFrames, "FrameVerifier::checksum_async: 1..kMaxFrames frames");
  CkFrames a{};
  for (size_t i = 0; i < ptrs.size(); ++i) a.ptr[i] = ptrs[i];
  std::lock_guard<std::mutex> lk(mu_);
  const int64_t base = take_results((int)ptrs.size());
  DeviceGuard dg(device_);
  launch_row(a, (int)ptrs.size(), base, stream);
  return base;
}

int64_t FrameVerifier::result(int64_t index) const {
  check(device_ >= 0 && index >= 0 && index < kResults, "FrameVerifier::result: bad index");
  return reinterpret_cast<volatile int64_t*>(results_)[index];
}

void FrameVerifier::settle(bool wait) {
  while (!pending_.empty()) {
    Pending& p = pending_.front();
    if (wait) {
      hip_check(hipEventSynchronize(p.ev), "hipEventSynchronize (verify)");
    } else {
      const hipError_t q = hipEventQuery(p.ev);
      if (q == hipErrorNotReady) return;
      hip_check(q, "hipEventQuery (verify)");
    }
    for (size_t i = 0; i < p.expect.size(); ++i) {
      if (result(p.base + (int64_t)i) == p.expect[i]) {
        h_ok_.fetch_add(1);
      } else {
        h_bad_.fetch_add(1);
        h_last_bad_.store(p.gevt[i]);
      }
    }
    free_ev_.push_back(p.ev);
    pending_.pop_front();
  }
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
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard dg(device_);
  settle(false);
  // results of pending launches may not be overwritten: with the ring nearly full, wait for the oldest
  while (!pending_.empty() && ((int64_t)pending_.size() + 1) * kMaxFrames > kResults) {
    hip_check(hipEventSynchronize(pending_.front().ev), "hipEventSynchronize (verify ring)");
    settle(false);
  }
  for (size_t a0 = 0; a0 < ptrs.size(); a0 += kMaxFrames) {
    const size_t n = std::min(ptrs.size() - a0, (size_t)kMaxFrames);
    CkFrames a{};
    for (size_t i = 0; i < n; ++i) a.ptr[i] = ptrs[a0 + i];
    const int64_t base = take_results((int)n);
    launch_row(a, (int)n, base, stream);
    Pending p;
    if (free_ev_.empty()) {
      hip_check(hipEventCreateWithFlags(&p.ev, hipEventDisableTiming), "hipEventCreate (verify)");
    } else {
      p.ev = free_ev_.back();
      free_ev_.pop_back();
    }
    hip_check(hipEventRecord(p.ev, reinterpret_cast<hipStream_t>(stream)), "hipEventRecord (verify)");
    p.base = base;
    p.expect.assign(expect.begin() + (int64_t)a0, expect.begin() + (int64_t)(a0 + n));
    p.gevt.assign(gevt.begin() + (int64_t)a0, gevt.begin() + (int64_t)(a0 + n));
    pending_.push_back(std::move(p));
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

std::array<int64_t, 4> FrameVerifier::counts() {
  if (device_ >= 0) {
    std::lock_guard<std::mutex> lk(mu_);
    DeviceGuard dg(device_);
    settle(true);
  }
  return {h_ok_.load(), h_bad_.load(), h_last_bad_.load(), acquires_.load()};
}

}  // namespace pr
