// End-to-end checks of frames that cross processes (and GPUs) through the queue fabric.
//
// Reference contract: every put/get moves an intact [rank, idx, data, photon_energy] item
// (psana_ray/producer.py:101, psana_ray/data_reader.py:35).  Here the data of a frame routed to
// another process is written into that consumer's ring by the PRODUCER's copy (fabric.h), over
// xGMI when the two GPUs differ, so its integrity on arrival is checked end to end:
//
//   producer: every `every`-th frame (rank-local idx % every == 0) it sends to another process
//             gets a 64-bit content checksum, computed on the copy stream right before the copy (so it covers
//             exactly the bytes copied), carried to the consumer in the notice's `aux` field with a
//             tag in the top byte;
//   consumer: a frame it takes whose aux carries the tag is re-summed from ITS ring slot on the
//             stream the caller will read it on, before that read; the sum lands in pinned host
//             memory and is compared on the host once that launch's event completed (verified /
//             mismatched counts plus the last mismatching gevt; no host sync per frame).
//
// The checksum is order-dependent (each 16-B word is mixed with its index, then the mixes are
// summed), so a stale, shifted or partially written frame changes it; the sum is associative, so
// the GPU can reduce it in any order and the host (CPU rings) computes the identical value.
//
// Visibility is explicit too: a consumer that takes frames another process wrote launches a
// system-scope acquire (buffer_inv sc0 sc1 on every XCD) on its read stream before the frames'
// first read, and copy_runs_kernel ends with a system-scope release (gather.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <array>
#include <atomic>
#include <deque>
#include <mutex>
#include <vector>

#include "common.h"

namespace pr {

constexpr uint64_t kCheckTag = 0xC5ull << 56;          // aux top byte of a checksummed frame
constexpr uint64_t kCheckMask = (1ull << 56) - 1;

__host__ __device__ __forceinline__ uint64_t ck_word(uint64_t lo, uint64_t hi, uint64_t q) {
  uint64_t h = (lo ^ ((q + 1) * 0x9E3779B97F4A7C15ull)) * 0xBF58476D1CE4E5B9ull;
  h += hi * 0x94D049BB133111EBull;
  h ^= h >> 31;
  h *= 0xD6E8FEB86659FD93ull;
  h ^= h >> 32;
  return h;
}
__host__ __device__ __forceinline__ int64_t ck_tag(uint64_t sum) { return (int64_t)((sum & kCheckMask) | kCheckTag); }
__host__ __device__ __forceinline__ bool ck_tagged(int64_t aux) {
  return ((uint64_t)aux & ~kCheckMask) == kCheckTag;
}

// The checksum of `bytes` bytes at host address p (a partial last 16-B word is zero-padded).
uint64_t frame_checksum_host(const void* p, int64_t bytes);

// Per-launch arguments of the device checksum kernels (kernarg block).
struct CkFrames {
  uint64_t ptr[kMaxFrames];
};

// Device launcher (verify.hip): out[f] = tagged checksum of frame f (pinned host memory), via a
// scratch row `part` of kMaxFrames x kCkPartials uint64 partials.
constexpr int kCkPartials = 128;
void launch_frame_checksums(const CkFrames& a, int nframes, int64_t n16, uint64_t part, uint64_t out,
                            uint64_t stream);
// System-scope acquire on every XCD (64 one-wave workgroups, dealt round-robin over the 8 XCDs).
void launch_acquire_fence(uint64_t stream);
// System-scope release on every XCD (the direct-write path: calibration kernels wrote peer memory).
void launch_release_fence(uint64_t stream);

class FrameVerifier {
 public:
  // device < 0: host (CPU) rings, everything on the CPU
  FrameVerifier(int device, int64_t frame_bytes);
  ~FrameVerifier();
  FrameVerifier(const FrameVerifier&) = delete;
  FrameVerifier& operator=(const FrameVerifier&) = delete;

  int device() const { return device_; }
  int64_t frame_bytes() const { return bytes_; }

  // producer, GPU: checksums of `ptrs` (frames in HBM) queued on `stream`; returns the index of the
  // first result in the pinned result ring (result(i) is valid once the stream passed this point)
  int64_t checksum_async(const std::vector<uint64_t>& ptrs, uint64_t stream);
  int64_t result(int64_t index) const;
  // consumer: compare frames against the tagged checksums their producer sent (GPU: the sums are
  // queued on `stream` and compared on the host once that launch's event completed -- at a later
  // verify() or counts(); host rings: now)
  void verify(const std::vector<uint64_t>& ptrs, const std::vector<int64_t>& expect,
              const std::vector<int64_t>& gevt, uint64_t stream);
  // consumer, GPU: explicit system-scope acquire on `stream` before reading peer-written frames
  void acquire(uint64_t stream);
  // {verified, mismatched, last mismatching gevt (-1 none), acquires}; GPU: waits for every
  // pending comparison's launch, so the count covers every frame verify() was called for
  std::array<int64_t, 4> counts();

  static constexpr int kRows = 64;          // scratch rows (rotating, one per launch)
  static constexpr int kResults = 65536;    // pinned results (rotating)

 private:
  struct Pending {
    hipEvent_t ev;
    int64_t base;
    std::vector<int64_t> expect, gevt;
  };
  // one checksum launch (mu_ held): a scratch row, ordered after that row's previous launch
  void launch_row(const CkFrames& a, int n, int64_t base, uint64_t stream);
  int64_t take_results(int n);
  void settle(bool wait);   // compare pending results whose launch completed (all, if wait); mu_ held
  int device_;
  int64_t bytes_;
  uint64_t* part_ = nullptr;       // device: kRows x kMaxFrames x kCkPartials
  int64_t* results_ = nullptr;     // pinned host: kResults
  std::deque<Pending> pending_;
  std::vector<hipEvent_t> free_ev_;
  // per scratch row: an event after its last launch.  Producer checksums (the fabric's copy stream)
  // and consumer checks (read streams) share the rows, so a row's next launch, on whatever stream,
  // waits for its previous one on the device (rows recycled after kRows launches were otherwise
  // overwritten by a launch on another stream while still in use: wrong sums, false mismatches)
  std::vector<hipEvent_t> row_ev_;
  std::mutex mu_;
  int64_t row_ = 0, res_next_ = 0;
  bool acquire_on_ = true;
  std::atomic<int64_t> h_ok_{0}, h_bad_{0}, h_last_bad_{-1}, acquires_{0};
};

}  // namespace pr
