// Native host runtime of psana_ray_amd: pinned staging memory, the HBM slot pool that backs
// the sharded shared queue, and the raw-run file reader (the data loader).
//
// Reference parity:
//  * SlotPool replaces the single-threaded Ray actor `Queue` (psana_ray/shared_queue.py:4-31):
//    bounded capacity with put->False backpressure (Q-4), FIFO get, non-blocking get->None,
//    size().  Unlike the actor it is sharded (one pool per GPU), lock-protected for many
//    threads, and every slot carries HIP events so producers, the queue fabric (peer copies) and
//    consumers order on-device work without host synchronisation.
//  * PinnedBuffer / memcpy_h2d_async implement the "stage raw events into pinned host pages
//    with hipMemcpyAsync on a side stream" path that replaces psana's CPU-side numpy frames
//    (psana_ray/producer.py:88).
//  * RawRunReader is the native event reader behind the raw-run file source (stands in for
//    psana's XTC reader when psana is absent).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace pr {

class FrameVerifier;   // verify.h

// ---------------------------------------------------------------------------------------
class PinnedBuffer {
 public:
  explicit PinnedBuffer(size_t bytes);
  ~PinnedBuffer();
  PinnedBuffer(const PinnedBuffer&) = delete;
  PinnedBuffer& operator=(const PinnedBuffer&) = delete;
  uint64_t ptr() const { return reinterpret_cast<uint64_t>(ptr_); }
  size_t bytes() const { return bytes_; }
  void* raw() const { return ptr_; }

 private:
  void* ptr_ = nullptr;
  size_t bytes_ = 0;
};

// ---------------------------------------------------------------------------------------
// One hipMalloc allocation of HBM (ring segments).  Ring memory is allocated here, not by the torch
// caching allocator, so every allocation is exactly one segment: HIP IPC export works per
// allocation, and opening an IPC handle of an allocation above 2 GiB hangs on this ROCm stack
// (measured: 2.08 GB attaches in 0.2 ms, 2.16 GB never returns; profiles/r2/ipc_attach.md).
class DeviceBuffer {
 public:
  DeviceBuffer(int64_t bytes, int device);
  ~DeviceBuffer();
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  uint64_t ptr() const { return reinterpret_cast<uint64_t>(ptr_); }
  int64_t bytes() const { return bytes_; }
  int device() const { return device_; }

 private:
  void* ptr_ = nullptr;
  int64_t bytes_ = 0;
  int device_ = 0;
};

// ---------------------------------------------------------------------------------------
enum SlotState : int {
  kFree = 0,
  kProducing = 1,
  kProduced = 2,
  kSending = 3,
  kReceiving = 4,
  kReady = 5,
  kLeased = 6,
};

struct SlotHeader {
  int64_t rank = -1;        // producer rank (reference item field 0)
  int64_t idx = -1;         // rank-local event index (reference item field 1)
  int64_t gevt = -1;        // global event id (new: lets consumers dedupe / order)
  double photon_energy = 0; // NaN encodes None (Q-16)
  int64_t aux = 0;          // free for the caller (e.g. timestamp)
};

struct PoolStats {
  int64_t produced = 0, routed_local = 0, sent = 0, received = 0, got = 0, released = 0;
  int64_t produce_full = 0;  // acquire attempts refused because the producer budget was full
};

class SlotPool {
 public:
  // device < 0: host-only pool (no events).  n_slots = producer_budget + consumer_budget.
  SlotPool(int producer_budget, int consumer_budget, int device);
  ~SlotPool();
  SlotPool(const SlotPool&) = delete;
  SlotPool& operator=(const SlotPool&) = delete;

  int n_slots() const { return n_; }
  // device (or host) address of every slot: rings are built from several allocations
  void set_slot_ptrs(const std::vector<uint64_t>& ptrs);
  uint64_t slot_ptr(int slot) const {
    check_slot(slot);
    return ptrs_.empty() ? 0 : ptrs_[(size_t)slot];
  }
  const std::vector<uint64_t>& slot_ptrs() const { return ptrs_; }
  int producer_budget() const { return pb_; }
  int consumer_budget() const { return cb_; }
  // Frames this producer delivered into consumers' read-ahead that no consumer has taken yet.  They
  // still count against the producer budget (queue_size stays ONE logical bound: the reference's
  // deque(maxlen) holds every item not yet got, psana_ray/shared_queue.py:7,11); the queue fabric
  // keeps this up to date from the consumers' `taken` counters.
  void set_external_held(int n);
  int producer_room() const;   // pb - producer_held - external_held

  // producer side
  int try_acquire_produce();
  int acquire_produce(double timeout_s);  // -1 on timeout
  void commit_produce(int slot, const SlotHeader& h, uint64_t stream);
  void abort_produce(int slot);
  std::vector<int> produced(int max_n) const;  // FIFO order, not popped
  int n_produced() const;
  int producer_held() const;

  // routing outcomes
  void route_local(int slot);
  void begin_send(int slot);
  void end_send(int slot, uint64_t stream);

  // consumer side
  int credits() const;
  int begin_recv();
  void end_recv(int slot, const SlotHeader& h, uint64_t stream);
  int try_get();
  int get(double timeout_s);
  void release(int slot, uint64_t stream);
  int n_ready() const;
  int consumer_held() const;

  // ordering helpers
  void wait_ready_on(int slot, uint64_t stream) const;  // stream waits for the slot's data
  void wait_free_on(int slot, uint64_t stream) const;   // stream waits until the slot may be rewritten
  void sync_ready(int slot) const;                      // host waits for the slot's data
  SlotHeader header(int slot) const;
  int state(int slot) const;
  PoolStats stats() const;
  void wake_all();  // wake blocked waiters (shutdown)
  void wake_producers();
  bool closed() const;

  // single-process mode: PRODUCED frames are routed to this pool's own consumer as soon as
  // consumer credit exists (on commit and on release), entirely in native code
  void set_auto_route(bool on);

  // batched calls: one native call AND one HIP event record per batch instead of per frame
  std::vector<int> get_batch(int max_n, double timeout_s, uint64_t stream);
  void release_batch(const std::vector<int>& slots, uint64_t stream);
  std::vector<SlotHeader> headers(const std::vector<int>& slots) const;
  std::vector<int> acquire_batch(int n, double timeout_s, uint64_t stream);  // all n or none
  void commit_batch(const std::vector<int>& slots, const std::vector<SlotHeader>& hdrs, uint64_t stream);
  void begin_send_batch(const std::vector<int>& slots, uint64_t stream);   // + stream waits for their data
  std::vector<int> begin_recv_batch(int n, uint64_t stream);              // + stream waits for free slots
  void end_send_batch(const std::vector<int>& slots, uint64_t stream);
  // queue fabric: copies the host has SEEN complete (event query) -- the slots are free with no
  // device-side wait (end_send_batch would record a free event behind every copy queued since on
  // that stream, each waiting for a later chunk's calibration).  to_external: the frames move from
  // producer_held to the external read-ahead count in the same locked step, so producer_room()
  // never reads high between the two (ADVICE r3 keeper race).
  void end_send_completed(const std::vector<int>& slots, bool to_external);
  void end_recv_batch(const std::vector<int>& slots, const std::vector<SlotHeader>& hdrs, uint64_t stream);
  int64_t event_records() const { return ev_records_; }

  // End-to-end checks of frames other processes wrote into this (consumer) ring (verify.h): every
  // get_batch -- and check_frames, which the single-frame get path calls -- issues a system-scope
  // acquire on the caller's stream when a taken frame came from another process, and re-sums the
  // frames whose header carries a producer checksum (aux tag), compared on the device.
  void set_verifier(std::shared_ptr<FrameVerifier> v);
  std::shared_ptr<FrameVerifier> verifier() const;
  void check_frames(const std::vector<int>& slots, uint64_t stream);

  // elastic fabric (fabric.h): another PROCESS writes granted slots, so a grant needs the slot's
  // previous readers to have finished on the host's view (event query), not just stream order
  std::vector<int> grant_batch(int max_n);                                    // FREE -> RECEIVING
  void complete_recv_batch(const std::vector<int>& slots, const std::vector<SlotHeader>& hdrs);  // -> READY
  void cancel_recv_batch(const std::vector<int>& slots);                      // RECEIVING -> FREE
  void unsend_batch(const std::vector<int>& slots);  // SENDING -> PRODUCED, back at the FIFO front
  // queue keeper: received frames (LEASED) go back on offer as this process's own production
  // (LEASED -> PRODUCED, headers kept; consumer budget -> producer budget).  Returns how many
  // moved (stops when the producer budget is full).
  int reoffer_batch(const std::vector<int>& slots, uint64_t stream);
  // queue keeper, atomically: up to max_n READY frames straight to PRODUCED (FIFO, headers and data
  // references kept), bounded by the producer room read under the same lock -- no frame is ever
  // leased without room to re-offer it (room read, lease and re-offer were three calls
  // the fabric thread could interleave with).  Returns how many moved.
  int relay_ready(int max_n);
  // Origins of consumed frames (elastic fabric): a received frame remembers the producer member it
  // came from (-1: routed locally); every frame a consumer takes (get / get_batch) appends its
  // origin to a log the fabric drains, so each producer learns how many of its frames were taken.
  void set_track_origins(bool on);
  void complete_recv_batch_from(const std::vector<int>& slots, const std::vector<SlotHeader>& hdrs, int64_t origin);
  std::vector<int64_t> take_got_origins();
  int64_t origin(int slot) const;
  // Consumer close: READY frames taken out of the FIFO to be handed back to a producer (LEASED,
  // not counted as got); free them with release() once a producer copied them out.
  std::vector<int> pop_ready_for_return(int max_n);
  // Producer: up to n free slots for frames handed back by a closing consumer (PRODUCING; may
  // exceed the logical budget by frames that were counted as external read-ahead), and their
  // commit at the FRONT of the produced FIFO (they were queued before anything produced now).
  std::vector<int> reclaim_batch(int n, uint64_t stream);
  void commit_front_batch(const std::vector<int>& slots, const std::vector<SlotHeader>& hdrs, uint64_t stream);

 private:
  void set_device() const;
  void check_slot(int slot) const;
  // Shared event ring: a batch records ONE event and every slot of the batch references it as
  // (index, generation).  A reference whose generation was overwritten is treated as complete:
  // the ring holds >= 4x the slots, so an event is re-recorded only after thousands of batches.
  struct EvRef {
    int idx = -1;
    uint64_t gen = 0;
  };
  EvRef record_shared_locked(uint64_t stream);
  void wait_ref(const EvRef& r, uint64_t stream) const;
  bool ref_live_locked(const EvRef& r) const { return r.idx >= 0 && ev_gen_[r.idx] == r.gen; }
  void route_pending_locked();
  int pop_ready_locked();

  int pb_, cb_, n_, device_;
  std::vector<uint64_t> ptrs_;
  mutable std::mutex mu_;
  std::condition_variable cv_produce_, cv_ready_;
  std::vector<int> state_;
  std::vector<SlotHeader> hdr_;
  std::vector<hipEvent_t> ev_;
  std::vector<uint64_t> ev_gen_;
  int ev_next_ = 0;
  int64_t ev_records_ = 0;
  std::vector<EvRef> ready_ref_, free_ref_;
  std::deque<int> free_list_, produced_fifo_, ready_fifo_;
  int producer_held_ = 0, consumer_held_ = 0, ext_held_ = 0;
  bool track_origins_ = false;
  std::vector<int64_t> origin_;
  std::vector<int64_t> got_origins_;
  bool closed_ = false;
  bool auto_route_ = false;
  std::shared_ptr<FrameVerifier> verifier_;
  PoolStats st_;
};

// ---------------------------------------------------------------------------------------
// A run file mapped into the address space and registered with HIP (page-locked), so the DMA
// engines copy event payloads straight out of the page cache / tmpfs into HBM: no CPU memcpy into
// a staging buffer (the pread path is CPU-bound at ~18 GB/s on a 16-core share; PCIe is ~57).
class MappedFile {
 public:
  // register: hipHostRegister the whole mapping (read-only); false = plain mmap (host reads only)
  MappedFile(const std::string& path, bool register_with_hip);
  ~MappedFile();
  MappedFile(const MappedFile&) = delete;
  MappedFile& operator=(const MappedFile&) = delete;
  uint64_t ptr() const { return reinterpret_cast<uint64_t>(base_); }
  int64_t bytes() const { return (int64_t)bytes_; }
  bool registered() const { return registered_; }
  double register_s() const { return register_s_; }

 private:
  void* base_ = nullptr;
  size_t bytes_ = 0;
  bool registered_ = false;
  double register_s_ = 0;
};

// ---------------------------------------------------------------------------------------
// Raw-run file: fixed-size records so event i is at header_bytes + i * record_bytes.
//   file header (4096 B): magic "PRAWRUN1", u32 version, u32 header_bytes, char det[64],
//   u32 ndim, u64 shape[4], u32 dtype_bytes, u64 n_events, u64 record_bytes
//   record: i64 gevt, f64 photon_energy, i64 timestamp, i64 reserved, then the raw frame
class RawRunReader {
 public:
  RawRunReader(const std::string& path, int n_threads);
  // Index mode (variable-size containers, e.g. XTC2 bigdata located through its small-data file):
  // event i's frame is `frame_bytes` at payload_off[i]; its metadata comes from the index.
  RawRunReader(const std::string& path, int n_threads, std::vector<int64_t> payload_off, std::vector<int64_t> gevt,
               std::vector<double> photon_energy, int64_t frame_bytes);
  ~RawRunReader();
  bool indexed() const { return !off_.empty(); }
  int64_t n_events() const { return n_events_; }
  int64_t frame_bytes() const { return frame_bytes_; }
  int64_t record_bytes() const { return record_bytes_; }
  int64_t header_bytes() const { return header_bytes_; }
  // Synchronously reads events[i] into dst_ptrs[i] (frame bytes) using the thread pool and
  // returns (gevt, photon_energy) per event.
  std::vector<std::pair<int64_t, double>> read(const std::vector<int64_t>& events,
                                               const std::vector<uint64_t>& dst_ptrs);

 private:
  int fd_ = -1;
  int n_threads_;
  int64_t n_events_ = 0, frame_bytes_ = 0, record_bytes_ = 0, header_bytes_ = 0;
  std::vector<int64_t> off_, gevt_;
  std::vector<double> pe_;
};

// ---------------------------------------------------------------------------------------
void memcpy_h2d_async(uint64_t dst, uint64_t src, size_t bytes, uint64_t stream);
void memcpy_h2d_batch(const std::vector<uint64_t>& dst, const std::vector<uint64_t>& src, size_t bytes,
                      uint64_t stream);

}  // namespace pr
