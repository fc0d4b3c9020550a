#include "runtime.h"
#include "verify.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <future>
#include <stdexcept>

#include "common.h"

namespace pr {

// ---------------------------------------------------------------------------------------
PinnedBuffer::PinnedBuffer(size_t bytes) : bytes_(bytes) {
  check(bytes > 0, "PinnedBuffer: size must be > 0");
  hip_check(hipHostMalloc(&ptr_, bytes, hipHostMallocDefault), "hipHostMalloc");
}

PinnedBuffer::~PinnedBuffer() {
  if (ptr_) (void)hipHostFree(ptr_);
}

// ---------------------------------------------------------------------------------------
DeviceBuffer::DeviceBuffer(int64_t bytes, int device) : bytes_(bytes), device_(device) {
  check(bytes > 0 && device >= 0, "DeviceBuffer: size must be > 0 on a device");
  DeviceGuard dg(device);
  hip_check(hipMalloc(&ptr_, (size_t)bytes), "hipMalloc (ring segment)");
}

DeviceBuffer::~DeviceBuffer() {
  if (ptr_ != nullptr) {
    DeviceGuard dg(device_);
    (void)hipFree(ptr_);
  }
}

// ---------------------------------------------------------------------------------------
SlotPool::SlotPool(int producer_budget, int consumer_budget, int device)
    : pb_(producer_budget), cb_(consumer_budget), n_(producer_budget + consumer_budget), device_(device) {
  check(producer_budget >= 0 && consumer_budget >= 0 && n_ > 0, "SlotPool: budgets must be >= 0 and sum > 0");
  state_.assign(n_, kFree);
  origin_.assign(n_, -1);
  hdr_.resize(n_);
  ready_ref_.resize(n_);
  free_ref_.resize(n_);
  for (int i = 0; i < n_; ++i) free_list_.push_back(i);
  if (device_ >= 0) {
    DeviceGuard dg(device_);
    const int ne = std::max(256, 4 * n_);
    ev_.resize(ne);
    ev_gen_.assign(ne, 0);
    for (int i = 0; i < ne; ++i)
      hip_check(hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming), "hipEventCreate");
  }
}

SlotPool::~SlotPool() {
  if (device_ >= 0) {
    DeviceGuard dg(device_);
    for (auto e : ev_) (void)hipEventDestroy(e);
  }
}

void SlotPool::set_device() const {
  if (device_ >= 0) hip_check(hipSetDevice(device_), "hipSetDevice");
}

void SlotPool::set_slot_ptrs(const std::vector<uint64_t>& ptrs) {
  check((int)ptrs.size() == n_, "SlotPool.set_slot_ptrs: one address per slot");
  for (uint64_t p : ptrs) check(p != 0, "SlotPool.set_slot_ptrs: null slot address");
  std::lock_guard<std::mutex> lk(mu_);
  ptrs_ = ptrs;
}

void SlotPool::check_slot(int slot) const {
  check(slot >= 0 && slot < n_, "SlotPool: slot index out of range");
}

SlotPool::EvRef SlotPool::record_shared_locked(uint64_t stream) {
  EvRef r;
  if (device_ < 0) return r;
  DeviceGuard dg(device_);
  r.idx = ev_next_;
  ev_next_ = (ev_next_ + 1) % (int)ev_.size();
  r.gen = ++ev_gen_[r.idx];
  hip_check(hipEventRecord(ev_[r.idx], reinterpret_cast<hipStream_t>(stream)), "hipEventRecord");
  ++ev_records_;
  return r;
}

void SlotPool::wait_ref(const EvRef& r, uint64_t stream) const {
  if (device_ < 0 || r.idx < 0) return;
  // an event that already completed needs no barrier packet: every packet between two producer
  // chunks on the compute queue delays the next chunk's dispatch (tools/gap_probe.py)
  const hipError_t q = hipEventQuery(ev_[r.idx]);
  if (q == hipSuccess) return;
  if (q != hipErrorNotReady) hip_check(q, "hipEventQuery (wait)");
  hip_check(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), ev_[r.idx], 0), "hipStreamWaitEvent");
}

static std::string state_msg(const char* op, int want, int got) {
  return std::string("SlotPool.") + op + ": slot in state " + std::to_string(got) + ", expected " +
         std::to_string(want);
}

int SlotPool::try_acquire_produce() {
  std::lock_guard<std::mutex> lk(mu_);
  if (producer_held_ + ext_held_ >= pb_ || free_list_.empty()) {
    ++st_.produce_full;
    return -1;
  }
  const int s = free_list_.front();
  free_list_.pop_front();
  state_[s] = kProducing;
  ++producer_held_;
  return s;
}

int SlotPool::acquire_produce(double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  const auto pred = [&] { return closed_ || (producer_held_ + ext_held_ < pb_ && !free_list_.empty()); };
  if (!pred()) ++st_.produce_full;
  if (timeout_s < 0) {
    cv_produce_.wait(lk, pred);
  } else if (!cv_produce_.wait_for(lk, std::chrono::duration<double>(timeout_s), pred)) {
    return -1;
  }
  if (closed_) return -1;
  const int s = free_list_.front();
  free_list_.pop_front();
  state_[s] = kProducing;
  ++producer_held_;
  return s;
}

void SlotPool::commit_produce(int slot, const SlotHeader& h, uint64_t stream) {
  check_slot(slot);
  std::lock_guard<std::mutex> lk(mu_);
  check(state_[slot] == kProducing, state_msg("commit_produce", kProducing, state_[slot]));
  hdr_[slot] = h;
  ready_ref_[slot] = record_shared_locked(stream);
  state_[slot] = kProduced;
  produced_fifo_.push_back(slot);
  ++st_.produced;
  if (auto_route_) route_pending_locked();
}

void SlotPool::abort_produce(int slot) {
  check_slot(slot);
  std::lock_guard<std::mutex> lk(mu_);
  check(state_[slot] == kProducing, state_msg("abort_produce", kProducing, state_[slot]));
  state_[slot] = kFree;
  --producer_held_;
  free_list_.push_front(slot);
  cv_produce_.notify_one();
}

std::vector<int> SlotPool::produced(int max_n) const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<int> out;
  for (int s : produced_fifo_) {
    if ((int)out.size() >= max_n) break;
    out.push_back(s);
  }
  return out;
}

int SlotPool::n_produced() const {
  std::lock_guard<std::mutex> lk(mu_);
  return (int)produced_fifo_.size();
}

int SlotPool::producer_held() const {
  std::lock_guard<std::mutex> lk(mu_);
  return producer_held_;
}

static void erase_value(std::deque<int>& q, int v) {
  for (auto it = q.begin(); it != q.end(); ++it)
    if (*it == v) {
      q.erase(it);
      return;
    }
  throw std::runtime_error("psana_ray_amd: SlotPool internal FIFO corruption");
}

void SlotPool::route_local(int slot) {
  check_slot(slot);
  std::lock_guard<std::mutex> lk(mu_);
  check(state_[slot] == kProduced, state_msg("route_local", kProduced, state_[slot]));
  check(consumer_held_ < cb_, "SlotPool.route_local: no consumer credit");
  erase_value(produced_fifo_, slot);
  state_[slot] = kReady;
  origin_[slot] = -1;
  --producer_held_;
  ++consumer_held_;
  ready_fifo_.push_back(slot);
  ++st_.routed_local;
  cv_ready_.notify_one();
  cv_produce_.notify_one();
}

void SlotPool::begin_send(int slot) {
  check_slot(slot);
  std::lock_guard<std::mutex> lk(mu_);
  check(state_[slot] == kProduced, state_msg("begin_send", kProduced, state_[slot]));
  erase_value(produced_fifo_, slot);
  state_[slot] = kSending;
}

void SlotPool::end_send(int slot, uint64_t stream) {
  check_slot(slot);
  std::lock_guard<std::mutex> lk(mu_);
  check(state_[slot] == kSending, state_msg("end_send", kSending, state_[slot]));
  free_ref_[slot] = record_shared_locked(stream);
  state_[slot] = kFree;
  --producer_held_;
  free_list_.push_back(slot);
  ++st_.sent;
  cv_produce_.notify_one();
}

int SlotPool::credits() const {
  std::lock_guard<std::mutex> lk(mu_);
  return cb_ - consumer_held_;
}

int SlotPool::begin_recv() {
  std::lock_guard<std::mutex> lk(mu_);
  check(consumer_held_ < cb_, "SlotPool.begin_recv: no consumer credit");
  check(!free_list_.empty(), "SlotPool.begin_recv: no free slot");
  const int s = free_list_.front();
  free_list_.pop_front();
  state_[s] = kReceiving;
  ++consumer_held_;
  return s;
}

void SlotPool::end_recv(int slot, const SlotHeader& h, uint64_t stream) {
  check_slot(slot);
  std::lock_guard<std::mutex> lk(mu_);
  check(state_[slot] == kReceiving, state_msg("end_recv", kReceiving, state_[slot]));
  hdr_[slot] = h;
  ready_ref_[slot] = record_shared_locked(stream);
  state_[slot] = kReady;
  ready_fifo_.push_back(slot);
  ++st_.received;
  cv_ready_.notify_one();
}

int SlotPool::try_get() {
  std::lock_guard<std::mutex> lk(mu_);
  if (ready_fifo_.empty()) return -1;
  return pop_ready_locked();
}

int SlotPool::get(double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  const auto pred = [&] { return closed_ || !ready_fifo_.empty(); };
  if (timeout_s < 0) {
    cv_ready_.wait(lk, pred);
  } else if (!cv_ready_.wait_for(lk, std::chrono::duration<double>(timeout_s), pred)) {
    return -1;
  }
  if (ready_fifo_.empty()) return -1;
  return pop_ready_locked();
}

void SlotPool::release(int slot, uint64_t stream) {
  check_slot(slot);
  std::lock_guard<std::mutex> lk(mu_);
  check(state_[slot] == kLeased, state_msg("release", kLeased, state_[slot]));
  free_ref_[slot] = record_shared_locked(stream);
  state_[slot] = kFree;
  --consumer_held_;
  free_list_.push_back(slot);
  ++st_.released;
  if (auto_route_) route_pending_locked();
  cv_produce_.notify_one();
}

int SlotPool::n_ready() const {
  std::lock_guard<std::mutex> lk(mu_);
  return (int)ready_fifo_.size();
}

int SlotPool::consumer_held() const {
  std::lock_guard<std::mutex> lk(mu_);
  return consumer_held_;
}

void SlotPool::wait_ready_on(int slot, uint64_t stream) const {
  check_slot(slot);
  if (device_ < 0) return;
  EvRef r;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!ref_live_locked(ready_ref_[slot])) return;
    r = ready_ref_[slot];
  }
  DeviceGuard dg(device_);
  wait_ref(r, stream);
}

void SlotPool::wait_free_on(int slot, uint64_t stream) const {
  check_slot(slot);
  if (device_ < 0) return;
  EvRef r;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!ref_live_locked(free_ref_[slot])) return;
    r = free_ref_[slot];
  }
  DeviceGuard dg(device_);
  wait_ref(r, stream);
}

void SlotPool::sync_ready(int slot) const {
  check_slot(slot);
  if (device_ < 0) return;
  hipEvent_t e;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!ref_live_locked(ready_ref_[slot])) return;
    e = ev_[ready_ref_[slot].idx];
  }
  DeviceGuard dg(device_);
  hip_check(hipEventSynchronize(e), "hipEventSynchronize");
}

std::vector<int> SlotPool::acquire_batch(int n, double timeout_s, uint64_t stream) {
  std::vector<int> out;
  std::vector<EvRef> waits;
  {
    std::unique_lock<std::mutex> lk(mu_);
    const auto pred = [&] { return closed_ || (producer_held_ + ext_held_ + n <= pb_ && (int)free_list_.size() >= n); };
    if (!pred()) {
      ++st_.produce_full;
      if (timeout_s < 0) cv_produce_.wait(lk, pred);
      else if (!cv_produce_.wait_for(lk, std::chrono::duration<double>(timeout_s), pred)) return out;
    }
    if (closed_) return out;
    for (int i = 0; i < n; ++i) {
      const int s = free_list_.front();
      free_list_.pop_front();
      state_[s] = kProducing;
      ++producer_held_;
      out.push_back(s);
      const EvRef r = free_ref_[s];
      if (!ref_live_locked(r)) continue;
      bool dup = false;
      for (const auto& w : waits) dup |= (w.idx == r.idx && w.gen == r.gen);
      if (!dup) waits.push_back(r);
    }
  }
  if (device_ >= 0 && !waits.empty()) {
    DeviceGuard dg(device_);
    for (const auto& w : waits) wait_ref(w, stream);
  }
  return out;
}

void SlotPool::commit_batch(const std::vector<int>& slots, const std::vector<SlotHeader>& hdrs, uint64_t stream) {
  check(slots.size() == hdrs.size(), "commit_batch: size mismatch");
  std::lock_guard<std::mutex> lk(mu_);
  for (int s : slots) {
    check_slot(s);
    check(state_[s] == kProducing, state_msg("commit_batch", kProducing, state_[s]));
  }
  const EvRef r = record_shared_locked(stream);
  for (size_t i = 0; i < slots.size(); ++i) {
    const int s = slots[i];
    hdr_[s] = hdrs[i];
    ready_ref_[s] = r;
    state_[s] = kProduced;
    produced_fifo_.push_back(s);
    ++st_.produced;
  }
  if (auto_route_) route_pending_locked();
}

void SlotPool::begin_send_batch(const std::vector<int>& slots, uint64_t stream) {
  std::vector<EvRef> waits;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (int s : slots) {
      check_slot(s);
      check(state_[s] == kProduced, state_msg("begin_send_batch", kProduced, state_[s]));
    }
    for (int s : slots) {
      erase_value(produced_fifo_, s);
      state_[s] = kSending;
      const EvRef r = ready_ref_[s];
      if (!ref_live_locked(r)) continue;
      bool dup = false;
      for (const auto& w : waits) dup |= (w.idx == r.idx && w.gen == r.gen);
      if (!dup) waits.push_back(r);
    }
  }
  if (device_ >= 0 && !waits.empty()) {
    DeviceGuard dg(device_);
    for (const auto& w : waits) wait_ref(w, stream);
  }
}

std::vector<int> SlotPool::begin_recv_batch(int n, uint64_t stream) {
  std::vector<int> out;
  std::vector<EvRef> waits;
  {
    std::lock_guard<std::mutex> lk(mu_);
    check(consumer_held_ + n <= cb_, "SlotPool.begin_recv_batch: not enough consumer credit");
    check((int)free_list_.size() >= n, "SlotPool.begin_recv_batch: not enough free slots");
    for (int i = 0; i < n; ++i) {
      const int s = free_list_.front();
      free_list_.pop_front();
      state_[s] = kReceiving;
      ++consumer_held_;
      out.push_back(s);
      const EvRef r = free_ref_[s];
      if (!ref_live_locked(r)) continue;
      bool dup = false;
      for (const auto& w : waits) dup |= (w.idx == r.idx && w.gen == r.gen);
      if (!dup) waits.push_back(r);
    }
  }
  if (device_ >= 0 && !waits.empty()) {
    DeviceGuard dg(device_);
    for (const auto& w : waits) wait_ref(w, stream);
  }
  return out;
}

void SlotPool::end_send_batch(const std::vector<int>& slots, uint64_t stream) {
  if (slots.empty()) return;
  std::lock_guard<std::mutex> lk(mu_);
  for (int s : slots) {
    check_slot(s);
    check(state_[s] == kSending, state_msg("end_send_batch", kSending, state_[s]));
  }
  const EvRef r = record_shared_locked(stream);
  for (int s : slots) {
    free_ref_[s] = r;
    state_[s] = kFree;
    --producer_held_;
    free_list_.push_back(s);
    ++st_.sent;
  }
  cv_produce_.notify_all();
}

void SlotPool::end_send_completed(const std::vector<int>& slots, bool to_external) {
  if (slots.empty()) return;
  std::lock_guard<std::mutex> lk(mu_);
  for (int s : slots) {
    check_slot(s);
    check(state_[s] == kSending, state_msg("end_send_completed", kSending, state_[s]));
  }
  for (int s : slots) {
    free_ref_[s] = EvRef{};   // the host saw the copy complete: the next writer needs no device wait
    state_[s] = kFree;
    free_list_.push_back(s);
    ++st_.sent;
  }
  producer_held_ -= (int)slots.size();
  if (to_external) ext_held_ += (int)slots.size();
  cv_produce_.notify_all();
}

void SlotPool::end_recv_batch(const std::vector<int>& slots, const std::vector<SlotHeader>& hdrs, uint64_t stream) {
  check(slots.size() == hdrs.size(), "end_recv_batch: size mismatch");
  if (slots.empty()) return;
  std::lock_guard<std::mutex> lk(mu_);
  for (int s : slots) {
    check_slot(s);
    check(state_[s] == kReceiving, state_msg("end_recv_batch", kReceiving, state_[s]));
  }
  const EvRef r = record_shared_locked(stream);
  for (size_t i = 0; i < slots.size(); ++i) {
    const int s = slots[i];
    hdr_[s] = hdrs[i];
    ready_ref_[s] = r;
    state_[s] = kReady;
    ready_fifo_.push_back(s);
    ++st_.received;
  }
  cv_ready_.notify_all();
}

SlotHeader SlotPool::header(int slot) const {
  check_slot(slot);
  std::lock_guard<std::mutex> lk(mu_);
  return hdr_[slot];
}

int SlotPool::state(int slot) const {
  check_slot(slot);
  std::lock_guard<std::mutex> lk(mu_);
  return state_[slot];
}

PoolStats SlotPool::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  return st_;
}

void SlotPool::route_pending_locked() {
  bool any = false;
  while (consumer_held_ < cb_ && !produced_fifo_.empty()) {
    const int s = produced_fifo_.front();
    produced_fifo_.pop_front();
    state_[s] = kReady;
    --producer_held_;
    ++consumer_held_;
    ready_fifo_.push_back(s);
    ++st_.routed_local;
    any = true;
  }
  if (any) {
    cv_ready_.notify_all();
    cv_produce_.notify_all();
  }
}

void SlotPool::set_auto_route(bool on) {
  std::lock_guard<std::mutex> lk(mu_);
  auto_route_ = on;
  if (on) route_pending_locked();
}

int SlotPool::pop_ready_locked() {
  const int s = ready_fifo_.front();
  ready_fifo_.pop_front();
  state_[s] = kLeased;
  ++st_.got;
  if (track_origins_) got_origins_.push_back(origin_[s]);
  return s;
}

void SlotPool::set_external_held(int n) {
  std::lock_guard<std::mutex> lk(mu_);
  const bool less = n < ext_held_;
  ext_held_ = std::max(0, n);
  if (less) cv_produce_.notify_all();
}

int SlotPool::producer_room() const {
  std::lock_guard<std::mutex> lk(mu_);
  return pb_ - producer_held_ - ext_held_;
}

void SlotPool::set_track_origins(bool on) {
  std::lock_guard<std::mutex> lk(mu_);
  track_origins_ = on;
}

void SlotPool::complete_recv_batch_from(const std::vector<int>& slots, const std::vector<SlotHeader>& hdrs,
                                        int64_t origin) {
  check(slots.size() == hdrs.size(), "complete_recv_batch: size mismatch");
  if (slots.empty()) return;
  std::lock_guard<std::mutex> lk(mu_);
  for (int s : slots) {
    check_slot(s);
    check(state_[s] == kReceiving, state_msg("complete_recv_batch", kReceiving, state_[s]));
  }
  for (size_t i = 0; i < slots.size(); ++i) {
    const int s = slots[i];
    hdr_[s] = hdrs[i];
    ready_ref_[s] = EvRef{};   // the writer completed its copy before the notice: nothing to wait on
    origin_[s] = origin;
    state_[s] = kReady;
    ready_fifo_.push_back(s);
    ++st_.received;
  }
  cv_ready_.notify_all();
}

std::vector<int64_t> SlotPool::take_got_origins() {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<int64_t> out;
  out.swap(got_origins_);
  return out;
}

int64_t SlotPool::origin(int slot) const {
  check_slot(slot);
  std::lock_guard<std::mutex> lk(mu_);
  return origin_[slot];
}

std::vector<int> SlotPool::pop_ready_for_return(int max_n) {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<int> out;
  while ((int)out.size() < max_n && !ready_fifo_.empty()) {
    const int s = ready_fifo_.front();
    ready_fifo_.pop_front();
    state_[s] = kLeased;
    out.push_back(s);
  }
  return out;
}

std::vector<int> SlotPool::reclaim_batch(int n, uint64_t stream) {
  std::vector<int> out;
  std::vector<EvRef> waits;
  {
    std::lock_guard<std::mutex> lk(mu_);
    while ((int)out.size() < n && producer_held_ < pb_ && !free_list_.empty()) {
      const int s = free_list_.front();
      free_list_.pop_front();
      state_[s] = kProducing;
      ++producer_held_;
      out.push_back(s);
      const EvRef r = free_ref_[s];
      if (!ref_live_locked(r)) continue;
      bool dup = false;
      for (const auto& w : waits) dup |= (w.idx == r.idx && w.gen == r.gen);
      if (!dup) waits.push_back(r);
    }
  }
  if (device_ >= 0 && !waits.empty()) {
    DeviceGuard dg(device_);
    for (const auto& w : waits) wait_ref(w, stream);
  }
  return out;
}

void SlotPool::commit_front_batch(const std::vector<int>& slots, const std::vector<SlotHeader>& hdrs,
                                  uint64_t stream) {
  check(slots.size() == hdrs.size(), "commit_front_batch: size mismatch");
  if (slots.empty()) return;
  std::lock_guard<std::mutex> lk(mu_);
  for (int s : slots) {
    check_slot(s);
    check(state_[s] == kProducing, state_msg("commit_front_batch", kProducing, state_[s]));
  }
  const EvRef r = record_shared_locked(stream);
  for (size_t i = slots.size(); i-- > 0;) {
    const int s = slots[i];
    hdr_[s] = hdrs[i];
    ready_ref_[s] = r;
    state_[s] = kProduced;
    produced_fifo_.push_front(s);
    ++st_.produced;
  }
  if (auto_route_) route_pending_locked();
}

std::vector<int> SlotPool::get_batch(int max_n, double timeout_s, uint64_t stream) {
  std::vector<int> out;
  std::vector<EvRef> waits;
  {
    std::unique_lock<std::mutex> lk(mu_);
    const auto pred = [&] { return closed_ || !ready_fifo_.empty(); };
    if (timeout_s > 0 && !pred()) cv_ready_.wait_for(lk, std::chrono::duration<double>(timeout_s), pred);
    while ((int)out.size() < max_n && !ready_fifo_.empty()) {
      const int s = pop_ready_locked();
      out.push_back(s);
      const EvRef r = ready_ref_[s];
      if (!ref_live_locked(r)) continue;
      bool dup = false;
      for (const auto& w : waits) dup |= (w.idx == r.idx && w.gen == r.gen);
      if (!dup) waits.push_back(r);
    }
  }
  if (device_ >= 0 && !waits.empty()) {
    DeviceGuard dg(device_);
    for (const auto& w : waits) wait_ref(w, stream);
  }
  if (!out.empty()) check_frames(out, stream);
  return out;
}

void SlotPool::set_verifier(std::shared_ptr<FrameVerifier> v) {
  std::lock_guard<std::mutex> lk(mu_);
  verifier_ = std::move(v);
}

std::shared_ptr<FrameVerifier> SlotPool::verifier() const {
  std::lock_guard<std::mutex> lk(mu_);
  return verifier_;
}

void SlotPool::check_frames(const std::vector<int>& slots, uint64_t stream) {
  std::shared_ptr<FrameVerifier> v;
  std::vector<uint64_t> ptrs;
  std::vector<int64_t> expect, gevt;
  bool remote = false;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!verifier_) return;
    v = verifier_;
    for (int s : slots) {
      check_slot(s);
      remote |= origin_[s] >= 0;
      if (ck_tagged(hdr_[s].aux) && !ptrs_.empty()) {
        ptrs.push_back(ptrs_[(size_t)s]);
        expect.push_back(hdr_[s].aux);
        gevt.push_back(hdr_[s].gevt);
      }
    }
  }
  if (remote || !ptrs.empty()) v->acquire(stream);
  if (!ptrs.empty()) v->verify(ptrs, expect, gevt, stream);
}

void SlotPool::release_batch(const std::vector<int>& slots, uint64_t stream) {
  std::lock_guard<std::mutex> lk(mu_);
  for (int slot : slots) {
    check_slot(slot);
    check(state_[slot] == kLeased, state_msg("release_batch", kLeased, state_[slot]));
  }
  const EvRef r = record_shared_locked(stream);
  for (int slot : slots) {
    free_ref_[slot] = r;
    state_[slot] = kFree;
    --consumer_held_;
    free_list_.push_back(slot);
    ++st_.released;
  }
  if (auto_route_) route_pending_locked();
  cv_produce_.notify_all();
}

std::vector<int> SlotPool::grant_batch(int max_n) {
  std::vector<int> out;
  std::lock_guard<std::mutex> lk(mu_);
  const int n = std::min(max_n, cb_ - consumer_held_);
  if (n <= 0) return out;
  DeviceGuard dg(device_);
  for (auto it = free_list_.begin(); it != free_list_.end() && (int)out.size() < n;) {
    const int s = *it;
    const EvRef r = free_ref_[s];
    if (device_ >= 0 && ref_live_locked(r)) {
      const hipError_t q = hipEventQuery(ev_[r.idx]);
      if (q == hipErrorNotReady) {
        ++it;
        continue;
      }
      hip_check(q, "hipEventQuery (grant)");
    }
    it = free_list_.erase(it);
    state_[s] = kReceiving;
    ++consumer_held_;
    out.push_back(s);
  }
  return out;
}

void SlotPool::complete_recv_batch(const std::vector<int>& slots, const std::vector<SlotHeader>& hdrs) {
  check(slots.size() == hdrs.size(), "complete_recv_batch: size mismatch");
  if (slots.empty()) return;
  std::lock_guard<std::mutex> lk(mu_);
  for (int s : slots) {
    check_slot(s);
    check(state_[s] == kReceiving, state_msg("complete_recv_batch", kReceiving, state_[s]));
  }
  for (size_t i = 0; i < slots.size(); ++i) {
    const int s = slots[i];
    hdr_[s] = hdrs[i];
    ready_ref_[s] = EvRef{};   // the writer completed its copy before the notice: nothing to wait on
    state_[s] = kReady;
    ready_fifo_.push_back(s);
    ++st_.received;
  }
  cv_ready_.notify_all();
}

void SlotPool::cancel_recv_batch(const std::vector<int>& slots) {
  if (slots.empty()) return;
  std::lock_guard<std::mutex> lk(mu_);
  for (int s : slots) {
    check_slot(s);
    check(state_[s] == kReceiving, state_msg("cancel_recv_batch", kReceiving, state_[s]));
  }
  for (int s : slots) {
    state_[s] = kFree;
    --consumer_held_;
    free_list_.push_back(s);
  }
  cv_produce_.notify_all();
}

void SlotPool::unsend_batch(const std::vector<int>& slots) {
  if (slots.empty()) return;
  std::lock_guard<std::mutex> lk(mu_);
  for (int s : slots) {
    check_slot(s);
    check(state_[s] == kSending, state_msg("unsend_batch", kSending, state_[s]));
  }
  for (auto it = slots.rbegin(); it != slots.rend(); ++it) {
    state_[*it] = kProduced;
    produced_fifo_.push_front(*it);
  }
}

int SlotPool::reoffer_batch(const std::vector<int>& slots, uint64_t stream) {
  std::lock_guard<std::mutex> lk(mu_);
  int n = 0;
  for (int s : slots) {
    check_slot(s);
    check(state_[s] == kLeased, state_msg("reoffer_batch", kLeased, state_[s]));
    if (producer_held_ + ext_held_ >= pb_) break;
    ready_ref_[s] = record_shared_locked(stream);
    state_[s] = kProduced;
    --consumer_held_;
    ++producer_held_;
    produced_fifo_.push_back(s);
    ++n;
  }
  if (n > 0) cv_produce_.notify_one();
  return n;
}

int SlotPool::relay_ready(int max_n) {
  std::lock_guard<std::mutex> lk(mu_);
  const int room = pb_ - producer_held_ - ext_held_;
  int n = std::min<int>(std::min(max_n, room), (int)ready_fifo_.size());
  for (int i = 0; i < n; ++i) {
    const int s = pop_ready_locked();   // counts as taken: its producer learns it left the queue
    state_[s] = kProduced;              // ready_ref_ (the frame's data) is kept
    --consumer_held_;
    ++producer_held_;
    produced_fifo_.push_back(s);
  }
  if (n > 0) cv_produce_.notify_one();
  return std::max(0, n);
}

std::vector<SlotHeader> SlotPool::headers(const std::vector<int>& slots) const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<SlotHeader> out;
  out.reserve(slots.size());
  for (int s : slots) {
    check_slot(s);
    out.push_back(hdr_[s]);
  }
  return out;
}

void SlotPool::wake_producers() {
  std::lock_guard<std::mutex> lk(mu_);
  cv_produce_.notify_all();
}

bool SlotPool::closed() const {
  std::lock_guard<std::mutex> lk(mu_);
  return closed_;
}

void SlotPool::wake_all() {
  std::lock_guard<std::mutex> lk(mu_);
  closed_ = true;
  cv_produce_.notify_all();
  cv_ready_.notify_all();
}

// ---------------------------------------------------------------------------------------
namespace {
struct RunHeader {
  char magic[8];
  uint32_t version;
  uint32_t header_bytes;
  char det[64];
  uint32_t ndim;
  uint32_t pad0;
  uint64_t shape[4];
  uint32_t dtype_bytes;
  uint32_t pad1;
  uint64_t n_events;
  uint64_t record_bytes;
};
constexpr int64_t kRecordHeaderBytes = 32;

void pread_full(int fd, void* dst, size_t n, off_t off) {
  char* p = static_cast<char*>(dst);
  while (n > 0) {
    const ssize_t r = ::pread(fd, p, n, off);
    if (r < 0 && errno == EINTR) continue;
    check(r > 0, "RawRunReader: short read");
    p += r;
    n -= (size_t)r;
    off += r;
  }
}
}  // namespace

MappedFile::MappedFile(const std::string& path, bool register_with_hip) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  check(fd >= 0, "MappedFile: cannot open " + path);
  struct stat sb;
  if (fstat(fd, &sb) != 0 || sb.st_size <= 0) {
    ::close(fd);
    throw std::runtime_error("psana_ray_amd: MappedFile: empty or unreadable " + path);
  }
  bytes_ = (size_t)sb.st_size;
  // MAP_POPULATE: fault the pages in now (registration pins them anyway)
  base_ = mmap(nullptr, bytes_, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
  ::close(fd);
  check(base_ != MAP_FAILED, "MappedFile: mmap failed for " + path);
  if (register_with_hip) {
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = hipHostRegister(base_, bytes_, hipHostRegisterReadOnly);
    if (e != hipSuccess) {
      munmap(base_, bytes_);
      base_ = nullptr;
      throw std::runtime_error(std::string("psana_ray_amd: MappedFile: hipHostRegister failed: ") +
                               hipGetErrorString(e));
    }
    registered_ = true;
    register_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
}

MappedFile::~MappedFile() {
  if (registered_) (void)hipHostUnregister(base_);
  if (base_ != nullptr) munmap(base_, bytes_);
}

RawRunReader::RawRunReader(const std::string& path, int n_threads) : n_threads_(n_threads < 1 ? 1 : n_threads) {
  fd_ = ::open(path.c_str(), O_RDONLY);
  check(fd_ >= 0, "RawRunReader: cannot open " + path);
  RunHeader h;
  pread_full(fd_, &h, sizeof(h), 0);
  check(std::memcmp(h.magic, "PRAWRUN1", 8) == 0, "RawRunReader: bad magic in " + path);
  header_bytes_ = h.header_bytes;
  n_events_ = (int64_t)h.n_events;
  record_bytes_ = (int64_t)h.record_bytes;
  frame_bytes_ = record_bytes_ - kRecordHeaderBytes;
  check(frame_bytes_ > 0, "RawRunReader: bad record size");
}

RawRunReader::RawRunReader(const std::string& path, int n_threads, std::vector<int64_t> payload_off,
                           std::vector<int64_t> gevt, std::vector<double> photon_energy, int64_t frame_bytes)
    : n_threads_(n_threads < 1 ? 1 : n_threads), off_(std::move(payload_off)), gevt_(std::move(gevt)),
      pe_(std::move(photon_energy)) {
  check(!off_.empty(), "RawRunReader: empty event index");
  check(off_.size() == gevt_.size() && off_.size() == pe_.size(), "RawRunReader: index columns differ in length");
  check(frame_bytes > 0, "RawRunReader: bad frame size");
  fd_ = ::open(path.c_str(), O_RDONLY);
  check(fd_ >= 0, "RawRunReader: cannot open " + path);
  struct stat sb;
  check(fstat(fd_, &sb) == 0, "RawRunReader: fstat failed");
  for (int64_t o : off_)
    check(o >= 0 && o + frame_bytes <= (int64_t)sb.st_size, "RawRunReader: index points past the end of " + path);
  n_events_ = (int64_t)off_.size();
  frame_bytes_ = frame_bytes;
}

RawRunReader::~RawRunReader() {
  if (fd_ >= 0) ::close(fd_);
}

std::vector<std::pair<int64_t, double>> RawRunReader::read(const std::vector<int64_t>& events,
                                                           const std::vector<uint64_t>& dst_ptrs) {
  check(events.size() == dst_ptrs.size(), "RawRunReader.read: events / dst size mismatch");
  const size_t n = events.size();
  std::vector<std::pair<int64_t, double>> meta(n);
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= n) return;
      check(events[i] >= 0 && events[i] < n_events_, "RawRunReader.read: event index out of range");
      if (!off_.empty()) {
        meta[i] = {gevt_[events[i]], pe_[events[i]]};
        pread_full(fd_, reinterpret_cast<void*>(dst_ptrs[i]), (size_t)frame_bytes_, (off_t)off_[events[i]]);
        continue;
      }
      const off_t off = (off_t)(header_bytes_ + events[i] * record_bytes_);
      int64_t rh[4];
      pread_full(fd_, rh, sizeof(rh), off);
      double pe;
      std::memcpy(&pe, &rh[1], sizeof(double));
      meta[i] = {rh[0], pe};
      pread_full(fd_, reinterpret_cast<void*>(dst_ptrs[i]), (size_t)frame_bytes_, off + kRecordHeaderBytes);
    }
  };
  const int nt = (int)std::min<size_t>((size_t)n_threads_, n);
  std::vector<std::future<void>> fs;
  for (int t = 1; t < nt; ++t) fs.push_back(std::async(std::launch::async, work));
  work();
  for (auto& f : fs) f.get();
  return meta;
}

// ---------------------------------------------------------------------------------------
// hipMemcpyDefault: pinned host -> HBM (the staging path) or HBM -> HBM (device-resident source)
void memcpy_h2d_async(uint64_t dst, uint64_t src, size_t bytes, uint64_t stream) {
  hip_check(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), bytes,
                           hipMemcpyDefault, reinterpret_cast<hipStream_t>(stream)),
            "hipMemcpyAsync");
}

void memcpy_h2d_batch(const std::vector<uint64_t>& dst, const std::vector<uint64_t>& src, size_t bytes,
                      uint64_t stream) {
  check(dst.size() == src.size(), "memcpy_h2d_batch: size mismatch");
  // coalesce runs that are contiguous on both sides into one copy
  size_t i = 0;
  while (i < dst.size()) {
    size_t j = i + 1;
    while (j < dst.size() && dst[j] == dst[j - 1] + bytes && src[j] == src[j - 1] + bytes) ++j;
    memcpy_h2d_async(dst[i], src[i], bytes * (j - i), stream);
    i = j;
  }
}

}  // namespace pr
