#include "xport_engine.h"

#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <cmath>

#include "common.h"
#include "trace.h"

namespace pr {

std::vector<int32_t> plan_round_native(const std::vector<int64_t>& offers, const std::vector<int64_t>& credits,
                                       int64_t round_id, int policy);

namespace {

constexpr uint64_t kMagic = 0x3152545843525350ull;  // "PSRCXTR1"
constexpr size_t kSegHeader = 4096;

struct SegHeader {
  uint64_t magic;
  int32_t world, vec_words;
  int64_t outbox_bytes;
  uint64_t block_bytes;
  std::atomic<uint64_t> ready;  // set last by the creator
};

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

void nap_ns(long ns) {
  timespec ts{0, ns};
  nanosleep(&ts, nullptr);
}

// A peer that exited is either gone (ESRCH) or a zombie its parent has not reaped yet (state Z/X
// in /proc/<pid>/stat) -- e.g. under multiprocessing until join().
bool pid_alive(pid_t pid) {
  if (kill(pid, 0) != 0 && errno == ESRCH) return false;
  char path[64];
  snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
  FILE* f = fopen(path, "r");
  if (f == nullptr) return true;  // no procfs view (other pid namespace): trust kill()
  char buf[512];
  const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[n] = 0;
  const char* rp = strrchr(buf, ')');   // comm may contain spaces / parentheses
  if (rp == nullptr || rp[1] == 0 || rp[2] == 0) return true;
  return rp[2] != 'Z' && rp[2] != 'X';
}

}  // namespace

// One cache line per contended word: the waiters of different ranks never share a line with
// the word a rank is writing.
struct ShmControl::Block {
  std::atomic<uint64_t> ctrl_seq;
  char pad0[56];
  std::atomic<uint64_t> data_seq;
  char pad1[56];
  std::atomic<int64_t> pid;
  std::atomic<uint32_t> failed;
  std::atomic<uint32_t> attached;
  char pad2[48];
  // followed by: int64 vec[2][vec_words], then the outbox (4 KiB aligned)
};
static_assert(sizeof(std::atomic<uint64_t>) == 8 && std::atomic<uint64_t>::is_always_lock_free,
              "lock-free 64-bit atomics are required in shared memory");

ShmControl::ShmControl(const std::string& name, bool create, int rank, int world, int vec_words,
                       int64_t outbox_bytes, double timeout_s)
    : name_(name), rank_(rank), world_(world), vec_words_(vec_words), outbox_bytes_(outbox_bytes),
      timeout_s_(timeout_s) {
  check(!name.empty() && name[0] == '/', "ShmControl: name must start with '/'");
  check(world >= 1 && rank >= 0 && rank < world, "ShmControl: bad rank/world");
  check(vec_words > 0 && outbox_bytes >= 0, "ShmControl: bad sizes");
  const size_t vec_off = round_up(sizeof(Block), 64);
  const size_t box_off = round_up(vec_off + 2 * (size_t)vec_words * sizeof(int64_t), 4096);
  block_bytes_ = round_up(box_off + (size_t)outbox_bytes, 4096);
  total_bytes_ = kSegHeader + block_bytes_ * (size_t)world;
  int fd = -1;
  if (create) {
    fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    check(fd >= 0, "ShmControl: shm_open(create " + name + ") failed: " + strerror(errno));
    if (ftruncate(fd, (off_t)total_bytes_) != 0) {
      const int e = errno;
      close(fd);
      shm_unlink(name.c_str());
      throw std::runtime_error(std::string("psana_ray_amd: ShmControl: ftruncate failed: ") + strerror(e));
    }
    owner_ = true;
  } else {
    const double t0 = now_s();
    while (true) {
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat sb;
        if (fstat(fd, &sb) == 0 && (size_t)sb.st_size >= total_bytes_) break;
        close(fd);
        fd = -1;
      }
      check(now_s() - t0 < timeout_s, "ShmControl: timed out attaching to " + name);
      nap_ns(1000000);
    }
  }
  void* p = mmap(nullptr, total_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    if (owner_) shm_unlink(name.c_str());
    throw std::runtime_error(std::string("psana_ray_amd: ShmControl: mmap failed: ") + strerror(errno));
  }
  base_ = static_cast<uint8_t*>(p);
  auto* h = reinterpret_cast<SegHeader*>(base_);
  if (create) {
    // ftruncate zero-filled the segment: every sequence word starts at 0
    h->magic = kMagic;
    h->world = world;
    h->vec_words = vec_words;
    h->outbox_bytes = outbox_bytes;
    h->block_bytes = block_bytes_;
    h->ready.store(1, std::memory_order_release);
  } else {
    const double t0 = now_s();
    while (h->ready.load(std::memory_order_acquire) != 1) {
      if (now_s() - t0 > timeout_s) {
        munmap(base_, total_bytes_);
        base_ = nullptr;
        throw std::runtime_error("psana_ray_amd: ShmControl: segment " + name + " never became ready");
      }
      nap_ns(100000);
    }
    if (h->magic != kMagic || h->world != world || h->vec_words != vec_words || h->outbox_bytes != outbox_bytes ||
        h->block_bytes != block_bytes_) {
      munmap(base_, total_bytes_);
      base_ = nullptr;
      throw std::runtime_error("psana_ray_amd: ShmControl: segment " + name +
                               " layout differs (world / max_offer / frame size must agree on every rank)");
    }
  }
  Block* me = block(rank_);
  me->pid.store((int64_t)getpid(), std::memory_order_relaxed);
  me->failed.store(0, std::memory_order_relaxed);
  me->attached.store(1, std::memory_order_release);
}

ShmControl::~ShmControl() {
  if (base_ != nullptr) munmap(base_, total_bytes_);
  if (owner_ && !unlinked_) shm_unlink(name_.c_str());
}

void ShmControl::unlink() {
  if (owner_ && !unlinked_) {
    shm_unlink(name_.c_str());
    unlinked_ = true;
  }
}

ShmControl::Block* ShmControl::block(int r) const {
  return reinterpret_cast<Block*>(base_ + kSegHeader + block_bytes_ * (size_t)r);
}

int64_t* ShmControl::vec_slot(int r, int64_t round) const {
  uint8_t* b = reinterpret_cast<uint8_t*>(block(r)) + round_up(sizeof(Block), 64);
  return reinterpret_cast<int64_t*>(b) + (size_t)(round & 1) * vec_words_;
}

uint8_t* ShmControl::outbox(int r) const {
  check(r >= 0 && r < world_, "ShmControl.outbox: rank out of range");
  const size_t vec_off = round_up(sizeof(Block), 64);
  const size_t box_off = round_up(vec_off + 2 * (size_t)vec_words_ * sizeof(int64_t), 4096);
  return reinterpret_cast<uint8_t*>(block(r)) + box_off;
}

void ShmControl::set_failed() {
  if (base_ != nullptr) block(rank_)->failed.store(1, std::memory_order_release);
}

void ShmControl::wait_seq(int peer, int which, uint64_t target) {
  Block* b = block(peer);
  std::atomic<uint64_t>& w = which == 0 ? b->ctrl_seq : b->data_seq;
  if (w.load(std::memory_order_acquire) >= target) return;
  // spin briefly (a peer usually arrives within microseconds), then yield, then nap: ranks
  // can outnumber cores (tests) and a spinning waiter must not starve the peer it waits for
  const double t0 = now_s();
  double last_pid_check = t0;
  for (uint64_t it = 1;; ++it) {
    if (w.load(std::memory_order_acquire) >= target) return;
    if (it < 256) {
      __builtin_ia32_pause();
      continue;
    }
    if (cancelled_.load(std::memory_order_relaxed))
      throw std::runtime_error("psana_ray_amd: shared-queue transport cancelled");
    if (b->failed.load(std::memory_order_acquire) != 0)
      throw std::runtime_error("psana_ray_amd: shared-queue peer rank " + std::to_string(peer) + " failed");
    const double t = now_s();
    if (t - t0 < 2e-4) {
      sched_yield();
    } else {
      nap_ns(t - t0 < 5e-3 ? 20000 : 200000);
    }
    if (t - last_pid_check > 0.05) {
      last_pid_check = t;
      const int64_t pid = b->pid.load(std::memory_order_relaxed);
      if (check_pids_ && pid > 0 && !pid_alive((pid_t)pid))
        throw std::runtime_error("psana_ray_amd: shared-queue peer rank " + std::to_string(peer) + " (pid " +
                                 std::to_string(pid) + ") died");
      if (t - t0 > timeout_s_)
        throw std::runtime_error("psana_ray_amd: shared-queue peer rank " + std::to_string(peer) +
                                 " did not answer within " + std::to_string(timeout_s_) + " s");
    }
  }
}

void ShmControl::allgather(int64_t round, const int64_t* vec, int64_t* out) {
  check(round >= 0, "ShmControl.allgather: negative round");
  // Double buffering by round parity is enough: a peer writes the buffer of round r+2 only
  // after it read everybody's round r+1 sequence, which this rank publishes only after it
  // finished reading round r.
  memcpy(vec_slot(rank_, round), vec, (size_t)vec_words_ * sizeof(int64_t));
  block(rank_)->ctrl_seq.store((uint64_t)round + 1, std::memory_order_release);
  for (int k = 0; k < world_; ++k) {
    const int r = (rank_ + k) % world_;
    if (r != rank_) wait_seq(r, 0, (uint64_t)round + 1);
    memcpy(out + (size_t)r * vec_words_, vec_slot(r, round), (size_t)vec_words_ * sizeof(int64_t));
  }
}

void ShmControl::publish_data(int64_t round) {
  block(rank_)->data_seq.store((uint64_t)round + 1, std::memory_order_release);
}

void ShmControl::wait_data(int peer, int64_t round) {
  if (peer != rank_) wait_seq(peer, 1, (uint64_t)round + 1);
}

// ---------------------------------------------------------------------------------------
TransportEngine::TransportEngine(SlotPool* pool, ShmControl* ctrl, RcclTransport* rccl, uint64_t ring_base,
                                 int64_t slot_bytes, int rank, int world, const std::vector<int>& producer_ranks,
                                 bool is_producer, bool is_consumer, int policy, int max_offer, bool loopback,
                                 uint64_t stream, int device)
    : pool_(pool), ctrl_(ctrl), rccl_(rccl), ring_base_(ring_base), slot_bytes_(slot_bytes), rank_(rank),
      world_(world), producer_ranks_(producer_ranks), is_producer_(is_producer), is_consumer_(is_consumer),
      policy_(policy), max_offer_(max_offer), loopback_(loopback), stream_(stream), device_(device) {
  check(pool != nullptr && ctrl != nullptr, "TransportEngine: pool and control plane are required");
  check(ctrl->world() == world && ctrl->rank() == rank, "TransportEngine: control plane rank/world mismatch");
  check(ctrl->vec_words() == vec_words_for(max_offer), "TransportEngine: control vector size mismatch");
  check(policy >= 0 && policy <= 2, "TransportEngine: unknown routing policy");
  check(slot_bytes > 0 && ring_base != 0, "TransportEngine: empty ring");
  if (rccl == nullptr)
    check(ctrl->outbox_bytes() >= (int64_t)max_offer * slot_bytes,
          "TransportEngine: host data plane needs max_offer * slot_bytes of outbox");
  else
    check(rccl->world() == world && rccl->rank() == rank, "TransportEngine: RCCL rank/world mismatch");
  for (int p : producer_ranks) check(p >= 0 && p < world, "TransportEngine: producer rank out of range");
  vec_.assign((size_t)vec_words_for(max_offer), 0);
  all_.assign((size_t)world * vec_.size(), 0);
  eos_from_.assign((size_t)world, false);
  if (!is_producer) producer_finished_.store(true);
  if (!is_consumer) consumer_closed_.store(true);
}

TransportEngine::~TransportEngine() {
  stop_.store(true);
  if (running_.load()) ctrl_->cancel();
  if (th_.joinable()) th_.join();
}

std::string TransportEngine::error() const {
  std::lock_guard<std::mutex> lk(mu_);
  return error_;
}

XportStats TransportEngine::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  return st_;
}

void TransportEngine::fail(const std::string& msg) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (error_.empty()) error_ = msg;
  }
  ctrl_->set_failed();
  if (rccl_ != nullptr) {
    try {
      rccl_->abort();   // never leave RCCL kernels waiting on a dead peer
    } catch (...) {
    }
  }
  pool_->wake_all();
}

int64_t TransportEngine::step() {
  const double t0 = now_s();
  const int W = (int)vec_.size();
  std::vector<int> offers;
  if (is_producer_) offers = pool_->produced(max_offer_);
  const bool closed = consumer_closed_.load();
  // the routing policy rides in bits 8..9: every rank must derive the SAME plan
  int64_t flags = (is_producer_ ? kProducer : 0) | (is_consumer_ ? kConsumer : 0) | ((int64_t)policy_ << 8);
  if (producer_finished_.load() && offers.empty() && pool_->n_produced() == 0) flags |= kEos;
  if (closed) flags |= kClosed;
  std::fill(vec_.begin(), vec_.end(), 0);
  vec_[0] = (int64_t)offers.size();
  vec_[1] = closed ? 0 : pool_->credits();
  vec_[2] = flags;
  vec_[3] = round_;
  if (!offers.empty()) {
    const std::vector<SlotHeader> hs = pool_->headers(offers);
    for (size_t i = 0; i < hs.size(); ++i) {
      int64_t* w = &vec_[kHdr + kPerOffer * i];
      w[0] = hs[i].rank;
      w[1] = hs[i].idx;
      w[2] = hs[i].gevt;
      memcpy(&w[3], &hs[i].photon_energy, sizeof(double));  // NaN bit pattern = None
    }
  }
  {
    trace::Range tr("transport.ctrl_allgather");
    ctrl_->allgather(round_, vec_.data(), all_.data());
  }
  // every rank has attached once round 0 completed: drop the name so nothing outlives the job
  if (round_ == 0) ctrl_->unlink();
  const double t1 = now_s();
  std::vector<int64_t> offer_n(world_), credits(world_);
  bool any_consumer = false;
  for (int r = 0; r < world_; ++r) {
    const int64_t* v = &all_[(size_t)r * W];
    check(v[3] == round_, "TransportEngine: ranks disagree on the round number");
    check(((v[2] >> 8) & 3) == policy_, "TransportEngine: ranks use different routing policies");
    offer_n[r] = v[0];
    credits[r] = v[1];
    if (v[2] & kEos) eos_from_[r] = true;
    if ((v[2] & kConsumer) && !(v[2] & kClosed)) any_consumer = true;
  }
  consumers_gone_.store(!any_consumer);
  const std::vector<int32_t> plan = plan_round_native(offer_n, credits, round_, policy_);
  const int n_plan = (int)plan.size() / 3;
  std::vector<int> local, send_slots, send_peer, recv_peer, recv_ord;
  std::vector<SlotHeader> recv_hdr;
  std::vector<int> ordinal(world_, 0);   // per-producer position in its outbox (host data plane)
  for (int k = 0; k < n_plan; ++k) {
    const int p = plan[3 * k], i = plan[3 * k + 1], c = plan[3 * k + 2];
    if (p == c && !loopback_) {
      if (p == rank_) local.push_back(offers[i]);
      continue;
    }
    const int ord = ordinal[p]++;
    if (p == rank_) {
      send_slots.push_back(offers[i]);
      send_peer.push_back(c);
    }
    if (c == rank_) {
      const int64_t* w = &all_[(size_t)p * W + kHdr + kPerOffer * i];
      SlotHeader h;
      h.rank = w[0];
      h.idx = w[1];
      h.gevt = w[2];
      memcpy(&h.photon_energy, &w[3], sizeof(double));
      recv_peer.push_back(p);
      recv_ord.push_back(ord);
      recv_hdr.push_back(h);
    }
  }
  for (int s : local) pool_->route_local(s);
  int64_t nb_sent = 0, nb_recv = 0;
  if (rccl_ != nullptr) {
    if (!send_slots.empty() || !recv_peer.empty())
      rccl_->round(pool_, ring_base_, slot_bytes_, send_slots, send_peer, recv_peer, recv_hdr, stream_);
    if (st_.rounds % 64 == 0) {
      const std::string e = rccl_->async_error();
      check(e.empty(), "RCCL asynchronous error: " + e);
    }
  } else {
    // host pools: copy through the shared-memory outboxes (CPU tests / CPU queues)
    if (!send_slots.empty()) {
      pool_->begin_send_batch(send_slots, 0);
      uint8_t* box = ctrl_->outbox(rank_);
      for (size_t j = 0; j < send_slots.size(); ++j)
        memcpy(box + (size_t)j * slot_bytes_, reinterpret_cast<const void*>(ring_base_ + (uint64_t)send_slots[j] * slot_bytes_),
               (size_t)slot_bytes_);
      pool_->end_send_batch(send_slots, 0);
    }
    ctrl_->publish_data(round_);
    if (!recv_peer.empty()) {
      const std::vector<int> rs = pool_->begin_recv_batch((int)recv_peer.size(), 0);
      check(rs.size() == recv_peer.size(), "TransportEngine: not enough free consumer slots (credit accounting)");
      std::vector<bool> waited(world_, false);
      for (size_t j = 0; j < rs.size(); ++j) {
        const int p = recv_peer[j];
        if (!waited[p]) {
          ctrl_->wait_data(p, round_);
          waited[p] = true;
        }
        memcpy(reinterpret_cast<void*>(ring_base_ + (uint64_t)rs[j] * slot_bytes_),
               ctrl_->outbox(p) + (size_t)recv_ord[j] * slot_bytes_, (size_t)slot_bytes_);
      }
      pool_->end_recv_batch(rs, recv_hdr, 0);
    }
  }
  nb_sent = (int64_t)send_slots.size() * slot_bytes_;
  nb_recv = (int64_t)recv_peer.size() * slot_bytes_;
  bool all_eos = true;
  for (int p : producer_ranks_) all_eos = all_eos && eos_from_[p];
  ++round_;
  const double t2 = now_s();
  {
    std::lock_guard<std::mutex> lk(mu_);
    ++st_.rounds;
    if (n_plan == 0) ++st_.idle_rounds;
    st_.frames_routed += n_plan;
    st_.frames_local += (int64_t)local.size();
    st_.frames_sent += (int64_t)send_slots.size();
    st_.frames_recv += (int64_t)recv_peer.size();
    st_.bytes_sent += nb_sent;
    st_.bytes_recv += nb_recv;
    st_.round_s += t2 - t0;
    st_.ctrl_s += t1 - t0;
    st_.data_s += t2 - t1;
  }
  if (all_eos) done_.store(true);
  return n_plan;
}

void TransportEngine::loop() {
  try {
    if (device_ >= 0) hip_check(hipSetDevice(device_), "hipSetDevice");
    double idle = 0;
    while (!done_.load() && !stop_.load()) {
      if (step() == 0) {
        // every rank sees the same (global) plan size, so all ranks back off together
        idle = idle > 0 ? std::min(1e-3, idle * 2) : 5e-5;
        nap_ns((long)(idle * 1e9));
      } else {
        idle = 0;
      }
    }
  } catch (const std::exception& e) {
    fail(e.what());
  } catch (...) {
    fail("unknown error in the transport engine");
  }
  pool_->wake_all();
  running_.store(false);
}

void TransportEngine::start() {
  check(!th_.joinable(), "TransportEngine: already started");
  running_.store(true);
  th_ = std::thread([this] { loop(); });
}

bool TransportEngine::join(double timeout_s) {
  if (!th_.joinable()) return true;
  const double t0 = now_s();
  while (running_.load()) {
    if (timeout_s >= 0 && now_s() - t0 > timeout_s) return false;
    nap_ns(1000000);
  }
  th_.join();
  return true;
}

}  // namespace pr
