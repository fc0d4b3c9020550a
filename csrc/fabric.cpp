#include "fabric.h"

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>

#include "common.h"
#include "kernels.h"
#include "lifecycle.h"
#include "streams.h"
#include "trace.h"

namespace pr {

namespace {

constexpr uint64_t kLinkMagic = 0x314B4E494C525350ull;  // "PSRLINK1"
constexpr int32_t kLinkVersion = 5;
constexpr int32_t kNoticeReturned = 1;   // the grant comes back unused (producer finished / closing)
constexpr int32_t kNoticeReclaimed = 2;  // a returned frame was copied out: its slot is free again
constexpr int32_t kNoticeRejected = 4;   // a returned frame was refused (EOS posted): route it elsewhere
constexpr double kPidCheckS = 0.05;
constexpr double kKeeperDebounceS = 0.1;   // a live producer's backlog must lack other credit this long

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void nap_ns(long ns) {
  timespec ts{0, ns};
  nanosleep(&ts, nullptr);
}

size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

struct Notice {
  int32_t slot;
  int32_t flags;
  int64_t rank, idx, gevt;
  double photon_energy;
  int64_t aux;
};
static_assert(sizeof(Notice) == 48, "Notice layout");

// The mailbox of one link.  Written by the consumer at creation; afterwards every field has ONE
// writer: grants/g_head, returns/r_head, taken and consumer_closed by the consumer, the rest by the
// producer.  Counters are monotonic; ring entries are written before the counter is released and
// read after it is acquired.  Every slot of the consumer ring has at most one open exchange on a
// link (granted and not answered, or returned and not answered), so no ring holds more than
// n_slots entries.
struct SegDesc {          // one allocation of an HBM consumer ring
  uint8_t handle[HIP_IPC_HANDLE_SIZE];
  int64_t offset;         // of slot `first` inside the allocation
  int32_t first, n;       // slots [first, first + n) are contiguous in it
};

struct alignas(64) LinkSeg {
  uint64_t magic;
  int32_t version;
  int32_t n_slots;        // slots of the consumer ring = capacity of the grant / notice rings
  int64_t slot_bytes;
  int64_t producer_mid, consumer_mid;
  int64_t consumer_pid;
  int32_t kind;           // 0 host shared memory, 1 HIP IPC
  int32_t consumer_device;
  int32_t n_segs;
  int32_t consumer_kind;  // 0 consumer, 1 queue keeper
  char consumer_pci[32];  // PCI bus id of the consumer ring's GPU (device indices differ between
                          // processes whose launcher restricts the visible GPUs)
  char ring_name[128];
  SegDesc segs[QueueFabric::kMaxSegments];
  std::atomic<uint64_t> ready;
  alignas(64) std::atomic<int64_t> producer_pid;       // 0 until the producer attached
  alignas(64) std::atomic<uint64_t> g_head;            // consumer -> producer
  alignas(64) std::atomic<uint64_t> g_tail;
  alignas(64) std::atomic<uint64_t> n_head;            // producer -> consumer
  alignas(64) std::atomic<uint64_t> n_tail;
  alignas(64) std::atomic<uint32_t> consumer_closed;
  alignas(64) std::atomic<uint32_t> producer_eos;
  std::atomic<uint32_t> producer_detached;
  std::atomic<uint32_t> producer_ack_closed;           // no copy into this ring is in flight any more
  std::atomic<int64_t> producer_backlog;               // frames waiting at the producer (demand hint)
  std::atomic<int64_t> producer_budget;                // its pool budget (keeper watermark)
  std::atomic<int64_t> producer_other_credit;          // credit it holds from non-keeper consumers
  alignas(64) std::atomic<uint64_t> taken;             // consumer: frames of this link it took (get)
  std::atomic<int64_t> consumer_ready;                 // consumer: frames ready to read in its whole shard
  std::atomic<uint32_t> consumer_self_fed;             // consumer: its own process produces (and feeds it)
  std::atomic<uint32_t> consumer_published;            // consumer: the two above hold real values (first pass)
  std::atomic<uint32_t> returns_final;                 // consumer (closing): no return will follow
  std::atomic<uint32_t> producer_seen_closed;          // producer: no frame notice will follow
  alignas(64) std::atomic<uint64_t> r_head;            // consumer -> producer: returned frames
  alignas(64) std::atomic<uint64_t> r_tail;
};
static_assert(std::atomic<uint64_t>::is_always_lock_free && std::atomic<int64_t>::is_always_lock_free,
              "lock-free 64-bit atomics are required in shared memory");

size_t grants_off() { return round_up(sizeof(LinkSeg), 64); }
size_t notices_off(int n) { return grants_off() + round_up((size_t)n * sizeof(int32_t), 64); }
size_t returns_off(int n) { return notices_off(n) + round_up((size_t)n * sizeof(Notice), 64); }
size_t seg_bytes(int n) { return round_up(returns_off(n) + (size_t)n * sizeof(Notice), 4096); }
int32_t* seg_grants(LinkSeg* s) { return reinterpret_cast<int32_t*>(reinterpret_cast<uint8_t*>(s) + grants_off()); }
Notice* seg_notices(LinkSeg* s) {
  return reinterpret_cast<Notice*>(reinterpret_cast<uint8_t*>(s) + notices_off(s->n_slots));
}
Notice* seg_returns(LinkSeg* s) {
  return reinterpret_cast<Notice*>(reinterpret_cast<uint8_t*>(s) + returns_off(s->n_slots));
}
Notice make_notice(int32_t slot, int32_t flags, const SlotHeader& h) {
  Notice nt;
  nt.slot = slot;
  nt.flags = flags;
  nt.rank = h.rank;
  nt.idx = h.idx;
  nt.gevt = h.gevt;
  nt.photon_energy = h.photon_energy;
  nt.aux = h.aux;
  return nt;
}
SlotHeader header_of(const Notice& nt) {
  SlotHeader hd;
  hd.rank = nt.rank;
  hd.idx = nt.idx;
  hd.gevt = nt.gevt;
  hd.photon_energy = nt.photon_energy;
  hd.aux = nt.aux;
  return hd;
}

}  // namespace

// A peer that exited is either gone (ESRCH) or a zombie its parent has not reaped yet (state Z/X
// in /proc/<pid>/stat), e.g. under multiprocessing until join().
bool pid_alive(int64_t pid) {
  if (pid <= 0) return false;
  if (kill((pid_t)pid, 0) != 0 && errno == ESRCH) return false;
  char path[64];
  snprintf(path, sizeof(path), "/proc/%lld/stat", (long long)pid);
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

bool shm_remove(const std::string& name) { return !name.empty() && shm_unlink(name.c_str()) == 0; }

// ---------------------------------------------------------------------------------------
ShmRegion::ShmRegion(const std::string& name, int64_t bytes, bool create, double timeout_s)
    : name_(name), bytes_(bytes) {
  check(!name.empty() && name[0] == '/' && name.size() < 120, "ShmRegion: name must start with '/' (< 120 chars)");
  check(bytes > 0, "ShmRegion: size must be > 0");
  int fd = -1;
  if (create) {
    fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    check(fd >= 0, "ShmRegion: shm_open(create " + name + ") failed: " + strerror(errno));
    if (ftruncate(fd, (off_t)bytes) != 0) {
      const int e = errno;
      close(fd);
      shm_unlink(name.c_str());
      throw std::runtime_error(std::string("psana_ray_amd: ShmRegion: ftruncate failed: ") + strerror(e));
    }
    owner_ = true;
  } else {
    const double t0 = now_s();
    while (true) {
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat sb;
        if (fstat(fd, &sb) == 0 && (int64_t)sb.st_size >= bytes) break;
        close(fd);
        fd = -1;
      }
      check(now_s() - t0 < timeout_s, "ShmRegion: timed out attaching to " + name);
      nap_ns(1000000);
    }
  }
  void* p = mmap(nullptr, (size_t)bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    if (owner_) shm_unlink(name.c_str());
    throw std::runtime_error(std::string("psana_ray_amd: ShmRegion: mmap failed: ") + strerror(errno));
  }
  base_ = static_cast<uint8_t*>(p);
}

ShmRegion::~ShmRegion() {
  if (base_ != nullptr) munmap(base_, (size_t)bytes_);
  if (owner_ && !unlinked_) shm_unlink(name_.c_str());
}

void ShmRegion::unlink() {
  if (owner_ && !unlinked_) {
    shm_unlink(name_.c_str());
    unlinked_ = true;
  }
}

// ---------------------------------------------------------------------------------------
struct QueueFabric::Link {
  int64_t peer = -1;
  bool outgoing = false;
  std::string name;
  LinkSeg* seg = nullptr;
  size_t map_bytes = 0;
  int n = 0;
  bool attached = false, dead = false, closed = false, eos = false, detached = false, named = true;
  bool keeper = false;                // the consumer end is a queue keeper
  int consumer_device = -1;           // outgoing: GPU of the consumer ring (-1: host shared memory)
  bool ipc = false;                   // outgoing: the consumer ring is IPC-mapped HBM
  bool kcopy = false;                 // outgoing: frames move by the copy kernel (kCopyKernel, 16-B frames)
  int peer_access = -1;               // outgoing, cross-GPU: hipDeviceCanAccessPeer (-1: same GPU / host)
  int link_type = -1, hops = -1;      // outgoing, cross-GPU: hipExtGetLinkTypeAndHopCount
  double t_added = 0, last_check = 0;
  int64_t frames = 0;
  // producer side (outgoing)
  std::deque<int> grants;
  uint64_t g_tail = 0, n_head = 0;
  std::vector<uint64_t> remote;       // address of every slot of the consumer ring (this process's view)
  std::vector<void*> ipc_ptrs;        // one mapping per ring segment
  std::unique_ptr<ShmRegion> remote_ring;
  hipStream_t stream = nullptr;       // this link's copy stream: copies to different consumers
                                      // (different xGMI links) run concurrently
  int inflight = 0;
  int direct = 0;                     // grants of this link in the direct pool (offered / taken / bound)
  bool eos_posted = false, acked_close = false;
  uint64_t r_tail = 0;
  int64_t noticed = 0;                // frames noticed on this link
  uint64_t taken_seen = 0;            // the consumer's `taken` counter, last read
  std::deque<Notice> returns;         // returned frames waiting for a free slot of this pool
  int reclaiming = 0;                 // copies of returned frames in flight
  // consumer side (incoming)
  uint64_t g_head = 0, n_tail = 0, r_head = 0, taken = 0;
  std::vector<uint8_t> owed;  // slot -> granted to this producer and not answered
  std::vector<uint8_t> ret;   // slot -> returned to this producer and not answered
  int64_t outstanding = 0, returned = 0;
  double starved_since = -1;  // keeper: since when this producer's backlog had no other credit

  ~Link() {
    if (seg != nullptr) munmap(seg, map_bytes);
  }
  LinkStatus status() const {
    LinkStatus s;
    s.peer = peer;
    s.outgoing = outgoing;
    s.attached = attached;
    s.eos = eos;
    s.detached = detached;
    s.dead = dead;
    s.closed = closed;
    s.keeper = keeper;
    s.outstanding = outgoing ? (int64_t)grants.size() : outstanding;
    s.frames = frames;
    s.taken = outgoing ? (int64_t)taken_seen : (int64_t)taken;
    s.consumer_device = outgoing ? consumer_device : -1;
    s.kernel_copy = outgoing && kcopy;
    s.peer_access = outgoing ? peer_access : -1;
    s.link_type = outgoing ? link_type : -1;
    s.hops = outgoing ? hops : -1;
    return s;
  }
};

struct QueueFabric::CopyGroup {
  hipEvent_t start = nullptr, end = nullptr;   // timing-enabled, on xstream_
  int pending = 0;                             // batches of this dispatch not retired yet
  bool timed = false;
  double t_issue = 0;
  int64_t bytes = 0;
  int32_t frames = 0, links = 0;
};

struct QueueFabric::Batch {
  std::shared_ptr<Link> link;
  hipStream_t stream = nullptr;
  std::vector<int> slots, rslots;
  std::vector<SlotHeader> hdrs;
  hipEvent_t ev = nullptr;                 // runtime engine / reclaims: this batch's own event
  std::shared_ptr<CopyGroup> grp;          // kernel engine: the dispatch it rode in
  double t_issue = 0;
  std::vector<std::pair<int, int64_t>> ck;  // (frame of the batch, pinned checksum result index)
  bool direct = false;                      // calibrated straight into the consumer's slots (no copy)
};

QueueFabric::QueueFabric(SlotPool* pool, int64_t slot_bytes, int device, bool is_producer, bool is_consumer,
                         int policy, int64_t self_mid)
    : pool_(pool), slot_bytes_(slot_bytes), device_(device), is_producer_(is_producer), is_consumer_(is_consumer),
      policy_(policy), self_mid_(self_mid) {
  check(pool != nullptr && slot_bytes > 0, "QueueFabric: empty ring");
  check((int)pool->slot_ptrs().size() == pool->n_slots(), "QueueFabric: the pool has no slot addresses");
  check(policy >= 0 && policy <= 4, "QueueFabric: unknown routing policy");
  check(is_producer || is_consumer, "QueueFabric: a member must produce or consume");
  if (is_consumer) pool_->set_track_origins(true);
  if (device_ >= 0) {
    DeviceGuard dg(device_);
    hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate (fabric)");
  }
  if (!is_producer) drained_.store(true);
  if (device_ < 0 || slot_bytes_ % 16 == 0) {   // the device checksum reads whole 16-B words
    verifier_ = std::make_shared<FrameVerifier>(device_, slot_bytes_);
    if (is_consumer) pool_->set_verifier(verifier_);
  }
  if (const char* e = getenv("PSANA_RAY_AMD_FAULT_CORRUPT")) corrupt_every_ = std::max(0L, atol(e));
  if (const char* e = getenv("PSANA_RAY_AMD_DIRECT_FENCE")) direct_fence_ = atoi(e);
  register_native_thread_owner(this, [this] { halt(); });
}

void QueueFabric::set_verify_every(int every) {
  check(!running_.load(), "QueueFabric: set_verify_every before start()");
  verify_every_ = std::max(0, every);
}

std::array<int64_t, 4> QueueFabric::verify_counts() const {
  return verifier_ ? verifier_->counts() : std::array<int64_t, 4>{0, 0, -1, 0};
}

void QueueFabric::set_direct(bool on) {
  check(!running_.load(), "QueueFabric: set_direct before start()");
  direct_on_ = on && is_producer_ && device_ >= 0 && copy_engine_ == kCopyKernel;
}

std::vector<QueueFabric::DirectGrant> QueueFabric::take_direct(int max_n) {
  std::vector<DirectGrant> out;
  if (!direct_on_ || max_n <= 0) return out;
  std::lock_guard<std::mutex> lk(dmu_);
  while ((int)out.size() < max_n && !d_free_.empty()) {
    auto e = std::move(d_free_.front());
    d_free_.pop_front();
    out.push_back({e.first, e.second.link->remote[(size_t)e.second.rslot]});
    d_taken_.push_back(std::move(e));
  }
  return out;
}

bool QueueFabric::direct_offering() const {
  const int policy = policy_.load();
  return direct_on_ && !finished_.load() && (policy == 2 || policy == 4);
}

void QueueFabric::bind_direct(const std::vector<int>& local_slots, const std::vector<int64_t>& tokens) {
  check(local_slots.size() == tokens.size(), "QueueFabric::bind_direct: size mismatch");
  d_inflight_.fetch_add((int64_t)tokens.size(), std::memory_order_relaxed);
  std::lock_guard<std::mutex> lk(dmu_);
  for (size_t i = 0; i < tokens.size(); ++i) {
    auto it = std::find_if(d_taken_.begin(), d_taken_.end(), [&](const auto& e) { return e.first == tokens[i]; });
    check(it != d_taken_.end(), "QueueFabric::bind_direct: unknown token");
    d_bound_.emplace_back(local_slots[i], std::move(it->second));
    d_taken_.erase(it);
  }
}

void QueueFabric::cancel_direct(const std::vector<int64_t>& tokens) {
  std::lock_guard<std::mutex> lk(dmu_);
  for (int64_t t : tokens) {
    auto it = std::find_if(d_taken_.begin(), d_taken_.end(), [&](const auto& e) { return e.first == t; });
    if (it == d_taken_.end()) continue;
    d_cancel_.push_back(std::move(*it));
    d_taken_.erase(it);
  }
}

// Fabric thread, every producer pass: cancelled grants back to their links, the offer pool purged
// of links that can no longer take frames, emptied when the policy keeps frames local (balanced /
// local_first / relay) or the producer finished, else refilled from the live remote consumers'
// grants (the link holding the most grants first, so the offers spread over the consumers).
int64_t QueueFabric::direct_pass() {
  const int policy = policy_.load();
  // only where the POLICY sends frames to other processes (spread, remote_only).  A producer with no
  // consumer of its own keeps the copy path: its frames are routed at completion to whichever
  // consumer has credit then, which keeps competing consumers balanced by their read speed (binding
  // at launch time skewed a fast / slow pair towards the slow one, 77 vs 123 frames)
  const bool want = direct_on_ && !finished_.load() && (policy == 2 || policy == 4);
  auto usable = [](const Link& l) {
    return l.attached && !l.dead && !l.closed && !l.eos_posted && !l.keeper && l.kcopy;
  };
  int64_t work = 0;
  std::lock_guard<std::mutex> lk(dmu_);
  for (auto& e : d_cancel_) {
    Link& l = *e.second.link;
    if (!l.dead && !l.closed) l.grants.push_front(e.second.rslot);
    --l.direct;
    ++work;
  }
  d_cancel_.clear();
  // the pool never holds more grants than the engine can use now (its free producer budget): a
  // budget full of frames waiting for a copy needs the consumers' grants for the copy path, or
  // nothing moves (the pool would keep every grant while the engine cannot take one)
  const int64_t target = want ? std::max<int64_t>(0, std::min<int64_t>(kDirectPool, pool_->producer_room())) : 0;
  int64_t keep = 0;
  for (auto it = d_free_.begin(); it != d_free_.end();) {
    Link& l = *it->second.link;
    if (want && usable(l) && keep < target) {
      ++keep;
      ++it;
      continue;
    }
    if (!l.dead && !l.closed) l.grants.push_front(it->second.rslot);   // EOS: returned with the others
    --l.direct;
    it = d_free_.erase(it);
    ++work;
  }
  if (!want) return work;
  // direct first: the offer pool refills (up to the engine's free budget) before the copy path
  // routes this pass's produced frames
  while ((int64_t)d_free_.size() < target) {
    Link* best = nullptr;
    std::shared_ptr<Link> bp;
    for (auto& lp : links_)
      if (lp->outgoing && usable(*lp) && !lp->grants.empty() && (best == nullptr || lp->grants.size() > best->grants.size())) {
        best = lp.get();
        bp = lp;
      }
    if (best == nullptr) break;
    const int rs = best->grants.front();
    best->grants.pop_front();
    ++best->direct;
    d_free_.emplace_back(d_next_++, DirectRec{bp, rs});
    ++work;
  }
  return work;
}

// Produced frames that were calibrated straight into consumer slots: no copy, only ordering.  The
// fabric's copy stream waits for their calibration (the slots' ready events), a system-scope release
// on every XCD writes back L2 lines of peer memory the calibration kernels left dirty, optional
// checksums read the frames back from the consumer rings, and each link's batch gets a completion
// event; step 3 notices the frames when it completes (or counts them lost if the consumer left).
void QueueFabric::issue_direct(std::vector<Batch>& db) {
  trace::Range tr("fabric.direct_dispatch");
  if (xstream_ == nullptr) xstream_ = acquire_stream(device_, xstream_kind_);
  std::vector<int> all;
  for (const Batch& b : db) all.insert(all.end(), b.slots.begin(), b.slots.end());
  pool_->begin_send_batch(all, reinterpret_cast<uint64_t>(xstream_));
  bool peer_gpu = false;   // a ring on another GPU was written: write back L2 lines of peer memory
  for (const Batch& b : db) peer_gpu |= b.link->consumer_device >= 0 && b.link->consumer_device != device_;
  if (peer_gpu || (direct_fence_ & 1)) launch_release_fence(reinterpret_cast<uint64_t>(xstream_));
  if (direct_fence_ & 2) launch_acquire_fence(reinterpret_cast<uint64_t>(xstream_));
  int64_t n = 0;
  for (Batch& b : db) {
    b.direct = true;   // before the checksums: they must read the frames in the consumer's ring
    start_checksums(b, reinterpret_cast<uint64_t>(xstream_));
    inject_corruption(b, reinterpret_cast<uint64_t>(xstream_));
  }
  for (Batch& b : db) {
    b.stream = xstream_;
    b.ev = take_event();
    hip_check(hipEventRecord(b.ev, xstream_), "hipEventRecord (direct frames)");
    b.link->inflight += (int)b.slots.size();
    n += (int64_t)b.slots.size();
    inflight_.push_back(std::move(b));
  }
  std::lock_guard<std::mutex> lk(mu_);
  st_.frames_direct += n;
  st_.batches += (int64_t)db.size();
}

// Producer: the frames of `b` that carry a content checksum to their consumer (every
// verify_every_-th frame of this producer by its rank-local idx -- so every producer's links are
// sampled, which gevt % N would not do for N producers sharing one gevt sequence -- and only
// frames that have none yet: a frame handed back by a closing consumer keeps its producer's
// checksum).  GPU: queued on `stream` ahead of the copy, results read
// when the copy completes (finish_checksums); host: computed now.
void QueueFabric::start_checksums(Batch& b, uint64_t stream) {
  if (verify_every_ <= 0 || !verifier_) return;
  std::vector<uint64_t> ptrs;
  std::vector<int> which;
  for (size_t i = 0; i < b.slots.size(); ++i) {
    const SlotHeader& h = b.hdrs[i];
    if (h.idx < 0 || h.idx % verify_every_ != 0 || ck_tagged(h.aux)) continue;
    if (device_ < 0) {
      const uint64_t src = b.direct ? b.link->remote[b.rslots[i]] : pool_->slot_ptr(b.slots[i]);
      b.hdrs[i].aux = ck_tag(frame_checksum_host(reinterpret_cast<const void*>(src), slot_bytes_));
      continue;
    }
    ptrs.push_back(b.direct ? b.link->remote[b.rslots[i]] : pool_->slot_ptr(b.slots[i]));
    which.push_back((int)i);
  }
  for (size_t a = 0; a < ptrs.size(); a += kMaxFrames) {
    const size_t n = std::min(ptrs.size() - a, (size_t)kMaxFrames);
    const int64_t base =
        verifier_->checksum_async(std::vector<uint64_t>(ptrs.begin() + a, ptrs.begin() + a + n), stream);
    for (size_t k = 0; k < n; ++k) b.ck.emplace_back(which[a + k], base + (int64_t)k);
  }
}

void QueueFabric::finish_checksums(Batch& b) {
  for (const auto& c : b.ck) b.hdrs[(size_t)c.first].aux = verifier_->result(c.second);
  int64_t n = 0;
  for (const SlotHeader& h : b.hdrs) n += ck_tagged(h.aux) ? 1 : 0;
  b.ck.clear();
  std::lock_guard<std::mutex> lk(mu_);
  st_.frames_checksummed += n;
}

// Test-only fault injection (PSANA_RAY_AMD_FAULT_CORRUPT=N): every N-th frame this producer sends to
// another process is damaged in the consumer's ring after its copy, so the consumer's checks must
// catch it (tests/test_fabric_verify.py).  Off (0) unless the variable is set.
void QueueFabric::inject_corruption(const Batch& b, uint64_t stream) {
  if (corrupt_every_ <= 0) return;
  const Link& l = *b.link;
  for (size_t i = 0; i < b.slots.size(); ++i) {
    if (++corrupt_count_ % corrupt_every_ != 0) continue;
    const uint64_t dst = l.remote[b.rslots[i]] + (uint64_t)(slot_bytes_ / 2 / 16 * 16);
    if (device_ < 0)
      memset(reinterpret_cast<void*>(dst), 0x5A, 16);
    else
      hip_check(hipMemsetAsync(reinterpret_cast<void*>(dst), 0x5A, 16, reinterpret_cast<hipStream_t>(stream)),
                "hipMemsetAsync (fault injection)");
    std::lock_guard<std::mutex> lk(mu_);
    ++st_.frames_corrupted;
  }
}

void QueueFabric::halt() {
  std::lock_guard<std::mutex> lk(halt_mu_);
  stop_.store(true);
  if (th_.joinable()) th_.join();
}

QueueFabric::~QueueFabric() {
  unregister_native_thread_owner(this);
  halt();
  try {
    DeviceGuard dg(device_);
    // copies still in flight complete into memory we keep mapped until here
    std::vector<std::shared_ptr<CopyGroup>> groups;
    for (auto& b : inflight_) {
      if (b.ev != nullptr) (void)hipEventSynchronize(b.ev);
      if (b.grp != nullptr && std::find(groups.begin(), groups.end(), b.grp) == groups.end()) groups.push_back(b.grp);
    }
    for (auto& g : groups) {
      (void)hipEventSynchronize(g->end);
      free_timed_.push_back(g->start);
      free_timed_.push_back(g->end);
    }
    inflight_.clear();
    if (xstream_ != nullptr) release_stream(device_, xstream_kind_, xstream_);   // synchronises it
    xstream_ = nullptr;
    for (auto& l : links_) {
      if (l->seg == nullptr) continue;
      if (l->outgoing) {
        if (l->attached) {
          l->seg->producer_ack_closed.store(1, std::memory_order_release);
          l->seg->producer_detached.store(1, std::memory_order_release);
        }
        release_out_link(*l);
      } else {
        l->seg->consumer_closed.store(1, std::memory_order_release);
        if (l->named) shm_remove(l->name);
      }
    }
    links_.clear();
    for (auto e : all_events_) (void)hipEventDestroy(e);
    for (auto e : free_timed_) (void)hipEventDestroy(e);
    if (stream_ != nullptr) (void)hipStreamDestroy(stream_);
  } catch (...) {
  }
}

std::string QueueFabric::last_link_error() const {
  std::lock_guard<std::mutex> lk(mu_);
  return link_error_;
}

std::string QueueFabric::error() const {
  std::lock_guard<std::mutex> lk(mu_);
  return error_;
}

FabricStats QueueFabric::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  return st_;
}

std::vector<LinkStatus> QueueFabric::links() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<LinkStatus> v = status_;
  v.insert(v.end(), retired_.begin(), retired_.end());
  return v;
}

void QueueFabric::fail(const std::string& msg) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (error_.empty()) error_ = msg;
  }
  pool_->wake_all();
}

void QueueFabric::export_host_ring(const std::string& shm_name) {
  check(is_consumer_, "QueueFabric: only a consumer exports its ring");
  check(shm_name.size() < 120, "QueueFabric: ring name too long");
  export_kind_ = 0;
  export_name_ = shm_name;
}

void QueueFabric::export_ipc_ring() {
  check(is_consumer_ && device_ >= 0, "QueueFabric: IPC export needs a GPU consumer");
  DeviceGuard dg(device_);
  segs_.clear();
  const int n = pool_->n_slots();
  uint64_t cur_base = 0, cur_first_ptr = 0;
  for (int s = 0; s < n; ++s) {
    const uint64_t p = pool_->slot_ptr(s);
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hip_check(hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(p)),
              "hipMemGetAddressRange (ring segment)");
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    check(p + (uint64_t)slot_bytes_ <= b + (uint64_t)size, "QueueFabric: a ring slot straddles two allocations");
    if (!segs_.empty() && b == cur_base && p == cur_first_ptr + (uint64_t)segs_.back().n * (uint64_t)slot_bytes_) {
      ++segs_.back().n;
      continue;
    }
    check((int)segs_.size() < kMaxSegments, "QueueFabric: ring has too many segments to export");
    check(size <= (size_t(2) << 30), "QueueFabric: ring allocations above 2 GiB cannot be opened over HIP IPC");
    SegExport e;
    hipIpcMemHandle_t h;
    hip_check(hipIpcGetMemHandle(&h, base), "hipIpcGetMemHandle (ring segment)");
    e.handle.assign(reinterpret_cast<const uint8_t*>(h.reserved),
                    reinterpret_cast<const uint8_t*>(h.reserved) + HIP_IPC_HANDLE_SIZE);
    e.offset = (int64_t)(p - b);
    e.first = s;
    e.n = 1;
    segs_.push_back(std::move(e));
    cur_base = b;
    cur_first_ptr = p;
  }
  export_kind_ = 1;
}

void QueueFabric::add_in_link(int64_t producer_mid, const std::string& name) {
  check(is_consumer_, "QueueFabric.add_in_link: not a consumer");
  check(export_kind_ >= 0, "QueueFabric.add_in_link: export the ring first");
  std::lock_guard<std::mutex> lk(ops_mu_);
  ops_.push_back(Op{0, producer_mid, name});
}

void QueueFabric::add_out_link(int64_t consumer_mid, const std::string& name) {
  check(is_producer_, "QueueFabric.add_out_link: not a producer");
  std::lock_guard<std::mutex> lk(ops_mu_);
  ops_.push_back(Op{1, consumer_mid, name});
}

void QueueFabric::drop_peer(int64_t mid) {
  std::lock_guard<std::mutex> lk(ops_mu_);
  ops_.push_back(Op{2, mid, ""});
}

void QueueFabric::set_policy(int policy) {
  check(policy >= 0 && policy <= 4, "QueueFabric: unknown routing policy");
  policy_.store(policy);
}

void QueueFabric::set_peer_grantable(int64_t mid, bool on) {
  std::lock_guard<std::mutex> lk(ops_mu_);
  ops_.push_back(Op{on ? 3 : 4, mid, ""});
}

void QueueFabric::set_copy_engine(int engine, int workgroups, int stream_kind) {
  check(engine == kCopyKernel || engine == kCopyRuntime, "QueueFabric: unknown copy engine");
  check(stream_kind == kStreamShared || stream_kind == kStreamDedicated || stream_kind == kStreamHighPriority,
        "QueueFabric: unknown stream kind");
  check(!running_.load(), "QueueFabric: set_copy_engine before start()");
  copy_engine_ = engine;
  if (workgroups > 0) copy_wgs_ = std::min(workgroups, 4096);
  xstream_kind_ = stream_kind;
}

std::vector<CopySample> QueueFabric::copy_samples() const {
  std::lock_guard<std::mutex> lk(mu_);
  return std::vector<CopySample>(samples_.begin(), samples_.end());
}

hipEvent_t QueueFabric::take_timed_event() {
  if (!free_timed_.empty()) {
    hipEvent_t e = free_timed_.back();
    free_timed_.pop_back();
    return e;
  }
  hipEvent_t e;
  hip_check(hipEventCreate(&e), "hipEventCreate (fabric copy timing)");
  return e;
}

// A dispatch whose end event completed: its device time becomes a sample (once).
void QueueFabric::finish_group(const std::shared_ptr<CopyGroup>& g) {
  if (g->timed) return;
  g->timed = true;
  float ms = 0.f;
  CopySample cs;
  if (hipEventElapsedTime(&ms, g->start, g->end) == hipSuccess) cs.dev_ms = ms;
  (void)hipGetLastError();
  cs.issue_to_done_ms = 1e3 * (now_s() - g->t_issue);
  cs.bytes = g->bytes;
  cs.frames = g->frames;
  cs.links = g->links;
  std::lock_guard<std::mutex> lk(mu_);
  st_.copy_dev_ms += cs.dev_ms;
  st_.copy_dev_bytes += cs.bytes;
  samples_.push_back(cs);
  while ((int)samples_.size() > kMaxSamples) samples_.pop_front();
}

hipEvent_t QueueFabric::take_event() {
  if (!free_events_.empty()) {
    hipEvent_t e = free_events_.back();
    free_events_.pop_back();
    return e;
  }
  hipEvent_t e;
  hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate (fabric)");
  all_events_.push_back(e);
  return e;
}

void QueueFabric::apply_ops() {
  std::vector<Op> ops;
  {
    std::lock_guard<std::mutex> lk(ops_mu_);
    ops.swap(ops_);
  }
  for (const Op& op : ops) {
    if (op.kind == 3 || op.kind == 4) {
      auto it = std::find(grantable_.begin(), grantable_.end(), op.mid);
      if (op.kind == 3 && it == grantable_.end()) grantable_.push_back(op.mid);
      if (op.kind == 4 && it != grantable_.end()) grantable_.erase(it);
      continue;
    }
    if (op.kind == 2) {
      for (auto& l : links_)
        if (l->peer == op.mid && !l->dead) {
          l->dead = true;
          std::lock_guard<std::mutex> lk(mu_);
          ++st_.peers_dead;
        }
      continue;
    }
    bool dup = false;
    for (auto& l : links_) dup |= (l->peer == op.mid && l->outgoing == (op.kind == 1));
    if (dup) continue;
    auto l = std::make_shared<Link>();
    l->peer = op.mid;
    l->outgoing = op.kind == 1;
    l->name = op.name;
    l->t_added = now_s();
    if (op.kind == 0) {
      // consumer: create the mailbox (a stale name from a crashed run is replaced)
      const int n = std::max(1, pool_->n_slots());
      const size_t bytes = seg_bytes(n);
      int fd = shm_open(op.name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0 && errno == EEXIST) {
        shm_unlink(op.name.c_str());
        fd = shm_open(op.name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      }
      check(fd >= 0, "QueueFabric: shm_open(create " + op.name + ") failed: " + strerror(errno));
      if (ftruncate(fd, (off_t)bytes) != 0) {
        const int e = errno;
        close(fd);
        shm_unlink(op.name.c_str());
        throw std::runtime_error(std::string("psana_ray_amd: QueueFabric: ftruncate failed: ") + strerror(e));
      }
      void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      close(fd);
      check(p != MAP_FAILED, "QueueFabric: mmap of a link mailbox failed");
      auto* s = static_cast<LinkSeg*>(p);   // zero-filled by ftruncate
      s->magic = kLinkMagic;
      s->version = kLinkVersion;
      s->n_slots = n;
      s->slot_bytes = slot_bytes_;
      s->producer_mid = op.mid;
      s->consumer_mid = self_mid_;
      s->consumer_pid = (int64_t)getpid();
      s->kind = export_kind_;
      s->consumer_device = device_;
      if (device_ >= 0 && hipDeviceGetPCIBusId(s->consumer_pci, (int)sizeof(s->consumer_pci), device_) != hipSuccess) {
        (void)hipGetLastError();
        s->consumer_pci[0] = 0;
      }
      s->consumer_kind = keeper_ ? 1 : 0;
      snprintf(s->ring_name, sizeof(s->ring_name), "%s", export_name_.c_str());
      s->n_segs = (int32_t)segs_.size();
      for (size_t k = 0; k < segs_.size(); ++k) {
        memcpy(s->segs[k].handle, segs_[k].handle.data(), HIP_IPC_HANDLE_SIZE);
        s->segs[k].offset = segs_[k].offset;
        s->segs[k].first = segs_[k].first;
        s->segs[k].n = segs_[k].n;
      }
      s->ready.store(1, std::memory_order_release);
      l->seg = s;
      l->map_bytes = bytes;
      l->n = n;
      l->owed.assign((size_t)pool_->n_slots(), 0);
      l->ret.assign((size_t)pool_->n_slots(), 0);
      l->keeper = keeper_;
    }
    links_.push_back(l);
    std::lock_guard<std::mutex> lk(mu_);
    ++st_.links_opened;
  }
}

bool QueueFabric::try_attach(Link& l, double now) {
  (void)now;
  if (l.seg == nullptr) {
    const int fd = shm_open(l.name.c_str(), O_RDWR, 0600);
    if (fd < 0) return false;   // the consumer has not created it yet
    struct stat sb;
    if (fstat(fd, &sb) != 0 || (size_t)sb.st_size < seg_bytes(1)) {
      close(fd);
      return false;
    }
    void* p = mmap(nullptr, (size_t)sb.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return false;
    auto* s = static_cast<LinkSeg*>(p);
    if (s->ready.load(std::memory_order_acquire) != 1 || (size_t)sb.st_size < seg_bytes(s->n_slots)) {
      munmap(p, (size_t)sb.st_size);
      return false;
    }
    l.seg = s;
    l.map_bytes = (size_t)sb.st_size;
  }
  LinkSeg* s = l.seg;
  check(s->magic == kLinkMagic && s->version == kLinkVersion, "QueueFabric: link mailbox " + l.name + " has a foreign layout");
  check(s->slot_bytes == slot_bytes_, "QueueFabric: consumer " + std::to_string(l.peer) +
                                          " has a different frame size (" + std::to_string(s->slot_bytes) + " vs " +
                                          std::to_string(slot_bytes_) + " bytes)");
  l.n = s->n_slots;
  l.remote.assign((size_t)l.n, 0);
  // a consumer ring this process cannot map (no peer path to that GPU, a runtime refusing the
  // handle, a vanished shared-memory ring) makes THIS link unusable -- never the fabric: the link is
  // dropped before the producer announces itself (so the consumer never grants to it) and the
  // error is kept
  try {
    if (s->kind == 0) {
      l.remote_ring.reset(new ShmRegion(std::string(s->ring_name), (int64_t)l.n * slot_bytes_, false, 5.0));
      for (int k = 0; k < l.n; ++k) l.remote[k] = l.remote_ring->ptr() + (uint64_t)k * (uint64_t)slot_bytes_;
    } else {
      check(device_ >= 0, "QueueFabric: a GPU consumer's ring can only be written by a GPU producer");
      check(s->n_segs >= 1 && s->n_segs <= kMaxSegments, "QueueFabric: bad segment table in " + l.name);
      hip_check(hipSetDevice(device_), "hipSetDevice");
      int ndev = 0;
      hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
      // the consumer's GPU in THIS process's numbering: by PCI bus id (its own index is only
      // meaningful when both processes see the same devices)
      int cdev = s->consumer_device;
      if (s->consumer_pci[0] != 0) {
        char mine[32];
        for (int d = 0; d < ndev; ++d)
          if (hipDeviceGetPCIBusId(mine, (int)sizeof(mine), d) == hipSuccess && strncmp(mine, s->consumer_pci, sizeof(mine)) == 0) {
            cdev = d;
            break;
          }
        (void)hipGetLastError();
      }
      l.consumer_device = cdev;
      if (cdev >= 0 && cdev < ndev && cdev != device_) {
        // the copy engine / blit kernels of THIS GPU write the consumer GPU's HBM over xGMI
        int can = 0;
        hip_check(hipDeviceCanAccessPeer(&can, device_, cdev), "hipDeviceCanAccessPeer");
        l.peer_access = can;
        uint32_t lt = 0, hc = 0;   // topology record (bench extra.links_rank0): 4 = xGMI, hops 1 = direct
        if (hipExtGetLinkTypeAndHopCount(device_, cdev, &lt, &hc) == hipSuccess) {
          l.link_type = (int)lt;
          l.hops = (int)hc;
        } else {
          (void)hipGetLastError();
        }
        check(can != 0, "GPU " + std::to_string(device_) + " has no peer access to GPU " + std::to_string(cdev) +
                            " (hipDeviceCanAccessPeer = 0)");
      }
      for (int k = 0; k < s->n_segs; ++k) {
        const SegDesc& d = s->segs[k];
        check(d.first >= 0 && d.n >= 1 && d.first + d.n <= l.n, "QueueFabric: bad segment in " + l.name);
        hipIpcMemHandle_t h;
        memcpy(h.reserved, d.handle, HIP_IPC_HANDLE_SIZE);
        void* p = nullptr;
        hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle (consumer ring)");
        l.ipc_ptrs.push_back(p);
        for (int j = 0; j < d.n; ++j)
          l.remote[d.first + j] = reinterpret_cast<uint64_t>(p) + (uint64_t)d.offset + (uint64_t)j * (uint64_t)slot_bytes_;
      }
      for (int k = 0; k < l.n; ++k) check(l.remote[k] != 0, "QueueFabric: segment table leaves a slot unmapped");
    }
  } catch (const std::exception& e) {
    if (device_ >= 0) (void)hipGetLastError();
    release_out_link(l);
    l.dead = true;
    std::lock_guard<std::mutex> lk(mu_);
    ++st_.links_failed;
    link_error_ = "link to consumer " + std::to_string(l.peer) + ": " + e.what();
    return false;
  }
  l.ipc = s->kind == 1;
  if (!l.ipc) l.consumer_device = -1;   // IPC rings: set above, in this process's device numbering
  // the copy kernel moves 16-B words between 16-B aligned slots; a slot size that is not a multiple
  // of 16 B or a misaligned ring takes the runtime engine on this link instead -- decided here, once,
  // never after frames were handed to a copy (FrameRing pads its slots to 256 B, so its rings always
  // qualify; the check guards rings built by other code)
  l.kcopy = device_ >= 0 && l.ipc && copy_engine_ == kCopyKernel && slot_bytes_ % 16 == 0;
  for (int k = 0; l.kcopy && k < l.n; ++k) l.kcopy = l.remote[k] % 16 == 0;
  for (uint64_t p : pool_->slot_ptrs()) l.kcopy = l.kcopy && p % 16 == 0;
  // a per-link copy stream only where the runtime copies: a host ring (pageable shared memory), or
  // the runtime engine; the kernel engine moves every link's frames on xstream_
  if (device_ >= 0 && l.stream == nullptr && !l.kcopy) {
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hip_check(hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking), "hipStreamCreate (fabric link)");
  }
  l.g_tail = s->g_tail.load(std::memory_order_acquire);
  l.n_head = s->n_head.load(std::memory_order_acquire);
  l.r_tail = s->r_tail.load(std::memory_order_acquire);
  l.keeper = s->consumer_kind == 1;
  s->producer_budget.store(pool_->producer_budget(), std::memory_order_relaxed);
  s->producer_pid.store((int64_t)getpid(), std::memory_order_release);
  l.attached = true;
  return true;
}

void QueueFabric::release_out_link(Link& l) {
  if ((!l.ipc_ptrs.empty() || l.stream != nullptr) && device_ >= 0) (void)hipSetDevice(device_);
  // kernel-engine copies towards this ring run on xstream_: none may still write it once unmapped
  if (l.inflight > 0 && xstream_ != nullptr) (void)hipStreamSynchronize(xstream_);
  if (l.stream != nullptr) {
    (void)hipStreamSynchronize(l.stream);
    (void)hipStreamDestroy(l.stream);
    l.stream = nullptr;
  }
  for (void* p : l.ipc_ptrs) (void)hipIpcCloseMemHandle(p);
  l.ipc_ptrs.clear();
  l.remote_ring.reset();
  l.remote.clear();
}

// Hand a read-ahead frame (consumer slot, LEASED) back: to `pref` when it can take it, else to any
// live producer that has not posted EOS.  False: nobody can (the caller drops it).
bool QueueFabric::post_return(Link* pref, int slot, const SlotHeader& h) {
  auto ok = [](const Link* l) {
    return l != nullptr && !l->outgoing && l->seg != nullptr && l->attached && !l->dead && !l->detached && !l->eos;
  };
  Link* to = ok(pref) ? pref : nullptr;
  if (to == nullptr)
    for (auto& lp : links_)
      if (ok(lp.get())) {
        to = lp.get();
        break;
      }
  if (to == nullptr) return false;
  LinkSeg* s = to->seg;
  seg_returns(s)[to->r_head % (uint64_t)to->n] = make_notice(slot, 0, h);
  ++to->r_head;
  s->r_head.store(to->r_head, std::memory_order_release);
  to->ret[slot] = 1;
  ++to->returned;
  ++returns_pending_;
  std::lock_guard<std::mutex> lk(mu_);
  ++st_.frames_returned;
  return true;
}

void QueueFabric::drop_returned(int slot) {
  pool_->release(slot, 0);
  std::lock_guard<std::mutex> lk(mu_);
  ++st_.frames_dropped;
}

// ---------------------------------------------------------------------------------------
int64_t QueueFabric::consumer_pass(double now) {
  int64_t work = 0;
  const bool closing = consumer_closed_.load();
  // 0. frames the reader took since the last pass: tell each producer (its budget counts them
  //    until then -- queue_size is one logical bound)
  int64_t tk_local = 0, tk_remote = 0;
  for (int64_t o : pool_->take_got_origins()) {
    if (o < 0) {
      ++tk_local;
      continue;
    }
    ++tk_remote;
    for (auto& lp : links_)
      if (!lp->outgoing && lp->peer == o) {
        ++lp->taken;
        break;
      }
  }
  if (tk_local + tk_remote > 0) {
    std::lock_guard<std::mutex> lk(mu_);
    st_.taken_local += tk_local;
    st_.taken_remote += tk_remote;
  }
  const int64_t ready_now = pool_->n_ready();   // demand signal for balanced producers (starving: 0)
  const uint32_t self_fed = (is_producer_ && !finished_.load() && policy_.load() != 3) ? 1u : 0u;
  for (auto& lp : links_)
    if (!lp->outgoing && lp->seg != nullptr) {
      lp->seg->consumer_ready.store(ready_now, std::memory_order_relaxed);
      lp->seg->consumer_self_fed.store(self_fed, std::memory_order_relaxed);
      lp->seg->taken.store(lp->taken, std::memory_order_release);
      lp->seg->consumer_published.store(1, std::memory_order_release);
    }
  // 1. notices: frames (-> READY), unused grants, answers to returned frames.  n_tail is stored only
  //    after the returns of this pass were posted (a closing consumer hands back every frame noticed
  //    before a producer sees n_tail catch up and acknowledges the close)
  std::vector<int> done_slots, ret_slots;
  std::vector<SlotHeader> done_hdr;
  std::vector<std::pair<Link*, uint64_t>> tails;
  std::vector<std::pair<Link*, Notice>> rejected;
  for (auto& lp : links_) {
    Link& l = *lp;
    if (l.outgoing || l.seg == nullptr) continue;
    LinkSeg* s = l.seg;
    if (!l.attached && s->producer_pid.load(std::memory_order_acquire) != 0) {
      l.attached = true;
      if (l.named) {   // both ends mapped it: nothing may outlive the two processes
        shm_remove(l.name);
        l.named = false;
      }
    }
    // EOS / detach flags BEFORE the notice head: a producer releases them after its last notice
    const bool eos_flag = s->producer_eos.load(std::memory_order_acquire) != 0;
    const bool det_flag = s->producer_detached.load(std::memory_order_acquire) != 0;
    const uint64_t h = s->n_head.load(std::memory_order_acquire);
    if (l.n_tail < h) {
      Notice* ns = seg_notices(s);
      done_slots.clear();
      ret_slots.clear();
      done_hdr.clear();
      int64_t reclaimed = 0;
      for (; l.n_tail < h; ++l.n_tail) {
        const Notice nt = ns[l.n_tail % (uint64_t)l.n];
        check(nt.slot >= 0 && nt.slot < (int)l.owed.size(),
              "QueueFabric: producer " + std::to_string(l.peer) + " answered a slot outside the ring");
        if (nt.flags & (kNoticeReclaimed | kNoticeRejected)) {
          check(l.ret[nt.slot], "QueueFabric: producer " + std::to_string(l.peer) +
                                    " answered a frame that was not returned to it");
          l.ret[nt.slot] = 0;
          --l.returned;
          --returns_pending_;
          if (nt.flags & kNoticeReclaimed) {
            pool_->release(nt.slot, 0);   // copied out by the producer: the slot is free again
            ++reclaimed;
          } else {
            rejected.emplace_back(&l, nt);
          }
          continue;
        }
        check(l.owed[nt.slot], "QueueFabric: producer " + std::to_string(l.peer) + " answered a slot it was never granted");
        l.owed[nt.slot] = 0;
        --l.outstanding;
        if (nt.flags & kNoticeReturned) {
          ret_slots.push_back(nt.slot);
        } else {
          done_slots.push_back(nt.slot);
          done_hdr.push_back(header_of(nt));
        }
      }
      tails.emplace_back(&l, l.n_tail);
      pool_->complete_recv_batch_from(done_slots, done_hdr, l.peer);
      pool_->cancel_recv_batch(ret_slots);
      l.frames += (int64_t)done_slots.size();
      work += (int64_t)(done_slots.size() + ret_slots.size()) + reclaimed;
      std::lock_guard<std::mutex> lk(mu_);
      st_.frames_recv += (int64_t)done_slots.size();
      st_.bytes_recv += (int64_t)done_slots.size() * slot_bytes_;
      st_.grants_returned += (int64_t)ret_slots.size();
    }
    if (eos_flag) l.eos = true;
    if (det_flag) l.detached = true;
    if (l.attached && !l.dead && now - l.last_check > kPidCheckS) {
      l.last_check = now;
      if (!pid_alive(s->producer_pid.load(std::memory_order_acquire))) {
        l.dead = true;
        std::lock_guard<std::mutex> lk(mu_);
        ++st_.peers_dead;
      }
    }
    if ((l.dead || l.detached) && l.outstanding > 0) {
      // the producer is gone: everything it still owed comes back (a dead process's copies
      // cannot land any more; a detached one synchronised them before leaving)
      std::vector<int> back;
      for (size_t i = 0; i < l.owed.size(); ++i)
        if (l.owed[i]) {
          back.push_back((int)i);
          l.owed[i] = 0;
        }
      pool_->cancel_recv_batch(back);
      l.outstanding = 0;
      std::lock_guard<std::mutex> lk(mu_);
      st_.grants_reclaimed += (int64_t)back.size();
      work += (int64_t)back.size();
    }
    if ((l.dead || l.detached) && l.returned > 0) {
      // returned frames it never answered: try the other producers
      for (size_t i = 0; i < l.ret.size(); ++i)
        if (l.ret[i]) {
          l.ret[i] = 0;
          --l.returned;
          --returns_pending_;
          const SlotHeader hd = pool_->header((int)i);
          if (!post_return(nullptr, (int)i, hd)) drop_returned((int)i);
          ++work;
        }
    }
    if ((l.dead || l.detached) && l.named) {
      shm_remove(l.name);
      l.named = false;
    }
  }
  for (auto& r : rejected) {   // that producer posted EOS meanwhile: another one, or drop
    {
      std::lock_guard<std::mutex> lk(mu_);
      ++st_.returns_rejected;
    }
    r.first->eos = true;   // it will not accept more (its EOS flag follows)
    if (!post_return(nullptr, r.second.slot, header_of(r.second))) drop_returned(r.second.slot);
    ++work;
  }
  // 2. closing: hand every frame that arrived and was not taken back to a producer.  Once every live
  //    producer confirmed it will notice no more frames (producer_seen_closed), nothing is ready
  //    and every return was answered, `returns_final` tells the producers no return will follow:
  //    only then may they acknowledge the close (a return can never reach a link whose producer
  //    already let go of it)
  if (closing) {
    const std::vector<int> back = pool_->pop_ready_for_return(1 << 30);
    for (int slot : back) {
      const int64_t o = pool_->origin(slot);
      Link* pref = nullptr;
      for (auto& lp : links_)
        if (!lp->outgoing && lp->peer == o) pref = lp.get();
      if (!post_return(pref, slot, pool_->header(slot))) drop_returned(slot);
      ++work;
    }
  }
  for (auto& t : tails) t.first->seg->n_tail.store(t.second, std::memory_order_release);
  if (closing && !closed_posted_) {
    for (auto& lp : links_)
      if (!lp->outgoing && lp->seg != nullptr) lp->seg->consumer_closed.store(1, std::memory_order_release);
    closed_posted_ = true;
  }
  if (closing && closed_posted_ && !returns_final_ && returns_pending_ == 0 && pool_->n_ready() == 0) {
    bool all_seen = true;
    for (auto& lp : links_) {
      const Link& l = *lp;
      if (l.outgoing || l.seg == nullptr || !l.attached || l.dead || l.detached) continue;
      if (l.seg->producer_seen_closed.load(std::memory_order_acquire) == 0 ||
          l.seg->n_head.load(std::memory_order_acquire) != l.n_tail)
        all_seen = false;
    }
    if (all_seen) {
      for (auto& lp : links_)
        if (!lp->outgoing && lp->seg != nullptr) lp->seg->returns_final.store(1, std::memory_order_release);
      returns_final_ = true;
      ++work;
    }
  }
  // 3. grants: free slots of this shard to the live producers that may still send, bounded by the
  //    read-ahead allowance (prefetch - noticed-but-untaken - outstanding)
  if (!closing) {
    std::vector<Link*> act;
    for (auto& lp : links_) {
      Link* l = lp.get();
      if (l->outgoing || !l->attached || l->eos || l->dead || l->detached) continue;
      if (grant_filter_.load()) {
        // queue keeper: producers that finished (draining), or live ones whose backlog nobody
        // else can take (no other credit)
        // (debounced: a consumer between two grant rounds holds no credit for a moment)
        const bool listed = std::find(grantable_.begin(), grantable_.end(), l->peer) != grantable_.end();
        const int64_t backlog = l->seg->producer_backlog.load(std::memory_order_relaxed);
        const int64_t other = l->seg->producer_other_credit.load(std::memory_order_relaxed);
        if (backlog > 0 && other <= 0) {
          if (l->starved_since < 0) l->starved_since = now;
        } else {
          l->starved_since = -1;
        }
        const bool starved = l->starved_since >= 0 && now - l->starved_since >= kKeeperDebounceS;
        if (!listed && !(backlog > 0 && starved)) continue;
      }
      act.push_back(l);
    }
    if (!act.empty()) {
      const int cb = pool_->consumer_budget();
      int64_t allowance = cb;
      const int pf = prefetch_.load();
      if (pf > 0) {
        int64_t held = pool_->n_ready();
        for (auto& lp : links_)
          if (!lp->outgoing) held += lp->outstanding;
        allowance = std::max<int64_t>(0, (int64_t)pf - held);
      }
      const int floor_g = std::max(kMinGrants, std::min(64, cb / (2 * (int)act.size())));
      std::vector<int64_t> want(act.size());
      int64_t total = 0;
      for (size_t i = 0; i < act.size(); ++i) {
        const int64_t backlog = std::max<int64_t>(0, act[i]->seg->producer_backlog.load(std::memory_order_relaxed));
        want[i] = std::max<int64_t>(0, std::min<int64_t>(cb, floor_g + backlog) - act[i]->outstanding);
        total += want[i];
      }
      total = std::min(total, allowance);
      if (total > 0) {
        const std::vector<int> slots = pool_->grant_batch((int)std::min<int64_t>(total, cb));
        size_t k = 0;
        std::vector<uint64_t> head(act.size());
        for (size_t i = 0; i < act.size(); ++i) head[i] = act[i]->g_head;
        // round-robin so concurrent demand shares the free slots
        while (k < slots.size()) {
          bool any = false;
          for (size_t i = 0; i < act.size() && k < slots.size(); ++i) {
            if (want[i] <= 0) continue;
            Link& l = *act[i];
            seg_grants(l.seg)[head[i] % (uint64_t)l.n] = slots[k];
            l.owed[slots[k]] = 1;
            ++l.outstanding;
            ++head[i];
            --want[i];
            ++k;
            any = true;
          }
          if (!any) break;
        }
        check(k == slots.size(), "QueueFabric: grant distribution left slots over");
        for (size_t i = 0; i < act.size(); ++i)
          if (head[i] != act[i]->g_head) {
            act[i]->g_head = head[i];
            act[i]->seg->g_head.store(head[i], std::memory_order_release);
          }
        work += (int64_t)slots.size();
        std::lock_guard<std::mutex> lk(mu_);
        st_.grants_given += (int64_t)slots.size();
      }
    }
  }
  // quiesced: no producer can still write into the ring and every returned frame was answered
  // (close() waits for this before freeing the ring)
  if (closing) {
    bool q = returns_pending_ == 0 && returns_final_;
    for (auto& lp : links_) {
      const Link& l = *lp;
      if (l.outgoing || l.seg == nullptr || !l.attached || l.dead || l.detached) continue;
      if (l.seg->producer_ack_closed.load(std::memory_order_acquire) == 0) q = false;
    }
    quiesced_.store(q);
  }
  return work;
}

int64_t QueueFabric::producer_pass(double now) {
  int64_t work = 0;
  const int policy = policy_.load();
  auto post_notice = [&](Link& l, const Notice& nt) {
    seg_notices(l.seg)[l.n_head % (uint64_t)l.n] = nt;
    ++l.n_head;
  };
  // 1. attach / liveness / incoming grants, taken counters and returned frames
  for (auto& lp : links_) {
    Link& l = *lp;
    if (!l.outgoing || l.dead) continue;
    if (!l.attached) {
      if (!try_attach(l, now)) continue;
      ++work;
    }
    LinkSeg* s = l.seg;
    if (now - l.last_check > kPidCheckS) {
      l.last_check = now;
      if (!pid_alive(s->consumer_pid)) {
        l.dead = true;
        std::lock_guard<std::mutex> lk(mu_);
        ++st_.peers_dead;
      }
    }
    if (l.dead) {
      l.grants.clear();
      l.returns.clear();
      continue;
    }
    // returns first: a closing consumer posts them before consumer_closed
    const uint64_t rh = s->r_head.load(std::memory_order_acquire);
    if (l.r_tail < rh) {
      const Notice* rs = seg_returns(s);
      for (; l.r_tail < rh; ++l.r_tail) {
        const Notice nt = rs[l.r_tail % (uint64_t)l.n];
        check(nt.slot >= 0 && nt.slot < l.n, "QueueFabric: consumer " + std::to_string(l.peer) +
                                                 " returned a slot outside its ring");
        l.returns.push_back(nt);
      }
      s->r_tail.store(l.r_tail, std::memory_order_release);
      ++work;
    }
    const uint64_t tk = s->taken.load(std::memory_order_acquire);
    if (tk != l.taken_seen) {
      l.taken_seen = tk;
      ++work;
    }
    if (!l.closed && s->consumer_closed.load(std::memory_order_acquire) != 0) {
      // from now on copies completing towards this link are requeued, never noticed
      l.closed = true;
      s->producer_seen_closed.store(1, std::memory_order_release);
    }
    if (l.closed) {
      l.grants.clear();
      continue;
    }
    const uint64_t h = s->g_head.load(std::memory_order_acquire);
    if (l.g_tail < h) {
      const int32_t* gs = seg_grants(s);
      for (; l.g_tail < h; ++l.g_tail) {
        const int32_t slot = gs[l.g_tail % (uint64_t)l.n];
        check(slot >= 0 && slot < (int32_t)l.remote.size(),
              "QueueFabric: consumer " + std::to_string(l.peer) + " granted a slot outside its ring");
        l.grants.push_back(slot);
      }
      s->g_tail.store(l.g_tail, std::memory_order_release);
      ++work;
    }
    if (l.eos_posted && !l.grants.empty()) {
      // grants that raced with our EOS: hand them straight back (the consumer must not keep
      // credit owed by a producer that will never send)
      for (int slot : l.grants) post_notice(l, make_notice(slot, kNoticeReturned, SlotHeader{}));
      {
        std::lock_guard<std::mutex> lk(mu_);
        st_.grants_returned += (int64_t)l.grants.size();
      }
      l.grants.clear();
      s->n_head.store(l.n_head, std::memory_order_release);
    }
  }
  // 2. returned frames: copy them back into this pool (front of the FIFO), or refuse them after EOS
  for (auto& lp : links_) {
    Link& l = *lp;
    if (!l.outgoing || l.dead || l.returns.empty()) continue;
    if (eos_any_) {
      for (const Notice& nt : l.returns) post_notice(l, make_notice(nt.slot, kNoticeRejected, header_of(nt)));
      l.returns.clear();
      l.seg->n_head.store(l.n_head, std::memory_order_release);
      ++work;
      continue;
    }
    const int want = (int)std::min<size_t>(l.returns.size(), 64);
    hipStream_t st = device_ >= 0 ? (l.stream != nullptr ? l.stream : stream_) : nullptr;
    const std::vector<int> mine = pool_->reclaim_batch(want, reinterpret_cast<uint64_t>(st));
    if (mine.empty()) continue;   // no free slot right now: retry next pass
    Batch b;
    b.link = lp;
    b.slots = mine;
    b.stream = st;
    b.t_issue = now;
    for (size_t i = 0; i < mine.size(); ++i) {
      const Notice nt = l.returns.front();
      l.returns.pop_front();
      b.rslots.push_back(nt.slot);
      b.hdrs.push_back(header_of(nt));
      if (device_ >= 0)
        hip_check(hipMemcpyAsync(reinterpret_cast<void*>(pool_->slot_ptr(mine[i])),
                                 reinterpret_cast<const void*>(l.remote[nt.slot]), (size_t)slot_bytes_,
                                 hipMemcpyDeviceToDevice, st),
                  "hipMemcpyAsync (returned frame -> producer pool)");
      else
        memcpy(reinterpret_cast<void*>(pool_->slot_ptr(mine[i])), reinterpret_cast<const void*>(l.remote[nt.slot]),
               (size_t)slot_bytes_);
    }
    if (device_ >= 0) {
      b.ev = take_event();
      hip_check(hipEventRecord(b.ev, st), "hipEventRecord (reclaim copy)");
    }
    l.reclaiming += (int)mine.size();
    reclaims_.push_back(std::move(b));
    work += (int64_t)mine.size();
  }
  for (auto it = reclaims_.begin(); it != reclaims_.end();) {
    Batch& b = *it;
    if (b.ev != nullptr) {
      const hipError_t q = hipEventQuery(b.ev);
      if (q == hipErrorNotReady) {
        ++it;
        continue;
      }
      hip_check(q, "hipEventQuery (reclaim copy)");
    }
    Link& l = *b.link;
    const int n = (int)b.slots.size();
    // the frames are ours again (even if that consumer died meanwhile: the copy completed)
    pool_->commit_front_batch(b.slots, b.hdrs, reinterpret_cast<uint64_t>(b.stream));
    l.reclaiming -= n;
    l.noticed = std::max<int64_t>((int64_t)l.taken_seen, l.noticed - n);
    if (!l.dead) {
      for (int i = 0; i < n; ++i) post_notice(l, make_notice(b.rslots[i], kNoticeReclaimed, b.hdrs[i]));
      l.seg->n_head.store(l.n_head, std::memory_order_release);
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      st_.frames_reclaimed += n;
    }
    if (b.ev != nullptr) free_events_.push_back(b.ev);
    it = reclaims_.erase(it);
    work += n;
  }
  // 3. completed copies: notice the frames, or requeue them if their consumer left meanwhile.
  //    Batches of one link complete in order (one stream per link); links are independent.
  std::vector<const Link*> blocked;
  for (auto it = inflight_.begin(); it != inflight_.end();) {
    Batch& b = *it;
    if (std::find(blocked.begin(), blocked.end(), b.link.get()) != blocked.end()) {
      ++it;
      continue;
    }
    hipEvent_t done_ev = b.grp != nullptr ? b.grp->end : b.ev;
    if (done_ev != nullptr) {
      const hipError_t q = hipEventQuery(done_ev);
      if (q == hipErrorNotReady) {
        blocked.push_back(b.link.get());
        ++it;
        continue;
      }
      hip_check(q, "hipEventQuery (frame copy)");
    }
    if (b.grp != nullptr) finish_group(b.grp);
    Link& l = *b.link;
    const int n = (int)b.slots.size();
    l.inflight -= n;
    if (b.direct) d_inflight_.fetch_sub(n, std::memory_order_relaxed);   // noticed, copied back or lost
    if (l.attached && !l.dead && !l.closed) {
      finish_checksums(b);
      for (int i = 0; i < n; ++i) post_notice(l, make_notice(b.rslots[i], 0, b.hdrs[i]));
      l.seg->n_head.store(l.n_head, std::memory_order_release);
      // the copy is complete (host-observed): free the slots with no device wait, and count the
      // frames as consumer read-ahead in the same locked step (step 5 recomputes the exact value)
      const bool ext = !l.acked_close;
      pool_->end_send_completed(b.slots, ext);
      l.frames += n;
      l.noticed += n;
      std::lock_guard<std::mutex> lk(mu_);
      st_.frames_sent += n;
      st_.bytes_sent += (int64_t)n * slot_bytes_;
      st_.copy_s += now - b.t_issue;
    } else if (b.direct && l.closed && !l.dead && l.attached) {
      // a consumer that CLOSED keeps its ring mapped until we acknowledge: copy the frames back
      // into their local slots (still ours, SENDING) and requeue them at the FIFO front, like a
      // copy that completed after the close (rare path: the fabric thread waits for it)
      CopyRuns cr{};
      cr.n = 0;
      for (int i = 0; i < n; ++i) {
        if (cr.n == kMaxCopyRuns) {
          launch_copy_runs(cr, kLocalCopyWgs, reinterpret_cast<uint64_t>(xstream_));
          cr.n = 0;
        }
        cr.src[cr.n] = l.remote[b.rslots[i]];
        cr.dst[cr.n] = pool_->slot_ptr(b.slots[i]);
        cr.n16[cr.n] = slot_bytes_ / 16;
        ++cr.n;
      }
      if (cr.n > 0) launch_copy_runs(cr, kLocalCopyWgs, reinterpret_cast<uint64_t>(xstream_));
      hip_check(hipStreamSynchronize(xstream_), "hipStreamSynchronize (direct frames back from a closed consumer)");
      pool_->unsend_batch(b.slots);
      std::lock_guard<std::mutex> lk(mu_);
      st_.frames_requeued += n;
    } else if (b.direct) {
      // the frame's data exists only in the ring of the consumer that died: lost (never noticed),
      // like the rest of that consumer's read-ahead
      pool_->end_send_completed(b.slots, false);
      std::lock_guard<std::mutex> lk(mu_);
      st_.frames_lost_direct += n;
    } else {
      pool_->unsend_batch(b.slots);
      std::lock_guard<std::mutex> lk(mu_);
      st_.frames_requeued += n;
    }
    if (b.ev != nullptr) free_events_.push_back(b.ev);
    if (b.grp != nullptr && --b.grp->pending == 0) {
      free_timed_.push_back(b.grp->start);
      free_timed_.push_back(b.grp->end);
    }
    it = inflight_.erase(it);
    work += n;
  }
  // 4. route produced frames (FIFO) to this process's own consumer or to granted remote slots.
  //    Keeper links are the last resort: a frame goes there only when no real consumer (and not
  //    this process's own) has credit for it.
  if (direct_on_) {
    work += direct_pass();
    // frames bound to a direct grant go to that grant's consumer, whatever the policy says now --
    // every committed one, wherever it sits in the produced FIFO (behind a copy backlog longer than
    // one pass's kMaxDispatch offers, a bound frame would hold its grant until the backlog drained,
    // and a backlog that needs those grants would never drain)
    std::vector<Batch> db;
    {
      std::lock_guard<std::mutex> lk(dmu_);
      for (auto it = d_bound_.begin(); it != d_bound_.end();) {
        if (pool_->state(it->first) != kProduced) {   // not committed yet
          ++it;
          continue;
        }
        Batch* b = nullptr;
        for (Batch& x : db)
          if (x.link == it->second.link) b = &x;
        if (b == nullptr) {
          db.emplace_back();
          b = &db.back();
          b->link = it->second.link;
          b->t_issue = now;
        }
        b->slots.push_back(it->first);
        b->rslots.push_back(it->second.rslot);
        --it->second.link->direct;
        it = d_bound_.erase(it);
      }
    }
    if (!db.empty()) {
      for (Batch& b : db) b.hdrs = pool_->headers(b.slots);
      for (const Batch& b : db) work += (int64_t)b.slots.size();
      issue_direct(db);
    }
  }
  std::vector<int> offers = pool_->produced(kMaxDispatch);
  if (direct_on_) {
    // a frame bound after the scan above and committed before produced() is still in d_bound_ (the
    // engine binds before it commits): never route it as a copy; the next pass issues it
    std::lock_guard<std::mutex> lk(dmu_);
    if (!d_bound_.empty()) {
      std::vector<int> rest;
      for (int sl : offers)
        if (std::find_if(d_bound_.begin(), d_bound_.end(), [&](const auto& e) { return e.first == sl; }) == d_bound_.end())
          rest.push_back(sl);
      offers.swap(rest);
    }
  }
  int64_t local_credit = (is_consumer_ && !consumer_closed_.load() && policy != 3) ? pool_->credits() : 0;
  std::vector<Link*> cands;
  for (auto& lp : links_)
    if (lp->outgoing && lp->attached && !lp->dead && !lp->closed && !lp->eos_posted) cands.push_back(lp.get());
  if (policy == 4) {
    // remote_only: frames cross to another process whenever a remote consumer is linked
    for (const Link* c : cands)
      if (!c->keeper) local_credit = 0;
  }
  if (!offers.empty()) {
    std::vector<int64_t> avail(cands.size());
    for (size_t i = 0; i < cands.size(); ++i) avail[i] = (int64_t)cands[i]->grants.size();
    if (policy == 2 && local_credit > 0) {
      // spread: the own producer must not take the consumer credit that the remote producers'
      // grants need.  A local route needs only credit, a grant needs a FREE slot whose release
      // event has completed -- so without a reservation the local route wins every race and all
      // frames stay local.  Keep each live remote producer's grant floor (consumer_pass) reserved.
      std::vector<const Link*> in;
      for (auto& lp : links_)
        if (!lp->outgoing && lp->attached && !lp->eos && !lp->dead && !lp->detached) in.push_back(lp.get());
      if (!in.empty()) {
        const int cb = pool_->consumer_budget();
        const int64_t floor_g = std::max(kMinGrants, std::min(64, cb / (2 * (int)in.size())));
        int64_t reserve = 0;
        for (const Link* l : in) reserve += std::max<int64_t>(0, floor_g - l->outstanding);
        local_credit = std::max<int64_t>(0, local_credit - reserve);
      }
    }
    std::vector<std::vector<int>> assign(cands.size());
    std::vector<int> local;
    const int K = (int)cands.size() + 1;   // position K-1 = this process's own consumer
    // balanced: a remote consumer-ONLY member (no producer of its own feeds it) with NOTHING to
    // read (its published ready count is 0) and credit here is starving -- competing consumers pull
    // from one queue in the reference (shared_queue.py:19-24), so it is fed first while our own
    // consumer has frames ready (a consumer-only rank next to a fast co-located consumer would
    // otherwise never see a frame; BASELINE config 3).  Consumers that produce for themselves are
    // left to their own producer, so the weak-scaling case stays local.  Each offer goes to the
    // starving member given the fewest in this pass (several starving members share); a copy to it
    // still in flight does not stop the feed (waiting for it idled the member one notice -> copy ->
    // notice round trip per refill), its grants -- its read-ahead bound -- do.
    std::vector<int> starving;
    if (policy == 0 && (local_credit <= 0 || pool_->n_ready() >= kFeedLocalReady))
      for (size_t i = 0; i < cands.size(); ++i)
        // (a link whose consumer has not published its demand yet -- every field still the zero of a
        // fresh mailbox -- is not starving: a self-fed prosumer would look like one)
        if (!cands[i]->keeper && avail[i] > 0 && cands[i]->seg->consumer_published.load(std::memory_order_acquire) != 0 &&
            cands[i]->seg->consumer_self_fed.load(std::memory_order_relaxed) == 0 &&
            cands[i]->seg->consumer_ready.load(std::memory_order_relaxed) == 0)
          starving.push_back((int)i);
    for (int s : offers) {
      int pick = -2;   // -2 none, -1 local, >= 0 remote
      int sp = -1;
      for (int i : starving)
        if (avail[i] > 0 && (sp < 0 || assign[i].size() < assign[sp].size())) sp = i;
      if (sp >= 0) {
        assign[sp].push_back(s);
        --avail[sp];
        continue;
      }
      if (policy == 2) {
        for (int t = 0; t < K && pick == -2; ++t) {
          const int p = (rr_ + t) % K;
          if (p == K - 1) {
            if (local_credit > 0) pick = -1;
          } else if (avail[p] > 0 && !cands[p]->keeper) {
            pick = p;
          }
          if (pick != -2) rr_ = (p + 1) % K;
        }
      } else {
        int best = -1;
        for (size_t i = 0; i < cands.size(); ++i)
          if (avail[i] > 0 && !cands[i]->keeper && (best < 0 || avail[i] > avail[best])) best = (int)i;
        const int64_t best_n = best >= 0 ? avail[best] : 0;
        if (local_credit > 0 && (policy == 1 || local_credit + kLocalSlack >= best_n)) pick = -1;
        else if (best >= 0) pick = best;
      }
      if (pick == -2)   // nobody else: a keeper with credit
        for (size_t i = 0; i < cands.size(); ++i)
          if (avail[i] > 0 && cands[i]->keeper) {
            pick = (int)i;
            break;
          }
      if (pick == -2) break;
      if (pick == -1) {
        local.push_back(s);
        --local_credit;
      } else {
        assign[pick].push_back(s);
        --avail[pick];
      }
    }
    for (int s : local) pool_->route_local(s);
    if (!local.empty()) {
      work += (int64_t)local.size();
      std::lock_guard<std::mutex> lk(mu_);
      st_.frames_local += (int64_t)local.size();
    }
    std::vector<Batch> kbatches;   // kernel engine: one dispatch for every link of this pass
    for (size_t i = 0; i < cands.size(); ++i) {
      if (assign[i].empty()) continue;
      Link& l = *cands[i];
      const std::vector<int>& slots = assign[i];
      const int n = (int)slots.size();
      Batch b;
      for (std::shared_ptr<Link>& lp : links_)
        if (lp.get() == &l) b.link = lp;
      b.slots = slots;
      b.hdrs = pool_->headers(slots);
      b.rslots.assign(l.grants.begin(), l.grants.begin() + n);
      l.grants.erase(l.grants.begin(), l.grants.begin() + n);
      b.t_issue = now;
      if (l.kcopy) {
        l.inflight += n;
        kbatches.push_back(std::move(b));
        work += n;
        continue;
      }
      if (device_ >= 0) {
        trace::Range tr("fabric.copy_batch");
        b.stream = l.stream != nullptr ? l.stream : stream_;
        pool_->begin_send_batch(slots, reinterpret_cast<uint64_t>(b.stream));   // stream waits for the frames
        start_checksums(b, reinterpret_cast<uint64_t>(b.stream));
        int a = 0;
        const uint64_t sb = (uint64_t)slot_bytes_;
        while (a < n) {   // coalesce runs contiguous on both sides
          int e = a + 1;
          while (e < n && pool_->slot_ptr(slots[e]) == pool_->slot_ptr(slots[e - 1]) + sb &&
                 l.remote[b.rslots[e]] == l.remote[b.rslots[e - 1]] + sb)
            ++e;
          hip_check(hipMemcpyAsync(reinterpret_cast<void*>(l.remote[b.rslots[a]]),
                                   reinterpret_cast<const void*>(pool_->slot_ptr(slots[a])), (size_t)sb * (size_t)(e - a),
                                   hipMemcpyDeviceToDevice, b.stream),
                    "hipMemcpyAsync (frame -> consumer ring)");
          a = e;
        }
        inject_corruption(b, reinterpret_cast<uint64_t>(b.stream));
        b.ev = take_event();
        hip_check(hipEventRecord(b.ev, b.stream), "hipEventRecord (frame copy)");
      } else {
        pool_->begin_send_batch(slots, 0);
        start_checksums(b, 0);
        for (int j = 0; j < n; ++j)
          memcpy(reinterpret_cast<void*>(l.remote[b.rslots[j]]), reinterpret_cast<const void*>(pool_->slot_ptr(slots[j])),
                 (size_t)slot_bytes_);
        inject_corruption(b, 0);
      }
      l.inflight += n;
      inflight_.push_back(std::move(b));
      {
        std::lock_guard<std::mutex> lk(mu_);
        ++st_.batches;
        ++st_.copy_launches;
      }
      work += n;
    }
    if (!kbatches.empty()) issue_copies(kbatches, now);
  }
  // 5. read-ahead accounting (frames noticed and not taken still count against this producer's
  //    budget), demand hints, close acknowledgements, end of stream
  int64_t readahead = 0, other_credit = local_credit;
  bool returns_open = !reclaims_.empty();
  for (auto& lp : links_) {
    const Link& l = *lp;
    if (!l.outgoing || !l.attached || l.dead) continue;
    if (!l.acked_close) readahead += std::max<int64_t>(0, l.noticed - (int64_t)l.taken_seen);
    if (!l.closed && !l.keeper && !l.eos_posted) other_credit += (int64_t)l.grants.size();
    returns_open |= !l.returns.empty() || l.reclaiming > 0;
  }
  pool_->set_external_held((int)std::min<int64_t>(readahead, 1 << 30));
  {
    std::lock_guard<std::mutex> lk(mu_);
    st_.readahead = readahead;
  }
  const int64_t backlog = pool_->n_produced();
  bool direct_idle = true;
  if (direct_on_) {
    std::lock_guard<std::mutex> lk(dmu_);
    direct_idle = d_free_.empty() && d_taken_.empty() && d_bound_.empty() && d_cancel_.empty();
  }
  const bool all_routed = finished_.load() && backlog == 0 && inflight_.empty() && !returns_open && direct_idle;
  bool drained = all_routed;
  for (auto& lp : links_) {
    Link& l = *lp;
    if (!l.outgoing || !l.attached) continue;
    LinkSeg* s = l.seg;
    if (!l.dead && !l.closed) {
      s->producer_backlog.store(backlog, std::memory_order_relaxed);
      s->producer_other_credit.store(other_credit, std::memory_order_relaxed);
    }
    // a closed link is acknowledged once nothing is in flight towards it, every returned frame was
    // answered and the consumer read every notice (so it has handed back every frame it received)
    const bool settled =
        l.inflight == 0 && l.direct == 0 && l.returns.empty() && l.reclaiming == 0 &&
        (l.dead || (s->returns_final.load(std::memory_order_acquire) != 0 &&
                    s->r_head.load(std::memory_order_acquire) == l.r_tail &&
                    s->n_tail.load(std::memory_order_acquire) == l.n_head));
    if ((l.dead || l.closed) && settled && !l.acked_close) {
      s->producer_ack_closed.store(1, std::memory_order_release);
      l.acked_close = true;
      release_out_link(l);
      if (l.dead) {   // nobody else will: the consumer died holding these names
        shm_remove(l.name);
        if (s->kind == 0) shm_remove(std::string(s->ring_name));
      }
      ++work;
    }
    if (all_routed && !l.dead && !l.closed && !l.eos_posted) {
      // give unused grants back, then EOS (released after the last notice)
      for (int slot : l.grants) post_notice(l, make_notice(slot, kNoticeReturned, SlotHeader{}));
      {
        std::lock_guard<std::mutex> lk(mu_);
        st_.grants_returned += (int64_t)l.grants.size();
      }
      l.grants.clear();
      s->n_head.store(l.n_head, std::memory_order_release);
      s->producer_eos.store(1, std::memory_order_release);
      l.eos_posted = true;
      l.eos = true;
      eos_any_ = true;
      ++work;
    }
  }
  // links still being created by their consumer do not hold frames: EOS reaches them on attach
  drained_.store(drained);
  return work;
}

int QueueFabric::copy_grid_for(const std::vector<int>& consumer_devices, int device, int per_peer) {
  bool local = false;
  std::vector<int> peers;
  for (int d : consumer_devices) {
    if (d == device) local = true;
    else if (std::find(peers.begin(), peers.end(), d) == peers.end()) peers.push_back(d);
  }
  const int w = (local ? kLocalCopyWgs : 0) + per_peer * (int)peers.size();
  return std::min(std::max(w, std::max(per_peer, 1)), kMaxCopyWgs);
}

int QueueFabric::copy_grid(const std::vector<Batch>& kb) const {
  std::vector<int> devs;
  devs.reserve(kb.size());
  for (const Batch& b : kb) devs.push_back(b.link->consumer_device);
  return copy_grid_for(devs, device_, copy_wgs_);
}

// Kernel engine: the frames of every link routed in this pass move in ONE copy_runs_kernel launch
// on xstream_ (its own hardware queue), ordered after the frames' calibration by event waits on
// that stream only.  Timing events bracket the copy itself, so each dispatch's device time is known.
void QueueFabric::issue_copies(std::vector<Batch>& kb, double now) {
  trace::Range tr("fabric.copy_dispatch");
  if (xstream_ == nullptr) xstream_ = acquire_stream(device_, xstream_kind_);
  check(slot_bytes_ % 16 == 0, "QueueFabric: frame size must be a multiple of 16 B for the copy kernel");
  std::vector<int> all;
  for (const Batch& b : kb) all.insert(all.end(), b.slots.begin(), b.slots.end());
  pool_->begin_send_batch(all, reinterpret_cast<uint64_t>(xstream_));   // xstream_ waits for their data
  for (Batch& b : kb) start_checksums(b, reinterpret_cast<uint64_t>(xstream_));   // ahead of the copy
  auto g = std::make_shared<CopyGroup>();
  g->start = take_timed_event();
  g->end = take_timed_event();
  g->t_issue = now;
  g->links = (int32_t)kb.size();
  hip_check(hipEventRecord(g->start, xstream_), "hipEventRecord (copy start)");
  CopyRuns cr{};
  cr.n = 0;
  const uint64_t sb = (uint64_t)slot_bytes_;
  int launches = 0;
  // grid: a copy inside this GPU's HBM (a consumer process on the same GPU) is bound by HBM and
  // takes kLocalCopyWgs workgroups; a copy over xGMI is bound by its point-to-point link (~150 GB/s),
  // so the grid grows by copy_wgs_ workgroups per distinct peer GPU this dispatch writes (7 links
  // out of an MI355X run concurrently) and leaves the other CUs to the calibration
  const int wgs = copy_grid(kb);
  auto flush = [&] {
    if (cr.n == 0) return;
    launch_copy_runs(cr, wgs, reinterpret_cast<uint64_t>(xstream_));
    cr.n = 0;
    ++launches;
  };
  for (const Batch& b : kb) {
    const Link& l = *b.link;
    const int n = (int)b.slots.size();
    int a = 0;
    while (a < n) {   // coalesce runs contiguous on both sides
      int e = a + 1;
      while (e < n && pool_->slot_ptr(b.slots[e]) == pool_->slot_ptr(b.slots[e - 1]) + sb &&
             l.remote[b.rslots[e]] == l.remote[b.rslots[e - 1]] + sb)
        ++e;
      if (cr.n == kMaxCopyRuns) flush();
      cr.src[cr.n] = pool_->slot_ptr(b.slots[a]);
      cr.dst[cr.n] = l.remote[b.rslots[a]];
      cr.n16[cr.n] = (int64_t)(sb * (uint64_t)(e - a) / 16u);
      ++cr.n;
      a = e;
    }
    g->frames += n;
    g->bytes += (int64_t)n * slot_bytes_;
  }
  flush();
  // another GPU's ring written: one system-scope release on every XCD before the completion signal
  // (a consumer on THIS GPU reads through the same L2: nothing to write back)
  bool peer_gpu = false;
  for (const Batch& b : kb) peer_gpu |= b.link->consumer_device >= 0 && b.link->consumer_device != device_;
  if (peer_gpu) launch_release_fence(reinterpret_cast<uint64_t>(xstream_));
  for (const Batch& b : kb) inject_corruption(b, reinterpret_cast<uint64_t>(xstream_));
  hip_check(hipEventRecord(g->end, xstream_), "hipEventRecord (copy end)");
  g->pending = (int)kb.size();
  for (Batch& b : kb) {
    b.stream = xstream_;
    b.grp = g;
    inflight_.push_back(std::move(b));
  }
  std::lock_guard<std::mutex> lk(mu_);
  st_.batches += (int64_t)kb.size();
  st_.copy_launches += launches;
}

void QueueFabric::publish_status() {
  std::vector<LinkStatus> v;
  v.reserve(links_.size());
  std::vector<std::shared_ptr<Link>> keep;
  std::vector<LinkStatus> gone;
  for (auto& lp : links_) {
    Link& l = *lp;
    // retire links that can never carry anything again
    const bool out_done = l.outgoing && (l.dead || l.closed) && l.acked_close && l.inflight == 0 && l.direct == 0;
    const bool out_never = l.outgoing && l.dead && !l.attached;
    const bool in_done = !l.outgoing && (l.dead || l.detached) && l.outstanding == 0 && !l.named;
    const bool in_never = !l.outgoing && l.dead && !l.attached;
    if (out_done || out_never || in_done || in_never) {
      if (in_never && l.named) {
        shm_remove(l.name);
        l.named = false;
      }
      gone.push_back(l.status());
      continue;
    }
    keep.push_back(lp);
    v.push_back(l.status());
  }
  links_.swap(keep);
  std::lock_guard<std::mutex> lk(mu_);
  status_.swap(v);
  retired_.insert(retired_.end(), gone.begin(), gone.end());
}

int64_t QueueFabric::step() {
  const double now = now_s();
  apply_ops();
  int64_t work = 0;
  if (is_consumer_) work += consumer_pass(now);
  if (is_producer_) work += producer_pass(now);
  publish_status();
  std::lock_guard<std::mutex> lk(mu_);
  ++st_.iterations;
  if (work == 0) ++st_.idle_iterations;
  return work;
}

void QueueFabric::loop() {
  try {
    if (device_ >= 0) hip_check(hipSetDevice(device_), "hipSetDevice");
    long nap = 0;
    while (!stop_.load()) {
      if (step() == 0) {
        nap = nap > 0 ? std::min(500000L, nap * 2) : 20000L;
        nap_ns(nap);
      } else {
        nap = 0;
      }
    }
  } catch (const std::exception& e) {
    fail(e.what());
  } catch (...) {
    fail("unknown error in the queue fabric");
  }
  running_.store(false);
}

void QueueFabric::start() {
  check(!th_.joinable(), "QueueFabric: already started");
  running_.store(true);
  th_ = std::thread([this] { loop(); });
}

bool QueueFabric::join(double timeout_s) {
  if (!th_.joinable()) return true;
  const double t0 = now_s();
  while (running_.load()) {
    if (timeout_s >= 0 && now_s() - t0 > timeout_s) return false;
    nap_ns(1000000);
  }
  std::lock_guard<std::mutex> lk(halt_mu_);   // never two joins of one thread (halt() at exit)
  if (th_.joinable()) th_.join();
  return true;
}

}  // namespace pr
