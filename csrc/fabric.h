// Elastic fabric of the shared queue: independent producer -> consumer LINKS.
//
// Reference semantics being provided (SURVEY R-10/R-11, P-02, C-01..C-03, §5 failure handling):
// psana-ray's queue is ONE named, detached Ray actor (psana_ray/shared_queue.py:4-35).  Producers
// put as soon as it exists and it buffers up to `maxsize` items with nobody reading
// (psana_ray/producer.py:98-111); any number of consumers get() from it at any time, from
// anywhere (shared_queue.py:19-24, README.md:23-35); a consumer that crashes affects nobody else;
// only the actor's death stops producers (producer.py:112-114).
//
// MI355X design: there is no central actor process.  Each producer process keeps the frames it
// calibrated in its OWN HBM slot pool (its share of queue_size), and each consumer owns an HBM
// shard.  Every (producer, consumer) pair that is alive at the same time gets a LINK -- a small
// POSIX shared-memory mailbox created by the consumer:
//
//   consumer --grants--> producer : ids of free slots of the consumer's shard (credit; it pulls)
//   producer --notices-> consumer : "slot s now holds frame (rank, idx, gevt, photon_energy)"
//                                   or "grant s returned unused"
//
// The frame bytes never pass through the mailbox.  A GPU consumer exports its ring allocation as
// a HIP IPC handle; the producer maps it and writes granted slots directly -- every frame routed in
// one fabric pass, to all its consumers, by ONE copy_runs_kernel launch on a stream that owns its
// hardware queue (csrc/gather.hip) -- over the point-to-point xGMI links when the processes sit on
// different GPUs (one hop, no staging, no rendezvous kernel on the receiver).  The notice is
// posted only after that copy has completed, so the consumer needs no device-side wait.  Host
// (CPU) consumers keep their ring in a named shared-memory region the producer maps and memcpy's
// into.  A producer that is also a consumer (co-located consumer, weak-scaling bench) routes to
// itself with zero copies.
//
// Because links are independent, membership is elastic and failures are isolated:
//   * producers run with no consumer at all (frames wait in their pool, backpressure when full);
//   * consumers attach at any time and any number of them (a new link per live producer);
//   * a consumer that dies or closes: its producers stop using its grants, and frames whose copy
//     was still in flight go back to the FRONT of the producer's FIFO for another consumer;
//   * a consumer that CLOSES hands the frames it received but never read back: it posts them on a
//     return ring, a live producer copies them out of the consumer's ring into its own pool and
//     queues them at the front of its FIFO for the other consumers (the reference's items stay
//     in the actor until somebody get()s them, psana_ray/shared_queue.py:19-24);
//   * a consumer that DIES loses only its read-ahead: grants are bounded so that (noticed but
//     unread + outstanding grants) <= `prefetch` (set_prefetch), i.e. item-granular like the
//     reference's one-item get(), not a whole shard;
//   * a producer that dies: its consumers take back the slots granted to it;
//   * a producer that finishes returns unused grants and posts EOS on every link.
// Liveness is the peer's pid (same host; zombies count as dead), checked every 50 ms.
//
// queue_size is ONE logical bound (the reference's deque(maxlen), shared_queue.py:7,11): a frame
// counts against its producer's budget from production until a consumer TAKES it (get), including
// while it sits in a consumer's read-ahead -- every consumer reports per link how many frames it
// took (`taken`), the producer feeds (noticed - taken) into SlotPool::set_external_held.  So a
// joining consumer adds landing space, never queue capacity.
//
// Queue keeper (keeper.py) links are marked in their mailbox: producers route to them only when no
// other consumer has credit, and the keeper grants to a LIVE producer only while nobody else can
// take its backlog (for 0.1 s in a row) -- so committed frames move into the
// keeper (and survive a producer crash, like puts into the detached actor) without competing with
// real consumers.
//
// Visibility of peer-written slots (SURVEY H-10; /opt/skills/guides/MI355X_MICROARCH.md:150-236):
// the frame bytes are written by the PRODUCER's copy (copy_runs_kernel, or hipMemcpyAsync D2D with
// the runtime engine: kernels or SDMA writing the consumer's HBM through the IPC mapping, over xGMI
// when the GPUs differ).
// The consumer is told only by a notice posted after hipEventQuery reported that copy complete,
// i.e. after the copy's end-of-operation release (agent scope: buffer_wbl2 -- dirty lines,
// including lines of peer memory, leave the producer GPU's L2).  The consumer reads a leased slot
// ONLY from kernels it launches after the host took the notice (get / get_batch return first);
// every kernel dispatch begins with the packet's acquire, which invalidates the consumer GPU's
// L1/L2 lines that may still hold the slot's previous frame -- the same kernel-boundary rule that
// makes one kernel's output visible to the next kernel on another XCD of the same GPU.  No
// persistent kernel polls ring slots, and nothing reads a slot between grant and notice.  This is
// what the bit-exact multi-process tests rely on (test_elastic_gpu.py: producer and consumer
// processes on one GPU, slots reused many times); a consumer that ever polled slots from a
// resident kernel would need an explicit agent acquire (Guideline 16) after its poll.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <array>
#include <atomic>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "runtime.h"
#include "verify.h"

namespace pr {

bool pid_alive(int64_t pid);
bool shm_remove(const std::string& name);   // shm_unlink, true when the name existed

// ---------------------------------------------------------------------------------------
// A named POSIX shared-memory region (the ring of a host consumer).
class ShmRegion {
 public:
  ShmRegion(const std::string& name, int64_t bytes, bool create, double timeout_s);
  ~ShmRegion();
  ShmRegion(const ShmRegion&) = delete;
  ShmRegion& operator=(const ShmRegion&) = delete;
  uint64_t ptr() const { return reinterpret_cast<uint64_t>(base_); }
  int64_t bytes() const { return bytes_; }
  const std::string& name() const { return name_; }
  void unlink();

 private:
  std::string name_;
  uint8_t* base_ = nullptr;
  int64_t bytes_ = 0;
  bool owner_ = false, unlinked_ = false;
};

// ---------------------------------------------------------------------------------------
struct FabricStats {
  int64_t iterations = 0, idle_iterations = 0;
  int64_t frames_local = 0;      // producer -> own consumer, zero copy
  int64_t frames_sent = 0;       // producer -> another process (noticed)
  int64_t frames_recv = 0;       // consumer <- another process
  int64_t frames_requeued = 0;   // copy finished after the consumer left: back to the FIFO
  int64_t grants_given = 0, grants_returned = 0, grants_reclaimed = 0;
  int64_t bytes_sent = 0, bytes_recv = 0, batches = 0;
  int64_t links_opened = 0, peers_dead = 0;
  int64_t links_failed = 0;      // consumer ring could not be mapped (link unusable, others unaffected)
  int64_t frames_returned = 0;   // consumer: read-ahead frames handed back to a producer on close
  int64_t frames_reclaimed = 0;  // producer: frames taken back from closing consumers (requeued)
  int64_t frames_dropped = 0;    // consumer: read-ahead frames no live producer could take back
  int64_t returns_rejected = 0;  // consumer: returns refused (that producer had posted EOS) and re-routed
  int64_t readahead = 0;         // producer: frames in consumers' read-ahead not taken yet (gauge)
  double copy_s = 0;             // sum over batches of issue -> completion observed (includes the wait
                                 // for the frames' calibration, which the copy is ordered after)
  int64_t copy_launches = 0;     // copy dispatches (kernel engine: one per fabric pass over all links)
  double copy_dev_ms = 0;        // sum of device time of the copies themselves (timing events)
  int64_t copy_dev_bytes = 0;    // bytes those timed copies moved
  int64_t taken_local = 0;       // consumer: frames taken (get) that its own process produced
  int64_t taken_remote = 0;      // consumer: frames taken that another process produced
  int64_t frames_direct = 0;       // producer: frames calibrated straight into a consumer's slot (no copy)
  int64_t frames_lost_direct = 0;  // producer: direct frames whose consumer left before their notice
  int64_t frames_checksummed = 0;  // producer: frames sent with a content checksum (verify.h)
  int64_t frames_corrupted = 0;    // producer: test-only fault injection (PSANA_RAY_AMD_FAULT_CORRUPT)
};

// One timed copy dispatch (fabric pass): device time of the copy, bytes, frames, host time from
// issue to completion observed (the latter includes the wait for the frames' calibration).
struct CopySample {
  double dev_ms = 0, issue_to_done_ms = 0;
  int64_t bytes = 0;
  int32_t frames = 0, links = 0;
};

struct LinkStatus {
  int64_t peer = -1;         // member id of the other end
  bool outgoing = false;     // true: this process produces into the peer's shard
  bool attached = false;     // both ends have mapped the mailbox
  bool eos = false;          // producer posted EOS (incoming: and every notice was taken)
  bool detached = false;     // producer left after EOS
  bool dead = false;         // the peer process exited
  bool closed = false;       // the consumer closed the link
  bool keeper = false;       // the consumer end is a queue keeper
  int64_t outstanding = 0;   // grants not answered yet
  int64_t frames = 0;        // frames moved over the link
  int64_t taken = 0;         // frames of this link the consumer took (get)
  int32_t consumer_device = -1;   // outgoing: the GPU of the consumer ring (-1 host)
  bool kernel_copy = false;       // outgoing: frames move by the copy kernel (else the runtime's copies)
  int32_t peer_access = -1;       // outgoing, other GPU: hipDeviceCanAccessPeer(this, consumer) (-1: n/a)
  int32_t link_type = -1;         // outgoing, other GPU: hipExtGetLinkTypeAndHopCount type (4 = xGMI)
  int32_t hops = -1;              //   and hop count (1 = a direct link)
};

class QueueFabric {
 public:
  // policy: 0 balanced (local unless a remote consumer has kLocalSlack more free slots granted, or is
  //           starving: nothing to read at all while this process's own consumer has frames ready),
  //         1 local_first, 2 spread (round-robin over every consumer with credit),
  //         3 relay (queue keeper: never to its own consumer side; most granted credit first),
  //         4 remote_only (never to its own consumer while a remote consumer link is attached:
  //           the bench's cross-GPU window, every frame crosses xGMI).
  // slot addresses come from the pool (SlotPool::set_slot_ptrs): rings are built from segments
  QueueFabric(SlotPool* pool, int64_t slot_bytes, int device, bool is_producer, bool is_consumer, int policy,
              int64_t self_mid);
  ~QueueFabric();
  QueueFabric(const QueueFabric&) = delete;
  QueueFabric& operator=(const QueueFabric&) = delete;

  // consumer role: how producers reach this ring (written into every link this process creates):
  // a host ring is one named shared-memory region; an HBM ring is exported as one HIP IPC handle
  // per allocation (segment) it is made of
  void export_host_ring(const std::string& shm_name);
  void export_ipc_ring();
  int export_segments() const { return (int)segs_.size(); }
  static constexpr int kMaxSegments = 256;
  // membership changes (any thread; applied by the engine thread)
  void add_in_link(int64_t producer_mid, const std::string& name);   // consumer: create mailbox
  void add_out_link(int64_t consumer_mid, const std::string& name);  // producer: open it
  void drop_peer(int64_t mid);                                        // peer gone (store view)
  void set_policy(int policy);
  // consumer role: grant only to producers marked grantable (queue keeper: absorbs the frames of
  // producers that finished and wait for consumers, never competes with live ones)
  void set_grant_filter(bool on) { grant_filter_.store(on); }
  void set_peer_grantable(int64_t mid, bool on);
  void set_producer_finished() { finished_.store(true); }
  void set_consumer_closed() { consumer_closed_.store(true); }
  // consumer role: bound on (frames noticed but not taken + grants outstanding), summed over links;
  // 0 = unbounded (only the ring's free slots limit grants).  A consumer that dies loses at most
  // this many frames plus the ones it had taken and not finished.
  void set_prefetch(int n) { prefetch_.store(n < 0 ? 0 : n); }
  int prefetch() const { return prefetch_.load(); }
  // consumer role: mark every mailbox this process creates as a queue keeper's (before links exist)
  void set_keeper(bool on) { keeper_ = on; }
  // consumer: true once no live producer can still be writing into this ring (every attached
  // producer acknowledged the close, detached or died) -- only then may the ring be freed
  bool consumer_quiesced() const { return quiesced_.load(); }
  // producer (GPU): how frames move into GPU consumer rings.
  //   kCopyKernel (default): every frame of one fabric pass, to all links, in ONE copy_runs_kernel
  //     launch on a stream that owns its hardware queue (a copy waiting for its frames' calibration
  //     blocks nothing else); `workgroups` bounds the CUs it takes from the pipeline.
  //   kCopyRuntime: hipMemcpyAsync per contiguous run on one ordinary stream per link (blit kernels
  //     or SDMA, HSA_ENABLE_SDMA) -- kept for A/B measurements.
  // Before start().
  static constexpr int kCopyKernel = 0, kCopyRuntime = 1;
  void set_copy_engine(int engine, int workgroups, int stream_kind = 1);   // kind: csrc/streams.h
  int copy_engine() const { return copy_engine_; }
  int copy_workgroups() const { return copy_wgs_; }
  // the newest timed copy dispatches (bounded), oldest first
  std::vector<CopySample> copy_samples() const;
  static constexpr int kMaxSamples = 4096;

  // End-to-end frame checks (verify.h).  Producer: every `every`-th frame (idx % every == 0, rank-local) sent
  // to another process carries a content checksum in its notice (0 = none).  Consumer: frames taken
  // from other processes get a system-scope acquire on the reader's stream, checksummed ones are
  // re-summed and compared.  Before start().
  void set_verify_every(int every);
  int verify_every() const { return verify_every_; }
  // consumer: {verified, mismatched, last mismatching gevt, acquires} (verify.h counts())
  std::array<int64_t, 4> verify_counts() const;

  // Producer, GPU, kernel engine: calibrate straight into granted consumer slots (VERDICT r5 next
  // #4; SURVEY 5.8 "the calib kernel writes directly into the ring slot").  While the routing policy
  // sends frames to other processes (spread, remote_only), the fabric thread keeps up to kDirectPool
  // grants of live remote consumers on offer.  The producer engine takes some for a chunk
  // (take_direct: the consumer-ring address each frame's calibration writes, over xGMI for another
  // GPU), binds them to the chunk's local slots BEFORE committing those (bind_direct: the local slot
  // then only carries the header and the queue_size accounting), and the fabric posts each frame's
  // notice once its calibration completed -- no copy pass.  Frames produced without a direct grant
  // keep the copy path.  A consumer that dies or closes while a direct frame is in flight loses
  // that frame (its data exists only in that consumer's ring; counted as frames_lost_direct).
  // Bound frames are issued as soon as they are committed, wherever they sit in the produced FIFO.
  // With the engine's direct headroom (engine.h) the engine waits for grants rather than queue
  // copies, which makes nearly every routed frame direct.
  struct DirectGrant {
    int64_t token;
    uint64_t ptr;
  };
  void set_direct(bool on);   // before start()
  bool direct() const { return direct_on_; }
  std::vector<DirectGrant> take_direct(int max_n);
  void bind_direct(const std::vector<int>& local_slots, const std::vector<int64_t>& tokens);
  void cancel_direct(const std::vector<int64_t>& tokens);   // taken and never launched
  static constexpr int kDirectPool = 128;
  // grants are on offer now (direct on, policy spread / remote_only, producer not finished)
  bool direct_offering() const;
  // direct frames that hold a local slot (bound to a grant, or dispatched and not yet complete)
  int64_t direct_inflight() const { return d_inflight_.load(std::memory_order_relaxed); }

  void start();
  void request_stop() { stop_.store(true); }
  bool join(double timeout_s);
  void halt();     // stop the progress thread and join it (process exit: halt_native_threads)
  int64_t step();  // one engine iteration on the caller's thread (tests); returns work items

  bool running() const { return running_.load(); }
  bool producer_drained() const { return drained_.load(); }
  std::string error() const;
  std::string last_link_error() const;   // why the last failed link could not be mapped
  FabricStats stats() const;
  std::vector<LinkStatus> links() const;
  int policy() const { return policy_.load(); }

  static constexpr int kLocalSlack = 64;
  static constexpr int kFeedLocalReady = 2;   // balanced: own consumer's ready frames before feeding a starving one
  // copy-kernel grid when every consumer of a dispatch sits on this GPU (2-rank-on-one-GPU A/B,
  // device-resident, remote_only window: 512 -> 100.4k / 105.2k fr/s, 256 -> 100.1k / 101.1k,
  // 128 -> 93.6k / 94.4k; profiles/r4/fabric_pass3)
  static constexpr int kLocalCopyWgs = 512;
  static constexpr int kMaxCopyWgs = 4096;
  // workgroups of one copy dispatch writing the rings on `consumer_devices` from GPU `device`:
  // kLocalCopyWgs if one of them is this GPU, plus `per_peer` per distinct other GPU (each is its
  // own xGMI link), capped at kMaxCopyWgs
  static int copy_grid_for(const std::vector<int>& consumer_devices, int device, int per_peer);
  static constexpr int kMinGrants = 4;      // grants kept at an idle producer (pipeline depth)
  static constexpr int kMaxDispatch = 64;   // produced frames routed per iteration

 private:
  struct Link;
  struct Batch;
  struct CopyGroup;   // one timed copy dispatch shared by the per-link batches it carries
  void loop();
  void fail(const std::string& msg);
  void apply_ops();
  int64_t consumer_pass(double now);
  int64_t producer_pass(double now);
  bool try_attach(Link& l, double now);
  void release_out_link(Link& l);
  void finish_in_link(Link& l);
  bool post_return(Link* pref, int slot, const SlotHeader& h);
  void drop_returned(int slot);
  void publish_status();
  hipEvent_t take_event();
  hipEvent_t take_timed_event();
  void issue_copies(std::vector<Batch>& kb, double now);
  int copy_grid(const std::vector<Batch>& kb) const;
  void finish_group(const std::shared_ptr<CopyGroup>& g);
  int64_t direct_pass();
  void issue_direct(std::vector<Batch>& db);
  void start_checksums(Batch& b, uint64_t stream);
  void finish_checksums(Batch& b);
  void inject_corruption(const Batch& b, uint64_t stream);

  SlotPool* pool_;
  int64_t slot_bytes_;
  int device_;
  bool is_producer_, is_consumer_;
  std::atomic<int> policy_;
  int64_t self_mid_;
  // ring export
  int export_kind_ = -1;  // 0 host shm, 1 ipc
  std::string export_name_;
  struct SegExport {
    std::vector<uint8_t> handle;
    int64_t offset = 0;
    int32_t first = 0, n = 0;
  };
  std::vector<SegExport> segs_;

  hipStream_t stream_ = nullptr;
  hipStream_t xstream_ = nullptr;   // kernel engine: the copy stream (own hardware queue, pooled)
  int copy_engine_ = kCopyKernel;
  int copy_wgs_ = 128;
  int verify_every_ = 0;
  std::shared_ptr<FrameVerifier> verifier_;
  int64_t corrupt_every_ = 0, corrupt_count_ = 0;   // test-only fault injection
  int direct_fence_ = 0;   // diagnostic (PSANA_RAY_AMD_DIRECT_FENCE): 1 release, 2 acquire around direct frames
  // direct grants (take_direct / bind_direct): offered, taken by the engine, bound to a local slot.
  // Every transition under dmu_; only the fabric thread adds offers or resolves them.
  struct DirectRec {
    std::shared_ptr<Link> link;
    int rslot = -1;
  };
  bool direct_on_ = false;
  std::mutex dmu_;
  std::deque<std::pair<int64_t, DirectRec>> d_free_;
  std::vector<std::pair<int64_t, DirectRec>> d_taken_, d_cancel_;
  std::vector<std::pair<int, DirectRec>> d_bound_;   // local slot -> grant
  int64_t d_next_ = 1;
  std::atomic<int64_t> d_inflight_{0};
  int xstream_kind_ = 1;            // kStreamDedicated
  std::vector<hipEvent_t> free_events_, all_events_;
  std::vector<hipEvent_t> free_timed_;          // timing-enabled events (copy groups)
  std::deque<CopySample> samples_;              // guarded by mu_
  std::vector<std::shared_ptr<Link>> links_;
  std::deque<Batch> inflight_;
  std::deque<Batch> reclaims_;   // producer: copies of returned frames back into this pool
  int rr_ = 0;
  int64_t returns_pending_ = 0;  // consumer: returned frames not answered yet
  bool eos_any_ = false;         // producer: EOS posted (returns are refused from then on)
  bool keeper_ = false;
  std::atomic<int> prefetch_{0};

  struct Op {
    int kind;  // 0 in, 1 out, 2 drop, 3 grantable on, 4 grantable off
    int64_t mid;
    std::string name;
  };
  std::mutex ops_mu_;
  std::vector<Op> ops_;
  std::vector<int64_t> grantable_;   // engine thread: peers a filtered consumer grants to

  std::atomic<bool> finished_{false}, consumer_closed_{false}, stop_{false}, running_{false}, drained_{false};
  std::mutex halt_mu_;   // halt() from the destructor and from halt_native_threads()
  bool closed_posted_ = false;   // consumer: consumer_closed stored in every mailbox
  bool returns_final_ = false;   // consumer: returns_final stored in every mailbox
  std::atomic<bool> quiesced_{false};
  std::atomic<bool> grant_filter_{false};
  std::vector<LinkStatus> retired_;
  std::thread th_;
  mutable std::mutex mu_;  // error_, st_, status_
  std::string error_, link_error_;
  FabricStats st_;
  std::vector<LinkStatus> status_;
};

}  // namespace pr
