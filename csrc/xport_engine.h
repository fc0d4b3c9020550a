// Native transport engine of the sharded shared queue (one per rank, world > 1 or loopback).
//
// Reference parity: psana-ray serialises every put/get of every rank through ONE single-threaded
// Ray actor (psana_ray/shared_queue.py:4-31) reached by a synchronous RPC per frame
// (psana_ray/producer.py:101, psana_ray/data_reader.py:35; SURVEY C-01/C-03) and synchronises
// ranks with MPI Barriers (producer.py:53,120; C-05/C-06).  Here every rank runs a C++ thread
// that executes bulk-synchronous transport ROUNDS with no Python and no GIL on the path:
//
//   1. offers  = up to max_offer PRODUCED slots of the local pool (+ their headers),
//      credits = free consumer slots, flags (producer / consumer / EOS / closed);
//   2. all-gather of the fixed-size control vectors through a node-local shared-memory segment
//      (ShmControl: one cache-line sequence word per rank, double-buffered vectors; a round costs
//      a few microseconds instead of a gloo TCP all-gather, 2.7 ms at 8 ranks measured here);
//   3. the deterministic routing plan (routing.cpp) -- identical on every rank, so sends and
//      receives match without further messages;
//   4. the data plane: on GPUs ONE grouped ncclSend/ncclRecv of whole HBM slots over xGMI on the
//      transport stream (RcclTransport::round, event-ordered, no host sync); on host pools (CPU
//      tests, BASELINE config 1 across processes) a copy through per-rank shared-memory outboxes.
//
// Failure detection: every wait is bounded and also watches the peers' pids and
// "failed" words, so a dead peer turns into an error on every rank within ~50 ms, the RCCL
// communicator is aborted and blocked producers / consumers are woken (-> QueuePeerError /
// DataReaderError, the reference's RayActorError path).
#pragma once

#include <stdint.h>

#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "runtime.h"
#include "transport.h"

namespace pr {

// ---------------------------------------------------------------------------------------
// Node-local control plane: POSIX shared memory, one block per rank.
class ShmControl {
 public:
  // create: rank 0 creates + initialises (O_EXCL); the others attach (retrying until `timeout_s`).
  ShmControl(const std::string& name, bool create, int rank, int world, int vec_words, int64_t outbox_bytes,
             double timeout_s);
  ~ShmControl();
  ShmControl(const ShmControl&) = delete;
  ShmControl& operator=(const ShmControl&) = delete;

  void unlink();  // remove the name (the mapping stays valid); safe to call more than once
  // All-gather of `vec_words` int64 per rank for round `round` (>= 0, consecutive per rank).
  // out: world * vec_words.  Throws on timeout / dead or failed peer.
  void allgather(int64_t round, const int64_t* vec, int64_t* out);
  void publish_data(int64_t round);            // my outbox holds round `round`'s frames
  void wait_data(int peer, int64_t round);     // peer's outbox holds round `round`'s frames
  uint8_t* outbox(int r) const;
  void set_failed();                           // tell peers this rank failed
  void cancel() { cancelled_.store(true); }    // make local waits throw (shutdown)
  int world() const { return world_; }
  int rank() const { return rank_; }
  int vec_words() const { return vec_words_; }
  int64_t outbox_bytes() const { return outbox_bytes_; }
  double timeout_s() const { return timeout_s_; }
  const std::string& name() const { return name_; }
  // Test hook: a peer whose pid stops existing is reported as dead (default on).
  void set_check_pids(bool on) { check_pids_ = on; }

 private:
  struct Block;
  Block* block(int r) const;
  int64_t* vec_slot(int r, int64_t round) const;
  void wait_seq(int peer, int which, uint64_t target);

  std::string name_;
  int rank_, world_, vec_words_;
  int64_t outbox_bytes_;
  double timeout_s_;
  size_t block_bytes_ = 0, total_bytes_ = 0;
  uint8_t* base_ = nullptr;
  bool owner_ = false, unlinked_ = false, check_pids_ = true;
  std::atomic<bool> cancelled_{false};
};

// ---------------------------------------------------------------------------------------
struct XportStats {
  int64_t rounds = 0, idle_rounds = 0, frames_routed = 0, frames_sent = 0, frames_recv = 0, frames_local = 0;
  int64_t bytes_sent = 0, bytes_recv = 0;
  double round_s = 0, ctrl_s = 0, data_s = 0;
};

class TransportEngine {
 public:
  // rccl == nullptr: host pool, frames move through the ShmControl outboxes.
  TransportEngine(SlotPool* pool, ShmControl* ctrl, RcclTransport* rccl, uint64_t ring_base, int64_t slot_bytes,
                  int rank, int world, const std::vector<int>& producer_ranks, bool is_producer, bool is_consumer,
                  int policy, int max_offer, bool loopback, uint64_t stream, int device);
  ~TransportEngine();
  TransportEngine(const TransportEngine&) = delete;
  TransportEngine& operator=(const TransportEngine&) = delete;

  void start();
  bool join(double timeout_s);  // true when the thread finished
  int64_t step();                // one round on the caller's thread (tests); returns frames planned

  void set_producer_finished() { producer_finished_.store(true); }
  void set_consumer_closed() { consumer_closed_.store(true); }
  void request_stop() { stop_.store(true); }
  bool done() const { return done_.load(); }
  bool consumers_gone() const { return consumers_gone_.load(); }
  bool running() const { return running_.load(); }
  std::string error() const;
  XportStats stats() const;

  static constexpr int kHdr = 4, kPerOffer = 4;
  static constexpr int64_t kProducer = 1, kConsumer = 2, kEos = 4, kClosed = 8;
  static int vec_words_for(int max_offer) { return kHdr + kPerOffer * max_offer; }

 private:
  void loop();
  void fail(const std::string& msg);

  SlotPool* pool_;
  ShmControl* ctrl_;
  RcclTransport* rccl_;
  uint64_t ring_base_;
  int64_t slot_bytes_;
  int rank_, world_;
  std::vector<int> producer_ranks_;
  bool is_producer_, is_consumer_;
  int policy_, max_offer_;
  bool loopback_;
  uint64_t stream_;
  int device_;
  int64_t round_ = 0;
  std::vector<int64_t> vec_, all_;
  std::vector<bool> eos_from_;
  std::atomic<bool> producer_finished_{false}, consumer_closed_{false}, stop_{false}, done_{false};
  std::atomic<bool> consumers_gone_{false}, running_{false};
  std::thread th_;
  mutable std::mutex mu_;
  std::string error_;
  XportStats st_;
};

}  // namespace pr
