// Native RCCL data plane of the sharded shared queue (frames GPU -> GPU over xGMI).
//
// Reference parity: psana-ray moves every frame with a synchronous Ray actor RPC through the
// object store (psana_ray/producer.py:101 put, psana_ray/data_reader.py:35 get; SURVEY C-01/C-03).
// Here a transport round's frames move as ONE RCCL group of ncclSend/ncclRecv on a dedicated
// stream: each frame is a whole HBM ring slot, sent straight from the producer's slot into a
// free slot of the consumer's shard (no staging copy, no host round trip).  The fused `round`
// also does the slot-pool bookkeeping and the HIP-event ordering of both ends, so the Python
// transport thread makes one native call (GIL released) per round instead of one torch
// P2POp per frame ("RCCL p2p over xGMI (C++: ncclSend/Recv, grouped)").
//
// The communicator is our own (ncclCommInitRank with an id broadcast over the gloo control
// group); RCCL is torch's own librccl, so one RCCL/HIP runtime is loaded per process.
#pragma once

#include <rccl/rccl.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "runtime.h"

namespace pr {

std::string rccl_version();
std::vector<uint8_t> rccl_unique_id();

class RcclTransport {
 public:
  RcclTransport(const std::vector<uint8_t>& id, int rank, int world, int device);
  ~RcclTransport();
  RcclTransport(const RcclTransport&) = delete;
  RcclTransport& operator=(const RcclTransport&) = delete;

  // Raw grouped exchange: sends sptr[i] (bytes) to speer[i], receives rptr[j] from rpeer[j].
  // Per peer pair, sends and receives match in issue order.
  void exchange(const std::vector<uint64_t>& sptr, const std::vector<int>& speer,
                const std::vector<uint64_t>& rptr, const std::vector<int>& rpeer, int64_t bytes,
                uint64_t stream);

  // One transport round on `stream`: stream waits for the send slots' data and for the recv
  // slots to be free, the group runs, then one event per direction marks completion
  // (end_send_batch frees the sent slots, end_recv_batch makes the received ones READY with
  // `recv_hdr`).  Returns the receive slots.
  std::vector<int> round(SlotPool* pool, uint64_t ring_base, int64_t slot_bytes,
                         const std::vector<int>& send_slots, const std::vector<int>& send_peer,
                         const std::vector<int>& recv_peer, const std::vector<SlotHeader>& recv_hdr,
                         uint64_t stream);

  // Asynchronous RCCL error (peer died mid-transfer, ...): empty string when healthy.
  std::string async_error();
  // Tear the communicator down without waiting for peers (after a failure).
  void abort();

  int rank() const { return rank_; }
  int world() const { return world_; }
  int64_t bytes_sent() const { return bytes_sent_; }
  int64_t bytes_recv() const { return bytes_recv_; }
  int64_t groups() const { return groups_; }

 private:
  ncclComm_t comm_ = nullptr;
  int rank_, world_, device_;
  bool aborted_ = false;
  int64_t bytes_sent_ = 0, bytes_recv_ = 0, groups_ = 0;
};

}  // namespace pr
