#include "transport.h"

#include <hip/hip_runtime.h>
#include <string.h>

#include "common.h"
#include "trace.h"

namespace pr {

static void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string("psana_ray_amd RCCL error in ") + what + ": " + ncclGetErrorString(r));
}

std::string rccl_version() {
  int v = 0;
  nccl_check(ncclGetVersion(&v), "ncclGetVersion");
  return std::to_string(v / 10000) + "." + std::to_string((v / 100) % 100) + "." + std::to_string(v % 100);
}

std::vector<uint8_t> rccl_unique_id() {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::vector<uint8_t> out(sizeof(id.internal));
  memcpy(out.data(), id.internal, sizeof(id.internal));
  return out;
}

RcclTransport::RcclTransport(const std::vector<uint8_t>& id, int rank, int world, int device)
    : rank_(rank), world_(world), device_(device) {
  ncclUniqueId uid;
  check(id.size() == sizeof(uid.internal), "RcclTransport: unique id has the wrong size");
  check(world >= 1 && rank >= 0 && rank < world, "RcclTransport: bad rank/world");
  memcpy(uid.internal, id.data(), sizeof(uid.internal));
  hip_check(hipSetDevice(device), "hipSetDevice");
  nccl_check(ncclCommInitRank(&comm_, world, uid, rank), "ncclCommInitRank");
}

RcclTransport::~RcclTransport() {
  if (comm_ == nullptr) return;
  if (aborted_) return;
  // destroy waits for outstanding work; a failed run calls abort() first
  ncclCommDestroy(comm_);
  comm_ = nullptr;
}

void RcclTransport::abort() {
  if (comm_ != nullptr && !aborted_) {
    aborted_ = true;
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

std::string RcclTransport::async_error() {
  if (comm_ == nullptr) return aborted_ ? "communicator aborted" : "no communicator";
  ncclResult_t r = ncclSuccess;
  if (ncclCommGetAsyncError(comm_, &r) != ncclSuccess) return "ncclCommGetAsyncError failed";
  return r == ncclSuccess ? std::string() : std::string(ncclGetErrorString(r));
}

void RcclTransport::exchange(const std::vector<uint64_t>& sptr, const std::vector<int>& speer,
                             const std::vector<uint64_t>& rptr, const std::vector<int>& rpeer, int64_t bytes,
                             uint64_t stream) {
  check(comm_ != nullptr, "RcclTransport: communicator is gone");
  check(sptr.size() == speer.size() && rptr.size() == rpeer.size(), "RcclTransport: list length mismatch");
  check(bytes > 0, "RcclTransport: empty message");
  if (sptr.empty() && rptr.empty()) return;
  for (int p : speer) check(p >= 0 && p < world_, "RcclTransport: send peer out of range");
  for (int p : rpeer) check(p >= 0 && p < world_, "RcclTransport: recv peer out of range");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  trace::Range tr("transport.rccl_group");
  nccl_check(ncclGroupStart(), "ncclGroupStart");
  for (size_t i = 0; i < sptr.size(); ++i)
    nccl_check(ncclSend(reinterpret_cast<const void*>(sptr[i]), (size_t)bytes, ncclUint8, speer[i], comm_, s),
               "ncclSend");
  for (size_t i = 0; i < rptr.size(); ++i)
    nccl_check(ncclRecv(reinterpret_cast<void*>(rptr[i]), (size_t)bytes, ncclUint8, rpeer[i], comm_, s),
               "ncclRecv");
  nccl_check(ncclGroupEnd(), "ncclGroupEnd");
  bytes_sent_ += (int64_t)sptr.size() * bytes;
  bytes_recv_ += (int64_t)rptr.size() * bytes;
  ++groups_;
}

std::vector<int> RcclTransport::round(SlotPool* pool, uint64_t ring_base, int64_t slot_bytes,
                                      const std::vector<int>& send_slots, const std::vector<int>& send_peer,
                                      const std::vector<int>& recv_peer, const std::vector<SlotHeader>& recv_hdr,
                                      uint64_t stream) {
  check(send_slots.size() == send_peer.size(), "round: send lists differ in length");
  check(recv_peer.size() == recv_hdr.size(), "round: recv lists differ in length");
  std::vector<int> recv_slots;
  if (send_slots.empty() && recv_peer.empty()) return recv_slots;
  pool->begin_send_batch(send_slots, stream);   // stream waits for the frames' data
  if (!recv_peer.empty()) recv_slots = pool->begin_recv_batch((int)recv_peer.size(), stream);
  check(recv_slots.size() == recv_peer.size(), "round: not enough free consumer slots (credit accounting)");
  std::vector<uint64_t> sptr(send_slots.size()), rptr(recv_slots.size());
  for (size_t i = 0; i < send_slots.size(); ++i) sptr[i] = ring_base + (uint64_t)send_slots[i] * slot_bytes;
  for (size_t i = 0; i < recv_slots.size(); ++i) rptr[i] = ring_base + (uint64_t)recv_slots[i] * slot_bytes;
  exchange(sptr, send_peer, rptr, recv_peer, slot_bytes, stream);
  pool->end_send_batch(send_slots, stream);
  pool->end_recv_batch(recv_slots, recv_hdr, stream);
  return recv_slots;
}

}  // namespace pr
