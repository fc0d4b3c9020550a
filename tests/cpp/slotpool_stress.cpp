// Host-side race / memory-safety stress of the native runtime, built with ThreadSanitizer or
// AddressSanitizer+UBSan by tools/sanitize_host.sh (CPU only: pools run with device = -1, so no
// HIP call is made and the sanitizers see only our code).
//
// SURVEY §5 "Race detection": the reference serialises everything through one single-threaded
// actor; here the slot pool is shared by a producer thread, a transport thread and consumer
// threads, so its state machine is exercised concurrently:
//   scenario 1 (transport): producer -> pool A --(transport thread: begin/end send+recv)--> pool B
//                           -> 2 consumer threads; checks every event arrives exactly once, in
//                           per-producer FIFO order per consumer.
//   scenario 2 (auto-route): producer thread + 3 consumer threads on ONE pool in single-process
//                           mode (routing inside commit/release), batch and single-slot calls mixed.
//   scenario 3 (fabric): 3 members in one process (producer / producer+consumer / consumer), each
//                           with its own pool, host ring in named shared memory and a QueueFabric
//                           thread; links created through the same mailbox protocol separate
//                           processes use; checks payload bytes, exactly-once delivery, per-producer
//                           FIFO order within a shard and EOS, for every routing policy.
//   scenario 4 (fabric, consumer leaves): the consumer-only member closes mid-stream, hands back its
//                           unread frames, and is
//                           dropped; producers requeue its in-flight frames; the surviving consumer
//                           gets every frame the leaver had not taken, and the stream still ends.
#include <stdint.h>
#include <stdio.h>

#include <unistd.h>

#include <atomic>
#include <chrono>
#include <memory>
#include <string>
#include <mutex>
#include <random>
#include <stdexcept>
#include <thread>
#include <vector>

#include "runtime.h"
#include "fabric.h"

using pr::SlotHeader;
using pr::SlotPool;

static void require(bool ok, const char* what) {
  if (!ok) {
    fprintf(stderr, "FAILED: %s\n", what);
    std::abort();
  }
}

static void scenario_transport(int64_t n_events) {
  SlotPool A(48, 0, -1);    // producer rank: producer budget only
  SlotPool B(0, 40, -1);    // consumer rank: consumer budget only
  std::atomic<bool> prod_done{false}, xport_done{false};
  std::vector<std::atomic<int>> seen(n_events);
  for (auto& s : seen) s.store(0);

  std::thread producer([&] {
    std::mt19937 rng(1);
    int64_t k = 0;
    while (k < n_events) {
      const int n = std::min<int64_t>(1 + rng() % 8, n_events - k);
      std::vector<int> slots = A.acquire_batch(n, 0.01, 0);
      if (slots.empty()) continue;
      std::vector<SlotHeader> h(slots.size());
      for (size_t i = 0; i < slots.size(); ++i) {
        h[i].rank = 0;
        h[i].idx = k + (int64_t)i;
        h[i].gevt = k + (int64_t)i;
        h[i].photon_energy = 1.0 * (double)(k + (int64_t)i);
      }
      A.commit_batch(slots, h, 0);
      k += (int64_t)slots.size();
    }
    prod_done.store(true);
  });

  std::thread transport([&] {
    int64_t moved = 0;
    while (moved < n_events) {
      std::vector<int> offers = A.produced(16);
      const int k = std::min<int>((int)offers.size(), B.credits());
      if (k == 0) {
        std::this_thread::yield();
        continue;
      }
      offers.resize(k);
      std::vector<SlotHeader> hdrs = A.headers(offers);
      A.begin_send_batch(offers, 0);
      std::vector<int> recv = B.begin_recv_batch(k, 0);
      require((int)recv.size() == k, "begin_recv_batch returned fewer slots than credits");
      A.end_send_batch(offers, 0);
      B.end_recv_batch(recv, hdrs, 0);
      moved += k;
    }
    xport_done.store(true);
  });

  std::mutex mu;
  int64_t last_idx[2] = {-1, -1};
  auto consumer = [&](int id) {
    std::mt19937 rng(100 + id);
    for (;;) {
      std::vector<int> got = B.get_batch(1 + rng() % 6, 0.01, 0);
      if (got.empty()) {
        if (xport_done.load() && B.n_ready() == 0) return;
        continue;
      }
      std::vector<SlotHeader> hs = B.headers(got);
      for (const auto& h : hs) {
        require(h.idx >= 0 && h.idx < (int64_t)seen.size(), "header idx out of range");
        require(h.photon_energy == 1.0 * (double)h.idx, "header corrupted in transit");
        seen[h.idx].fetch_add(1);
        std::lock_guard<std::mutex> lk(mu);
        require(h.idx > last_idx[id], "per-consumer FIFO order violated");
        last_idx[id] = h.idx;
      }
      B.release_batch(got, 0);
    }
  };
  std::thread c0(consumer, 0), c1(consumer, 1);
  producer.join();
  transport.join();
  c0.join();
  c1.join();
  for (int64_t i = 0; i < n_events; ++i) require(seen[i].load() == 1, "event lost or duplicated");
  require(A.producer_held() == 0 && B.consumer_held() == 0, "slots leaked");
  printf("transport scenario: %lld events OK\n", (long long)n_events);
}

static void scenario_auto_route(int64_t n_events) {
  SlotPool P(24, 32, -1);
  P.set_auto_route(true);
  std::atomic<bool> done{false};
  std::vector<std::atomic<int>> seen(n_events);
  for (auto& s : seen) s.store(0);
  std::thread producer([&] {
    std::mt19937 rng(7);
    int64_t k = 0;
    while (k < n_events) {
      if (rng() % 2) {   // single-slot API
        const int s = P.acquire_produce(0.01);
        if (s < 0) continue;
        SlotHeader h;
        h.rank = 0;
        h.idx = k;
        h.gevt = k;
        P.commit_produce(s, h, 0);
        ++k;
      } else {           // batch API
        const int n = std::min<int64_t>(1 + rng() % 5, n_events - k);
        std::vector<int> slots = P.acquire_batch(n, 0.01, 0);
        if (slots.empty()) continue;
        std::vector<SlotHeader> h(slots.size());
        for (size_t i = 0; i < slots.size(); ++i) h[i].idx = h[i].gevt = k + (int64_t)i;
        P.commit_batch(slots, h, 0);
        k += (int64_t)slots.size();
      }
    }
    done.store(true);
  });
  auto consumer = [&](int id) {
    std::mt19937 rng(50 + id);
    for (;;) {
      if (rng() % 2) {
        const int s = P.get(0.005);
        if (s < 0) {
          if (done.load() && P.n_ready() == 0 && P.n_produced() == 0) return;
          continue;
        }
        seen[P.header(s).idx].fetch_add(1);
        P.release(s, 0);
      } else {
        std::vector<int> got = P.get_batch(1 + rng() % 4, 0.005, 0);
        if (got.empty()) {
          if (done.load() && P.n_ready() == 0 && P.n_produced() == 0) return;
          continue;
        }
        for (const auto& h : P.headers(got)) seen[h.idx].fetch_add(1);
        P.release_batch(got, 0);
      }
    }
  };
  std::thread c0(consumer, 0), c1(consumer, 1), c2(consumer, 2);
  producer.join();
  c0.join();
  c1.join();
  c2.join();
  for (int64_t i = 0; i < n_events; ++i) require(seen[i].load() == 1, "auto-route: event lost or duplicated");
  printf("auto-route scenario: %lld events OK\n", (long long)n_events);
}

// Members of one fabric "session" inside this process (the same mailboxes other processes use).
struct Member {
  std::unique_ptr<SlotPool> pool;
  std::unique_ptr<pr::ShmRegion> ring;
  std::unique_ptr<pr::QueueFabric> fab;
  bool prod = false, cons = false;
};

static void scenario_fabric(int64_t n_per_producer, int policy, bool leave) {
  const int M = 3;
  const int64_t slot_bytes = 192;
  const bool is_p[M] = {true, true, false}, is_c[M] = {false, true, true};
  const std::string tok = "/psq-stress-" + std::to_string((long long)getpid()) + "-" + std::to_string(policy) +
                          (leave ? "L" : "");
  std::vector<Member> m(M);
  for (int r = 0; r < M; ++r) {
    m[r].prod = is_p[r];
    m[r].cons = is_c[r];
    m[r].pool.reset(new SlotPool(is_p[r] ? 12 : 0, is_c[r] ? 10 : 0, -1));
    m[r].ring.reset(new pr::ShmRegion(tok + "-r" + std::to_string(r), (int64_t)m[r].pool->n_slots() * slot_bytes,
                                      true, 5.0));
    std::vector<uint64_t> ptrs((size_t)m[r].pool->n_slots());
    for (size_t k = 0; k < ptrs.size(); ++k) ptrs[k] = m[r].ring->ptr() + k * (uint64_t)slot_bytes;
    m[r].pool->set_slot_ptrs(ptrs);
    m[r].fab.reset(new pr::QueueFabric(m[r].pool.get(), slot_bytes, -1, is_p[r], is_c[r], policy, r));
    if (is_c[r]) m[r].fab->export_host_ring(m[r].ring->name());
  }
  for (int p = 0; p < M; ++p)
    for (int c = 0; c < M; ++c) {
      if (p == c || !is_p[p] || !is_c[c]) continue;
      const std::string name = tok + "-" + std::to_string(p) + "-" + std::to_string(c);
      m[c].fab->add_in_link(p, name);
      m[p].fab->add_out_link(c, name);
    }
  for (auto& x : m) x.fab->start();
  auto payload = [](int64_t rank, int64_t idx, int64_t j) { return (uint8_t)(rank * 131 + idx * 7 + j * 3); };
  std::vector<std::thread> th;
  std::atomic<int> finished{0};
  for (int r = 0; r < M; ++r) {
    if (!is_p[r]) continue;
    th.emplace_back([&, r] {
      uint8_t* base = reinterpret_cast<uint8_t*>(m[r].ring->ptr());
      for (int64_t k = 0; k < n_per_producer;) {
        const int s = m[r].pool->acquire_produce(0.01);
        if (s < 0) continue;
        uint8_t* d = base + (size_t)s * slot_bytes;
        for (int64_t j = 0; j < slot_bytes; ++j) d[j] = payload(r, k, j);
        SlotHeader h;
        h.rank = r;
        h.idx = k;
        h.gevt = 1000 * r + k;
        h.photon_energy = 0.5 * (double)k;
        m[r].pool->commit_produce(s, h, 0);
        ++k;
      }
      m[r].fab->set_producer_finished();
      finished.fetch_add(1);
    });
  }
  std::vector<std::atomic<int>> seen(2 * n_per_producer);
  for (auto& x : seen) x.store(0);
  std::atomic<int64_t> taken_by_leaver{0};
  auto stream_done = [&](int r) {
    // every producer drained (posted EOS) and every link into r saw it
    if (finished.load() < 2) return false;
    for (int p = 0; p < M; ++p)
      if (is_p[p] && !m[p].fab->producer_drained()) return false;
    for (const auto& ls : m[r].fab->links())
      if (!ls.outgoing && ls.attached && !(ls.eos || ls.dead || ls.detached)) return false;
    return true;
  };
  for (int r = 0; r < M; ++r) {
    if (!is_c[r]) continue;
    th.emplace_back([&, r] {
      const bool leaver = leave && r == 2;
      int64_t last[2] = {-1, -1};
      const uint8_t* base = reinterpret_cast<const uint8_t*>(m[r].ring->ptr());
      int64_t got = 0;
      for (;;) {
        if (leaver && got >= n_per_producer / 4) {
          // close mid-stream: producers stop writing here and requeue what was in flight
          m[r].fab->set_consumer_closed();
          while (!m[r].fab->consumer_quiesced()) std::this_thread::sleep_for(std::chrono::microseconds(200));
          for (int p = 0; p < M; ++p)
            if (p != r) m[p].fab->drop_peer(r);
          taken_by_leaver.store(got);
          return;
        }
        const int s = m[r].pool->get(0.005);
        if (s < 0) {
          require(m[r].fab->error().empty(), "fabric failed");
          if (stream_done(r) && m[r].pool->n_ready() == 0) return;
          continue;
        }
        const SlotHeader h = m[r].pool->header(s);
        require(h.rank >= 0 && h.rank < 2 && h.idx >= 0 && h.idx < n_per_producer, "fabric: header out of range");
        require(h.gevt == 1000 * h.rank + h.idx && h.photon_energy == 0.5 * (double)h.idx, "fabric: header corrupted");
        if (!leave) require(h.idx > last[h.rank], "fabric: per-producer FIFO order violated within a shard");
        last[h.rank] = h.idx;
        const uint8_t* d = base + (size_t)s * slot_bytes;
        for (int64_t j = 0; j < slot_bytes; ++j) require(d[j] == payload(h.rank, h.idx, j), "fabric: payload corrupted");
        seen[h.rank * n_per_producer + h.idx].fetch_add(1);
        ++got;
        m[r].pool->release(s, 0);
      }
    });
  }
  for (auto& t : th) t.join();
  for (auto& x : m) require(x.fab->error().empty(), "fabric reported an error");
  int64_t lost = 0;
  for (size_t i = 0; i < seen.size(); ++i) {
    require(seen[i].load() <= 1, "fabric: event duplicated");
    lost += seen[i].load() == 0;
  }
  // the leaver hands the frames it received and did not take back to the producers (they are
  // still producing when it leaves): nothing may be lost
  require(lost == 0, "fabric: events lost");
  if (leave) require(m[2].fab->stats().frames_returned == m[0].fab->stats().frames_reclaimed +
                                                             m[1].fab->stats().frames_reclaimed,
                     "fabric: returned frames not all reclaimed");
  const pr::FabricStats s1 = m[1].fab->stats();
  printf("fabric scenario (policy %d%s): %lld events, %lld lost, %lld sent by member 1, %lld requeued\n", policy,
         leave ? ", consumer leaves" : "", (long long)seen.size(), (long long)lost, (long long)s1.frames_sent,
         (long long)(m[0].fab->stats().frames_requeued + s1.frames_requeued));
  for (auto& x : m) {
    x.fab->request_stop();
    require(x.fab->join(30.0), "fabric thread did not stop");
  }
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 20000;
  try {
    scenario_transport(n);
    scenario_auto_route(n);
    for (int policy = 0; policy < 3; ++policy) scenario_fabric(std::max<int64_t>(200, n / 8), policy, false);
    scenario_fabric(std::max<int64_t>(400, n / 8), 2, true);
  } catch (const std::exception& e) {
    fprintf(stderr, "FAILED with exception: %s\n", e.what());
    return 1;
  }
  printf("SLOTPOOL_STRESS_OK\n");
  return 0;
}
