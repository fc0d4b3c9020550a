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
//   scenario 3 (routing): random plan_round inputs; every plan respects offers and credits.
//   scenario 4 (transport engine): 3 ranks in one process (producer / producer+consumer /
//                           consumer), each with its own pool, its own mapping of ONE shared-memory
//                           control segment and a TransportEngine thread; host data plane through
//                           the outboxes; checks payload bytes, exactly-once delivery and EOS.
#include <stdint.h>
#include <stdio.h>

#include <unistd.h>

#include <atomic>
#include <memory>
#include <string>
#include <mutex>
#include <random>
#include <stdexcept>
#include <thread>
#include <vector>

#include "runtime.h"
#include "xport_engine.h"

namespace pr {
std::vector<int32_t> plan_round_native(const std::vector<int64_t>& offers_in, const std::vector<int64_t>& credits_in,
                                       int64_t round_id, int policy);
}

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

static void scenario_routing(int iters) {
  std::mt19937 rng(3);
  for (int it = 0; it < iters; ++it) {
    const int world = 1 + rng() % 8;
    std::vector<int64_t> offers(world), credits(world);
    for (int r = 0; r < world; ++r) {
      offers[r] = (int64_t)(rng() % 70) - 3;    // includes negative garbage
      credits[r] = (int64_t)(rng() % 70) - 3;
    }
    for (int policy = 0; policy < 3; ++policy) {
      const std::vector<int32_t> flat = pr::plan_round_native(offers, credits, it, policy);
      require(flat.size() % 3 == 0, "plan is not a list of triples");
      std::vector<int64_t> used_off(world, 0), used_cred(world, 0);
      for (size_t k = 0; k < flat.size(); k += 3) {
        const int p = flat[k], i = flat[k + 1], c = flat[k + 2];
        require(p >= 0 && p < world && c >= 0 && c < world, "plan rank out of range");
        require(i == used_off[p], "offers of a producer must be consumed in FIFO order");
        ++used_off[p];
        ++used_cred[c];
      }
      int64_t tot_off = 0, tot_cred = 0, moved = (int64_t)flat.size() / 3;
      for (int r = 0; r < world; ++r) {
        require(used_off[r] <= std::max<int64_t>(0, offers[r]), "plan exceeds offers");
        require(used_cred[r] <= std::max<int64_t>(0, credits[r]), "plan exceeds credits");
        tot_off += std::max<int64_t>(0, offers[r]);
        tot_cred += std::max<int64_t>(0, credits[r]);
      }
      require(moved == std::min(tot_off, tot_cred), "plan is not maximal");
    }
  }
  printf("routing scenario: %d random rounds x 3 policies OK\n", iters);
}

static void scenario_engine(int64_t n_per_producer, int policy) {
  const int world = 3, max_offer = 8;
  const int64_t slot_bytes = 192;
  const bool is_p[world] = {true, true, false}, is_c[world] = {false, true, true};
  const std::vector<int> prods = {0, 1};
  const std::string name = "/psray-stress-" + std::to_string((long long)getpid()) + "-" + std::to_string(policy);
  std::vector<std::unique_ptr<SlotPool>> pools;
  std::vector<std::vector<uint8_t>> rings;
  std::vector<std::unique_ptr<pr::ShmControl>> ctrls;
  std::vector<std::unique_ptr<pr::TransportEngine>> engines;
  for (int r = 0; r < world; ++r) {
    pools.emplace_back(new SlotPool(is_p[r] ? 12 : 0, is_c[r] ? 10 : 0, -1));
    rings.emplace_back((size_t)pools[r]->n_slots() * slot_bytes);
  }
  for (int r = 0; r < world; ++r)
    ctrls.emplace_back(new pr::ShmControl(name, r == 0, r, world, pr::TransportEngine::vec_words_for(max_offer),
                                          max_offer * slot_bytes, 60.0));
  for (int r = 0; r < world; ++r)
    engines.emplace_back(new pr::TransportEngine(pools[r].get(), ctrls[r].get(), nullptr,
                                                 (uint64_t)(uintptr_t)rings[r].data(), slot_bytes, r, world, prods,
                                                 is_p[r], is_c[r], policy, max_offer, false, 0, -1));
  for (auto& e : engines) e->start();
  auto payload = [](int64_t rank, int64_t idx, int64_t j) { return (uint8_t)(rank * 131 + idx * 7 + j * 3); };
  std::vector<std::thread> th;
  for (int r = 0; r < world; ++r) {
    if (!is_p[r]) continue;
    th.emplace_back([&, r] {
      for (int64_t k = 0; k < n_per_producer;) {
        const int s = pools[r]->acquire_produce(0.01);
        if (s < 0) continue;
        uint8_t* d = rings[r].data() + (size_t)s * slot_bytes;
        for (int64_t j = 0; j < slot_bytes; ++j) d[j] = payload(r, k, j);
        SlotHeader h;
        h.rank = r;
        h.idx = k;
        h.gevt = 1000 * r + k;
        h.photon_energy = 0.5 * (double)k;
        pools[r]->commit_produce(s, h, 0);
        ++k;
      }
      engines[r]->set_producer_finished();
    });
  }
  std::vector<std::atomic<int>> seen(2 * n_per_producer);
  for (auto& x : seen) x.store(0);
  for (int r = 0; r < world; ++r) {
    if (!is_c[r]) continue;
    th.emplace_back([&, r] {
      int64_t last[2] = {-1, -1};
      for (;;) {
        const int s = pools[r]->get(0.005);
        if (s < 0) {
          const std::string e = engines[r]->error();
          require(e.empty(), "transport engine failed");
          if (engines[r]->done() && pools[r]->n_ready() == 0) return;
          continue;
        }
        const SlotHeader h = pools[r]->header(s);
        require(h.rank >= 0 && h.rank < 2 && h.idx >= 0 && h.idx < n_per_producer, "engine: header out of range");
        require(h.gevt == 1000 * h.rank + h.idx && h.photon_energy == 0.5 * (double)h.idx, "engine: header corrupted");
        require(h.idx > last[h.rank], "engine: per-producer FIFO order violated within a shard");
        last[h.rank] = h.idx;
        const uint8_t* d = rings[r].data() + (size_t)s * slot_bytes;
        for (int64_t j = 0; j < slot_bytes; ++j) {
          if (d[j] != payload(h.rank, h.idx, j))
            fprintf(stderr, "consumer %d: frame (%lld,%lld) byte %lld = %d, want %d (slot %d)\n", r, (long long)h.rank,
                    (long long)h.idx, (long long)j, (int)d[j], (int)payload(h.rank, h.idx, j), s);
          require(d[j] == payload(h.rank, h.idx, j), "engine: payload corrupted");
        }
        seen[h.rank * n_per_producer + h.idx].fetch_add(1);
        pools[r]->release(s, 0);
      }
    });
  }
  for (auto& t : th) t.join();
  for (auto& e : engines) require(e->join(60.0), "engine did not finish");
  for (auto& e : engines) require(e->error().empty(), "engine reported an error");
  for (size_t i = 0; i < seen.size(); ++i) require(seen[i].load() == 1, "engine: event lost or duplicated");
  const pr::XportStats s1 = engines[1]->stats();
  printf("engine scenario (policy %d): %lld events OK (%lld rounds, %lld sent by rank 1)\n", policy, (long long)seen.size(),
         (long long)s1.rounds, (long long)s1.frames_sent);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 20000;
  try {
    scenario_transport(n);
    scenario_auto_route(n);
    scenario_routing(2000);
    for (int policy = 0; policy < 3; ++policy) scenario_engine(std::max<int64_t>(200, n / 8), policy);
  } catch (const std::exception& e) {
    fprintf(stderr, "FAILED with exception: %s\n", e.what());
    return 1;
  }
  printf("SLOTPOOL_STRESS_OK\n");
  return 0;
}
