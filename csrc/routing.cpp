// Deterministic per-round routing of producer offers onto consumer credits (native; mirrors
// psana_ray_amd/parallel/routing.py, which remains the documented reference implementation and
// the oracle of tests/test_routing.py).
//
// Every rank runs this on identical all-gathered inputs, so all ranks derive the same plan and the
// RCCL sends / receives match without extra messages.  Policies: 0 balanced (water-filling by
// free slots, the producer's own shard counting kLocalSlack extra; ties -> own GPU then cyclic),
// 1 local_first (own GPU first, overflow water-filled), 2 spread (strict round robin over
// consumers with credit).
#include <stdint.h>

#include <vector>

#include "common.h"

namespace pr {

// balanced: credit bonus of the producer's own consumer shard (routing.py LOCAL_SLACK)
static constexpr int64_t kLocalSlack = 64;

std::vector<int32_t> plan_round_native(const std::vector<int64_t>& offers_in, const std::vector<int64_t>& credits_in,
                                       int64_t round_id, int policy) {
  const int world = (int)offers_in.size();
  check(world == (int)credits_in.size(), "plan_round: offers/credits size mismatch");
  check(policy >= 0 && policy <= 2, "plan_round: unknown policy");
  std::vector<int64_t> cred(world), left(world), nxt(world, 0);
  int64_t total_cred = 0;
  for (int r = 0; r < world; ++r) {
    cred[r] = credits_in[r] > 0 ? credits_in[r] : 0;
    left[r] = offers_in[r] > 0 ? offers_in[r] : 0;
    total_cred += cred[r];
  }
  std::vector<int> order(world);
  for (int k = 0; k < world; ++k) order[k] = (int)((round_id + k) % world);
  std::vector<int32_t> plan;   // flattened (producer, offer index, consumer)
  auto emit = [&](int p, int c) {
    plan.push_back(p);
    plan.push_back((int32_t)nxt[p]);
    plan.push_back(c);
    ++nxt[p];
    --left[p];
    --cred[c];
    --total_cred;
  };
  if (policy == 1) {
    for (int p : order) {
      const int64_t take = left[p] < cred[p] ? left[p] : cred[p];
      for (int64_t t = 0; t < take; ++t) emit(p, p);
    }
  }
  if (policy == 2) {
    std::vector<int> cursor(world);
    for (int p = 0; p < world; ++p) cursor[p] = (int)((p + round_id) % world);
    bool active = true;
    while (active) {
      active = false;
      for (int p : order) {
        if (left[p] == 0 || total_cred == 0) continue;
        for (int k = 0; k < world; ++k) {
          const int c = (cursor[p] + k) % world;
          if (cred[c] > 0) {
            emit(p, c);
            cursor[p] = (c + 1) % world;
            active = true;
            break;
          }
        }
      }
    }
    return plan;
  }
  // balanced water-filling (and local_first's overflow)
  while (true) {
    bool progressed = false;
    for (int p : order) {
      if (left[p] == 0) continue;
      int best = -1, best_k = 0;
      int64_t best_cred = 0;
      for (int k = 0; k < world; ++k) {
        const int c = (p + k) % world;
        if (cred[c] <= 0) continue;
        const int64_t eff = cred[c] + ((k == 0 && policy == 0) ? kLocalSlack : 0);
        if (best < 0 || eff > best_cred) {   // most credit first; ties: smallest k (own GPU first)
          best = c;
          best_cred = eff;
          best_k = k;
        }
      }
      (void)best_k;
      if (best < 0) return plan;
      emit(p, best);
      progressed = true;
    }
    if (!progressed) return plan;
  }
}

}  // namespace pr
