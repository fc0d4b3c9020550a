"""Deterministic per-round frame routing (producer offers x consumer credits -> assignments).

The reference shares ONE queue between all producers and all competing consumers
(psana_ray/shared_queue.py:19-24, P-02): whichever consumer calls ``get`` first wins, and a full
queue makes ``put`` return False (backpressure, :11-14).  In the sharded HBM design each consumer
GPU owns a ring shard; every transport round all ranks all-gather (offers, credits) and run THIS
function on identical inputs, so every rank derives the same plan without further messages and
the RCCL sends/recvs match by construction.

Policies:
  balanced     water-filling: each frame goes to the consumer with the most free slots (ties:
               the producer's own GPU, then the next ranks cyclically), where the producer's own
               shard counts LOCAL_SLACK extra slots: a frame leaves its GPU only when another
               shard is more than two chunks emptier.  Fast consumers accumulate more credits and
               therefore receive more frames -- the competing-consumer load balancing of the
               reference, without a central actor -- while near-balanced ranks (the weak-scaling
               steady state) keep their frames local instead of trading them over xGMI.
  local_first  a producer's frames stay on its own GPU while that shard has credit (zero-copy),
               the overflow is water-filled to the others.
  spread       strict round robin over consumers with credit (maximises xGMI link use).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

POLICIES = ("balanced", "local_first", "spread")

Assignment = Tuple[int, int, int]  # (producer rank, offer index, consumer rank)

# balanced policy: credit bonus of the producer's own consumer shard (two producer chunks); the
# native plan (csrc/routing.cpp) uses the same constant
LOCAL_SLACK = 64


def plan_round(offers: Sequence[int], credits: Sequence[int], round_id: int, policy: str = "balanced") -> List[Assignment]:
    if policy not in POLICIES:
        raise ValueError(f"unknown routing policy {policy!r}; choose from {POLICIES}")
    world = len(offers)
    assert len(credits) == world
    cred = [max(0, int(c)) for c in credits]
    nxt = [0] * world                       # next offer index per producer
    left = [max(0, int(o)) for o in offers]
    plan: List[Assignment] = []
    order = [(round_id + k) % world for k in range(world)]  # fairness: rotate who goes first

    if policy == "local_first":
        for p in order:
            take = min(left[p], cred[p])
            for _ in range(take):
                plan.append((p, nxt[p], p))
                nxt[p] += 1
            left[p] -= take
            cred[p] -= take

    if policy == "spread":
        cursor = [(p + round_id) % world for p in range(world)]
        active = True
        while active:
            active = False
            for p in order:
                if left[p] == 0 or sum(cred) == 0:
                    continue
                for k in range(world):
                    c = (cursor[p] + k) % world
                    if cred[c] > 0:
                        plan.append((p, nxt[p], c))
                        nxt[p] += 1
                        left[p] -= 1
                        cred[c] -= 1
                        cursor[p] = (c + 1) % world
                        active = True
                        break
        return plan

    # balanced water-filling (also the overflow stage of local_first)
    while True:
        progressed = False
        for p in order:
            if left[p] == 0:
                continue
            best, best_key = -1, None
            for k in range(world):
                c = (p + k) % world
                if cred[c] <= 0:
                    continue
                bonus = LOCAL_SLACK if (k == 0 and policy == "balanced") else 0
                key = (-(cred[c] + bonus), k)   # most credit first, then own GPU (k=0), then cyclic
                if best_key is None or key < best_key:
                    best, best_key = c, key
            if best < 0:
                return plan
            plan.append((p, nxt[p], best))
            nxt[p] += 1
            left[p] -= 1
            cred[best] -= 1
            progressed = True
        if not progressed:
            return plan
