"""Randomised membership churn over the queue fabric (one process, host rings, real native threads):
producers with random budgets, consumers with random rings / read-ahead that join late, leave
gracefully (hand-back) or die (their fabric stops dead, the others drop them), and one survivor
that drains the stream.  Checked for every seed: no frame is delivered twice, and the only frames
missing are ones a DEAD consumer had received and not taken (bounded by its read-ahead) -- a
graceful leave loses nothing (reference: one deque in a detached actor, psana_ray/shared_queue.py)."""
import os
import random
import threading
import time

import pytest

from tests.test_fabric_links import _member


def _run(C, seed):
    rng = random.Random(seed)
    sb = 64
    tok = f"/psq-fz-{os.getpid()}-{seed}"
    n_prod = rng.randint(1, 3)
    n_cons = rng.randint(2, 4)
    per_prod = rng.randint(60, 160)
    mids = iter(range(100))
    prods, cons = [], []
    for _ in range(n_prod):
        m = next(mids)
        pool, ring, fab = _member(C, tok, m, rng.randint(4, 16), 0, sb, rng.choice([0, 1, 2]))
        prods.append(dict(mid=m, pool=pool, ring=ring, fab=fab, k=0))
    specs = []
    for i in range(n_cons):
        fate = "survive" if i == 0 else rng.choice(["close", "die", "close"])
        specs.append(dict(fate=fate, join_at=0 if i == 0 else rng.randint(0, per_prod // 2),
                          stop_at=rng.randint(5, 40), cb=rng.randint(4, 24), prefetch=rng.choice([0, 2, 5, 9])))
    seen = {}
    lock = threading.Lock()
    lost_budget = [0]

    def link(p, c):
        name = f"{tok}-{p['mid']}-{c['mid']}"
        c["fab"].add_in_link(p["mid"], name)
        p["fab"].add_out_link(c["mid"], name)

    def join(spec):
        m = next(mids)
        pool, ring, fab = _member(C, tok, m, 0, spec["cb"], sb, 0)
        fab.set_prefetch(spec["prefetch"])
        c = dict(mid=m, pool=pool, ring=ring, fab=fab, spec=spec, got=0, done=False)
        for p in prods:
            link(p, c)
        fab.start()
        cons.append(c)
        return c

    def reader(c):
        spec = c["spec"]
        pool = c["pool"]
        while True:
            if spec["fate"] != "survive" and c["got"] >= spec["stop_at"]:
                break
            s = pool.try_get()
            if s >= 0:
                h = pool.header(s)
                with lock:
                    seen[(h.rank, h.idx)] = seen.get((h.rank, h.idx), 0) + 1
                pool.release(s, 0)
                c["got"] += 1
                continue
            if all(p["fab"].producer_drained for p in prods):   # the stream ended for everybody
                links = [ls for ls in c["fab"].links() if not ls.outgoing]
                if pool.n_ready() == 0 and all(ls.eos or ls.dead or ls.detached for ls in links if ls.attached):
                    break
            time.sleep(0.0005)
        fab = c["fab"]
        if spec["fate"] == "close":
            fab.set_consumer_closed()
            t0 = time.time()
            while not fab.consumer_quiesced and time.time() - t0 < 30:
                time.sleep(0.001)
            assert fab.consumer_quiesced, f"seed {seed}: a closing consumer never quiesced"
            st = fab.stats()
            assert st.frames_dropped == 0 or all(p["fab"].producer_drained for p in prods), \
                f"seed {seed}: frames dropped while producers could take them back"
            with lock:
                lost_budget[0] += st.frames_dropped
        elif spec["fate"] == "die":
            # the process "dies": its fabric stops on the spot; what it had received is gone
            with lock:
                lost_budget[0] += pool.n_ready() + spec["cb"]
            fab.request_stop()
            fab.join(10.0)
            for p in prods:
                p["fab"].drop_peer(c["mid"])
        c["done"] = True

    for p in prods:
        p["fab"].start()
    threads = []
    pending = sorted(specs, key=lambda s: s["join_at"])
    while pending and pending[0]["join_at"] == 0:
        c = join(pending.pop(0))
        threads.append(threading.Thread(target=reader, args=(c,)))
        threads[-1].start()
    t_end = time.time() + 120
    while any(p["k"] < per_prod for p in prods) and time.time() < t_end:
        for r, p in enumerate(prods):
            if p["k"] < per_prod:
                s = p["pool"].try_acquire_produce()
                if s >= 0:
                    p["pool"].commit_produce(s, C.SlotHeader(r, p["k"], p["k"], 1.0, 0), 0)
                    p["k"] += 1
                    if p["k"] == per_prod:
                        p["fab"].set_producer_finished()
        done = min(p["k"] for p in prods)
        while pending and pending[0]["join_at"] <= done:
            c = join(pending.pop(0))
            threads.append(threading.Thread(target=reader, args=(c,)))
            threads[-1].start()
        time.sleep(0.0002)
    for spec in pending:   # stream already produced: join late anyway
        c = join(spec)
        threads.append(threading.Thread(target=reader, args=(c,)))
        threads[-1].start()
    for th in threads:
        th.join(60)
    try:
        assert all(p["k"] == per_prod for p in prods), f"seed {seed}: producers blocked"
        assert not any(th.is_alive() for th in threads), f"seed {seed}: a reader hung"
        for m in prods + cons:
            assert not m["fab"].error(), (seed, m["fab"].error())
        dup = {k: v for k, v in seen.items() if v > 1}
        assert not dup, f"seed {seed}: delivered twice: {sorted(dup)[:8]}"
        expect = {(r, k) for r in range(n_prod) for k in range(per_prod)}
        lost = expect - set(seen)
        assert len(lost) <= lost_budget[0], \
            f"seed {seed}: lost {len(lost)} frames, more than the dead consumers held ({lost_budget[0]})"
        if not any(s["fate"] == "die" for s in specs):
            assert not lost, f"seed {seed}: lost {sorted(lost)[:8]} with graceful leaves only"
    finally:
        for m in prods + cons:
            m["fab"].request_stop()
        for m in prods + cons:
            m["fab"].join(10.0)


@pytest.mark.parametrize("seed", list(range(12)))
def test_fabric_membership_churn(native, seed):
    _run(native, seed)
