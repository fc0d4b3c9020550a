"""Queue semantics of the elastic fabric (csrc/fabric.cpp), one process, host rings on the CPU.

Reference: ONE bounded deque in a detached actor (psana_ray/shared_queue.py:4-35) -- put() fails
once queue_size items wait (:11-14), get() pops exactly one item for whoever asks (:19-24), and an
item nobody got stays in the queue.  Checked here:
  * queue_size is ONE logical bound: consumers that join add landing space, not capacity;
  * a consumer's read-ahead is bounded by its prefetch (what a crash can lose);
  * a consumer that closes hands every frame it received but did not take back to a producer, and
    the other consumers get them -- exactly once, nothing dropped;
  * remote_only routing sends every frame to another process;
  * producers route to a queue keeper only when no real consumer has credit."""
import os
import time

import pytest

from tests.test_fabric_links import _member


def _link(tok, prod, pid, cons, cid):
    name = f"{tok}-{pid}-{cid}"
    cons.add_in_link(pid, name)
    prod.add_out_link(cid, name)


def _wait(cond, timeout=30.0, what="condition"):
    t0 = time.time()
    while not cond():
        if time.time() - t0 > timeout:
            raise AssertionError(f"timed out waiting for {what}")
        time.sleep(0.005)


def _produce(C, pool, n, k0=0):
    """Commit up to n frames (idx k0..) as long as the pool has room; returns how many."""
    k = 0
    while k < n:
        s = pool.try_acquire_produce()
        if s < 0:
            break
        pool.commit_produce(s, C.SlotHeader(0, k0 + k, k0 + k, 1.0, 0), 0)
        k += 1
    return k


@pytest.fixture
def tok():
    return f"/psq-sem-{os.getpid()}-{time.monotonic_ns() % 100000}"


def _stop(*fabs):
    for f in fabs:
        f.request_stop()
    for f in fabs:
        f.join(10.0)


def test_queue_size_is_one_global_bound(native, tok):
    C = native
    sb = 128
    pp, _pr, pf = _member(C, tok, 0, 8, 0, sb, 0)
    cons = [_member(C, tok, 1 + i, 0, 16, sb, 0) for i in range(3)]
    for i, (_p, _r, f) in enumerate(cons):
        _link(tok, pf, 0, f, 1 + i)
    fabs = [pf] + [f for _, _, f in cons]
    for f in fabs:
        f.start()
    try:
        produced = 0
        t0 = time.time()
        while time.time() - t0 < 2.0:   # nobody reads: production must stop at queue_size frames
            produced += _produce(C, pp, 100, produced)
            time.sleep(0.01)
        ready = sum(p.n_ready() for p, _, _ in cons)
        assert produced == 8, f"produced {produced} frames into a queue of 8"
        assert ready + pp.n_produced() == 8 and pp.producer_room() == 0
        # one consumer takes 3 frames: exactly 3 more may be produced
        p1 = cons[0][0] if cons[0][0].n_ready() >= 3 else next(p for p, _, _ in cons if p.n_ready() >= 1)
        taken = 0
        while taken < 3:
            for p, _, _ in cons:
                s = p.try_get()
                if s >= 0:
                    p.release(s, 0)
                    taken += 1
                    if taken == 3:
                        break
        _wait(lambda: pp.producer_room() == 3, what="the producer to see the frames taken")
        assert _produce(C, pp, 100, produced) == 3
        assert p1 is not None
    finally:
        _stop(*fabs)


def test_prefetch_bounds_a_consumers_read_ahead(native, tok):
    C = native
    sb = 128
    pp, _pr, pf = _member(C, tok, 0, 64, 0, sb, 0)
    cp, _cr, cf = _member(C, tok, 1, 0, 32, sb, 0)
    cf.set_prefetch(5)
    _link(tok, pf, 0, cf, 1)
    for f in (pf, cf):
        f.start()
    try:
        assert _produce(C, pp, 40) == 40
        _wait(lambda: cp.n_ready() == 5, what="the read-ahead to fill")
        time.sleep(0.3)
        assert cp.n_ready() == 5 and pp.n_produced() == 35, (cp.n_ready(), pp.n_produced())
        got = []
        while len(got) < 40:
            s = cp.try_get()
            if s >= 0:
                got.append(cp.header(s).idx)
                cp.release(s, 0)
                assert cp.n_ready() <= 5
        assert got == list(range(40))
    finally:
        _stop(pf, cf)


def test_closing_consumer_hands_unread_frames_back(native, tok):
    C = native
    sb = 128
    n = 60
    pp, _pr, pf = _member(C, tok, 0, 32, 0, sb, 0)
    ap, _ar, af = _member(C, tok, 1, 0, 16, sb, 0)
    bp, _br, bf = _member(C, tok, 2, 0, 16, sb, 0)
    af.set_prefetch(8)
    bf.set_prefetch(8)
    _link(tok, pf, 0, af, 1)
    for f in (pf, af):
        f.start()
    try:
        k = _produce(C, pp, n)
        _wait(lambda: ap.n_ready() == 8, what="A's read-ahead")
        got_a = []
        for _ in range(3):
            s = ap.try_get()
            got_a.append(ap.header(s).idx)
            ap.release(s, 0)
        _wait(lambda: ap.n_ready() == 8, what="A's read-ahead to refill")
        # A stops reading and leaves with 8 frames delivered and not taken
        af.set_consumer_closed()
        _wait(lambda: af.consumer_quiesced, what="A to quiesce")
        sa = af.stats()
        assert sa.frames_returned == 8 and sa.frames_dropped == 0, (sa.frames_returned, sa.frames_dropped)
        assert ap.n_ready() == 0 and ap.consumer_held() == 0
        # B joins later and gets everything else, A's returned frames first
        _link(tok, pf, 0, bf, 2)
        bf.start()
        got_b = []
        t0 = time.time()
        while len(got_a) + len(got_b) < n and time.time() - t0 < 30:
            k += _produce(C, pp, n - k, k)
            s = bp.try_get()
            if s >= 0:
                got_b.append(bp.header(s).idx)
                bp.release(s, 0)
        assert sorted(got_a + got_b) == list(range(n)), "exactly-once delivery violated"
        assert got_b[:8] == list(range(3, 11)), got_b[:12]
        assert pf.stats().frames_reclaimed == 8
    finally:
        _stop(pf, af, bf)


def test_remote_only_routes_every_frame_across(native, tok):
    C = native
    sb = 128
    pp, _pr, pf = _member(C, tok, 0, 16, 16, sb, 4)       # prosumer, remote_only
    rp, _rr, rf = _member(C, tok, 1, 0, 16, sb, 0)
    pf.export_host_ring(f"{tok}-r0")
    _link(tok, pf, 0, rf, 1)
    for f in (pf, rf):
        f.start()
    try:
        _wait(lambda: any(ls.attached for ls in pf.links() if ls.outgoing), what="the link")
        n, k, got = 50, 0, []
        t0 = time.time()
        while len(got) < n and time.time() - t0 < 30:
            k += _produce(C, pp, n - k, k)
            s = rp.try_get()
            if s >= 0:
                got.append(rp.header(s).idx)
                rp.release(s, 0)
            assert pp.try_get() < 0, "remote_only delivered a frame to the producer's own consumer"
        assert sorted(got) == list(range(n))
        st = pf.stats()
        assert st.frames_local == 0 and st.frames_sent == n
    finally:
        _stop(pf, rf)


def test_keeper_links_are_the_last_resort(native, tok):
    C = native
    sb = 128
    pp, _pr, pf = _member(C, tok, 0, 16, 0, sb, 0)
    cp, _cr, cf = _member(C, tok, 1, 0, 16, sb, 0)
    kp, _kr, kf = _member(C, tok, 2, 0, 16, sb, 0)
    kf.set_keeper(True)
    kf.set_grant_filter(True)
    _link(tok, pf, 0, cf, 1)
    _link(tok, pf, 0, kf, 2)
    for f in (pf, cf, kf):
        f.start()
    try:
        _wait(lambda: sum(ls.attached for ls in pf.links() if ls.outgoing) == 2, what="both links")
        assert any(ls.keeper for ls in pf.links() if ls.outgoing and ls.peer == 2)
        # a reading consumer with credit: the keeper receives nothing
        n, k, got = 40, 0, []
        t0 = time.time()
        while len(got) < n and time.time() - t0 < 30:
            k += _produce(C, pp, n - k, k)
            s = cp.try_get()
            if s >= 0:
                got.append(cp.header(s).idx)
                cp.release(s, 0)
        assert sorted(got) == list(range(n)) and kp.n_ready() == 0
        # the consumer leaves: the keeper now takes the backlog of the LIVE producer
        cf.set_consumer_closed()
        _wait(lambda: cf.consumer_quiesced, what="the consumer to close")
        k += _produce(C, pp, 10, k)
        _wait(lambda: kp.n_ready() == 10, what="the keeper to pull the backlog")
        assert kf.stats().frames_recv == 10
    finally:
        _stop(pf, cf, kf)


def test_balanced_feeds_a_starving_consumer_only_rank(native, tok):
    """BASELINE config 3 shape: a producer with its OWN fast consumer (prosumer) and a consumer-only
    member.  balanced keeps frames local while every consumer has something to read, but a consumer
    with nothing to read at all gets frames (the reference's competing consumers pull from one
    queue, shared_queue.py:19-24) -- before, it starved forever next to a fast local consumer."""
    C = native
    sb = 128
    pp, _pr, pf = _member(C, tok, 0, 32, 32, sb, 0)    # prosumer, balanced
    cp, _cr, cf = _member(C, tok, 1, 0, 32, sb, 0)      # consumer only
    _link(tok, pf, 0, cf, 1)
    for f in (pf, cf):
        f.start()
    try:
        produced = local = remote = 0
        t0 = time.time()
        while time.time() - t0 < 5.0 and remote < 20:
            produced += _produce(C, pp, 8, produced)
            for pool, is_local in ((pp, True), (cp, False)):
                while True:   # both consumers take everything they have, at once (fast readers)
                    s = pool.try_get()
                    if s < 0:
                        break
                    pool.release(s, 0)
                    if is_local:
                        local += 1
                    else:
                        remote += 1
            time.sleep(0.002)
        assert remote >= 20, f"the consumer-only member got {remote} frames (local {local})"
        assert local > 0
    finally:
        _stop(pf, cf)


def test_balanced_shares_between_two_starving_consumer_only_members(native, tok):
    """Two consumer-only members next to a prosumer: every offer goes to the starving member given
    the fewest in the pass, so neither starves (the first-listed member used to take every offer
    while it had grants)."""
    C = native
    sb = 128
    pp, _pr, pf = _member(C, tok, 0, 32, 32, sb, 0)    # prosumer, balanced
    ap, _ar, af = _member(C, tok, 1, 0, 32, sb, 0)      # consumer only
    bp, _br, bf = _member(C, tok, 2, 0, 32, sb, 0)      # consumer only
    _link(tok, pf, 0, af, 1)
    _link(tok, pf, 0, bf, 2)
    for f in (pf, af, bf):
        f.start()
    try:
        produced = 0
        got = {"local": 0, "a": 0, "b": 0}
        t0 = time.time()
        while time.time() - t0 < 5.0 and min(got["a"], got["b"]) < 20:
            produced += _produce(C, pp, 8, produced)
            for pool, key in ((pp, "local"), (ap, "a"), (bp, "b")):
                while True:
                    s = pool.try_get()
                    if s < 0:
                        break
                    pool.release(s, 0)
                    got[key] += 1
            time.sleep(0.002)
        assert got["a"] >= 20 and got["b"] >= 20, got
    finally:
        _stop(pf, af, bf)
