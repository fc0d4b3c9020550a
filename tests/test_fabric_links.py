"""Queue fabric (csrc/fabric.cpp) link-level behaviour, one process, host rings on the CPU:
a consumer whose ring cannot be mapped costs only its own link (the reference's isolation: one
bad consumer never stops a producer, psana_ray/producer.py:112-114), and the frames go to the
consumers that can be reached, exactly once."""
import os
import time

import pytest


def _member(C, tok, r, pb, cb, slot_bytes, policy, ring_name=None):
    pool = C.SlotPool(pb, cb, -1)
    ring = C.ShmRegion(f"{tok}-r{r}", pool.n_slots * slot_bytes, True, 5.0)
    pool.set_slot_ptrs([ring.ptr + k * slot_bytes for k in range(pool.n_slots)])
    fab = C.QueueFabric(pool, slot_bytes, -1, pb > 0, cb > 0, policy, r)
    if cb > 0:
        fab.export_host_ring(ring_name or ring.name)
    return pool, ring, fab


def test_unmappable_consumer_ring_drops_only_its_link(native):
    C = native
    slot_bytes, n = 256, 60
    tok = f"/psq-linktest-{os.getpid()}"
    pp, pr_, pf = _member(C, tok, 0, 8, 0, slot_bytes, 2)                       # producer, spread
    gp, gr, gf = _member(C, tok, 1, 0, 8, slot_bytes, 0)                        # good consumer
    bp, br, bf = _member(C, tok, 2, 0, 8, slot_bytes, 0, ring_name=f"{tok}-no-such-ring")   # bad ring
    for c, fab in ((1, gf), (2, bf)):
        name = f"{tok}-0-{c}"
        fab.add_in_link(0, name)
        pf.add_out_link(c, name)
    for f in (pf, gf, bf):
        f.start()
    try:
        got = []
        k = 0
        t0 = time.time()
        while len(got) < n and time.time() - t0 < 60:
            if k < n:
                s = pp.try_acquire_produce()
                if s >= 0:
                    pp.commit_produce(s, C.SlotHeader(0, k, k, 1.0, 0), 0)
                    k += 1
            s = gp.try_get()
            if s >= 0:
                got.append(gp.header(s).idx)
                gp.release(s, 0)
            assert not pf.error() and not gf.error(), (pf.error(), gf.error())
        assert sorted(got) == list(range(n)), "the reachable consumer must receive every frame exactly once"
        st = pf.stats()
        assert st.links_failed == 1
        assert "no-such-ring" in pf.last_link_error()
        dead = [ls for ls in pf.links() if ls.outgoing and ls.peer == 2]
        assert dead and dead[0].dead and not dead[0].attached
    finally:
        for f in (pf, gf, bf):
            f.request_stop()
        for f in (pf, gf, bf):
            f.join(10.0)
