"""Native SlotPool state machine (host pools: no HIP events) -- the HBM ring's bookkeeping."""
import threading
import time

import pytest


def test_budgets_and_states(native):
    C = native
    p = C.SlotPool(2, 3, -1)
    assert p.n_slots == 5 and p.credits() == 3
    a, b = p.try_acquire_produce(), p.try_acquire_produce()
    assert a >= 0 and b >= 0 and p.try_acquire_produce() == -1   # producer budget
    h = C.SlotHeader(1, 2, 3, 9.5)
    p.commit_produce(a, h, 0)
    assert p.produced(10) == [a] and p.n_produced() == 1
    p.route_local(a)
    assert p.n_ready() == 1 and p.credits() == 2
    s = p.try_get()
    assert s == a and p.header(s).gevt == 3
    p.release(s, 0)
    assert p.credits() == 3
    with pytest.raises(RuntimeError):
        p.release(s, 0)                      # double release is rejected
    p.abort_produce(b)


def test_auto_route_and_batches(native):
    C = native
    p = C.SlotPool(4, 2, -1)
    p.set_auto_route(True)
    slots = [p.try_acquire_produce() for _ in range(4)]
    for i, s in enumerate(slots):
        p.commit_produce(s, C.SlotHeader(0, i, i, 0.0), 0)
    assert p.n_ready() == 2 and p.n_produced() == 2        # consumer budget caps routing
    got = p.get_batch(8, 0.0, 0)
    assert len(got) == 2
    assert [h.idx for h in p.headers(got)] == [0, 1]       # FIFO
    p.release_batch(got, 0)
    assert p.n_ready() == 2                                # pending frames routed on release
    got2 = p.get_batch(8, 0.0, 0)
    assert [h.idx for h in p.headers(got2)] == [2, 3]


def test_blocking_acquire_wakes_on_release(native):
    C = native
    p = C.SlotPool(1, 1, -1)
    p.set_auto_route(True)
    s = p.acquire_produce(1.0)
    p.commit_produce(s, C.SlotHeader(0, 0, 0, 0.0), 0)
    s2 = p.acquire_produce(1.0)
    p.commit_produce(s2, C.SlotHeader(0, 1, 1, 0.0), 0)   # held: consumer full
    t0 = time.time()
    out = []
    th = threading.Thread(target=lambda: out.append(p.acquire_produce(5.0)))
    th.start()
    time.sleep(0.2)
    g = p.try_get()
    p.release(g, 0)                                        # frees consumer credit -> s2 routed -> producer slot
    th.join(5)
    assert out and out[0] >= 0 and time.time() - t0 < 4.0
    assert p.acquire_produce(0.05) == -1                   # timeout path


def test_wake_all_unblocks(native):
    p = native.SlotPool(1, 1, -1)
    out = []
    th = threading.Thread(target=lambda: out.append(p.get(10.0)))
    th.start()
    time.sleep(0.1)
    p.wake_all()
    th.join(5)
    assert out == [-1]


def test_relay_ready_moves_at_most_the_producer_room(native):
    """The keeper's re-offer: READY frames go back on offer in ONE locked step,
    never more than the producer room at that moment, headers kept -- no lease-then-reoffer window
    in which the fabric thread can shrink the room."""
    C = native
    p = C.SlotPool(3, 4, -1)
    slots = [p.try_acquire_produce() for _ in range(3)]
    for i, s in enumerate(slots):
        p.commit_produce(s, C.SlotHeader(0, i, 100 + i, 0.0), 0)
        p.route_local(s)
    assert p.n_ready() == 3 and p.producer_room() == 3
    held = [p.try_acquire_produce(), p.try_acquire_produce()]   # room 1 left
    assert all(h >= 0 for h in held) and p.producer_room() == 1
    assert p.relay_ready(64) == 1
    assert p.n_ready() == 2 and p.n_produced() == 1 and p.producer_room() == 0
    moved = p.produced(10)
    assert [h.gevt for h in p.headers(moved)] == [100]          # FIFO, header kept
    assert p.relay_ready(64) == 0                                # no room: nothing moves
    for h in held:
        p.abort_produce(h)
    assert p.relay_ready(1) == 1 and p.n_ready() == 1            # bounded by max_n
