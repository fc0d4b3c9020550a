"""Reference queue semantics (psana_ray/shared_queue.py:4-38) on the in-process CPU queue."""
import threading

from psana_ray_amd.queue.cpu_queue import Queue, create_queue, drop_queue, get_queue
import pytest


def test_bounded_backpressure_not_drop_oldest():
    q = Queue(maxsize=3)
    assert [q.put(i) for i in range(3)] == [True, True, True]
    assert q.put(99) is False            # Q-4: full -> False, nothing dropped
    assert q.size() == 3
    assert [q.get() for _ in range(3)] == [0, 1, 2]   # FIFO


def test_get_nonblocking_none_when_empty():
    q = Queue(maxsize=2)
    assert q.get() is None
    assert q.size() == 0


def test_get_with_timeout_wakes_on_put():
    q = Queue(maxsize=2)
    out = []
    t = threading.Thread(target=lambda: out.append(q.get(timeout=5.0)))
    t.start()
    q.put("x")
    t.join(5)
    assert out == ["x"]


def test_default_maxsize_is_reference_default():
    assert Queue().maxsize == 100


def test_create_queue_attach_if_exists():
    drop_queue("qa", "ns")
    a = create_queue("qa", "ns", maxsize=5)
    b = create_queue("qa", "ns", maxsize=50)   # Q-5: existing queue reused, maxsize ignored
    assert a is b and b.maxsize == 5
    assert get_queue("qa", "ns") is a
    with pytest.raises(ValueError):
        get_queue("missing", "ns")
    drop_queue("qa", "ns")


def test_concurrent_producers_consumers_exactly_once():
    q = Queue(maxsize=8)
    N, P = 500, 4
    got = []
    lock = threading.Lock()

    def prod(r):
        for i in range(N):
            while not q.put((r, i)):
                pass

    def cons():
        while True:
            x = q.get(timeout=0.5)
            if x is None:
                return
            with lock:
                got.append(x)

    ts = [threading.Thread(target=prod, args=(r,)) for r in range(P)] + [threading.Thread(target=cons) for _ in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    assert sorted(got) == sorted((r, i) for r in range(P) for i in range(N))


def test_wait_not_full_wakes_on_get():
    import threading

    from psana_ray_amd.queue.cpu_queue import Queue

    q = Queue(maxsize=1)
    assert q.put(1) and not q.put(2)
    assert q.wait_not_full(0.01) is False
    t = threading.Timer(0.05, q.get)
    t.start()
    assert q.wait_not_full(5.0) is True
    assert q.put(2)


def test_config1_bench_runs():
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "bench/config1_cpu_queue.py", "--frames", "500", "--queue-size", "16"],
                       cwd=root, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["frames"] == 500 and d["frames_per_s"] > 0
