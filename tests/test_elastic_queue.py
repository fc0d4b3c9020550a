"""Elastic, fault-isolated shared queue (reference: one named detached Ray actor,
psana_ray/shared_queue.py:19-35, producer.py:43-48,98-130, README.md:23-35).

Separate OS processes on the CPU -- the producer CLI and DataReader consumers -- meeting at a
rendezvous store; frames move through the native fabric's shared-memory links:
  (a) a producer runs with NO consumer, buffers its frames, a consumer started 10 s later drains
      all of them plus EOS, and the producer exits 0 (drain before exit);
  (b) a consumer that joins mid-stream receives frames; delivery stays exactly-once;
  (c) kill -9 of one of two consumers mid-stream (default ring and read-ahead): the survivor gets
      every frame not already in the dead consumer's read-ahead (<= its prefetch), plus EOS, and
      the producer exits 0; a consumer that LEAVES normally hands its read-ahead back (no loss);
  (d) a second producer job attaches to the live queue; one consumer receives both jobs' frames
      exactly once;
  plus: a producer that nobody drains fails after --timeout with a clear message (rc 1).
Every frame is checked bit-exactly against the fp32 golden calibration."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT + (os.pathsep + os.environ["PYTHONPATH"] if os.environ.get("PYTHONPATH") else ""))
ENV.pop("LOCAL_RANK", None)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def store_port():
    port = _port()
    p = subprocess.Popen([sys.executable, "-m", "psana_ray_amd.server", "--host", "127.0.0.1", "--port", str(port),
                          "--log_level", "WARNING"], env=ENV, cwd=ROOT)
    t0 = time.time()
    while time.time() - t0 < 30:
        with socket.socket() as s:
            if s.connect_ex(("127.0.0.1", port)) == 0:
                break
        time.sleep(0.1)
    yield port
    p.terminate()
    try:
        p.wait(10)
    except subprocess.TimeoutExpired:
        p.kill()


def producer(port, n_events, *extra, queue_size=16, chunk=4, timeout=60, detector="tiny_epix", mode="calib", env=None):
    cmd = [sys.executable, "-m", "psana_ray_amd.producer", "--exp", "synthetic", "--run", "2", "--detector_name",
           detector, *(("--calib",) if mode == "calib" else ()), "--device", "cpu", "--ray_address", f"127.0.0.1:{port}",
           "--num_events",
           str(n_events), "--queue_size", str(queue_size), "--chunk", str(chunk), "--timeout", str(timeout),
           "--metrics_interval", "0", "--log_level", "INFO", *extra]
    return subprocess.Popen(cmd, env={**ENV, **(env or {})}, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                            text=True)


def consumer(port, out, *extra):
    cmd = [sys.executable, os.path.join(ROOT, "tests", "_elastic_consumer.py"), "--address", f"127.0.0.1:{port}",
           "--out", str(out), *extra]
    return subprocess.Popen(cmd, env=ENV, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def records(path):
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]


def frames(recs):
    fr = [r for r in recs if "gevt" in r]
    assert all(r["ok"] for r in fr), "frame content differs from the golden calibration"
    return [r["gevt"] for r in fr]


def finish(p, timeout=180):
    try:
        out, _ = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        p.kill()
        out, _ = p.communicate()
        raise AssertionError(f"process did not finish:\n{out[-3000:]}")
    return p.returncode, out


def test_producer_first_consumer_ten_seconds_later(store_port, tmp_path):
    prod = producer(store_port, 24, queue_size=32)
    time.sleep(10.0)
    assert prod.poll() is None, "the producer must wait for a consumer to drain its frames"
    c = consumer(store_port, tmp_path / "c.jsonl")
    rc_c, out_c = finish(c)
    rc_p, out_p = finish(prod)
    assert rc_c == 0, out_c
    assert rc_p == 0, out_p
    recs = records(tmp_path / "c.jsonl")
    assert sorted(frames(recs)) == list(range(24))
    assert recs[-1].get("eos") is True


def test_odd_sized_image_frames_cross_processes(store_port, tmp_path):
    """Image frames of 612 B (tiny_odd: 9 x 17 pixels, not a multiple of 16 B) through host rings."""
    prod = producer(store_port, 20, detector="tiny_odd", mode="image")
    c = consumer(store_port, tmp_path / "c.jsonl", "--mode", "image", "--verify", "synthetic:2:tiny_odd:1")
    rc_c, out_c = finish(c)
    rc_p, out_p = finish(prod)
    assert rc_c == 0, out_c
    assert rc_p == 0, out_p
    recs = records(tmp_path / "c.jsonl")
    assert sorted(frames(recs)) == list(range(20))
    assert recs[-1].get("eos") is True


def test_consumer_joins_mid_stream(store_port, tmp_path):
    n = 300
    prod = producer(store_port, n)
    c1 = consumer(store_port, tmp_path / "c1.jsonl", "--sleep", "0.04", "--slots", "4")
    c2 = consumer(store_port, tmp_path / "c2.jsonl", "--sleep", "0.04", "--slots", "4")
    t0 = time.time()
    while len(frames(records(tmp_path / "c1.jsonl"))) < 10 and time.time() - t0 < 30:
        time.sleep(0.05)
    c3 = consumer(store_port, tmp_path / "c3.jsonl", "--sleep", "0.04", "--slots", "4")
    for c in (c1, c2, c3):
        rc, out = finish(c)
        assert rc == 0, out
    rc_p, out_p = finish(prod)
    assert rc_p == 0, out_p
    got = [frames(records(tmp_path / f"c{i}.jsonl")) for i in (1, 2, 3)]
    assert len(got[2]) > 0, "the late consumer received nothing"
    allg = got[0] + got[1] + got[2]
    assert sorted(allg) == list(range(n)), "exactly-once delivery violated"
    for i in (1, 2, 3):
        assert records(tmp_path / f"c{i}.jsonl")[-1].get("eos") is True


def test_kill9_consumer_survivor_gets_the_rest(store_port, tmp_path):
    """Default ring and read-ahead (no --slots): a killed consumer loses at most its prefetch --
    the frames delivered to it and not read -- not a shard (reference: get() pops one item,
    psana_ray/shared_queue.py:19-24, examples/psana_consumer.py:41-47)."""
    from psana_ray_amd.config import DEFAULT_PREFETCH

    n = 240
    prod = producer(store_port, n, queue_size=100)
    a = consumer(store_port, tmp_path / "a.jsonl", "--sleep", "0.01", "--die_after", "12")
    b = consumer(store_port, tmp_path / "b.jsonl", "--sleep", "0.01")
    rc_a, _ = finish(a)
    assert rc_a == -9
    rc_b, out_b = finish(b)
    rc_p, out_p = finish(prod)
    assert rc_b == 0, out_b
    assert rc_p == 0, out_p
    ga, gb = frames(records(tmp_path / "a.jsonl")), frames(records(tmp_path / "b.jsonl"))
    assert len(ga) == 12
    assert not set(ga) & set(gb), "a frame was delivered twice"
    lost = set(range(n)) - set(ga) - set(gb)
    assert len(lost) <= DEFAULT_PREFETCH, f"lost {len(lost)} frames, more than the dead consumer's prefetch"
    assert records(tmp_path / "b.jsonl")[-1].get("eos") is True
    assert "died" in out_p, out_p[-2000:]


def test_consumer_that_leaves_hands_its_read_ahead_back(store_port, tmp_path):
    """A consumer that stops after 10 frames and closes: the frames delivered into its ring and not
    read go back to the producer, the other consumer receives them -- nothing lost, exactly once."""
    n = 200
    prod = producer(store_port, n, queue_size=64)
    a = consumer(store_port, tmp_path / "a.jsonl", "--sleep", "0.02", "--stop_after", "10")
    b = consumer(store_port, tmp_path / "b.jsonl", "--sleep", "0.02")
    rc_a, out_a = finish(a)
    rc_b, out_b = finish(b)
    rc_p, out_p = finish(prod)
    assert (rc_a, rc_b, rc_p) == (0, 0, 0), (out_a[-2000:], out_b[-2000:], out_p[-2000:])
    ra = records(tmp_path / "a.jsonl")
    ga, gb = frames(ra), frames(records(tmp_path / "b.jsonl"))
    assert len(ga) == 10
    assert sorted(ga + gb) == list(range(n)), "a frame was lost or delivered twice"
    closed = ra[-1]
    assert closed.get("closed") and closed["frames_dropped"] == 0 and closed["frames_returned"] > 0, closed


def test_second_producer_job_attaches(store_port, tmp_path):
    c = consumer(store_port, tmp_path / "c.jsonl", "--sleep", "0.01", "--slots", "4")
    p1 = producer(store_port, 80)
    time.sleep(1.0)
    p2 = producer(store_port, 1080, "--start_event", "1000")
    rc_c, out_c = finish(c)
    rc1, out1 = finish(p1)
    rc2, out2 = finish(p2)
    assert (rc1, rc2, rc_c) == (0, 0, 0), (out1[-2000:], out2[-2000:], out_c[-2000:])
    got = frames(records(tmp_path / "c.jsonl"))
    assert sorted(got) == list(range(80)) + list(range(1000, 1080))


def test_undrained_producer_times_out_with_a_clear_message(store_port):
    p = producer(store_port, 8, timeout=3)
    rc, out = finish(p)
    assert rc == 1
    assert "were not taken by any consumer within --timeout" in out


def test_competing_consumers_share_by_speed(store_port, tmp_path):
    """P-02 (reference: consumers compete for one actor's items, so a faster consumer takes more):
    at the DEFAULT ring and read-ahead, a consumer holds at most its prefetch (and the producer's
    queue_size bounds what waits anywhere), so the fast one takes clearly more, both finish within
    one read-ahead window of each other, and every frame arrives exactly once."""
    n = 200
    fast = consumer(store_port, tmp_path / "fast.jsonl", "--sleep", "0.002")
    slow = consumer(store_port, tmp_path / "slow.jsonl", "--sleep", "0.05")
    time.sleep(1.0)   # both attached before the stream starts
    prod = producer(store_port, n)
    for c in (fast, slow):
        rc, out = finish(c)
        assert rc == 0, out
    rc_p, out_p = finish(prod)
    assert rc_p == 0, out_p
    gf, gs = frames(records(tmp_path / "fast.jsonl")), frames(records(tmp_path / "slow.jsonl"))
    assert sorted(gf + gs) == list(range(n)), "exactly-once delivery violated"
    assert len(gs) > 0, "the slow consumer should still receive frames"
    assert len(gf) > 2 * len(gs), (len(gf), len(gs))
    # the slow one cannot have hoarded: it ends at most one read-ahead (its unread frames, <= the
    # producer's queue_size of 16 here) after the fast one
    t_fast = records(tmp_path / "fast.jsonl")[-1]["t_end"]
    t_slow = records(tmp_path / "slow.jsonl")[-1]["t_end"]
    assert t_slow - t_fast <= 16 * 0.05 + 2.0, (t_slow - t_fast)


def keeper(port, *extra):
    cmd = [sys.executable, "-m", "psana_ray_amd.keeper", "--ray_address", f"127.0.0.1:{port}", "--slots", "64",
           "--timeout", "60", "--log_level", "INFO", *extra]
    return subprocess.Popen(cmd, env=ENV, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def test_keeper_holds_frames_after_the_producer_exits(store_port, tmp_path):
    """R-11 (the reference's queue is a DETACHED actor, shared_queue.py:35): with a keeper in the
    session the producer drains into it and exits 0 without any consumer; a consumer started
    afterwards receives every frame exactly once, bit-exact, plus EOS; the keeper then leaves."""
    prod = producer(store_port, 40, queue_size=48)   # the queue holds the run (reference: maxsize)
    time.sleep(1.0)
    kp = keeper(store_port)
    rc_p, out_p = finish(prod, timeout=60)
    assert rc_p == 0, out_p
    assert kp.poll() is None, "the keeper must stay while it holds frames"
    time.sleep(2.0)
    c = consumer(store_port, tmp_path / "c.jsonl")
    rc_c, out_c = finish(c)
    rc_k, out_k = finish(kp)
    assert rc_c == 0, out_c
    assert rc_k == 0, out_k
    recs = records(tmp_path / "c.jsonl")
    assert sorted(frames(recs)) == list(range(40))
    assert recs[-1].get("eos") is True
    assert "keeper done: kept=40" in out_k, out_k[-2000:]


def test_keeper_with_a_live_consumer_stays_out_of_the_way(store_port, tmp_path):
    """Keeper and consumer both present from the start: the consumer receives every frame exactly
    once (frames the keeper took after the producer finished are relayed on), and both exit 0."""
    c = consumer(store_port, tmp_path / "c.jsonl")
    prod = producer(store_port, 64, queue_size=16)
    time.sleep(1.0)
    kp = keeper(store_port)
    rc_p, out_p = finish(prod)
    rc_c, out_c = finish(c)
    rc_k, out_k = finish(kp)
    assert (rc_p, rc_c, rc_k) == (0, 0, 0), (out_p[-1500:], out_c[-1500:], out_k[-1500:])
    recs = records(tmp_path / "c.jsonl")
    assert sorted(frames(recs)) == list(range(64))
    assert recs[-1].get("eos") is True


def hang_producer(port, n, *extra):
    cmd = [sys.executable, os.path.join(ROOT, "tests", "_hang_producer.py"), "--address", f"127.0.0.1:{port}",
           "--n", str(n), *extra]
    return subprocess.Popen(cmd, env=ENV, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def wait_line(p, prefix, timeout=60):
    t0 = time.time()
    while time.time() - t0 < timeout:
        line = p.stdout.readline()
        if line.startswith(prefix):
            return line
        if not line and p.poll() is not None:
            break
    raise AssertionError(f"no {prefix!r} line from the process")


def test_keeper_keeps_committed_frames_across_a_producer_crash(store_port, tmp_path):
    """R-11: a LIVE producer's committed frames move into the keeper while no consumer can take
    them, so a kill -9 of the producer loses none of them (<= one chunk in flight is allowed); a
    consumer started afterwards receives them, bit-exact, exactly once."""
    kp = keeper(store_port)
    time.sleep(1.0)
    n, chunk = 40, 4
    hp = hang_producer(store_port, n, "--chunk", str(chunk), "--queue_size", "16")
    wait_line(hp, "COMMITTED")
    time.sleep(1.5)
    hp.kill()
    hp.wait(10)
    c = consumer(store_port, tmp_path / "c.jsonl")
    rc_c, out_c = finish(c)
    rc_k, out_k = finish(kp)
    assert rc_c == 0, out_c[-2000:]
    assert rc_k == 0, out_k[-2000:]
    got = frames(records(tmp_path / "c.jsonl"))
    assert len(got) == len(set(got)) and set(got) <= set(range(n)), got
    assert len(got) >= n - chunk, f"only {len(got)} of {n} committed frames survived the producer"


def test_keeper_holds_more_than_its_receive_slots(store_port, tmp_path):
    """a producer draining MORE frames than the keeper's --slots into a keeper with
    no consumer -- every frame reaches a late consumer (the keeper leases only what it can re-offer;
    the frames in its receive ring still count against the producer's queue_size until taken, so
    the queue holds queue_size + keeper slots = 40 here)."""
    prod = producer(store_port, 40, queue_size=16)
    time.sleep(1.0)
    kp = keeper(store_port, "--slots", "24")
    rc_p, out_p = finish(prod, timeout=60)
    assert rc_p == 0, out_p[-2000:]
    c = consumer(store_port, tmp_path / "c.jsonl")
    rc_c, out_c = finish(c)
    rc_k, out_k = finish(kp)
    assert (rc_c, rc_k) == (0, 0), (out_c[-2000:], out_k[-2000:])
    recs = records(tmp_path / "c.jsonl")
    assert sorted(frames(recs)) == list(range(40))
    assert recs[-1].get("eos") is True
