"""Elastic shared queue between separate GPU processes on ONE MI355X: the producer CLI on cuda:0
writes frames into DataReader consumers' HBM rings through HIP IPC peer copies (the same path that
crosses xGMI when the processes sit on different GPUs).  Frames are checked bit-exactly against
the fp32 golden calibration; the scenarios are the CPU ones of test_elastic_queue.py."""
import os
import time

import pytest

from tests.test_elastic_queue import consumer, finish, frames, records, store_port  # noqa: F401

pytestmark = pytest.mark.gpu


def gpu_producer(port, n_events, *extra, queue_size=16, chunk=4, timeout=60, env=None):
    from tests.test_elastic_queue import producer

    p = producer(port, n_events, "--device", "cuda:0", *extra, queue_size=queue_size, chunk=chunk, timeout=timeout,
                 env=env)
    return p


def test_gpu_producer_first_consumer_later(store_port, tmp_path):  # noqa: F811
    prod = gpu_producer(store_port, 24, queue_size=32)
    time.sleep(3.0)
    assert prod.poll() is None
    c = consumer(store_port, tmp_path / "c.jsonl", "--device", "cuda:0", "--gen_device", "cuda")
    rc_c, out_c = finish(c, 120)
    rc_p, out_p = finish(prod, 120)
    assert rc_c == 0, out_c[-3000:]
    assert rc_p == 0, out_p[-3000:]
    recs = records(tmp_path / "c.jsonl")
    assert sorted(frames(recs)) == list(range(24))
    assert recs[-1].get("eos") is True


GPU_C = ("--device", "cuda:0", "--gen_device", "cuda")


def test_gpu_kill9_consumer_survivor_gets_the_rest(store_port, tmp_path):  # noqa: F811
    """Default ring and read-ahead: the killed consumer loses at most its prefetch."""
    from psana_ray_amd.config import DEFAULT_PREFETCH

    n = 240
    prod = gpu_producer(store_port, n, queue_size=100)
    a = consumer(store_port, tmp_path / "a.jsonl", *GPU_C, "--sleep", "0.01", "--die_after", "16")
    b = consumer(store_port, tmp_path / "b.jsonl", *GPU_C, "--sleep", "0.01")
    rc_a, _ = finish(a, 120)
    assert rc_a == -9
    rc_b, out_b = finish(b, 120)
    rc_p, out_p = finish(prod, 120)
    assert rc_b == 0, out_b[-3000:]
    assert rc_p == 0, out_p[-3000:]
    ga, gb = frames(records(tmp_path / "a.jsonl")), frames(records(tmp_path / "b.jsonl"))
    assert len(ga) == 16
    assert not set(ga) & set(gb)
    lost = set(range(n)) - set(ga) - set(gb)
    assert len(lost) <= DEFAULT_PREFETCH, lost
    assert records(tmp_path / "b.jsonl")[-1].get("eos") is True


def test_gpu_consumer_that_leaves_hands_its_read_ahead_back(store_port, tmp_path):  # noqa: F811
    """HBM read-ahead handed back on close: the producer copies the unread frames out of the
    leaving consumer's ring (IPC) and the other consumer receives them, bit-exact, exactly once."""
    n = 200
    prod = gpu_producer(store_port, n, queue_size=64)
    a = consumer(store_port, tmp_path / "a.jsonl", *GPU_C, "--sleep", "0.02", "--stop_after", "10")
    b = consumer(store_port, tmp_path / "b.jsonl", *GPU_C, "--sleep", "0.02")
    rc_a, out_a = finish(a, 120)
    rc_b, out_b = finish(b, 120)
    rc_p, out_p = finish(prod, 120)
    assert (rc_a, rc_b, rc_p) == (0, 0, 0), (out_a[-2000:], out_b[-2000:], out_p[-2000:])
    ra = records(tmp_path / "a.jsonl")
    ga, gb = frames(ra), frames(records(tmp_path / "b.jsonl"))
    assert len(ga) == 10
    assert sorted(ga + gb) == list(range(n))
    assert ra[-1].get("closed") and ra[-1]["frames_dropped"] == 0 and ra[-1]["frames_returned"] > 0, ra[-1]


def test_gpu_competing_consumers_default_read_ahead(store_port, tmp_path):  # noqa: F811
    """Fast and slow HBM consumers at the default ring: exactly once, the fast one takes more, and
    the slow one finishes within one read-ahead window of the fast one."""
    n = 200
    fast = consumer(store_port, tmp_path / "fast.jsonl", *GPU_C, "--sleep", "0.002")
    slow = consumer(store_port, tmp_path / "slow.jsonl", *GPU_C, "--sleep", "0.05")
    time.sleep(3.0)
    prod = gpu_producer(store_port, n)
    for c in (fast, slow):
        rc, out = finish(c, 120)
        assert rc == 0, out[-2000:]
    rc_p, out_p = finish(prod, 120)
    assert rc_p == 0, out_p[-2000:]
    gf, gs = frames(records(tmp_path / "fast.jsonl")), frames(records(tmp_path / "slow.jsonl"))
    assert sorted(gf + gs) == list(range(n))
    assert len(gf) > 2 * len(gs) and len(gs) > 0, (len(gf), len(gs))
    t_fast = records(tmp_path / "fast.jsonl")[-1]["t_end"]
    t_slow = records(tmp_path / "slow.jsonl")[-1]["t_end"]
    assert t_slow - t_fast <= 16 * 0.05 + 3.0, (t_slow - t_fast)


def test_gpu_keeper_keeps_committed_frames_across_a_producer_crash(store_port, tmp_path):  # noqa: F811
    """A live GPU producer's committed frames move into the keeper's HBM ring while nobody else can
    take them; kill -9 of the producer loses none of them (<= one chunk in flight allowed)."""
    from tests.test_elastic_queue import hang_producer, keeper, wait_line

    kp = keeper(store_port, "--device", "cuda:0")
    time.sleep(2.0)
    n, chunk = 40, 4
    hp = hang_producer(store_port, n, "--chunk", str(chunk), "--queue_size", "16", "--device", "cuda:0")
    wait_line(hp, "COMMITTED", timeout=120)
    time.sleep(2.0)
    hp.kill()
    hp.wait(10)
    c = consumer(store_port, tmp_path / "c.jsonl", *GPU_C)
    rc_c, out_c = finish(c, 120)
    rc_k, out_k = finish(kp, 120)
    assert rc_c == 0, out_c[-2000:]
    assert rc_k == 0, out_k[-2000:]
    got = frames(records(tmp_path / "c.jsonl"))
    assert len(got) == len(set(got)) and set(got) <= set(range(n)), got
    assert len(got) >= n - chunk, f"only {len(got)} of {n} committed frames survived the producer"


def test_gpu_keeper_holds_frames_after_the_producer_exits(store_port, tmp_path):  # noqa: F811
    """R-11 on HBM: the producer drains into the keeper's HBM ring (IPC peer copies) and exits with
    no consumer; a consumer started later receives every frame bit-exactly, plus EOS."""
    from tests.test_elastic_queue import keeper

    prod = gpu_producer(store_port, 40, queue_size=48)
    time.sleep(2.0)
    kp = keeper(store_port, "--device", "cuda:0")
    rc_p, out_p = finish(prod, 120)
    assert rc_p == 0, out_p[-3000:]
    assert kp.poll() is None, "the keeper must stay while it holds frames"
    c = consumer(store_port, tmp_path / "c.jsonl", "--device", "cuda:0", "--gen_device", "cuda")
    rc_c, out_c = finish(c, 120)
    rc_k, out_k = finish(kp, 120)
    assert rc_c == 0, out_c[-3000:]
    assert rc_k == 0, out_k[-3000:]
    recs = records(tmp_path / "c.jsonl")
    assert sorted(frames(recs)) == list(range(40))
    assert recs[-1].get("eos") is True
    assert "keeper done: kept=40" in out_k, out_k[-2000:]


def test_gpu_odd_sized_image_frames_cross_processes(store_port, tmp_path):  # noqa: F811
    """Image frames of 612 B (9 x 17 pixels: not a multiple of 16 B) between two GPU processes
    (ADVICE r4): ring slots are 256-B strided (FrameRing.slot_bytes), so every slot stays aligned for
    the calibration kernels and the fabric's copy kernel moves whole slots -- every frame bit-exact,
    then EOS.  (A ring whose slots are not 16-B multiples is copied by the runtime engine instead:
    the engine is chosen per link at attach, csrc/fabric.cpp.)"""
    from tests.test_elastic_queue import producer

    prod = producer(store_port, 30, "--device", "cuda:0", queue_size=16, detector="tiny_odd", mode="image")
    c = consumer(store_port, tmp_path / "c.jsonl", "--device", "cuda:0", "--gen_device", "cuda", "--mode", "image",
                 "--verify", "synthetic:2:tiny_odd:1")
    rc_c, out_c = finish(c, 120)
    rc_p, out_p = finish(prod, 120)
    assert rc_c == 0, out_c[-3000:]
    assert rc_p == 0, out_p[-3000:]
    recs = records(tmp_path / "c.jsonl")
    assert sorted(frames(recs)) == list(range(30))
    assert recs[-1].get("eos") is True


@pytest.mark.parametrize("headroom", ["", "0"])
def test_gpu_direct_writes_consumer_that_leaves(store_port, tmp_path, headroom):  # noqa: F811
    """Direct writes (csrc/fabric.h take_direct): with --route spread the producer calibrates frames
    straight into its consumers' slots.  A consumer that CLOSES hands back the direct frames still in
    flight by copy-back (requeued: the survivor receives them, every frame exactly once, bit-exact).
    headroom "" = the default (config.FABRIC_DIRECT_HEADROOM slots kept for direct frames, the engine
    waits for grants, engine.h), "0" = grants only when on offer at launch."""
    n = 200
    prod = gpu_producer(store_port, n, "--route", "spread", queue_size=64,
                        env={"PSANA_RAY_AMD_FABRIC_DIRECT_HEADROOM": headroom})
    a = consumer(store_port, tmp_path / "a.jsonl", *GPU_C, "--sleep", "0.02", "--stop_after", "10")
    b = consumer(store_port, tmp_path / "b.jsonl", *GPU_C, "--sleep", "0.02")
    rc_a, out_a = finish(a, 120)
    rc_b, out_b = finish(b, 120)
    rc_p, out_p = finish(prod, 120)
    assert (rc_a, rc_b, rc_p) == (0, 0, 0), (out_a[-2000:], out_b[-2000:], out_p[-2000:])
    ga, gb = frames(records(tmp_path / "a.jsonl")), frames(records(tmp_path / "b.jsonl"))
    assert len(ga) == 10
    assert sorted(ga + gb) == list(range(n))
    assert _direct_frames(out_p) > 0, out_p[-2000:]


def _direct_frames(out):
    import re

    m = re.search(r"\((\d+) calibrated straight into the consumer's slot", out)
    return int(m.group(1)) if m else 0


@pytest.mark.parametrize("headroom", ["", "0"])
def test_gpu_direct_writes_killed_consumer(store_port, tmp_path, headroom):  # noqa: F811
    """Direct writes with a consumer killed by -9: the frames in flight into its ring are lost with
    its read-ahead (at most the prefetch bound), the survivor gets the rest exactly once."""
    from psana_ray_amd.config import DEFAULT_PREFETCH

    n = 240
    prod = gpu_producer(store_port, n, "--route", "spread", queue_size=100,
                        env={"PSANA_RAY_AMD_FABRIC_DIRECT_HEADROOM": headroom})
    a = consumer(store_port, tmp_path / "a.jsonl", *GPU_C, "--sleep", "0.01", "--die_after", "16")
    b = consumer(store_port, tmp_path / "b.jsonl", *GPU_C, "--sleep", "0.01")
    rc_a, _ = finish(a, 120)
    assert rc_a == -9
    rc_b, out_b = finish(b, 120)
    rc_p, out_p = finish(prod, 120)
    assert rc_b == 0, out_b[-3000:]
    assert rc_p == 0, out_p[-3000:]
    ga, gb = frames(records(tmp_path / "a.jsonl")), frames(records(tmp_path / "b.jsonl"))
    assert not set(ga) & set(gb)
    lost = set(range(n)) - set(ga) - set(gb)
    assert len(lost) <= DEFAULT_PREFETCH, lost
    assert _direct_frames(out_p) > 0, out_p[-2000:]
