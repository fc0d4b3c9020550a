"""Elastic shared queue between separate GPU processes on ONE MI355X: the producer CLI on cuda:0
writes frames into DataReader consumers' HBM rings through HIP IPC peer copies (the same path that
crosses xGMI when the processes sit on different GPUs).  Frames are checked bit-exactly against
the fp32 golden calibration; the scenarios are the CPU ones of test_elastic_queue.py."""
import os
import time

import pytest

from tests.test_elastic_queue import consumer, finish, frames, records, store_port  # noqa: F401

pytestmark = pytest.mark.gpu


def gpu_producer(port, n_events, *extra, queue_size=16, chunk=4, timeout=60):
    from tests.test_elastic_queue import producer

    p = producer(port, n_events, "--device", "cuda:0", *extra, queue_size=queue_size, chunk=chunk, timeout=timeout)
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


def test_gpu_kill9_consumer_survivor_gets_the_rest(store_port, tmp_path):  # noqa: F811
    n, slots_a = 160, 4
    prod = gpu_producer(store_port, n)
    a = consumer(store_port, tmp_path / "a.jsonl", "--device", "cuda:0", "--gen_device", "cuda", "--sleep", "0.01", "--slots", str(slots_a),
                 "--die_after", "16")
    b = consumer(store_port, tmp_path / "b.jsonl", "--device", "cuda:0", "--gen_device", "cuda", "--sleep", "0.01", "--slots", "4")
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
    assert len(lost) <= slots_a, lost
    assert records(tmp_path / "b.jsonl")[-1].get("eos") is True


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
