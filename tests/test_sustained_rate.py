"""Sustained-rate accounting of bench.py: production is counted at completion,
frames READY before the window opened are excluded, and the rate runs between chunk completions."""
import threading
import time

import torch

from psana_ray_amd.utils.metrics import sustained_rate


def test_sustained_rate_excludes_frames_ready_before_t0():
    # 10 chunks of 4 frames completed every 0.1 s from t=0.0; window (0.35, 0.75]
    log = [(4 * (i + 1), 0.1 * i) for i in range(10)]
    frames, rate = sustained_rate(log, 0.35, 0.75)
    # chunks at 0.4, 0.5, 0.6, 0.7 are inside; the 16 frames done by 0.3 are not counted
    assert frames == 16
    assert abs(rate - 16 / 0.4) < 1e-9      # from the completion at 0.3 to the one at 0.7


def test_sustained_rate_window_length_independent():
    log = [(64 * (i + 1), 0.005 * i) for i in range(2000)]   # steady 12.8k frames/s
    _, short = sustained_rate(log, 1.0013, 1.0513)
    _, long = sustained_rate(log, 1.0013, 5.5013)
    assert abs(short / long - 1) < 1e-9 and abs(long - 12800) < 1e-6


def test_sustained_rate_nothing_inside():
    log = [(4, 0.0), (8, 0.1)]
    assert sustained_rate(log, 0.2, 0.3) == (0, None)
    assert sustained_rate([], 0.0, 1.0) == (0, None)


def test_frames_ready_at_t0_are_not_counted(native):
    """A producer fills the queue with no consumer reading; a window that opens afterwards and
    drains those frames measures no production (the reference's one put == one delivered frame)."""
    from psana_ray_amd.models import Calibrator, Mode
    from psana_ray_amd.pipeline import ProducerPipeline
    from psana_ray_amd.queue import FrameRing, QueueEndpoint
    from psana_ray_amd.source import SyntheticRun

    src = SyntheticRun("synthetic", 0, "tiny_epix", n_events=24, pool_frames=4, pinned=False)
    cal = Calibrator(src.consts, torch.device("cpu"), Mode.calib)
    ring = FrameRing(cal.out_shape, cal.out_dtype, "cpu", 24, 24)
    ep = QueueEndpoint(ring)
    prod = ProducerPipeline(src, cal, ep, chunk=4)
    th = threading.Thread(target=prod.run)
    th.start()
    th.join(60)
    assert prod.produced == 24 and ep.size() == 24       # all READY, nobody read
    t0 = prod.clock()
    got = 0
    while got < 24:
        it = ep.get(timeout=1.0)
        assert it is not None
        it.release()
        got += 1
    t1 = prod.clock()
    _, lg = prod.completion_log(0)
    assert len(lg) == 6 and all(t <= t0 for _, t in lg)
    frames, rate = sustained_rate(lg, t0, t1)
    assert frames == 0 and rate is None     # 24 frames consumed inside the window, none produced there
    assert t1 > t0 and time.perf_counter() >= t1
