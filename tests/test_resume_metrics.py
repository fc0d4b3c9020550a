"""Resume cursor (--start_event) and the sampled metrics / tracing utilities."""
import json
import logging
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from psana_ray_amd.models import Calibrator, Mode
from psana_ray_amd.ops import reference
from psana_ray_amd.pipeline import ProducerPipeline
from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint
from psana_ray_amd.source import SyntheticRun
from psana_ray_amd.source.synthetic import first_local_event
from psana_ray_amd.utils import Registry, Reporter, trace_range
from psana_ray_amd.utils.metrics import rates

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("size", [1, 2, 3, 4])
@pytest.mark.parametrize("start", [0, 1, 7, 11])
def test_seek_covers_the_tail_exactly_once(size, start):
    n = 23
    got = []
    for r in range(size):
        src = SyntheticRun("synthetic", 0, "tiny_plain", rank=r, size=size, n_events=n, pool_frames=4,
                           gen_device="cpu")
        k0 = src.seek(start)
        assert k0 == first_local_event(start, r, size)
        while True:
            evs = src.next_events(5)
            if not evs:
                break
            for e in evs:
                assert e.gevt == r + e.idx * size
            got += [e.gevt for e in evs]
    assert sorted(got) == list(range(start, n))


def _drain(ep):
    out = []
    while True:
        try:
            it = ep.get(timeout=0.2)
        except EndOfStream:
            return out
        if it is not None:
            with it:
                out.append((it.idx, it.gevt, it.data.clone()))


def _resume_run(device, engine_expected):
    n, start = 40, 13
    src = SyntheticRun("synthetic", 2, "tiny_epix", n_events=n, pool_frames=8, pinned=device.type == "cuda",
                       gen_device="cpu")
    src.seek(start)
    cal = Calibrator(src.consts, device, Mode.calib)
    ring = FrameRing(cal.out_shape, cal.out_dtype, device, 16, 64)
    ep = QueueEndpoint(ring)
    prod = ProducerPipeline(src, cal, ep, chunk=8)
    assert (prod.engine is not None) == engine_expected
    prod.run()
    items = _drain(ep)
    if device.type == "cuda":
        torch.cuda.synchronize()
    assert [g for _, g, _ in items] == list(range(start, n))
    ref = reference.calibrate_reference(torch.from_numpy(src.pool.astype(np.int32)), src.consts)
    for idx, _, data in items:
        assert torch.equal(data.cpu(), ref[idx % 8]), f"event {idx}: wrong pool frame after resume"
    m = prod.metrics()
    assert m["frames_produced"] == n - start


def test_resume_python_path_cpu():
    _resume_run(torch.device("cpu"), engine_expected=False)


@pytest.mark.gpu
def test_resume_native_engine_gpu(cuda_device, native):
    _resume_run(cuda_device, engine_expected=True)


def test_registry_rates_and_reporter(tmp_path, caplog):
    reg = Registry()
    c = {"frames_produced": 0}
    reg.register("producer", lambda: dict(c, ready=3))
    reg.register("broken", lambda: 1 / 0)
    path = tmp_path / "m.jsonl"
    rep = Reporter(reg, rank=5, interval=0, json_path=str(path))
    rep.sample()
    c["frames_produced"] = 1000
    with caplog.at_level(logging.INFO, logger="psana_ray_amd.metrics"):
        rec = rep.sample()
    assert rec["producer.frames_produced"] == 1000 and rec["broken.error"] == 1.0
    assert rec["producer.frames_produced_per_s"] > 0
    assert any("rank 5" in r.message and "producer.ready=3" in r.message for r in caplog.records)
    lines = [json.loads(l) for l in path.read_text().splitlines()]
    assert len(lines) == 2 and lines[-1]["rank"] == 5
    assert rates({"a.frames": 0.0}, {"a.frames": 10.0}, 2.0) == {"a.frames_per_s": 5.0}


def test_trace_range_is_safe_without_profiler():
    with trace_range("test.range"):
        x = 1
    assert x == 1


def test_producer_cli_resume_and_metrics(native, tmp_path):
    path = tmp_path / "metrics.jsonl"
    r = subprocess.run([sys.executable, "-m", "psana_ray_amd.producer", "--exp", "synthetic", "--run", "1",
                        "--detector_name", "tiny_epix", "--calib", "--num_events", "30", "--start_event", "11",
                        "--local", "--consumer_task", "peakfind", "--device", "cpu", "--metrics_interval", "0.2",
                        "--metrics_json", str(path)],
                       cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "resuming at global event 11" in r.stderr
    last = json.loads(path.read_text().splitlines()[-1])
    assert last["producer.frames_produced"] == 19
    assert last["consumer.frames_consumed"] == 19
