#!/usr/bin/env python3
"""BASELINE config 1: synthetic 256x256 float32 frames through the in-process CPU queue,
1 producer + 1 consumer, no GPU (the plumbing configuration of BASELINE.json).

The producer thread mirrors the reference hot loop (psana_ray/producer.py:88-111): build the
item ``[rank, idx, frame, photon_energy]`` and ``put`` it, backing off while the queue is full;
the consumer mirrors ``DataReader.read`` (psana_ray/data_reader.py:31-37) on the same named queue
(``create_queue`` / ``DataReader`` in-process attach).  The reference's exponential backoff
(0.1 s base) and 1 s consumer poll are kept selectable (``--reference-timing``) to show what they
cost; the default uses the event-driven waits this framework replaces them with.

Prints one JSON line: frames/s through the queue.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=20000)
    ap.add_argument("--queue-size", type=int, default=400)
    ap.add_argument("--shape", type=int, nargs=2, default=(256, 256))
    ap.add_argument("--pool", type=int, default=64, help="distinct pre-generated frames (cycled)")
    ap.add_argument("--copy", action="store_true", help="producer copies each frame (fresh array per event)")
    ap.add_argument("--reference-timing", action="store_true",
                    help="reference backoff (0.1 s x 2^n + U(0,0.5)) and 1 s consumer poll instead of waits")
    a = ap.parse_args(argv)

    from psana_ray_amd.data_reader import DataReader
    from psana_ray_amd.producer import backoff_delays
    from psana_ray_amd.shared_queue import create_queue, drop_queue

    rng = np.random.default_rng(0)
    pool = rng.normal(100.0, 5.0, size=(a.pool, 1, *a.shape)).astype(np.float32)   # ndim 3 (producer.py:96-97)
    name, ns = "bench_cfg1", "bench"
    q = create_queue(name, ns, a.queue_size)
    full_waits = [0]

    def produce():
        for idx in range(a.frames):
            frame = pool[idx % a.pool]
            item = [0, idx, frame.copy() if a.copy else frame, 9500.0]
            retries = 0
            while not q.put(item):
                full_waits[0] += 1
                if a.reference_timing:
                    d, j = backoff_delays(retries)
                    time.sleep(d + np.random.uniform(0, j))
                    retries += 1
                else:
                    q.wait_not_full(0.05)
        q.put(None)   # end-of-stream sentinel (producer.py:122-128)

    got = 0
    t0 = time.perf_counter()
    pt = threading.Thread(target=produce, daemon=True)
    pt.start()
    with DataReader(queue_name=name, ray_namespace=ns) as reader:
        while True:
            item = reader.read(timeout=None if a.reference_timing else 0.05)
            if item is None:
                if a.reference_timing:
                    time.sleep(1.0)   # examples/psana_consumer.py:40
                if not pt.is_alive() and q.size() == 0:
                    break
                continue
            got += 1
            if got == a.frames:
                break
    dt = time.perf_counter() - t0
    pt.join(timeout=10)
    drop_queue(name, ns)
    res = {"config": "BASELINE config 1: synthetic %dx%d float32, in-process CPU queue, 1 producer + 1 consumer"
           % tuple(a.shape), "frames": got, "seconds": round(dt, 4), "frames_per_s": round(got / dt, 1),
           "GB_per_s": round(got * pool[0].nbytes / dt / 1e9, 3), "queue_size": a.queue_size,
           "queue_full_waits": full_waits[0], "reference_timing": a.reference_timing, "copy": a.copy}
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
