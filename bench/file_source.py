#!/usr/bin/env python3
"""Raw-run file source throughput: file (page cache / tmpfs) -> native pread thread pool -> pinned
staging -> H2D -> calibration + common mode -> shared queue -> on-GPU peak finder, one GPU.

The reference reads XTC2 through psana's C++ reader; here the whole per-chunk loop is the native
producer engine (csrc/engine.cpp, set_file_source).  Prints one JSON line."""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--dir", default="/dev/shm/psana_ray_file_bench")
    ap.add_argument("--detector", default="epix10k2M")
    ap.add_argument("--threads", type=int, default=16, help="reader pread threads")
    ap.add_argument("--chunk", type=int, default=32)
    ap.add_argument("--common-mode", default="default")
    ap.add_argument("--no-numa", action="store_true", help="do not bind to the GPU's NUMA node")
    ap.add_argument("--format", choices=["praw", "xtc2"], default="praw",
                    help="fixed-record raw-run file, or XTC2-style bigdata + smalldata index")
    a = ap.parse_args(argv)

    import torch

    from psana_ray_amd.config import CommonModeParams, PeakFinderParams
    from psana_ray_amd.models import Calibrator, Mode
    from psana_ray_amd.pipeline import PeakFinderConsumer, ProducerPipeline
    from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint
    from psana_ray_amd.source import RawFileRun, make_synthetic_run, make_synthetic_xtc2_run, open_xtc2_run

    from psana_ray_amd.parallel.launch import bind_numa_to_device

    dev = torch.device("cuda:0")
    numa = None if a.no_numa else bind_numa_to_device(dev)
    shutil.rmtree(a.dir, ignore_errors=True)
    try:
        if a.format == "xtc2":
            make_synthetic_xtc2_run(a.dir, "bench", 1, a.detector, n_events=a.frames, chunk=32)
            t_scan = time.perf_counter()
            src = open_xtc2_run(a.dir, "bench", 1, a.detector, n_threads=a.threads, pinned=False)
            t_scan = time.perf_counter() - t_scan
        else:
            path = make_synthetic_run(a.dir, "bench", 1, a.detector, n_events=a.frames, chunk=32)
            t_scan = 0.0
            src = RawFileRun(path, a.detector, exp="bench", run=1, n_threads=a.threads, pinned=False)
        cal = Calibrator(src.consts, dev, Mode.calib, common_mode=CommonModeParams.parse(a.common_mode))
        ring = FrameRing(cal.out_shape, cal.out_dtype, dev, 4 * a.chunk + 32, 400)
        ep = QueueEndpoint(ring)
        prod = ProducerPipeline(src, cal, ep, chunk=a.chunk)
        cons = PeakFinderConsumer(ep, cal.out_shape, PeakFinderParams(), batch=32)
        t0 = time.perf_counter()
        th = threading.Thread(target=prod.run, daemon=True)
        th.start()
        n = 0
        t_first, n_first = None, 0
        while True:
            try:
                n += cons.poll(timeout=0.05)
            except EndOfStream:
                break
            if t_first is None and n > 0:
                t_first, n_first = time.perf_counter(), n     # steady state: after the pipeline filled
        peaks = cons.synchronize()
        dt = time.perf_counter() - t0
        steady = (n - n_first) / max(1e-9, time.perf_counter() - t_first) if t_first is not None else 0.0
        th.join()
        st = prod.engine.timing() if prod.engine is not None else None
        print(json.dumps({"bench": f"{a.format} file source, 1 GPU", "detector": a.detector, "frames": n,
                          "index_scan_s": round(t_scan, 4),
                          "seconds": round(dt, 4), "frames_per_s": round(n / dt, 1),
                          "steady_frames_per_s": round(steady, 1),
                          "GB_per_s_raw": round(n * src.spec.raw_frame_bytes / dt / 1e9, 2),
                          "native_engine": prod.engine is not None, "zero_copy": prod.zero_copy, "reader_threads": a.threads, "peaks": peaks, "numa": numa,
                          "engine_span_frame_kernel_copies": prod.engine.copy_stats(),
                          "engine_host_s_stage_acquire_launch_commit_total": st}))
    finally:
        shutil.rmtree(a.dir, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
