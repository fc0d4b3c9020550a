"""One GPU, one process: synthetic epix10k2M raw frames -> pinned host -> HIP calibration (with
common mode) -> HBM ring -> on-GPU peak finder.  The minimum end-to-end slice.

    python examples/single_gpu_pipeline.py --events 2000
"""
import argparse
import threading
import time

from psana_ray_amd.config import CommonModeParams, PeakFinderParams
from psana_ray_amd.models import Calibrator, Mode
from psana_ray_amd.pipeline import PeakFinderConsumer, ProducerPipeline
from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint
from psana_ray_amd.source import SyntheticRun

ap = argparse.ArgumentParser()
ap.add_argument("--events", type=int, default=2000)
ap.add_argument("--detector", default="epix10k2M")
ap.add_argument("--device", default="cuda:0")
a = ap.parse_args()

src = SyntheticRun("synthetic", 0, a.detector, n_events=a.events, pool_frames=32, pinned=a.device != "cpu")
cal = Calibrator(src.consts, a.device, Mode.calib, common_mode=CommonModeParams())
ring = FrameRing(cal.out_shape, cal.out_dtype, a.device, producer_slots=64, consumer_slots=400)
ep = QueueEndpoint(ring)
prod = ProducerPipeline(src, cal, ep, chunk=16)
cons = PeakFinderConsumer(ep, cal.out_shape, PeakFinderParams(), batch=32)
t0 = time.time()
th = threading.Thread(target=prod.run)
th.start()
n = 0
while True:
    try:
        n += cons.poll(timeout=0.1)
    except EndOfStream:
        break
th.join()
peaks = cons.synchronize()
dt = time.time() - t0
print(f"{n} frames in {dt:.2f} s = {n / dt:.0f} frames/s, {peaks} peaks ({peaks / max(n, 1):.1f}/frame)")
