"""Producer process for the crash-persistence tests: joins the queue session like the producer CLI,
commits exactly --n frames of the synthetic run (chunk by chunk, without ever finishing the
stream), prints ``COMMITTED <n>`` and then waits to be killed -- a producer that dies mid-stream
with frames it already put (reference: items put into the detached actor survive their producer,
psana_ray/shared_queue.py:35, producer.py:101)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--address", required=True)
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--chunk", type=int, default=4)
    ap.add_argument("--queue_size", type=int, default=16)
    ap.add_argument("--device", default="cpu")
    a = ap.parse_args()

    import torch

    from psana_ray_amd.models import Calibrator, Mode
    from psana_ray_amd.pipeline import ProducerPipeline
    from psana_ray_amd.producer import initialize_queue
    from psana_ray_amd.queue import FrameRing, QueueEndpoint
    from psana_ray_amd.queue.session import QueueSession
    from psana_ray_amd.producer import build_calibrator
    from psana_ray_amd.source import SyntheticRun

    device = torch.device(a.device)
    gpu = device.type == "cuda"
    if gpu:
        torch.cuda.set_device(device)
    # the same synthetic run as the producer CLI's (--exp synthetic --run 2, one rank)
    src = SyntheticRun("synthetic", 2, "tiny_epix", rank=0, size=1, pinned=gpu, gen_device="cuda" if gpu else "cpu")
    cal = build_calibrator(src, device, Mode.calib, None, "auto")   # the producer CLI's default calibration
    store, meta = initialize_queue(a.address, "default", "my", a.queue_size, 0, 1, 1, cal.out_shape, "float32",
                                   device.type, timeout_s=30)
    sess = QueueSession(store, "default", "my", meta, "producer", device=device.index if gpu else -1, rank=0)
    ring = FrameRing(cal.out_shape, cal.out_dtype, device, a.queue_size, 0)
    ep = QueueEndpoint(ring, sess, is_producer=True, is_consumer=False).start()
    pipe = ProducerPipeline(src, cal, ep, rank=0, chunk=a.chunk)
    if pipe.engine is not None:   # GPU: the native engine, stopped after n frames (never finishes the stream)
        pipe.engine.start(-1, a.n, 0)
        while pipe.engine.running:
            time.sleep(0.01)
        assert int(pipe.engine.frames) == a.n, pipe.engine.error()
    else:
        while pipe.frames < a.n:
            pipe.chunk = min(a.chunk, a.n - pipe.frames)
            assert pipe.step() > 0
    print(f"COMMITTED {a.n}", flush=True)
    while True:   # never finish(): the session sees a LIVE producer until it is killed
        time.sleep(1.0)


if __name__ == "__main__":
    main()
