"""Experiment: the producer engine's copy->calibrate pipeline WITHOUT queue/consumer, vs pure copies.
Rotating raw buffers, copies on a side stream, CM calibration on a compute stream, cross-stream
events exactly like csrc/engine.cpp."""
import time
import numpy as np
import torch
from psana_ray_amd.config import CommonModeParams
from psana_ray_amd.models import Calibrator, Mode
from psana_ray_amd.ops import _ext
from psana_ray_amd.source import SyntheticRun

C = _ext.load()
dev = torch.device("cuda:0")
src = SyntheticRun("synthetic", 0, "epix10k2M", pool_frames=64, pinned=True, gen_device="cuda")
ptrs, _ = src.cycled_frames()
fb = src.spec.raw_frame_bytes
for nbuf in (3, 6):
    for cm in (None, CommonModeParams()):
        cal = Calibrator(src.consts, dev, Mode.calib, common_mode=cm)
        chunk = 16
        raw = torch.empty((nbuf, chunk, *src.spec.frame_shape), dtype=torch.uint16, device=dev)
        out = torch.empty((64, *src.spec.frame_shape), dtype=torch.float32, device=dev)
        h2d, comp = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
        bfree = [torch.cuda.Event() for _ in range(nbuf)]
        hdone = [torch.cuda.Event() for _ in range(nbuf)]
        used = [False] * nbuf
        def run(nchunks):
            for c in range(nchunks):
                b = c % nbuf
                if used[b]:
                    h2d.wait_event(bfree[b])
                used[b] = True
                k0 = (c * chunk) % 64
                C.memcpy_h2d_async(int(raw[b].data_ptr()), ptrs[k0], chunk * fb, int(h2d.cuda_stream))
                hdone[b].record(h2d)
                comp.wait_event(hdone[b])
                o0 = (c * chunk) % 64
                cal.run_ptrs([int(raw[b, i].data_ptr()) for i in range(chunk)],
                             [int(out[(o0 + i) % 64].data_ptr()) for i in range(chunk)], comp)
                bfree[b].record(comp)
            torch.cuda.synchronize()
        run(4)
        t0 = time.perf_counter()
        run(40)
        dt = time.perf_counter() - t0
        print(f"nbuf={nbuf} cm={'on' if cm else 'off'}: {40 * chunk / dt:.0f} frames/s, H2D {40 * chunk * fb / dt / 1e9:.1f} GB/s",
              flush=True)
