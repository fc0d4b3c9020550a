#!/usr/bin/env python3
"""Counter workload for the SHIPPED kernels in production form: every phase launches
its kernel REPEAT times on 64 epix10k2M frames (the producer's chunk), in this order --

  cm        calib_cm_net_kernel, calib mode + common mode (K-01..K-04)
  cm_image  the same kernel with the fused K-05 image write-out (image mode + common mode)
  peakfind  peakfind_range_kernel on 64 calibrated frames (consumer batch; self-resetting scratch)
  h2d       copy_h2d_kernel: 64 raw frames from pinned host memory into HBM (32 workgroups)
  xcopy     copy_runs_kernel: 64 calibrated frames HBM -> HBM in one launch (the fabric's copy)

Run it under rocprofv3 (--pmc passes, and --kernel-trace --stats for durations);
tools/pmc_table.py turns the CSVs into the per-kernel table.  Writes the phase list to
``--phases`` (JSON) so the summary can label dispatches."""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psana_ray_amd.config import CommonModeParams, PeakFinderParams  # noqa: E402
from psana_ray_amd.models import Calibrator, Mode  # noqa: E402
from psana_ray_amd.ops import _ext, kernels  # noqa: E402
from psana_ray_amd.source import SyntheticRun  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--repeat", type=int, default=4)
ap.add_argument("--phases", default=None)
ap.add_argument("--xcopy-wgs", type=int, default=128)
a = ap.parse_args()
C = _ext.load()
dev = torch.device("cuda:0")
F = 64
src = SyntheticRun("synthetic", 0, "epix10k2M", pool_frames=8, pinned=True, gen_device="cuda")
pool = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16).to(dev)
raw = pool.repeat(F // pool.shape[0] + 1, 1, 1, 1)[:F].contiguous()
out = torch.empty((F, *src.spec.frame_shape), dtype=torch.float32, device=dev)
out2 = torch.empty_like(out)
rl, ol = [raw[i] for i in range(F)], [out[i] for i in range(F)]
s = _ext.stream_handle()
cm = CommonModeParams()
calcm = Calibrator(src.consts, dev, Mode.calib, common_mode=cm)
calim = Calibrator(src.consts, dev, Mode.image, common_mode=cm)
img = torch.empty((F, *calim.out_shape), dtype=torch.float32, device=dev)
il = [img[i] for i in range(F)]
pf = PeakFinderParams()
peaks = torch.empty((F, pf.max_peaks, 8), dtype=torch.float32, device=dev)
counts = torch.empty((F,), dtype=torch.int32, device=dev)
summ = torch.empty((F, 2), dtype=torch.float32, device=dev)
scratch = torch.zeros(kernels.PF_SCRATCH_WORDS, dtype=torch.int32, device=dev)
# pinned host source of the staging copy: the pool cycled into one 64-frame span
fb = src.spec.raw_frame_bytes
host = C.PinnedBuffer(F * fb)
hv = np.frombuffer(host, dtype=np.uint16).reshape(F, *src.spec.frame_shape)
for i in range(F):
    hv[i] = src.pool[i % src.pool_frames]
stage = torch.empty((F, *src.spec.frame_shape), dtype=torch.uint16, device=dev)
calcm.run(rl, ol)   # warm up (tables resident, code loaded)
calim.run(rl, il)
torch.cuda.synchronize()
phases = []


def phase(name, fn, frames, bytes_per_frame):
    for _ in range(a.repeat):
        fn()
    phases.append({"name": name, "dispatches": a.repeat, "frames": frames, "bytes_per_frame_nominal": bytes_per_frame})


npix = src.spec.npix
phase("cm", lambda: calcm.run(rl, ol), F, {"read_raw": 2 * npix, "read_tables_nominal": 8 * npix, "write": 4 * npix})
phase("cm_image", lambda: calim.run(rl, il), F,
      {"read_raw": 2 * npix, "read_tables_nominal": 8 * npix, "write": 4 * int(np.prod(calim.out_shape))})
phase("peakfind", lambda: kernels.peakfind(ol, src.spec.frame_shape, pf, peaks, counts, summ, scratch=scratch), F,
      {"read": 4 * npix})
phase("h2d", lambda: C.copy_h2d_kernel(int(stage.data_ptr()), int(host.ptr), F * fb, 32, s), F,
      {"read_host": fb, "write": fb})
ob = out.numel() * 4 // F
phase("xcopy", lambda: C.copy_runs([int(out.data_ptr())], [int(out2.data_ptr())], [F * ob], a.xcopy_wgs, s), F,
      {"read": ob, "write": ob})
torch.cuda.synchronize()
assert torch.equal(stage, raw), "copy_h2d_kernel output differs"
assert torch.equal(out2.view(torch.int32), out.view(torch.int32)), "copy_runs_kernel output differs"
if a.phases:
    Path(a.phases).write_text(json.dumps(phases, indent=1))
print("done", json.dumps([p["name"] for p in phases]))
