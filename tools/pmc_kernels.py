"""Workload for counter collection (rocprofv3 --pmc): each hot kernel launched 4x eagerly on 32
epix10k2M frames -- calib_basic (K-01/02/04), calib_cm (+K-03 common mode), calib_image (fused
raw -> image, K-05), peakfind (K-07) -- plus the u16->f32 stream with calib's traffic (bandwidth
reference).  tools/pmc_summary.py turns the counter CSVs into a per-kernel table."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psana_ray_amd.config import CommonModeParams, PeakFinderParams  # noqa: E402
from psana_ray_amd.models import Calibrator, Mode  # noqa: E402
from psana_ray_amd.ops import _ext, kernels  # noqa: E402
from psana_ray_amd.source import SyntheticRun  # noqa: E402

C = _ext.load()
dev = torch.device("cuda:0")
F = 32
src = SyntheticRun("synthetic", 0, "epix10k2M", pool_frames=8, pinned=False, gen_device="cuda")
pool = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16).to(dev)
raw = pool.repeat(4, 1, 1, 1)[:F].contiguous()
out = torch.empty((F, *src.spec.frame_shape), dtype=torch.float32, device=dev)
rl, ol = [raw[i] for i in range(F)], [out[i] for i in range(F)]
rp, op = [int(t.data_ptr()) for t in rl], [int(t.data_ptr()) for t in ol]
s = _ext.stream_handle()
cal = Calibrator(src.consts, dev, Mode.calib)
calcm = Calibrator(src.consts, dev, Mode.calib, common_mode=CommonModeParams())
cali = Calibrator(src.consts, dev, Mode.image)
img = torch.empty((F, *cali.out_shape), dtype=torch.float32, device=dev)
il = [img[i] for i in range(F)]
pf = PeakFinderParams()
peaks = torch.empty((F, pf.max_peaks, 8), dtype=torch.float32, device=dev)
counts = torch.empty((F,), dtype=torch.int32, device=dev)
summ = torch.empty((F, 2), dtype=torch.float32, device=dev)
calcm.run(rl, ol)
for _ in range(4):
    C.convert_u16_f32(rp, op, src.spec.npix, s)
    cal.run(rl, ol)
    cali.run(rl, il)
    calcm.run(rl, ol)
    kernels.peakfind(ol, src.spec.frame_shape, pf, peaks, counts, summ)
torch.cuda.synchronize()
print("done")
