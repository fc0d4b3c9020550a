"""Tiny driver for counter collection: a few launches of calib_basic (epix, 32 frames) and of the
u16->f32 bandwidth reference with identical traffic."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch
from psana_ray_amd.models import Calibrator, Mode
from psana_ray_amd.ops import _ext
from psana_ray_amd.source import SyntheticRun

C = _ext.load()
dev = torch.device("cuda:0")
src = SyntheticRun("synthetic", 0, "epix10k2M", pool_frames=8, pinned=False, gen_device="cuda")
pool = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16).to(dev)
F = 32
raw = pool.repeat(4, 1, 1, 1)[:F].contiguous()
out = torch.empty((F, *src.spec.frame_shape), dtype=torch.float32, device=dev)
cal = Calibrator(src.consts, dev, Mode.calib)
rp = [int(raw[i].data_ptr()) for i in range(F)]
op = [int(out[i].data_ptr()) for i in range(F)]
s = int(torch.cuda.current_stream().cuda_stream)
for _ in range(5):
    cal.run_ptrs(rp, op)
    C.convert_u16_f32(rp, op, src.spec.npix, s)
torch.cuda.synchronize()
print("done")
