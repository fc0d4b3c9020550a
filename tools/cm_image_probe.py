#!/usr/bin/env python3
"""Fused common-mode -> image kernel vs panel alignment in the image: times calib_cm in image mode
for epix10k2M quad geometries with different panel gaps (10 px: panel runs start at arbitrary
4-B offsets; 16 px: every run starts 64-B aligned) against frame mode.

    python tools/cm_image_probe.py
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psana_ray_amd.config import CommonModeParams  # noqa: E402
from psana_ray_amd.models import Calibrator, Mode  # noqa: E402
from psana_ray_amd.models.geometry import Geometry, _epix_quads, _panel_grid  # noqa: E402
from psana_ray_amd.source import SyntheticRun  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "bench"))
from kernels import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    F = 32
    src = SyntheticRun("synthetic", 0, "epix10k2M", pool_frames=8, pinned=False, gen_device="cuda")
    spec = src.spec
    pool = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16).to(dev)
    raw = pool.repeat(4, 1, 1, 1)[:F].contiguous()
    rl = [raw[i] for i in range(F)]
    res = {}
    cal = Calibrator(src.consts, dev, Mode.calib, common_mode=CommonModeParams())
    out = torch.empty((F, *cal.out_shape), dtype=torch.float32, device=dev)
    res["frame_us"] = round(timeit(lambda: cal.run(rl, [out[i] for i in range(F)]))[0] * 1e6 / F, 3)
    layouts = [("quads_gap10", lambda: _epix_quads(spec, 10)), ("quads_gap16", lambda: _epix_quads(spec, 16)),
               ("grid_unrotated_gap16", lambda: _panel_grid(spec, 16))]
    for gap, make in layouts:
        rows, cols, shape = make()
        geo = Geometry(spec, tuple(int(s) for s in shape), rows, cols)
        place = geo.panel_placement().reshape(-1, 3)
        c = Calibrator(src.consts, dev, Mode.image, common_mode=CommonModeParams(), geometry=geo)
        img = torch.empty((F, *c.out_shape), dtype=torch.float32, device=dev)
        il = [img[i] for i in range(F)]
        res[f"image_gap{gap}_us"] = round(timeit(lambda: c.run(rl, il))[0] * 1e6 / F, 3)
        res[f"image_gap{gap}_base_mod16"] = sorted(set((place[:, 0] % 16).tolist()))
        res[f"image_gap{gap}_shape"] = list(shape)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
