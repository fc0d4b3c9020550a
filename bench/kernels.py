#!/usr/bin/env python3
"""Per-kernel micro-benchmarks on one MI355X (epix10k2M unless --detector), with rooflines.

Times each HIP kernel over a batch of frames with HIP events (median of --iters) and reports
frames/s, effective HBM GB/s (algorithmic bytes: raw u16 in + f32 out, + f32 in for the peak
finder / assembly) and the fraction of the measured 6.29 TB/s HBM roof
(/opt/skills/guides/MI355X_MICROARCH.md:36).  Also times the pinned host -> HBM copy.
Writes one JSON line per kernel (and to --json-out).
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np
import torch

from psana_ray_amd.config import CommonModeParams, PeakFinderParams
from psana_ray_amd.models import Calibrator, Mode
from psana_ray_amd.ops import _ext, kernels
from psana_ray_amd.source import SyntheticRun

HBM_ROOF = 6.29e12


def timeit(fn, iters=20, warmup=5, reps=8):
    """Median/min GPU seconds of one ``fn()``.

    ``fn`` is captured ``reps`` times into a HIP graph and the graph is replayed between events, so
    the number is device time only (the Python wrappers' argument validation costs more host time
    than some of these kernels take on the GPU; eager event timing would measure the host).
    Falls back to eager timing when capture is impossible."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    g = None
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001 - report and time eagerly
        print(json.dumps({"warning": f"graph capture failed ({e}); eager timing"}), flush=True)
        g, reps = None, 1
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        if g is not None:
            g.replay()
        else:
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3 / reps)
    return statistics.median(ts), min(ts)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--detector", default="epix10k2M")
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--only", default=None, help="comma list of kernels to run")
    a = ap.parse_args(argv)
    dev = torch.device("cuda:0")
    F = a.frames
    src = SyntheticRun("synthetic", 0, a.detector, pool_frames=min(F, 16), pinned=True, gen_device="cuda")
    spec = src.spec
    pool = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16)
    raw = pool.to(dev).repeat((F + pool.shape[0] - 1) // pool.shape[0], 1, 1, 1)[:F].contiguous()
    rl = [raw[i] for i in range(F)]
    out = torch.empty((F, *spec.frame_shape), dtype=torch.float32, device=dev)
    ol = [out[i] for i in range(F)]
    npix = spec.npix
    results = []
    only = set(a.only.split(",")) if a.only else None

    def report(name, t, nbytes, extra=None):
        med, best = t
        r = {"kernel": name, "detector": spec.name, "frames": F, "ms_median": round(med * 1e3, 4),
             "us_per_frame": round(med * 1e6 / F, 3), "frames_per_s": round(F / med, 1),
             "GB_per_s": round(nbytes / med / 1e9, 1), "hbm_roof_frac": round(nbytes / med / HBM_ROOF, 3)}
        if extra:
            r.update(extra)
        results.append(r)
        print(json.dumps(r), flush=True)

    def want(k):
        return only is None or k in only

    cal = Calibrator(src.consts, dev, Mode.calib)
    if want("calib_basic"):
        report("calib_basic", timeit(lambda: cal.run(rl, ol), a.iters), F * npix * 6)
    if want("calib_basic"):
        C = _ext.load()
        rp = [int(t.data_ptr()) for t in rl]
        op = [int(t.data_ptr()) for t in ol]
        report("convert_u16_f32 (bandwidth reference)",
               timeit(lambda: C.convert_u16_f32(rp, op, npix, _ext.stream_handle()), a.iters), F * npix * 6)
    if want("calib_cm") and spec.kind != "plain":
        for name, flags in (("rows+cols", 3), ("rows", 1), ("cols", 2), ("memory phases only", 0)):
            c = Calibrator(src.consts, dev, Mode.calib, common_mode=CommonModeParams(flags=flags))
            report(f"calib_cm({name})", timeit(lambda: c.run(rl, ol), a.iters), F * npix * 6)
    if want("calib_cm_image") and spec.kind != "plain":
        # image mode with common mode: the CM kernel writes the assembled image from LDS + gap fill
        c = Calibrator(src.consts, dev, Mode.image, common_mode=CommonModeParams())
        img = torch.empty((F, *c.out_shape), dtype=torch.float32, device=dev)
        il = [img[i] for i in range(F)]
        report("calib_cm_image(fused)", timeit(lambda: c.run(rl, il), a.iters), F * npix * 2 + img.numel() * 4)
    if want("calib_image") and spec.kind != "plain":
        C = _ext.load()
        cali = Calibrator(src.consts, dev, Mode.image)
        tm = cali.tile_map
        img = torch.empty((F, *cali.out_shape), dtype=torch.float32, device=dev)
        il = [img[i] for i in range(F)]
        nout = int(np.prod(cali.out_shape))
        op = [int(t.data_ptr()) for t in ol]
        ip = [int(t.data_ptr()) for t in il]
        extra = {"image_shape": list(cali.out_shape),
                 "tile_direct_frac": round(tm.direct_px / max(1, tm.staged_px + tm.direct_px), 4)}
        report("calib_image(fused, tiles)", timeit(lambda: cali.run(rl, il), a.iters), F * (npix * 2 + nout * 4), extra)
        report("assemble(index map)", timeit(lambda: kernels.assemble(ol, il, cali.idx, npix), a.iters),
               F * (npix * 4 + nout * 4))
        report("assemble(tiles)",
               timeit(lambda: C.image_tiles(op, ip, False, spec.kernel_kind, 0, 0, npix, spec.panel_rows,
                                            spec.panel_cols, int(cali._tiles.data_ptr()), tm.n_tiles, tm.tiles_x,
                                            int(cali._codes.data_ptr()), tm.image_shape[0], tm.image_shape[1],
                                            _ext.stream_handle()), a.iters),
               F * (npix * 4 + nout * 4))
    if want("peakfind"):
        cal.run(rl, ol)
        p = PeakFinderParams()
        peaks = torch.empty((F, p.max_peaks, 8), dtype=torch.float32, device=dev)
        counts = torch.zeros(F, dtype=torch.int32, device=dev)
        summ = torch.zeros((F, 2), dtype=torch.float32, device=dev)
        C = _ext.load()
        sums = torch.zeros(F, dtype=torch.float32, device=dev)
        op = [int(t.data_ptr()) for t in ol]
        report("read_f32 reference (K=16)",
               timeit(lambda: C.read_f32(op, npix, 16, False, int(sums.data_ptr()), _ext.stream_handle()), a.iters),
               F * npix * 4)
        report("peakfind", timeit(lambda: kernels.peakfind(ol, spec.frame_shape, p, peaks, counts, summ), a.iters),
               F * npix * 4, {"peaks_per_frame": float(counts.float().mean())})
    if want("h2d"):
        C = _ext.load()
        hp = src.pool
        n = hp.shape[0]

        def h2d():
            C.memcpy_h2d_batch([int(raw[i].data_ptr()) for i in range(F)],
                               [int(hp[i % n].ctypes.data) for i in range(F)], spec.raw_frame_bytes, _ext.stream_handle())
        med, best = timeit(h2d, a.iters)
        r = {"kernel": "h2d_pinned", "detector": spec.name, "frames": F, "ms_median": round(med * 1e3, 4),
             "frames_per_s": round(F / med, 1), "GB_per_s": round(F * spec.raw_frame_bytes / med / 1e9, 1)}
        results.append(r)
        print(json.dumps(r), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            for r in results:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
