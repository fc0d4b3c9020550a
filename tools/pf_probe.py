#!/usr/bin/env python3
"""Peak-finder probe: device time per epix10k2M frame of the shipped peak finder on 32 (or
--frames) calibrated frames (graph-replayed, event-timed), repeated --repeat times with the record
count checked against the first launch.

    python tools/pf_probe.py --repeat 2
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psana_ray_amd.config import PeakFinderParams  # noqa: E402
from psana_ray_amd.models import Calibrator, Mode  # noqa: E402
from psana_ray_amd.ops import _ext, kernels  # noqa: E402
from psana_ray_amd.source import SyntheticRun  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--thr", type=float, default=None, help="thr_peak (default: PeakFinderParams)")
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--total", action="store_true", help="bump a running peak total (as the pipeline consumer does)")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    C = _ext.load()
    dev = torch.device("cuda:0")
    F = a.frames
    src = SyntheticRun("synthetic", 0, "epix10k2M", pool_frames=8, pinned=False, gen_device="cuda")
    cal = Calibrator(src.consts, dev, Mode.calib)
    raw = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16).to(dev)
    frames = [cal(raw[i % raw.shape[0]]).contiguous() for i in range(F)]
    # every buffer distinct and cold-ish: 32 x 8.65 MB
    frames = [f.clone() for f in frames]
    pp = PeakFinderParams() if a.thr is None else PeakFinderParams(thr_peak=a.thr)
    P, H, W = src.spec.frame_shape
    peaks = torch.zeros((F, pp.max_peaks, 8), dtype=torch.float32, device=dev)
    counts = torch.zeros(F, dtype=torch.int32, device=dev)
    summary = torch.zeros((F, 2), dtype=torch.float32, device=dev)
    scratch = torch.zeros(kernels.PF_SCRATCH_WORDS, dtype=torch.int32, device=dev)
    total = torch.zeros((), dtype=torch.int64, device=dev)
    total_ptr = int(total.data_ptr()) if a.total else 0
    ptrs = [int(f.data_ptr()) for f in frames]

    def launch(var):
        C.peakfind(ptrs, P, H, W, float(pp.thr_peak), float(pp.son_min), int(pp.radius),
                   int(pp.max_peaks), int(peaks.data_ptr()), int(counts.data_ptr()), int(summary.data_ptr()),
                   _ext.stream_handle(), total_ptr, int(scratch.data_ptr()))

    launch(0)
    torch.cuda.synchronize()
    ref_counts, ref_sum = counts.clone(), summary.clone()
    for var in range(a.repeat):
        launch(var)
        torch.cuda.synchronize()
        same = bool(torch.equal(counts, ref_counts)) and bool(torch.allclose(summary, ref_sum, rtol=1e-5))
        for _ in range(3):
            launch(var)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(8):
                launch(var)
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(15):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 8)
        ts.sort()
        above = float(ref_sum[0, 0])
        res = {"run": var, "frames": F, "same_counts": same, "peaks_frame0": int(ref_counts[0]),
               "thr_peak": float(pp.thr_peak), "above_thr_frame0": int(above),
               "candidate_density": round(above / float(P * H * W), 5),
               "us_per_frame": round(1e3 * ts[len(ts) // 2] / F, 3)}
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "a") as f:
                f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
