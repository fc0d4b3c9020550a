#!/usr/bin/env python3
"""Common-mode kernel probe: device time of calib_cm on 32 epix10k2M frames for each phase mix
(flags 0 = decode/pedestal/gain/store only, 1 = + row medians, 2 = + column medians, 3 = both),
graph-replayed and event-timed.  Under ``rocprofv3 --pmc SQ_INSTS_VALU ...`` the dispatches run in
the order flags 0,1,2,3 (``--pmc-pass``: each flag value launched 3 times, no graphs), so per-phase
VALU / LDS instruction counts can be read off the counter CSV.

    python tools/cm_probe.py [--pmc-pass] [--mode image] [--no-gaps]

``--mode image``: the same kernel writing the assembled image (fused K-05 placement, the plan's
gap table unless ``--no-gaps`` -- the producer's zero-filled HBM ring launches without it).
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psana_ray_amd.config import CommonModeParams  # noqa: E402
from psana_ray_amd.models import Calibrator, Mode  # noqa: E402
from psana_ray_amd.ops import _ext, reference  # noqa: E402
from psana_ray_amd.source import SyntheticRun  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pmc-pass", action="store_true")
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--detector", default="epix10k2M")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--repeat", type=int, default=1, help="timing rounds (one JSON line each)")
    ap.add_argument("--mode", default="calib", choices=["calib", "image"])
    ap.add_argument("--no-gaps", action="store_true", help="image mode: no gap fill (ring launches)")
    a = ap.parse_args()
    C = _ext.load()
    dev = torch.device("cuda:0")
    F = a.frames
    src = SyntheticRun("synthetic", 0, a.detector, pool_frames=8, pinned=False, gen_device="cuda")
    pool = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16).to(dev)
    raw = pool.repeat((F + 7) // 8, 1, 1, 1)[:F].contiguous()
    cm = CommonModeParams()
    image = a.mode == "image"
    cal = Calibrator(src.consts, dev, Mode.image if image else Mode.calib, common_mode=cm)
    out = torch.empty((F, *cal.out_shape), dtype=torch.float32, device=dev)
    rp = [int(raw[i].data_ptr()) for i in range(F)]
    op = [int(out[i].data_ptr()) for i in range(F)]
    p = cal.plan
    spec = src.spec
    if image and a.no_gaps:
        out.zero_()
        p.n_gap_runs = 0
    def launch(flags):
        # the stream is read at call time: under graph capture it is the capture stream
        if image:
            p.cm_flags = int(flags)
            C.run_calib_plan(p, rp, op, _ext.stream_handle())
            return
        C.calib_cm(rp, op, p.ped, p.gf, p.elig, spec.kernel_kind, spec.n_panels, spec.panel_rows,
                   spec.panel_cols, spec.asic_rows, spec.asic_cols, float(cm.thr), float(cm.maxcorr),
                   int(cm.npix_min), int(flags), int(p.bank_cols), _ext.stream_handle(), p.ped_sg)

    # correctness of the full kernel against the golden model (1 frame)
    launch(3)
    torch.cuda.synchronize()
    ref = reference.calibrate_reference(torch.from_numpy(src.pool[:1].astype(np.int32)), src.consts, None, cal.cm)
    if image:
        g = cal.geometry
        ref = reference.assemble_reference(ref, g.rows, g.cols, g.image_shape, None)
    exact = bool(torch.equal(out[0].cpu().view(-1), ref[0].reshape(-1)))
    if a.pmc_pass:
        for flags in (0, 1, 2, 3):
            for _ in range(3):
                launch(flags)
        torch.cuda.synchronize()
        print(json.dumps({"pmc_pass": True, "exact": exact}))
        return 0
    for rnd in range(a.repeat):
        res = measure(launch, F, rnd, exact)
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "a") as f:
                f.write(line + "\n")
    return 0


def measure(launch, F, rnd, exact):
    res = {"round": rnd, "exact_vs_golden": exact, "frames": F}
    for flags in (0, 1, 2, 3):
        for _ in range(3):
            launch(flags)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(8):
                launch(flags)
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
        res[f"us_per_frame_flags{flags}"] = round(1e3 * ts[len(ts) // 2] / F, 3)
    return res


if __name__ == "__main__":
    sys.exit(main())
