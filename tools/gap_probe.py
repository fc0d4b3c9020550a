#!/usr/bin/env python3
"""Launch-gap probe: what separates two producer chunks on the device?  64-frame epix10k2M
common-mode launches (production flags), 24 per variant, event-timed end to end:
  plain      back-to-back on one stream
  events2    + two timing-event records after every launch (a chunk's ready + completion events)
  events2nt  + two events without timing
  wait       + one stream wait on an event another stream recorded long ago (a slot-release wait)
  all        events2 + wait (the engine's per-chunk packet mix)
  two        launches alternate over two streams (no events)
  three      over three streams

    python tools/gap_probe.py [--frames 64] [--n 24]
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
from psana_ray_amd.ops import _ext  # noqa: E402
from psana_ray_amd.source import SyntheticRun  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--n", type=int, default=24)
    a = ap.parse_args()
    C = _ext.load()
    dev = torch.device("cuda:0")
    F = a.frames
    src = SyntheticRun("synthetic", 0, "epix10k2M", pool_frames=8, pinned=False, gen_device="cuda")
    pool = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16).to(dev)
    raw = pool.repeat((F + 7) // 8, 1, 1, 1)[:F].contiguous()
    outs = [torch.empty((F, *src.spec.frame_shape), dtype=torch.float32, device=dev) for _ in range(3)]
    rp = [int(raw[i].data_ptr()) for i in range(F)]
    cm = CommonModeParams()
    cal = Calibrator(src.consts, dev, Mode.calib, common_mode=cm)
    p, spec = cal.plan, src.spec
    streams = [torch.cuda.Stream(device=dev) for _ in range(3)]
    other = torch.cuda.Stream(device=dev)
    old = torch.cuda.Event()
    old.record(other)
    torch.cuda.synchronize()

    def launch(k, st):
        op = [int(outs[k % 3][i].data_ptr()) for i in range(F)]
        C.calib_cm(rp, op, p.ped, p.gf, p.elig, spec.kernel_kind, spec.n_panels, spec.panel_rows,
                   spec.panel_cols, spec.asic_rows, spec.asic_cols, float(cm.thr), float(cm.maxcorr),
                   int(cm.npix_min), 3, int(p.bank_cols), int(st.cuda_stream))

    def run(variant):
        ns = {"two": 2, "three": 3}.get(variant, 1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(streams[0])
        for st in streams[1:ns]:
            st.wait_event(e0)
        for k in range(a.n):
            st = streams[k % ns]
            if variant in ("wait", "all"):
                st.wait_event(old)
            launch(k, st)
            if variant in ("events2", "all"):
                torch.cuda.Event(enable_timing=True).record(st)
                torch.cuda.Event(enable_timing=True).record(st)
            elif variant == "events2nt":
                torch.cuda.Event().record(st)
                torch.cuda.Event().record(st)
        for st in streams[1:ns]:
            streams[0].wait_stream(st)
        e1.record(streams[0])
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.n   # us per launch

    for v in ("plain", "events2"):   # warm
        run(v)
    res = {"frames": F, "launches": a.n}
    for rnd in range(3):
        for v in ("plain", "events2", "events2nt", "wait", "all", "two", "three"):
            res.setdefault(v, []).append(round(run(v), 1))
    res = {k: (sorted(v)[1] if isinstance(v, list) else v) for k, v in res.items()}
    res["us_per_frame_plain"] = round(res["plain"] / F, 3)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
