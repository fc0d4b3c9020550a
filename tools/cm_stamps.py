#!/usr/bin/env python3
"""Phase stamps of the epix10k2M common-mode kernel (diagnostic build only).

Needs an extension built with -DPR_CM_STAMPS=1:
    python tools/build_variant.py stamps common_mode.hip -DPR_CM_STAMPS=1
and run with that .so in place of the shipped one (tools/gpu_stamps.sh does both steps on the box).

Every wave of the production kernel records the shader clock at its phase boundaries; this tool
launches one 64-frame dispatch per flag mix (after warm-up launches) and reports, per phase, the
median / p90 duration over waves, split by wave index (wave 3 has no median work), the workgroup
lifetime and how many workgroups were resident over the dispatch (real-time clock).

    python tools/cm_stamps.py [--frames 64] [--json-out FILE]
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

WORDS = 16
# shader-clock stamp k sits in word 4 + k
PHASES = [
    ("p0_load_decode", 0, 1),
    ("bar1", 1, 2),
    ("rows", 2, 3),
    ("bar2", 3, 4),
    ("cols", 4, 5),
    ("bar3", 5, 6),
    ("p3_gain_out", 6, 7),
    ("flush(bar+stores)", 7, 8),
    ("  out_barrier", 7, 9),
    ("  place_or_flush", 9, 8),
    ("  place", 9, 10),
    ("  gaps", 10, 8),
]


def analyse(rec, nwaves, sclk_ghz):
    w = rec.reshape(-1, nwaves, WORDS)
    out = {}
    st = w[:, :, 4:].astype(np.int64)
    for name, a, b in PHASES:
        if not (st[:, :, a].any() and st[:, :, b].any()):
            continue   # phase not run (flags 0: no median phases)
        d = (st[:, :, b] - st[:, :, a]) / (sclk_ghz * 1e3)   # us
        row = {}
        for wi in range(nwaves):
            x = d[:, wi]
            row[f"w{wi}"] = [round(float(np.median(x)), 3), round(float(np.percentile(x, 90)), 3)]
        out[name] = row
    life_sclk = (st[:, :, 8] - st[:, :, 0]) / (sclk_ghz * 1e3)
    out["lifetime_sclk_us"] = [round(float(np.median(life_sclk)), 3), round(float(np.percentile(life_sclk, 90)), 3)]
    rt0 = w[:, 0, 0].astype(np.int64)
    rt1 = w[:, :, 1].max(axis=1).astype(np.int64)
    t0 = rt0.min()
    life = (rt1 - rt0) / 100.0   # 100 MHz -> us
    out["lifetime_rt_us"] = [round(float(np.median(life)), 3), round(float(np.percentile(life, 90)), 3)]
    span = (rt1.max() - t0) / 100.0
    out["dispatch_span_us"] = round(float(span), 2)
    # resident workgroups over time (10-ns bins)
    ev = np.zeros(int(rt1.max() - t0) + 2, dtype=np.int64)
    np.add.at(ev, rt0 - t0, 1)
    np.add.at(ev, rt1 - t0, -1)
    live = np.cumsum(ev)
    out["resident_wg_median_max"] = [int(np.median(live[: len(live) - 1])), int(live.max())]
    hw = w[:, :, 2].astype(np.int64)
    xcc = w[:, :, 3].astype(np.int64) & 0xF
    out["xcc_histogram"] = np.bincount(xcc[:, 0], minlength=8).tolist()
    # shader clock vs real time over the workgroups (sanity of sclk_ghz)
    rts = (w[:, 0, 1].astype(np.int64) - w[:, 0, 0].astype(np.int64)) / 100.0
    scl = (st[:, 0, 8] - st[:, 0, 0]) / 1e3
    ok = rts > 1.0
    out["sclk_ghz_est"] = round(float(np.median(scl[ok] / rts[ok])), 3) if ok.any() else None
    out["simd_of_wave0"] = np.bincount((hw[:, 0] >> 4) & 3, minlength=4).tolist()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--sclk-ghz", type=float, default=0.0, help="0: estimate from the real-time clock")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    C = _ext.load()
    dev = torch.device("cuda:0")
    F = a.frames
    src = SyntheticRun("synthetic", 0, "epix10k2M", pool_frames=8, pinned=False, gen_device="cuda")
    pool = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16).to(dev)
    raw = pool.repeat((F + 7) // 8, 1, 1, 1)[:F].contiguous()
    out = torch.empty((F, *src.spec.frame_shape), dtype=torch.float32, device=dev)
    rp = [int(raw[i].data_ptr()) for i in range(F)]
    op = [int(out[i].data_ptr()) for i in range(F)]
    cm = CommonModeParams()
    cal = Calibrator(src.consts, dev, Mode.calib, common_mode=cm)
    p = cal.plan
    spec = src.spec
    ntiles = spec.n_panels * (spec.panel_rows // spec.asic_rows) * (spec.panel_cols // 48)
    nwaves = 4
    buf = torch.zeros(ntiles * F * nwaves * WORDS, dtype=torch.int64, device=dev)

    def launch(flags):
        C.calib_cm(rp, op, p.ped, p.gf, p.elig, spec.kernel_kind, spec.n_panels, spec.panel_rows,
                   spec.panel_cols, spec.asic_rows, spec.asic_cols, float(cm.thr), float(cm.maxcorr),
                   int(cm.npix_min), int(flags), int(p.bank_cols), _ext.stream_handle(), p.ped_sg)

    res = {"frames": F, "tiles": ntiles}
    # image mode (production geometry): the same kernel placing the tile into the assembled image
    cal_img = Calibrator(src.consts, dev, Mode.image, common_mode=cm)
    img = torch.empty((F, *cal_img.out_shape), dtype=torch.float32, device=dev)
    rl, il = [raw[i] for i in range(F)], [img[i] for i in range(F)]
    runs = [(3, launch), (0, launch), ("image", lambda _f: cal_img.run(rl, il)), (3, launch)]
    for flags, fn in runs:
        C.cm_set_stamp_buffer(0)
        for _ in range(5):
            fn(flags)
        torch.cuda.synchronize()
        C.cm_set_stamp_buffer(int(buf.data_ptr()))
        buf.zero_()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        fn(flags)
        ev1.record()
        torch.cuda.synchronize()
        C.cm_set_stamp_buffer(0)
        rec = buf.cpu().numpy().view(np.uint64)
        r = {"event_us_per_frame": round(ev0.elapsed_time(ev1) * 1e3 / F, 3)}
        first = analyse(rec, nwaves, 2.4)
        ghz = a.sclk_ghz or first.get("sclk_ghz_est") or 2.4
        r.update(analyse(rec, nwaves, ghz))
        r["sclk_ghz_used"] = ghz
        key = f"flags{flags}" if flags != "image" else "image_flags3"
        key += "_again" if key in res else ""
        res[key] = r
        print(json.dumps({key: r}), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
