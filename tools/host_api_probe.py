#!/usr/bin/env python3
"""Host-side cost of the HIP calls the producer engine makes per chunk, with and without pending
cross-stream work: does hipStreamWaitEvent / a kernel launch / hipEventQuery block the calling
thread while the awaited event is still pending on another stream?

    python tools/host_api_probe.py
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psana_ray_amd.config import CommonModeParams  # noqa: E402
from psana_ray_amd.models import Calibrator, Mode  # noqa: E402
from psana_ray_amd.ops import _ext  # noqa: E402
from psana_ray_amd.source import SyntheticRun  # noqa: E402


def main():
    C = _ext.load()
    dev = torch.device("cuda:0")
    F = 64
    src = SyntheticRun("synthetic", 0, "epix10k2M", pool_frames=8, pinned=False, gen_device="cuda")
    pool = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16).to(dev)
    raw = pool.repeat(F // 8, 1, 1, 1).contiguous()
    out = torch.empty((F, *src.spec.frame_shape), dtype=torch.float32, device=dev)
    rp = [int(raw[i].data_ptr()) for i in range(F)]
    op = [int(out[i].data_ptr()) for i in range(F)]
    cm = CommonModeParams()
    cal = Calibrator(src.consts, dev, Mode.calib, common_mode=cm)
    p, spec = cal.plan, src.spec
    A, B = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)

    def launch(st):
        C.calib_cm(rp, op, p.ped, p.gf, p.elig, spec.kernel_kind, spec.n_panels, spec.panel_rows,
                   spec.panel_cols, spec.asic_rows, spec.asic_cols, float(cm.thr), float(cm.maxcorr),
                   int(cm.npix_min), 3, int(p.bank_cols), int(st.cuda_stream))

    def us(f):
        t = time.perf_counter()
        f()
        return (time.perf_counter() - t) * 1e6

    for _ in range(3):
        launch(A)
    torch.cuda.synchronize()
    res = {}
    for rnd in range(5):
        r = {}
        # idle device
        r["launch_idle"] = us(lambda: launch(A))
        torch.cuda.synchronize()
        ev = torch.cuda.Event()
        ev.record(B)
        torch.cuda.synchronize()
        r["wait_done_event"] = us(lambda: A.wait_event(ev))
        # B busy for ~10 launches; A waits on B's event, then launches
        for _ in range(10):
            launch(B)
        eb = torch.cuda.Event()
        eb.record(B)
        r["query_pending"] = us(lambda: eb.query())
        r["wait_pending_event"] = us(lambda: A.wait_event(eb))
        r["launch_behind_pending_wait"] = us(lambda: launch(A))
        r["record_behind_pending_wait"] = us(lambda: torch.cuda.Event().record(A))
        r["launch_other_stream_busy"] = us(lambda: launch(B))
        t = time.perf_counter()
        torch.cuda.synchronize()
        r["sync_after_us"] = (time.perf_counter() - t) * 1e6
        for k, v in r.items():
            res.setdefault(k, []).append(round(v, 1))
    print(json.dumps({k: sorted(v)[len(v) // 2] for k, v in res.items()}))
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
