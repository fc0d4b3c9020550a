#!/usr/bin/env python3
"""Producer PROCESS -> consumer PROCESS throughput through the elastic queue fabric on one GPU.

The producer CLI (epix10k2M, calib + common mode, pinned host source, copy kernel staging) runs as
its own process on cuda:0; this script joins the same queue as a DataReader on cuda:0 and drains
it with zero-copy batch leases.  Every frame crosses the process boundary as a HIP IPC peer copy
(hipMemcpyAsync device->device into the consumer's ring) -- the data path of a cross-GPU link,
except that on one GPU the copy stays inside HBM instead of crossing xGMI.  Reports the
steady-state frames/s between the first and last 10 % of the frames, to compare with the
single-process pipeline (bench.py, zero-copy local route).

    python bench/fabric_ipc.py --frames 4000
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--frames", type=int, default=4000)
    ap.add_argument("--detector", default="epix10k2M")
    ap.add_argument("--queue_size", type=int, default=400)
    ap.add_argument("--slots", type=int, default=256, help="consumer shard slots")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--log-dir", default=None, help="write the producer's log here")
    a = ap.parse_args(argv)
    import torch

    from psana_ray_amd.data_reader import DataReader
    from psana_ray_amd.queue import EndOfStream

    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT)
    server = subprocess.Popen([sys.executable, "-m", "psana_ray_amd.server", "--host", "127.0.0.1", "--port", str(port),
                               "--log_level", "WARNING"], env=env)
    prod = None
    try:
        t0 = time.time()
        while time.time() - t0 < 30:
            with socket.socket() as s:
                if s.connect_ex(("127.0.0.1", port)) == 0:
                    break
            time.sleep(0.1)
        prod = subprocess.Popen([sys.executable, "-m", "psana_ray_amd.producer", "--exp", "synthetic", "--run", "0",
                                 "--detector_name", a.detector, "--calib", "--common_mode", "default", "--num_events",
                                 str(a.frames), "--queue_size", str(a.queue_size), "--device", "cuda:0",
                                 "--ray_address", f"127.0.0.1:{port}", "--timeout", "120", "--metrics_interval", "0",
                                 "--log_level", "INFO"], env=env,
                                stdout=open(os.path.join(a.log_dir, "producer.log"), "w") if a.log_dir else None,
                                stderr=subprocess.STDOUT if a.log_dir else None)
        stamps = []
        with DataReader(f"127.0.0.1:{port}", device="cuda:0", timeout_s=120, slots=a.slots) as r:
            ep = r.endpoint
            stream = torch.cuda.Stream()
            n = 0
            t_last, n_last, t_print = time.time(), 0, time.time()
            while True:
                try:
                    slots = ep.get_batch(a.batch, 0.05, stream)
                except EndOfStream:
                    break
                if slots:
                    ep.release_batch(slots, stream)
                    n += len(slots)
                    stamps.append((time.perf_counter(), n))
                now = time.time()
                if now - t_print > 5:
                    print(f"fabric_ipc: {n} frames, links {[(x.peer, x.attached, x.eos, x.outstanding) for x in ep.links()]}, "
                          f"stats {ep.metrics()}", flush=True)
                    t_print = now
                if n != n_last:
                    t_last, n_last = now, n
                elif now - t_last > 60:
                    print(f"fabric_ipc: STALLED at {n} frames: {ep.stats()}", flush=True)
                    break
            stream.synchronize()
            st = ep.stats()
        rc = prod.wait(120)
    finally:
        if prod is not None and prod.poll() is None:
            prod.kill()
        server.terminate()
    lo, hi = int(0.1 * n), int(0.9 * n)
    w = [(t, k) for t, k in stamps if lo <= k <= hi]
    rate = (w[-1][1] - w[0][1]) / (w[-1][0] - w[0][0]) if len(w) > 1 else float("nan")
    frame_bytes = st.get("bytes_recv", 0) / max(1, st.get("frames_recv", 1))
    out = {"bench": "fabric_ipc_same_gpu", "frames": n, "producer_rc": rc, "frames_per_s": round(rate, 1),
           "GB_per_s_ipc": round(rate * frame_bytes / 1e9, 2), "frames_recv": st.get("frames_recv"),
           "grants_given": st.get("grants_given"), "detector": a.detector,
           "note": "producer and consumer are separate processes on cuda:0; frames move by HIP IPC D2D copies "
                   "inside HBM (the cross-GPU path minus xGMI)"}
    line = json.dumps(out)
    print(line)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")
    return 0 if (rc == 0 and n == a.frames) else 1


if __name__ == "__main__":
    sys.exit(main())
