"""Consumer process for the elastic-queue tests: reads frames with DataReader.lease() until the end
of the stream, checks every frame against the fp32 golden calibration of the synthetic run, and
appends one JSON line per frame to --out (flushed, so a consumer killed mid-stream leaves its
record).  --die_after N: SIGKILL itself after N frames (fault injection, no goodbye)."""
import argparse
import json
import os
import signal
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--address", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--queue_name", default="my")
    ap.add_argument("--namespace", default="default")
    ap.add_argument("--slots", type=int, default=None)
    ap.add_argument("--prefetch", type=int, default=None)
    ap.add_argument("--die_after", type=int, default=-1)
    ap.add_argument("--stop_after", type=int, default=-1,
                    help="leave normally (DataReader.close) after N frames: unread frames go back to the queue")
    ap.add_argument("--sleep", type=float, default=0.0, help="seconds per frame (a slow consumer)")
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--verify", default="synthetic:2:tiny_epix:1", help="exp:run:detector:n_producers")
    ap.add_argument("--timeout", type=float, default=60.0)
    ap.add_argument("--gen_device", default="cpu", help="device the producer generated its synthetic pool on")
    ap.add_argument("--mode", default="calib", choices=["calib", "image"], help="the producer's retrieval mode")
    a = ap.parse_args()

    import numpy as np
    import torch

    from psana_ray_amd.config import resolve_common_mode
    from psana_ray_amd.data_reader import DataReader, EndOfStream
    from psana_ray_amd.ops import reference
    from psana_ray_amd.source import SyntheticRun

    exp, run, det, size = a.verify.split(":")
    refs = {}

    def ref_frame(rank, idx):
        if rank not in refs:
            src = SyntheticRun(exp, int(run), det, rank=rank, size=int(size), pool_frames=32, gen_device=a.gen_device)
            # the producer CLI's default common mode (--common_mode auto: on for epix10ka)
            cm = resolve_common_mode("auto", src.consts.spec)
            ref = reference.calibrate_reference(torch.from_numpy(src.pool.astype(np.int32)), src.consts, None, cm)
            if a.mode == "image":
                from psana_ray_amd.models.geometry import make_geometry

                geo = make_geometry(src.consts.spec)
                ref = reference.assemble_reference(ref, geo.rows, geo.cols, geo.image_shape)
            refs[rank] = ref
        return refs[rank][idx % 32]

    out = open(a.out, "w", buffering=1)
    n = 0
    with DataReader(a.address, queue_name=a.queue_name, ray_namespace=a.namespace, device=a.device,
                    timeout_s=a.timeout, slots=a.slots, prefetch=a.prefetch) as r:
        out.write(json.dumps({"joined": r.consumer_id, "pid": os.getpid()}) + "\n")
        t0 = time.time()
        while True:
            try:
                it = r.lease(timeout=0.5)
            except EndOfStream:
                out.write(json.dumps({"eos": True, "t": time.time() - t0, "t_end": time.time()}) + "\n")
                break
            if it is None:
                continue
            ok = bool(torch.equal(it.data.cpu(), ref_frame(it.rank, it.idx)))
            rec = {"rank": it.rank, "idx": it.idx, "gevt": it.gevt, "ok": ok}
            it.release()
            out.write(json.dumps(rec) + "\n")
            n += 1
            if a.sleep:
                time.sleep(a.sleep)
            if a.die_after >= 0 and n >= a.die_after:
                out.flush()
                os.kill(os.getpid(), signal.SIGKILL)
            if a.stop_after >= 0 and n >= a.stop_after:
                if a.sleep:
                    time.sleep(0.5)   # let the read-ahead refill: close() must hand it back
                break
        ep = r.endpoint
    if a.stop_after >= 0 and ep is not None:
        st = ep.metrics()   # the counters as of the close (returns answered)
        out.write(json.dumps({"closed": True, **{k: st.get(k) for k in ("frames_returned", "frames_dropped")}}) + "\n")
    out.close()


if __name__ == "__main__":
    main()
