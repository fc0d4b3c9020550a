#!/usr/bin/env python3
"""Flagship benchmark: detector frames/sec (whole node) through the shared queue, epix10k2M.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 it is launched by
``torch.distributed.run`` with one rank per GPU.  One STEP = every rank's consumer takes
``--batch`` frames out of the sharded shared queue and runs the on-GPU peak finder on them.
Behind it, every rank's producer streams raw epix10k2M frames from a pinned host pool through
hipMemcpyAsync (side stream) into HBM, calibrates them with the HIP kernels (pedestal + gain
switching + common mode + mask) directly into ring slots, and the transport routes them to the
consumer shards (RCCL send/recv over xGMI for N > 1, balanced routing).  W untimed warmup
steps, then exactly K timed steps bracketed by a barrier + device synchronisation; the time is
the MAX over ranks; rank 0 prints ONE JSON line.  ``value`` = total frames/s of the node.

Synthetic data: random-init calibration constants and a pre-generated pool of raw frames
(cycled), because no LCLS data / psana exists offline (BASELINE.json).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import threading
import time

METRIC = "detector frames/sec (whole node) through SharedQueue, epix10k2M at 1/2/4/8 GPUs"


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32, help="frames per rank per step (consumer batch)")
    ap.add_argument("--detector", default="epix10k2M")
    ap.add_argument("--mode", default="calib", choices=["calib", "image", "raw"])
    ap.add_argument("--common-mode", default="default", help="off | default | flags,thr,maxcorr,npix_min[,bank]")
    ap.add_argument("--consumer", default="peakfind", choices=["peakfind", "none"])
    ap.add_argument("--route", default="balanced", choices=["balanced", "local_first", "spread"])
    ap.add_argument("--queue-size", type=int, default=None,
                    help="logical (global) queue capacity; default 400 per GPU (README.md:20 example, weak scaling: "
                         "constant queue depth per consumer shard). BASELINE config 3: --gpus 8 --queue-size 400")
    ap.add_argument("--source", default="host", choices=["host", "device"],
                    help="host: pinned host pool + H2D (real pipeline); device: raw frames already in HBM")
    ap.add_argument("--chunk", type=int, default=32,
                    help="frames per producer kernel launch / H2D copy (32: 13.0k vs 16: 11.7k fr/s, profiles/bench_ab_r1.md)")
    ap.add_argument("--pool-frames", type=int, default=64)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--producers", type=int, default=0,
                    help="producer ranks P (ranks < P produce, every rank consumes; 0 = all).  BASELINE config 3: "
                         "--gpus 8 --producers 4")
    ap.add_argument("--hbm-fraction", type=float, default=0.8, help="cap of free HBM used for queue slots")
    ap.add_argument("--loopback", action="store_true",
                    help="N=1 only: route frames through the multi-GPU transport (gloo control round + RCCL "
                         "send/recv to self) instead of the zero-copy local route; exercises the N>1 data path")
    ap.add_argument("--copy-engine", default="blit", choices=["blit", "sdma"],
                    help="host->HBM staging copies: blit kernels (HSA_ENABLE_SDMA=0; 12.7k vs 12.2k fr/s on the same "
                         "box, profiles/bench_ab_r1.md) or the SDMA engines.  An HSA_ENABLE_SDMA already in the "
                         "environment wins")
    ap.add_argument("--transport", action="store_true",
                    help="N=1 only: run the multi-GPU transport rounds (control all-gather, routing) with frames "
                         "routed to this rank itself -- the per-rank steady state of N>1 weak scaling")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: protocol rehearsal with gloo and the golden models (tests only; not a benchmark)")
    return ap.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    from psana_ray_amd.utils.runtime_env import select_copy_engine

    select_copy_engine(args.copy_engine)   # before the HIP runtime initialises (first torch.cuda call)
    import numpy as np
    import torch
    import torch.distributed as dist

    from psana_ray_amd.config import CommonModeParams, PeakFinderParams
    from psana_ray_amd.models import Calibrator, Mode
    from psana_ray_amd.parallel.comm import init_groups
    from psana_ray_amd.parallel.launch import bind_numa_to_device, detect
    from psana_ray_amd.pipeline import PeakFinderConsumer, ProducerPipeline
    from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint
    from psana_ray_amd.queue.ring import physical_slots
    from psana_ray_amd.source import SyntheticRun

    sys.setswitchinterval(5e-4)   # short GIL hand-off: transport / consumer threads stay responsive
    li = detect()
    world, rank = li.size, li.rank
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print(f"bench.py: --gpus {args.gpus} needs a launcher (torch.distributed.run) with one rank per GPU",
                  file=sys.stderr)
            return 2
    if args.device == "cpu":
        device = torch.device("cpu")
        numa = None
    else:
        if not torch.cuda.is_available():
            print("bench.py needs a HIP device", file=sys.stderr)
            return 2
        device = torch.device(f"cuda:{li.local_rank % torch.cuda.device_count()}")
        torch.cuda.set_device(device)
        numa = bind_numa_to_device(device)
    gpu = device.type == "cuda"

    comm = None
    coord = None
    if world > 1:
        # single-node contract (rendezvous on 127.0.0.1): keep gloo's control traffic on loopback
        # instead of whatever interface the container hostname resolves to (or fails to)
        if os.environ.get("MASTER_ADDR", "127.0.0.1") in ("127.0.0.1", "localhost") and os.path.isdir("/sys/class/net/lo"):
            os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        comm = init_groups(rank, world, device)
        coord = dist.new_group(backend="gloo")
    elif args.loopback or args.transport:
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        comm = init_groups(0, 1, device, master_addr="127.0.0.1", master_port=port)

    def barrier():
        if coord is not None:
            dist.barrier(group=coord)

    mode = Mode(args.mode)
    cm = CommonModeParams.parse(args.common_mode) if mode != Mode.raw else None
    n_prod = args.producers or world
    if not 1 <= n_prod <= world:
        print(f"bench.py: --producers must be in [1, {world}]", file=sys.stderr)
        return 2
    is_prod = rank < n_prod
    # producers shard the run round-robin among themselves (P-01); consumer-only ranks need the
    # calibration constants (same seed) but no raw pool
    src = SyntheticRun("synthetic", 0, args.detector, rank=rank if is_prod else 0, size=n_prod,
                       pool_frames=args.pool_frames if is_prod else 1,
                       pinned=(args.source == "host" and gpu and is_prod), gen_device=str(device))
    cal = Calibrator(src.consts, device, mode, common_mode=cm)
    if args.queue_size is None:
        args.queue_size = 400 * world
    share = max(1, math.ceil(args.queue_size / world))
    # slack for frames waiting to be routed / in flight over xGMI (a round can hold max_offer frames)
    producer_slots = (4 * args.chunk + args.batch + (64 if comm is not None else 0)) if is_prod else 1
    # queue_size is the LOGICAL capacity (deque(maxlen), shared_queue.py:7); physical HBM slots are
    # capped by free memory (config 4: Jungfrau-16M x 400000 would need 26.8 TB)
    cslots = physical_slots(share, cal.out_frame_bytes, device, args.hbm_fraction, producer_slots)
    ring = FrameRing(cal.out_shape, cal.out_dtype, device, producer_slots, cslots)
    ep = QueueEndpoint(ring, rank, world, comm, producer_ranks=list(range(n_prod)), route=args.route, max_offer=64,
                       is_producer=is_prod, loopback=args.loopback)
    if args.source == "device":
        # raw pool resident in HBM: isolates the GPU pipeline from PCIe (secondary number)
        dev_pool = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16).to(device)

        class _DevSrc:
            spec = src.spec
            size = n_prod
            calibrated = False

            def __init__(self):
                self.k = 0

            def cycled_frames(self):
                return [int(dev_pool[j].data_ptr()) for j in range(dev_pool.shape[0])], \
                    [float(v) for v in src.pool_pe]

            def n_local_events(self):
                return None

            def next_events(self, n):
                from psana_ray_amd.source.synthetic import RawEvent
                out = []
                for _ in range(n):
                    j = self.k % dev_pool.shape[0]
                    out.append(RawEvent(rank + self.k * n_prod, self.k, dev_pool[j], int(dev_pool[j].data_ptr()), 9.5))
                    self.k += 1
                return out

        source = _DevSrc()
    else:
        source = src
    prod = ProducerPipeline(source, cal, ep, rank=rank, chunk=args.chunk) if is_prod else None
    consumer = PeakFinderConsumer(ep, cal.out_shape, PeakFinderParams(), batch=args.batch) \
        if args.consumer == "peakfind" else None

    stop = threading.Event()
    ep.start()
    pt = threading.Thread(target=prod.run if prod is not None else ep.finish, kwargs=dict(stop=stop) if prod else {},
                          name="producer", daemon=True)
    pt.start()

    def consume(n_frames):
        got = 0
        while got < n_frames:
            if consumer is not None:
                got += consumer.poll(timeout=0.05, max_items=n_frames - got)
            else:
                it = ep.get(timeout=0.05)
                if it is not None:
                    it.release()
                    got += 1
            if ep.failed is not None:
                raise RuntimeError(f"transport failed: {ep.failed!r}")
        return got

    def sync():
        if gpu:
            torch.cuda.synchronize(device)

    B = args.batch
    consume(args.warmup * B)
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    p0 = prod.produced if prod is not None else 0
    consume(args.steps * B)
    sync()
    t1 = time.perf_counter()
    p1 = prod.produced if prod is not None else 0
    barrier()
    dt = t1 - t0
    produced_window = p1 - p0
    if coord is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=coord)
        dt = float(t[0])
        pw = torch.tensor([produced_window], dtype=torch.int64)
        dist.all_reduce(pw, op=dist.ReduceOp.SUM, group=coord)
        produced_window = int(pw[0])
    stop.set()
    # drain until every producer's EOS arrived
    while True:
        try:
            if consumer is not None:
                consumer.poll(timeout=0.05)
            else:
                it = ep.get(timeout=0.05)
                if it is not None:
                    it.release()
        except EndOfStream:
            break
        if ep.failed is not None:
            break
    pt.join(timeout=60)
    ep.join(timeout=60)
    peaks = consumer.synchronize() if consumer is not None else 0
    total = world * args.steps * B
    # sustained throughput through the queue: frames can only leave as fast as they enter, so a
    # ring that was already (partly) full at t0 must not count -- report min(consumed, produced)
    value = min(total, produced_window) / dt
    st = ep.stats()
    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * dt / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "float32" if mode != Mode.raw else "uint16",
        "data": "synthetic (random-init calibration constants, pre-generated raw epix10k2M pool cycled "
                + ("from pinned host memory via hipMemcpyAsync)" if args.source == "host" and gpu
                   else "from HBM)" if gpu else "on the CPU; gloo protocol rehearsal, not a benchmark)"),
        "config": {
            "model": args.detector,
            "global_batch": world * B,
            "seq_len": None,
            "parallelism": f"dp{world}",
            "frame_shape": list(cal.out_shape),
            "mode": args.mode,
            "common_mode": args.common_mode,
            "consumer": args.consumer,
            "route": args.route,
            "queue_size": args.queue_size,
            "source": args.source,
            "chunk": args.chunk,
            "loopback": args.loopback,
            "transport": bool(args.transport or world > 1 or args.loopback),
            "producer_ranks": n_prod,
        },
        "extra": {
            "producer_frames_per_s_rank0": round((p1 - p0) / max(dt, 1e-9), 1),
            "consumed_frames_per_s": round(total / dt, 1),
            "produced_frames_per_s": round(produced_window / dt, 1),
            "frame_bytes": ring.frame_bytes,
            "queue_slots_physical_rank0": cslots,
            "ring_GB_rank0": round(ring.storage.numel() * ring.storage.element_size() / 1e9, 1),
            "GB_per_s_out": round(value * ring.frame_bytes / 1e9, 2),
            "peaks_found_rank0": peaks,
            "queue_full_waits_rank0": prod.full_waits if prod is not None else 0,
            "transport_rounds_rank0": st.get("rounds", 0),
            "transport_round_ms_rank0": round(st.get("round_ms", 0.0), 3),
            "transport_ctrl_ms_rank0": round(st.get("ctrl_ms", 0.0), 4),
            "transport_driver": ep.xport,
            "bytes_sent_rank0": st.get("bytes_sent", 0),
            "numa_node": numa,
            "copy_engine": "blit" if os.environ.get("HSA_ENABLE_SDMA") == "0" else "sdma",
            "cpus_allowed": len(os.sched_getaffinity(0)),
            "producer_host_s_stage_acquire_launch_commit_total": (
                [round(x, 4) for x in prod.engine.timing()] if prod is not None and prod.engine is not None
                else None),
            "producer_gpu_ms_h2d_chunks_calib_chunks": (
                [round(x, 3) for x in prod.engine.gpu_timing()]
                if prod is not None and prod.engine is not None and prod.engine.gpu_timing_enabled else None),
        },
    }
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    sys.stdout.flush()
    if comm is not None:
        # never let a communicator teardown hang the run after the result line
        clean = ep.failed is None and not pt.is_alive()
        wd = threading.Timer(60.0, lambda: os._exit(0 if clean else 3))
        wd.daemon = True
        wd.start()
        if clean:
            ep.close()
            comm.close()
            dist.destroy_process_group()
        else:
            comm.abort()
        wd.cancel()
        if not clean:
            os._exit(3)
    return 0


if __name__ == "__main__":
    sys.exit(main())
