#!/usr/bin/env python3
"""Flagship benchmark: detector frames/sec (whole node) through the shared queue, epix10k2M.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``.  For N > 1 it runs either
under a launcher (``torch.distributed.run`` / mpirun / Slurm: one rank per GPU) or, typed as is,
starts its N ranks itself as child processes before any GPU call (``self_launch``).  One STEP = every rank's consumer takes
``--batch`` frames out of its shard of the shared queue and runs the on-GPU peak finder on them.
Behind it, every producer rank streams raw epix10k2M frames from a pinned host pool into HBM
(our copy kernel on a side stream), calibrates them with the HIP kernels (pedestal + gain
switching + common mode + mask) directly into its ring slots, and the queue routes them to the
consumer shards.  A steady-state gate (untimed windows of ~0.25 s until two consecutive ones agree
within 3 % on every rank, bounded at 10 s; ``extra.steady_gate``), then W untimed warmup steps,
then exactly K timed steps bracketed by a barrier + device synchronisation; the time is the MAX
over ranks; rank 0 prints ONE JSON line (with every rank's GPU and fabric links, peer access and
xGMI link type / hops, under ``extra.topology``).  ``value``
= total frames/s of the node (headline phase: ``--route``, default balanced -- frames stay on the
GPU that produced them unless another shard is starving).

N > 1: every rank is a member of one queue session on torchrun's store and links to every other
rank through the elastic fabric (csrc/fabric.h).  After the headline window a SECOND fixed-step
window runs with ``route=remote_only`` (a producer never keeps a frame on its own GPU while a
consumer on another GPU is linked: every frame crosses xGMI as a HIP-IPC peer copy); its frames/s,
cross-GPU GB/s and bytes per rank are reported under ``extra.xgmi_phase`` (``--cross-steps 0``
skips it).  The run is self-validating: it exits non-zero (after printing its line) when a link
failed or never attached, when less than 90% of that window's frames crossed GPUs, or when a frame
arrived with contents that differ from what its producer sent (every 64th frame a producer sends
to another process carries a content checksum the consumer re-sums from its own ring,
``extra.frame_checks``; csrc/verify.h).

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
    from psana_ray_amd.config import CONSUMER_BATCH

    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None,
                    help=f"frames per rank per step (consumer batch; default {CONSUMER_BATCH}, 32 when ranks share a GPU)")
    ap.add_argument("--detector", default="epix10k2M")
    ap.add_argument("--mode", default="calib", choices=["calib", "image", "raw"])
    ap.add_argument("--common-mode", default="auto",
                    help="auto (the producer CLI's default: on for epix10ka) | off | default | "
                         "flags,thr,maxcorr,npix_min[,bank]")
    ap.add_argument("--consumer", default="peakfind", choices=["peakfind", "none"])
    ap.add_argument("--consumer-streams", type=int, default=None,
                    help="peak-finder consumer streams (default config.CONSUMER_STREAMS)")
    ap.add_argument("--gap-fill", action="store_true",
                    help="image mode: zero the panel gaps of every frame even in a zero-filled ring (A/B)")
    ap.add_argument("--route", default="balanced", choices=["balanced", "local_first", "spread", "remote_only"],
                    help="routing policy of the headline window")
    ap.add_argument("--cross-steps", type=int, default=None,
                    help="N > 1: steps of the second, route=remote_only window that pushes frames across GPUs over xGMI "
                         "(default: --steps; 0 skips it)")
    ap.add_argument("--queue-size", type=int, default=None,
                    help="logical (global) queue capacity; default 400 per GPU (README.md:20 example, weak scaling: "
                         "constant queue depth per consumer shard). BASELINE config 3: --gpus 8 --queue-size 400")
    ap.add_argument("--source", default="host", choices=["host", "device"],
                    help="host: pinned host pool + H2D (real pipeline); device: raw frames already in HBM")
    ap.add_argument("--chunk", type=int, default=64,
                    help="frames per producer kernel launch / H2D copy (device-resident: 64 134.0-139.0k vs "
                         "32 132.0-134.5k vs 16 119.9k fr/s; host-staged 13.03k vs 12.90k; profiles/r2/pipeline_chunks.md)")
    ap.add_argument("--pool-frames", type=int, default=64)
    ap.add_argument("--compute-streams", type=int, default=None,
                    help="producer chunks alternate over this many HIP streams (default: config.PRODUCER_STREAMS)")
    ap.add_argument("--stream-kind", default=None, choices=["shared", "dedicated", "high"],
                    help="hardware-queue placement of the producer streams (default: config.PRODUCER_STREAM_KIND)")
    ap.add_argument("--consumer-stream-kind", default=None, choices=["shared", "dedicated", "high"],
                    help="placement of the peak finder's streams (default: config.CONSUMER_STREAM_KIND)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--preroll-s", type=float, default=0.0,
                    help="fixed untimed streaming before the steady-state gate (the gate alone is the default)")
    ap.add_argument("--gate-tol", type=float, default=0.03,
                    help="steady-state gate: untimed windows of --gate-window-s until two consecutive ones agree within "
                         "this fraction on EVERY rank (then the --warmup steps, then the timed window); 0 disables")
    ap.add_argument("--gate-window-s", type=float, default=0.25, help="target length of one gate window")
    ap.add_argument("--gate-max-s", type=float, default=10.0, help="bound of the gate (the run goes on unconverged)")
    ap.add_argument("--producers", type=int, default=0,
                    help="producer ranks P (ranks < P produce, every rank consumes; 0 = all).  BASELINE config 3: "
                         "--gpus 8 --producers 4")
    ap.add_argument("--hbm-fraction", type=float, default=0.8, help="cap of free HBM used for queue slots")
    ap.add_argument("--copy-engine", default="blit", choices=["blit", "sdma"],
                    help="runtime copies (HBM->HBM peer copies of the cross-GPU window): blit kernels "
                         "(HSA_ENABLE_SDMA=0) or the SDMA engines.  An HSA_ENABLE_SDMA already in the environment wins")
    ap.add_argument("--fabric-copy", default=None, choices=["kernel", "runtime"],
                    help="N > 1: how producers move frames into other ranks' rings: one copy_runs_kernel launch per "
                         "fabric pass on its own hardware queue (default, config.FABRIC_COPY_ENGINE) or hipMemcpyAsync "
                         "per run on one ordinary stream per link (round-3 path)")
    ap.add_argument("--fabric-copy-stream", default=None, choices=["shared", "dedicated", "high"],
                    help="hardware-queue placement of the fabric copy stream (default config.FABRIC_COPY_STREAM)")
    ap.add_argument("--fabric-copy-wgs", type=int, default=None,
                    help="fabric copy kernel workgroups per peer GPU link (default config.FABRIC_COPY_WORKGROUPS)")
    ap.add_argument("--verify-every", type=int, default=None,
                    help="every N-th frame a producer sends to another process carries a content checksum its "
                         "consumer verifies (default config.FABRIC_VERIFY_EVERY = 64; 0 off; "
                         "$PSANA_RAY_AMD_VERIFY_EVERY)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: protocol rehearsal with gloo and the golden models (tests only; not a benchmark)")
    return ap.parse_args(argv)


def _wait_links(ep, n_members: int, expect_in: int, expect_out: int, timeout_s: float = 120.0) -> dict:
    """Wait until every member registered and every link of this rank attached.  A link whose
    consumer ring could not be mapped is dropped by the fabric (only that link); after
    ``timeout_s`` the run goes on with the links it has (the headline's balanced route keeps frames
    on their own GPU) and the result records what was missing."""
    t0 = time.time()
    while True:
        ls = ep.links()
        n_in = sum(1 for x in ls if not x.outgoing and x.attached)
        n_out = sum(1 for x in ls if x.outgoing and x.attached)
        n_fail = int(ep.metrics().get("links_failed", 0))
        members = len(ep.session.members) + 1
        if members == n_members and n_in >= expect_in and n_out + n_fail >= expect_out:
            return {"complete": n_fail == 0 and n_out >= expect_out, "in": n_in, "out": n_out, "failed": n_fail}
        if ep.failed is not None:
            raise RuntimeError(f"queue fabric failed while linking: {ep.failed}")
        if time.time() - t0 > timeout_s:
            print(f"bench.py: links incomplete after {timeout_s:.0f} s (members {members}/{n_members}, in "
                  f"{n_in}/{expect_in}, out {n_out}/{expect_out}, failed {n_fail}); going on without them",
                  file=sys.stderr, flush=True)
            return {"complete": False, "in": n_in, "out": n_out, "failed": n_fail}
        time.sleep(0.01)


def _topology(ep, device, allsum) -> dict:
    """Per-rank topology evidence for the result line: every rank's GPU and its
    outgoing fabric links (consumer GPU, copy engine, hipDeviceCanAccessPeer, hipExtGetLinkType-
    AndHopCount type / hops -- 4 = xGMI, hops 1 = a direct link), plus rank 0's view of the peer
    access / link-type / hop matrices of every visible GPU."""
    links = [{"peer": int(x.peer), "consumer_device": int(x.consumer_device), "attached": bool(x.attached),
              "kernel_copy": bool(getattr(x, "kernel_copy", False)), "peer_access": int(getattr(x, "peer_access", -1)),
              "link_type": int(getattr(x, "link_type", -1)), "hops": int(getattr(x, "hops", -1))}
             for x in ep.links() if x.outgoing]
    out = {"device_per_rank": allsum(device.index if device.type == "cuda" else -1),
           "outgoing_links_per_rank": allsum(links)}
    if device.type == "cuda":
        from psana_ray_amd.ops import _ext

        out["rank0_view"] = _ext.load().device_topology()
    return out


def _pct(v, q):
    if not v:
        return None
    v = sorted(v)
    return v[min(len(v) - 1, int(round(q * (len(v) - 1))))]


def _copy_stats(samples) -> dict:
    """p50 / p99 of a window's fabric copy dispatches (endpoint.copy_samples tuples)."""
    if not samples:
        return {"dispatches": 0}
    dev = [s[0] for s in samples]
    lat = [s[1] for s in samples]
    byts = sum(s[2] for s in samples)
    frames = [s[3] for s in samples]
    return {"dispatches": len(samples), "frames_per_dispatch_mean": round(sum(frames) / len(frames), 1),
            "dev_ms_p50": round(_pct(dev, 0.5), 4), "dev_ms_p99": round(_pct(dev, 0.99), 4),
            "dev_GB_per_s": round(byts / max(1e-9, sum(dev) * 1e-3) / 1e9, 1),
            "issue_to_done_ms_p50": round(_pct(lat, 0.5), 3), "issue_to_done_ms_p99": round(_pct(lat, 0.99), 3),
            "ms_per_64_frames_dev_p50": round(64 * _pct([d / max(1, f) for d, f in zip(dev, frames)], 0.5), 4)}


def resolve_shape(args, gpu: bool):
    """(ranks per GPU, consumer batch, producer compute streams) of this launch: explicit flags, else
    the library's resolution (pipeline.resolve_consumer_batch / resolve_producer_streams)."""
    from psana_ray_amd.parallel.launch import ranks_per_gpu
    from psana_ray_amd.pipeline import resolve_consumer_batch, resolve_producer_streams

    share = ranks_per_gpu() if gpu else 1
    where = "device" if args.source == "device" else "staged"
    return share, resolve_consumer_batch(args.batch, share), resolve_producer_streams(where, args.compute_streams, share)


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def self_launch(n: int, argv) -> int:
    """``python bench.py --gpus N`` with N > 1 and no launcher around it: start the N ranks here, as
    CHILD processes with the env a torchrun / mpirun launch gives them (RANK, WORLD_SIZE,
    LOCAL_RANK, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), one per GPU.  The reference's
    launch shape is the same (``mpirun -n 4 psana-ray-producer``, README.md:20; every rank reads
    its own rank and size, psana_ray/producer.py:138-140).

    This parent never touches the GPU (no torch.cuda call, no HIP runtime) and never execs: it
    waits for the children, forwards nothing itself (rank 0 prints the one JSON line on the
    inherited stdout), and returns the worst child exit code.  When one rank fails, the others are
    given 30 s to notice (their collectives fail) and are then killed by PID, so a lost rank cannot
    hang the job until gloo's 600-s timeout."""
    import signal
    import subprocess

    port = _free_port()
    script = os.path.abspath(__file__)
    procs = []

    def die_with_parent():   # in the child, before exec: a parent killed by its caller takes its ranks along
        try:
            import ctypes

            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGKILL)   # PR_SET_PDEATHSIG
        except Exception:
            pass

    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(n),
                    "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                    "PSANA_RAY_SELF_LAUNCHED": "1"})
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=env, stdout=subprocess.PIPE,
                                      text=True, bufsize=1, preexec_fn=die_with_parent))

    def on_signal(signo, frame):   # SIGTERM / SIGINT of the launcher: the ranks go too, then we do
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGKILL)
        sys.exit(128 + signo)

    signal.signal(signal.SIGTERM, on_signal)
    signal.signal(signal.SIGINT, on_signal)
    print(f"bench.py: self-launched {n} ranks (pids {[p.pid for p in procs]}, rendezvous 127.0.0.1:{port})",
          file=sys.stderr, flush=True)

    def forward(p):
        # the result line to stdout; everything else a rank writes there (gloo's "[Gloo] Rank r is
        # connected to ..." banner) to stderr, so stdout carries exactly ONE line
        for line in p.stdout:
            dst = sys.stdout if line.startswith("{") else sys.stderr
            dst.write(line)
            dst.flush()

    fwd = [threading.Thread(target=forward, args=(p,), daemon=True) for p in procs]
    for t in fwd:
        t.start()
    rcs = [None] * n
    first_fail = None
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
                if rcs[i] not in (None, 0) and first_fail is None:
                    first_fail = time.monotonic()
                    print(f"bench.py: rank {i} exited with {rcs[i]}", file=sys.stderr, flush=True)
        if first_fail is not None and time.monotonic() - first_fail > 30.0:
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.send_signal(signal.SIGKILL)
                    rcs[i] = p.wait()
                    print(f"bench.py: killed rank {i} (pid {p.pid}) after a peer failed", file=sys.stderr, flush=True)
        time.sleep(0.05)
    for t in fwd:
        t.join(timeout=10)
    bad = [rc for rc in rcs if rc != 0]
    if not bad:
        return 0
    # a signal death (negative rc) maps to 128 + signo, like a shell
    return max((128 - rc) if rc < 0 else rc for rc in bad)


def main(argv=None):
    args = parse(argv)
    from psana_ray_amd.parallel.launch import detect as _detect

    if args.gpus > 1 and _detect().launcher == "single":
        return self_launch(args.gpus, sys.argv[1:] if argv is None else list(argv))
    from psana_ray_amd.utils.runtime_env import select_copy_engine

    select_copy_engine(args.copy_engine)   # before the HIP runtime initialises (first torch.cuda call)
    if args.verify_every is not None:
        os.environ["PSANA_RAY_AMD_VERIFY_EVERY"] = str(max(0, args.verify_every))
    import numpy as np
    import torch
    import torch.distributed as dist

    from psana_ray_amd.config import CONSUMER_STREAM_KIND, PeakFinderParams
    from psana_ray_amd.models import Mode
    from psana_ray_amd.producer import build_calibrator
    from psana_ray_amd.parallel.launch import bind_numa_to_device, detect
    from psana_ray_amd.pipeline import PeakFinderConsumer, ProducerPipeline
    from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint
    from psana_ray_amd.queue.ring import physical_slots
    from psana_ray_amd.queue.session import QueueSession, create_or_attach
    from psana_ray_amd.source import SyntheticRun
    from psana_ray_amd.utils.metrics import sustained_rate

    sys.setswitchinterval(5e-4)   # short GIL hand-off: fabric / consumer threads stay responsive
    li = detect()
    world, rank = li.size, li.rank
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s); N > 1 needs "
              f"torch.distributed.run with one rank per GPU", file=sys.stderr)
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
    # ranks sharing one GPU (rehearsals of an N-rank launch on fewer GPUs): the library's pipeline
    # shape (config.pipeline_shape: 3 producer streams and 32-frame batches there), the same
    # resolution psana-ray-producer / psana-ray-consumer make
    gpu_share, args.batch, compute_streams = resolve_shape(args, gpu)
    if gpu and gpu_share > 1 and rank == 0:
        print(f"bench.py: WARNING: {world} ranks on {torch.cuda.device_count()} visible GPU(s): {gpu_share} ranks "
              f"share a GPU (config.ranks_per_gpu); n_gpus reports distinct devices", file=sys.stderr, flush=True)

    coord = None
    store = None
    if world > 1:
        # single-node contract (rendezvous on 127.0.0.1): keep gloo's control traffic on loopback
        # instead of whatever interface the container hostname resolves to (or fails to)
        if os.environ.get("MASTER_ADDR", "127.0.0.1") in ("127.0.0.1", "localhost") and os.path.isdir("/sys/class/net/lo"):
            os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        import datetime

        # gloo prints its "[Gloo] Rank r is connected to ..." banner on fd 1 while connecting: send
        # it to stderr so stdout carries only the result line (torchrun launches included)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=600))
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        coord = dist.group.WORLD
        store = dist.distributed_c10d._get_default_store()

    def barrier():
        if coord is not None:
            dist.barrier(group=coord)

    mode = Mode(args.mode)
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
    # the producer CLI's own construction (same mode / common-mode resolution as psana-ray-producer)
    cal = build_calibrator(src, device, mode, None, args.common_mode)
    if args.queue_size is None:
        args.queue_size = 400 * world
    share = max(1, math.ceil(args.queue_size / world))
    # slack for frames waiting to be routed / copied to another GPU
    producer_slots = (4 * args.chunk + args.batch + (64 if world > 1 else 0)) if is_prod else 0
    if is_prod and world > 1 and gpu:
        from psana_ray_amd.config import fabric_direct_headroom
        producer_slots += fabric_direct_headroom(cal.out_frame_bytes)   # slots kept for direct frames (engine.h)
    # queue_size is the LOGICAL capacity (deque(maxlen), shared_queue.py:7); physical HBM slots are
    # capped by free memory (config 4: Jungfrau-16M x 400000 would need 26.8 TB)
    cslots = physical_slots(share, cal.out_frame_bytes, device, args.hbm_fraction, producer_slots)
    sess = None
    if world > 1:
        meta = create_or_attach(store, "bench", "queue",
                                {"queue_size": args.queue_size, "num_consumers": world, "n_producers": n_prod,
                                 "frame_shape": list(cal.out_shape), "dtype": str(cal.out_dtype).split(".")[-1],
                                 "device_kind": device.type})
        sess = QueueSession(store, "bench", "queue", meta, "prosumer" if is_prod else "consumer",
                            device=device.index if gpu else -1, rank=rank)
    ring = FrameRing(cal.out_shape, cal.out_dtype, device, producer_slots, cslots,
                     shm_name=sess.ring_name() if (sess is not None and not gpu) else None)
    ep = QueueEndpoint(ring, sess, is_producer=is_prod, is_consumer=True, route=args.route,
                       copy_engine=args.fabric_copy, copy_workgroups=args.fabric_copy_wgs,
                       copy_stream=args.fabric_copy_stream)
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
    cs_kw = {} if args.compute_streams is None else {"compute_streams": args.compute_streams}
    if args.stream_kind is not None:
        cs_kw["stream_kind"] = args.stream_kind
    sk_kw = {} if args.consumer_stream_kind is None else {"stream_kind": args.consumer_stream_kind}
    if args.consumer_streams is not None:
        sk_kw["streams"] = args.consumer_streams
    if args.gap_fill:
        cs_kw["gap_fill"] = True
    cs_kw["compute_streams"] = compute_streams
    prod = ProducerPipeline(source, cal, ep, rank=rank, chunk=args.chunk, ranks_per_gpu=gpu_share, **cs_kw) \
        if is_prod else None
    consumer = PeakFinderConsumer(ep, cal.out_shape, PeakFinderParams(), batch=args.batch, ranks_per_gpu=gpu_share,
                                  **sk_kw) if args.consumer == "peakfind" else None

    stop = threading.Event()
    ep.start()
    linking = None
    if sess is not None:
        linking = _wait_links(ep, world, n_prod - (1 if is_prod else 0), (world - 1) if is_prod else 0)
        fab = getattr(ep, "_fabric", None)
        if fab is not None and fab.last_link_error():
            linking["last_link_error"] = fab.last_link_error()
        barrier()
    pt = threading.Thread(target=prod.run if prod is not None else ep.finish, kwargs=dict(stop=stop) if prod else {},
                          name="producer", daemon=True)
    pt.start()

    def consume(n_frames, stall_s=90.0):
        """Take n_frames; a rank that receives nothing for stall_s fails loudly instead of hanging the
        job (a starved consumer would block every barrier after it)."""
        got = 0
        t_last = time.monotonic()
        while got < n_frames:
            g0 = got
            if consumer is not None:
                got += consumer.poll(timeout=0.05, max_items=n_frames - got)
            else:
                it = ep.get(timeout=0.05)
                if it is not None:
                    it.release()
                    got += 1
            if ep.failed is not None:
                raise RuntimeError(f"queue fabric failed: {ep.failed!r}")
            if got > g0:
                t_last = time.monotonic()
            elif time.monotonic() - t_last > stall_s:
                raise RuntimeError(f"bench.py rank {rank}: no frame for {stall_s:.0f} s ({got}/{n_frames} of this "
                                   f"request; fabric {ep.metrics()})")
        return got

    def csync():
        """This rank's consumer work issued so far has finished (its stream, not the device: a
        device-wide synchronize would also drain the producer's queued copies and kernels, and the
        frames they complete would then be consumed inside the window for free -- VERDICT r2 #1)."""
        if gpu:
            if consumer is not None:
                consumer.sync_streams()
            else:
                torch.cuda.current_stream(device).synchronize()

    # the mark is recorded on an idle consumer stream right after csync(): it completes once every
    # consumer batch issued before it has (both streams were synchronised)
    cstream = (consumer.stream if consumer is not None else torch.cuda.current_stream(device)) if gpu else None

    def window(steps, takes=True, sit_out=False):
        """``steps`` timed steps between barriers, in steady state.  Returns (host seconds, max over
        ranks; sustained frames/s of the node = min(sum over producers of the production rate,
        frames consumed / seconds); frames completed by the producers inside the window (sum);
        details; fabric counters before and after on this rank).

        Production is counted at DEVICE COMPLETION (one timing event per producer chunk) and only
        for chunks that completed after t0: frames already READY when the window opened are
        excluded, and the rate runs between two chunk completions (utils.metrics.sustained_rate),
        so a short window and a long one measure the same steady state.  ``takes=False``: this rank
        consumes nothing in the window (a lone producer's own consumer in the remote_only window)."""
        mine = steps * B if takes else 0
        csync()
        barrier()
        csync()
        c0 = ep.metrics()
        m0 = prod.clock(cstream) if prod is not None else None
        t0 = time.perf_counter()
        consume(mine)
        csync()
        if sit_out:
            barrier()   # some rank takes nothing: its window ends when the others' does (every rank calls it)
        t1 = time.perf_counter()
        m1 = prod.clock(cstream) if prod is not None else None
        c1 = ep.metrics()
        if gpu:
            torch.cuda.synchronize(device)   # untimed: the whole device is idle-consistent before the barrier
        barrier()
        dt = t1 - t0
        fr_p, rate_p = 0, 0.0
        if prod is not None:
            _, lg = prod.completion_log(0)
            fr_p, r = sustained_rate(lg, m0, m1)
            # fewer than two chunk completions around the window (a producer slower than one chunk
            # per window): frames completed inside it over the whole window
            rate_p = r if r is not None else fr_p / max(dt, 1e-9)
        if coord is not None:
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=coord)
            dt = float(t[0])
            v = torch.tensor([rate_p, float(fr_p), float(mine)], dtype=torch.float64)
            dist.all_reduce(v, op=dist.ReduceOp.SUM, group=coord)
            rate_sum, fr_sum, taken = float(v[0]), int(v[1]), int(v[2])
        else:
            rate_sum, fr_sum, taken = rate_p, fr_p, mine
        consumed_rate = taken / dt
        value = min(rate_sum, consumed_rate)
        det = {"production_frames_per_s": round(rate_sum, 1), "consumer_frames_per_s": round(consumed_rate, 1),
               "produced_in_window": fr_sum, "produced_in_window_rank0": fr_p}
        return dt, value, fr_sum, det, c0, c1

    def allsum(x):
        if coord is None:
            return [x]
        out = [None] * world
        dist.all_gather_object(out, x, group=coord)
        return out

    def steady_gate():
        """Untimed windows until two consecutive ones agree within --gate-tol on every rank (the
        queue's start-up backlog drained, clocks and the routing settled), bounded by --gate-max-s.
        Each window takes ~--gate-window-s worth of frames at the last measured rate; the decision
        is collective (all-reduce), so every rank leaves the gate after the same window."""
        t_start = time.perf_counter()
        n = max(4, args.warmup) * B
        prev, rates, it, converged = None, [], 0, False
        while True:
            csync()
            barrier()
            t0 = time.perf_counter()
            consume(n)
            csync()
            r = n / max(1e-9, time.perf_counter() - t0)
            it += 1
            rates.append(round(r, 1))
            agree = prev is not None and abs(r - prev) <= args.gate_tol * prev
            prev = r
            n = max(B, int(round(r * args.gate_window_s / B)) * B)
            flags = [0.0 if agree else 1.0, time.perf_counter() - t_start]
            if coord is not None:
                t = torch.tensor(flags, dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=coord)
                flags = [float(t[0]), float(t[1])]
            if flags[0] == 0.0:
                converged = True
                break
            if flags[1] > args.gate_max_s:
                break
        return {"tol": args.gate_tol, "iterations": it, "converged": converged,
                "seconds": round(time.perf_counter() - t_start, 3), "window_rates": rates[-8:]}

    B = args.batch
    t_pre = time.perf_counter()
    while time.perf_counter() - t_pre < args.preroll_s:
        consume(B)
    gate = steady_gate() if args.gate_tol > 0 else None
    barrier()
    consume(args.warmup * B)
    # producers < ranks (BASELINE config 3): every rank's window ends with the slowest consumer's, so
    # the producers' rate and the node's consumption cover the same interval (a producer whose own
    # consumer finished early would otherwise report its rate over a shorter, emptier-queue window)
    dt, value, produced_window, rate_detail, c0, c1 = window(args.steps, sit_out=n_prod < world)

    cross = None
    cross_steps = args.steps if args.cross_steps is None else args.cross_steps
    if world > 1 and cross_steps > 0:
        ep.set_route("remote_only")
        # a LONE producer's own consumer receives nothing under remote_only (no other producer can
        # feed it): it sits the window out and the consumer-only ranks take every frame (BASELINE
        # config 3 with --producers 1)
        takes = not (is_prod and n_prod == 1)
        # drain what the headline policy already put into this shard (FIFO), then warm up: the
        # window must see frames routed by the new policy, not the old backlog
        consume(int(ep.metrics().get("ready", 0)) + (max(2, args.warmup // 2) * B if takes else 0))
        xdt, xval, xpw, xdet, x0, x1 = window(cross_steps, takes, sit_out=n_prod == 1)
        sent = allsum(int(x1.get("bytes_sent", 0) - x0.get("bytes_sent", 0)))
        fr_sent = allsum(int(x1.get("frames_sent", 0) - x0.get("frames_sent", 0)))
        fr_local = allsum(int(x1.get("frames_local", 0) - x0.get("frames_local", 0)))
        fr_recv = allsum(int(x1.get("frames_recv", 0) - x0.get("frames_recv", 0)))
        tk_rem = allsum(int(x1.get("taken_remote", 0) - x0.get("taken_remote", 0)))
        tk_loc = allsum(int(x1.get("taken_local", 0) - x0.get("taken_local", 0)))
        cms = allsum(round(float(x1.get("copy_ms_per_batch", 0.0)), 3))
        # the window's copy dispatches: device time of the copy alone (timing events around it) and
        # host issue -> completion (includes the wait for the frames' calibration)
        n_new = int(x1.get("copy_launches", 0) - x0.get("copy_launches", 0))
        smp = ep.copy_samples()[-n_new:] if n_new > 0 else []
        copy_detail = allsum(_copy_stats(smp))
        fb = ring.frame_bytes
        per_link = allsum({str(int(l.peer)): round(int(l.frames) * fb / 1e9, 3) for l in ep.links() if l.outgoing})
        keys = ("grants_given", "grants_returned", "grants_reclaimed", "frames_recv", "frames_requeued")
        fab = allsum({k: int(x1.get(k, 0) - x0.get(k, 0)) for k in keys} |
                     {"credits": int(x1.get("credits", 0)), "ready": int(x1.get("ready", 0)),
                      "held": int(x1.get("held", 0)),
                      "links": [[int(l.peer), bool(l.outgoing), int(l.outstanding), int(l.frames)] for l in ep.links()]})
        cross = {
            "route": "remote_only", "steps": cross_steps, "ms_per_step": round(1e3 * xdt / cross_steps, 4),
            "frames_per_s": round(xval, 2), **xdet,
            "cross_gpu_GB_per_s": round(sum(sent) / xdt / 1e9, 2),
            # of the frames consumers TOOK in the window, the share another process produced (a
            # consumer's read-ahead at t0 counts where it came from; sends inside the window alone
            # miss it when the window is short)
            "cross_gpu_fraction": round(sum(tk_rem) / max(1, sum(tk_rem) + sum(tk_loc)), 3),
            "sent_cross_fraction": round(sum(fr_sent) / max(1, sum(fr_sent) + sum(fr_local)), 3),
            "taken_remote_per_rank": tk_rem, "taken_local_per_rank": tk_loc,
            "received_cross_per_consumed": round(sum(fr_recv) / max(1, sum(allsum(cross_steps * B if takes else 0))),
                                                 3),
            "bytes_sent_per_rank": sent, "frames_sent_per_rank": fr_sent, "frames_local_per_rank": fr_local,
            # of the frames sent: calibrated straight into the consumer's slot (no copy pass;
            # csrc/fabric.h take_direct), and direct frames lost to a consumer that left
            "frames_direct_per_rank": allsum(int(x1.get("frames_direct", 0) - x0.get("frames_direct", 0))),
            "frames_lost_direct_per_rank": allsum(int(x1.get("frames_lost_direct", 0))),
            "direct_headroom_slots": int(getattr(getattr(prod, "engine", None), "direct_headroom", 0)),
            "copy_ms_per_batch_per_rank": cms,
            "copy_dispatch_per_rank": copy_detail,
            "link_GB_total_per_rank": per_link,
            "fabric_copy": list(getattr(ep, "copy_engine", ("", 0))),
            "fabric_per_rank": fab,
            "data_plane": "HIP IPC peer writes into the consumer's ring over xGMI ("
                          + ("one copy_runs_kernel launch per fabric pass, own hardware queue"
                             if getattr(ep, "copy_engine", ("kernel",))[0] == "kernel"
                             else "hipMemcpyAsync per run, one stream per link") + ")",
        }
        ep.set_route(args.route)
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
    topology = _topology(ep, device, allsum) if sess is not None or gpu else None
    peaks = consumer.synchronize() if consumer is not None else 0
    if gpu:
        torch.cuda.synchronize(device)   # every verify launch on the consumer streams has completed
    st = ep.stats()
    # end-to-end checks of frames that crossed processes (csrc/verify.h): consumer-side re-sums of the
    # frames whose producer attached a checksum, and the acquires issued before peer-written reads
    checks = None
    if sess is not None:
        vc = allsum(ep.verify_counts())
        checks = {"verify_every": ep._fabric.verify_every() if ep._fabric is not None else None,
                  "frames_verified": sum(v["verified"] for v in vc),
                  "frames_mismatched": sum(v["mismatched"] for v in vc),
                  "verified_per_rank": [v["verified"] for v in vc],
                  "mismatched_per_rank": [v["mismatched"] for v in vc],
                  "last_bad_gevt_per_rank": [v["last_bad_gevt"] for v in vc],
                  "acquires_per_rank": [v["acquires"] for v in vc],
                  "checksummed_sent_per_rank": allsum(int(st.get("frames_checksummed", 0))),
                  "corrupted_injected_per_rank": allsum(int(st.get("frames_corrupted", 0)))}
        if cross is not None:
            cross["frames_verified"] = checks["frames_verified"]
            cross["frames_mismatched"] = checks["frames_mismatched"]
    # per rank over the whole run: the share of the frames it consumed that arrived from another
    # process (consumer-only ranks of BASELINE config 3 receive every frame over the fabric)
    recv_share = consumed_per_rank = None
    if sess is not None:
        got = int(st.get("got", 0))
        consumed_per_rank = allsum(got)
        recv_share = [round(x, 3) for x in allsum(int(st.get("frames_recv", 0)) / max(1, got))]
    copies = prod.engine.copy_stats() if (prod is not None and prod.engine is not None) else None
    # n_gpus = DISTINCT devices the ranks ran on (2 ranks sharing the one GPU of a box report 1);
    # n_ranks = world size
    devs = topology["device_per_rank"] if topology is not None else [device.index if gpu else -1]
    n_devices = len({d for d in devs if d is not None and d >= 0})
    if not gpu:
        staging = "host memory (CPU rehearsal)"
    elif args.source == "device":
        staging = "raw frames resident in HBM (no host staging)"
    elif copies is not None and copies[2] > 0:
        staging = "pinned host memory -> HBM by copy_h2d_kernel"
    else:
        staging = "pinned host memory -> HBM by hipMemcpyAsync (" + \
                  ("blit kernels" if os.environ.get("HSA_ENABLE_SDMA") == "0" else "SDMA") + ")"
    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": n_devices,
        "n_ranks": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * dt / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "float32" if mode != Mode.raw else "uint16",
        "data": "synthetic (random-init calibration constants, pre-generated raw " + args.detector
                + " pool cycled; " + staging + ")" + ("" if gpu else "; gloo protocol rehearsal, not a benchmark"),
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
            "ranks_per_gpu": gpu_share,
            "launch": "self-launched children" if os.environ.get("PSANA_RAY_SELF_LAUNCHED") == "1"
                      else li.launcher,
            "producer_ranks": n_prod,
            "queue": "local (single process)" if sess is None else "elastic fabric session",
        },
        "extra": {
            **rate_detail,
            "timing": "t0/t1: barrier + consumer-stream synchronize (steady state; a device-wide synchronize "
                      "would drain the producer pipeline into the window), device-wide synchronize after t1; "
                      "production counted at device completion of each chunk, chunks ready at t0 excluded",
            "frame_bytes": ring.frame_bytes,
            "queue_slots_physical_rank0": cslots,
            "ring_GB_rank0": round(ring.nbytes / 1e9, 1),
            "GB_per_s_out": round(value * ring.frame_bytes / 1e9, 2),
            "peaks_found_rank0": peaks,
            "queue_full_waits_rank0": prod.full_waits if prod is not None else 0,
            "frames_local_rank0_headline": int(c1.get("frames_local", 0) - c0.get("frames_local", 0)),
            "recv_cross_per_consumed_per_rank": recv_share,
            "consumed_per_rank": consumed_per_rank,
            "frames_sent_rank0_headline": int(c1.get("frames_sent", 0) - c0.get("frames_sent", 0)),
            "bytes_sent_rank0": st.get("bytes_sent", 0),
            "xgmi_phase": cross,
            "frame_checks": checks,
            "links_rank0": linking,
            "topology": topology,
            "steady_gate": gate,
            "staging": staging,
            "staging_copies_span_frame_kernel": copies,
            "numa_node": numa,
            "cpus_allowed": len(os.sched_getaffinity(0)),
            "producer_streams": list(prod.stream_config) if prod is not None and prod.stream_config else None,
            "consumer_stream_kind": args.consumer_stream_kind or CONSUMER_STREAM_KIND,
            "producer_host_s_stage_acquire_launch_commit_total": (
                [round(x, 4) for x in prod.engine.timing()] if prod is not None and prod.engine is not None
                else None),
        },
    }
    # self-validation: every link attached, none failed, and the cross window
    # really crossed GPUs -- otherwise the line is printed for diagnosis but the run fails
    problems = []
    if sess is not None:
        failed_links = sum(allsum(int(ep.metrics().get("links_failed", 0))))
        if failed_links:
            problems.append(f"{failed_links} fabric link(s) failed")
        if linking is not None and not all(allsum(bool(linking.get("complete")))):
            problems.append("some rank's links never completed")
        if checks is not None and checks["frames_mismatched"] > 0:
            problems.append(f"{checks['frames_mismatched']} frame(s) arrived with contents that differ from what "
                            f"their producer sent (last gevt per rank {checks['last_bad_gevt_per_rank']})")
        if cross is not None and cross["cross_gpu_fraction"] < 0.9:
            problems.append(f"only {cross['cross_gpu_fraction']:.3f} of the cross window's frames crossed GPUs")
    result["extra"]["validation"] = problems or "ok"
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    sys.stdout.flush()
    if sess is not None:
        # never let a teardown hang the run after the result line: the watchdog exits NON-zero
        clean = ep.failed is None and not pt.is_alive()

        def _teardown_timeout():
            print(f"bench.py rank {rank}: teardown timed out", file=sys.stderr, flush=True)
            os._exit(3)

        wd = threading.Timer(60.0, _teardown_timeout)
        wd.daemon = True
        wd.start()
        ep.close()
        barrier()
        dist.destroy_process_group()
        wd.cancel()
        if not clean:
            print(f"bench.py rank {rank}: queue fabric reported {ep.failed!r}", file=sys.stderr, flush=True)
            return 3
    if problems:
        print(f"bench.py rank {rank}: INVALID run: {'; '.join(problems)}", file=sys.stderr, flush=True)
        return 4
    return 0


if __name__ == "__main__":
    sys.exit(main())
