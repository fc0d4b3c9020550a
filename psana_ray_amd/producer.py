"""``psana-ray-producer``: MPI-launched producer ranks streaming calibrated detector frames into
the shared queue (reference parity: psana_ray/producer.py, console script setup.py:22-26).

    mpirun -n 4 psana-ray-producer --exp mfxl1038923 --run 58 --detector_name epix10k2M --queue_size 400

The 13 reference flags keep their exact names, types and defaults (producer.py:17-33; SURVEY
2.6).  Image mode stays the default; ``--calib`` selects per-panel frames (Q-11).  Additive
flags (``--device``, ``--common_mode``, ``--consumer_task``, ...) have defaults that reproduce
the reference behaviour.  Rank/size come from the MPI launcher environment (no mpi4py).

Per rank: event source (psana / raw-run file / synthetic) -> pinned host pages -> hipMemcpyAsync
on a side stream -> gfx950 calibration kernels (pedestal, gain switching, common mode, masks,
geometry) writing into HBM ring slots -> sharded queue -> consumers, with explicit per-producer
end-of-stream (no global barrier, Q-7/Q-8) and SIGINT handling on every rank (Q-14).
"""
from __future__ import annotations

import argparse
import logging
import math
import signal
import sys
import threading
import traceback
from typing import Optional

import numpy as np

from .config import (BACKOFF_BASE_S, BACKOFF_JITTER_S, BACKOFF_MAX_S, DEFAULT_LOG_LEVEL,
                     DEFAULT_NUM_CONSUMERS,
                     DEFAULT_QUEUE_NAME, DEFAULT_QUEUE_SIZE, DEFAULT_RAY_ADDRESS, DEFAULT_RAY_NAMESPACE, LOG_LEVELS,
                     QUEUE_LOOKUP_DELAY_S, QUEUE_LOOKUP_RETRIES, CommonModeParams, PeakFinderParams,
                     resolve_common_mode)

log = logging.getLogger("psana_ray_amd.producer")


def build_parser() -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser(description="PsanaWrapper Data Producer")
    # ---- reference flags: identical names / types / defaults (psana_ray/producer.py:19-32)
    parser.add_argument("--exp", type=str, required=True, help="Experiment name")
    parser.add_argument("--run", type=int, required=True, help="Run number")
    parser.add_argument("--detector_name", type=str, required=True, help="Detector name")
    parser.add_argument("--calib", action="store_true", help="Use calib mode")
    parser.add_argument("--uses_bad_pixel_mask", action="store_true", help="Use bad pixel mask")
    parser.add_argument("--manual_mask_path", type=str, default=None, help="Path to a manual mask in npy")
    parser.add_argument("--ray_address", type=str, default=DEFAULT_RAY_ADDRESS, help="Address of the Ray cluster")
    parser.add_argument("--ray_namespace", type=str, default=DEFAULT_RAY_NAMESPACE,
                        help="Ray namespace to use for both queues")
    parser.add_argument("--queue_name", type=str, default=DEFAULT_QUEUE_NAME, help="Queue name")
    parser.add_argument("--queue_size", type=int, default=DEFAULT_QUEUE_SIZE, help="Maximum queue size")
    parser.add_argument("--num_consumers", type=int, default=DEFAULT_NUM_CONSUMERS,
                        help="Number of consumer processes expected.")
    parser.add_argument("--max_steps", type=int, default=None, help="Maximum number of steps before terminating")
    parser.add_argument("--log_level", type=str, default=DEFAULT_LOG_LEVEL, choices=LOG_LEVELS, help="Logging level")
    # ---- additive flags (MI355X framework)
    g = parser.add_argument_group("psana_ray_amd")
    g.add_argument("--device", type=str, default="auto", help="auto | cpu | cuda[:i] (auto: GPU local_rank)")
    g.add_argument("--mode", type=str, default=None, choices=["raw", "calib", "image"],
                   help="override the retrieval mode (default: image, or calib with --calib)")
    g.add_argument("--common_mode", type=str, default="auto",
                   help="common-mode correction: auto (default: on for detectors whose psana calib applies it -- "
                        "epix10ka -- off otherwise) | off | default | flags,thr,maxcorr,npix_min[,bank_cols]")
    g.add_argument("--psana_calibrated", action="store_true",
                   help="psana_wrapper runs: take psana's CPU-calibrated frames even when the wrapper can provide "
                        "raw frames and constants (default: raw frames calibrated by the HIP kernels)")
    g.add_argument("--psana_private_constants", action="store_true",
                   help="psana_wrapper runs without a calib_constants() hook: read psana2's calibration constants "
                        "through its PRIVATE detector accessors (det.raw._pedestals / _gain / _status / ...); "
                        "without it such a run falls back to psana's CPU calibration")
    g.add_argument("--psana_handle_shard", default="explicit", choices=["explicit", "psana"],
                   help="psana_wrapper runs whose raw frames come from the run's own event loop (no raw retrieval "
                        "mode): explicit = rank r keeps every size-th event from r (default); psana = the loop is "
                        "already sharded over the MPI ranks by psana")
    g.add_argument("--num_events", type=int, default=None, help="events in a synthetic run (default: endless)")
    g.add_argument("--data_dir", type=str, default=None, help="raw-run files directory (or $PSANA_RAY_DATA)")
    g.add_argument("--chunk", type=int, default=64, help="frames per H2D copy / kernel launch (<= 64)")
    g.add_argument("--route", type=str, default="balanced", choices=["balanced", "local_first", "spread"])
    g.add_argument("--consumer_task", type=str, default="none", choices=["none", "peakfind"],
                   help="also consume on every producer rank (co-located consumer, BASELINE config 5)")
    g.add_argument("--producer_slots", type=int, default=None,
                   help="calibrated frames a rank may hold until a consumer takes them (default: its share of "
                        "--queue_size, at least 2 x --chunk)")
    g.add_argument("--hbm_fraction", type=float, default=0.8, help="cap of free HBM used for ring slots")
    g.add_argument("--timeout", type=float, default=300.0, help="rendezvous / peer timeout in seconds")
    g.add_argument("--calibrate_on_read", action="store_true",
                   help="capacity tier: the ring holds RAW u16 frames (half the HBM and xGMI bytes of f32); "
                        "consumers calibrate on read with the same constants / mode / masks / common mode")
    g.add_argument("--start_event", type=int, default=0,
                   help="resume: first global event id to produce (frames carry gevt, so consumers can dedupe)")
    g.add_argument("--metrics_interval", type=float, default=10.0,
                   help="seconds between metric summary lines (rates, queue depth); 0 disables")
    g.add_argument("--metrics_json", type=str, default=None, help="append per-interval metrics as JSON lines")
    g.add_argument("--metrics_port", type=int, default=None, help="Prometheus exporter port (if installed)")
    g.add_argument("--panel_shards", type=int, default=1,
                   help="split every frame's panels over groups of this many ranks (SP analog for Jungfrau-16M-"
                        "scale frames): a group walks the same events, each rank stages/calibrates/queues 1/N "
                        "of the panels; needs --calib or --mode raw (source/shard.py)")
    g.add_argument("--copy_engine", type=str, default="blit", choices=["blit", "sdma"],
                   help="host->HBM staging copies: blit kernels (default, measured faster in the pipeline) or "
                        "the SDMA engines (utils/runtime_env.py)")
    g.add_argument("--local", action="store_true",
                   help="single-process queue: no rendezvous; requires --consumer_task (no external consumers)")
    return parser


def parse_arguments(argv=None):
    return build_parser().parse_args(argv)


def backoff_delays(retries: int):
    """The reference's full-queue backoff schedule (producer.py:84-111): 0.1, 0.2, 0.4, 0.8, 1.6, then
    2.0 s forever, each plus U(0, 0.5) s jitter.  Returns (delay without jitter, jitter bound)."""
    delay = min(BACKOFF_MAX_S, BACKOFF_BASE_S * (2 ** retries))
    return delay, BACKOFF_JITTER_S


def initialize_queue(ray_address, ray_namespace, queue_name, queue_size, rank, size, num_consumers, frame_shape,
                     dtype, device_kind, extra=None, max_retries=QUEUE_LOOKUP_RETRIES,
                     retry_delay=QUEUE_LOOKUP_DELAY_S, timeout_s=300.0):
    """Reach the rendezvous store and create -- or attach to (producer.py:43-45) -- the live session
    of the named queue.  Returns ``(store, meta)``, or None on failure after logging the reason
    (producer.py:35-71)."""
    from .parallel.rendezvous import open_store
    from .queue.session import create_or_attach

    try:
        store = open_store(ray_address, spawn_if_absent=True, timeout_s=timeout_s, retries=max_retries,
                           retry_delay_s=retry_delay)
        meta = {"queue_size": int(queue_size), "num_consumers": int(num_consumers), "n_producers": int(size),
                "frame_shape": list(frame_shape), "dtype": dtype, "device_kind": device_kind}
        meta.update(extra or {})
        meta = create_or_attach(store, ray_namespace, queue_name, meta, timeout_s=timeout_s)
        log.info("Rank %d: Successfully connected to shared queue.", rank)
        return store, meta
    except Exception as e:  # noqa: BLE001 - reference: log + None (producer.py:69-71)
        log.error("Rank %d: Error in initialize_queue: %s", rank, e)
        return None


initialize_ray = initialize_queue   # reference name (producer.py:35), kept for API parity


def load_masks(source, uses_bad_pixel_mask: bool, manual_mask_path: Optional[str]):
    """Combined mask (truthy keeps, producer.py:81-82,92-95): bad-pixel AND manual."""
    mask = None
    if uses_bad_pixel_mask:
        mask = np.asarray(source.create_bad_pixel_mask()).astype(bool)
    if manual_mask_path is not None:
        manual = np.load(manual_mask_path).astype(bool)   # allow_pickle stays False
        full = getattr(source, "full_spec", None)        # panel shard: a whole-detector mask is sliced
        if full is not None and manual.shape == tuple(full.frame_shape):
            manual = manual[source.lo:source.hi]
        if mask is None:
            mask = manual
        elif manual.shape == mask.shape:
            mask = mask & manual
        else:
            raise ValueError(f"manual mask {manual.shape} and bad-pixel mask {mask.shape} differ in shape")
    return mask


def _read_recipe(args, read_mode, read_cm) -> dict:
    """What a consumer needs to reproduce this producer's calibration (--calibrate_on_read)."""
    return {"exp": args.exp, "run": args.run, "detector_name": args.detector_name, "mode": read_mode.value,
            "common_mode": None if read_cm is None else [read_cm.flags, read_cm.thr, read_cm.maxcorr,
                                                          read_cm.npix_min, read_cm.bank_cols],
            "uses_bad_pixel_mask": bool(args.uses_bad_pixel_mask), "manual_mask_path": args.manual_mask_path,
            "data_dir": args.data_dir}


def produce_data(pipeline, max_steps=None, stop=None):
    """Run one rank's producer pipeline (producer.py:78-130); returns frames produced."""
    from .queue.endpoint import QueuePeerError

    try:
        return pipeline.run(max_steps=max_steps, stop=stop)
    except QueuePeerError:
        log.error("Rank %d: Queue fabric failed. Exiting...", pipeline.rank)   # producer.py:113
        return pipeline.frames


def build_calibrator(source, device, mode, mask, common_mode_text):
    """The Calibrator a producer rank runs for ``source`` (None for a source whose frames arrive
    calibrated).  One place for the producer CLI and bench.py, so the headline measures what the
    CLI runs."""
    from .models.calibrator import Calibrator
    from .models.detector import Mode

    if getattr(source, "calibrated", False):
        return None
    cm = resolve_common_mode(common_mode_text, source.consts.spec) if mode != Mode.raw else None
    return Calibrator(source.consts, device, mode, mask=mask, common_mode=cm,
                      geometry=getattr(source, "geometry", None))


def main(argv=None) -> int:
    args = parse_arguments(argv)
    logging.basicConfig(level=getattr(logging, args.log_level),
                        format="%(asctime)s - %(levelname)s - %(message)s")   # producer.py:135-136
    from .utils.runtime_env import select_copy_engine

    select_copy_engine(args.copy_engine)   # before the HIP runtime initialises
    import torch

    from .models.detector import Mode
    from .parallel.launch import bind_numa_to_device, detect, device_for
    from .pipeline import PeakFinderConsumer, ProducerPipeline
    from .queue.endpoint import EndOfStream, QueueEndpoint
    from .queue.ring import FrameRing, physical_slots
    from .queue.session import QueueSession
    from .source import NoSourceError, open_source
    from .utils.metrics import Registry, Reporter

    li = detect()
    rank, size = li.rank, li.size
    device = device_for(li.local_rank, args.device)
    if device.type == "cuda":
        torch.cuda.set_device(device)
        bind_numa_to_device(device)
        from .parallel.launch import ranks_per_gpu

        log.info("Rank %d: %s launch, %d local rank(s), %d rank(s) per GPU", rank, li.launcher, li.local_size,
                 ranks_per_gpu(local_size=li.local_size))
    stop = threading.Event()

    def signal_handler(sig, frame):   # every rank (Q-14): stop producing, advertise EOS, exit cleanly
        log.error("Ctrl+C pressed. Shutting down...")
        stop.set()

    signal.signal(signal.SIGINT, signal_handler)

    mode = Mode(args.mode) if args.mode else (Mode.calib if args.calib else Mode.image)   # producer.py:156-159
    read_mode = mode
    if args.calibrate_on_read:
        if args.local or args.consumer_task != "none":
            log.error("--calibrate_on_read needs separate consumers (DataReader); it does not apply to --local "
                      "or a co-located --consumer_task")
            return 2
        mode = Mode.raw   # frames travel raw; DataReader applies read_mode
    shards = int(args.panel_shards)
    if shards > 1:
        from .source.shard import PanelShardSource, shard_layout

        if read_mode == Mode.image or args.calibrate_on_read:
            log.error("--panel_shards queues per-panel shards: use --calib (or --mode raw), without "
                      "--calibrate_on_read (image assembly needs every panel of the frame)")
            return 2
        group, n_groups, shard = shard_layout(rank, size, shards)   # events over groups, panels within
        try:
            source = open_source(args.exp, args.run, args.detector_name, rank=group, size=n_groups,
                                 n_events=args.num_events, pinned=device.type == "cuda", data_dir=args.data_dir,
                                 mode=Mode.raw, prefer_raw=True, psana_private_constants=args.psana_private_constants,
                                 psana_handle_shard=args.psana_handle_shard)
        except NoSourceError as e:
            log.error("Rank %d: %s", rank, e)
            return 2
        if getattr(source, "calibrated", False):
            log.error("--panel_shards needs raw frames (a psana-calibrated source cannot be split into panel shards)")
            return 2
        source = PanelShardSource(source, shard, shards)
        log.info("Rank %d: panel shard %d/%d (panels %d:%d) of event group %d/%d", rank, shard, shards, source.lo,
                 source.hi, group, n_groups)
    else:
        try:
            source = open_source(args.exp, args.run, args.detector_name, rank=rank, size=size,
                                 n_events=args.num_events, pinned=device.type == "cuda", data_dir=args.data_dir,
                                 mode=read_mode if not args.calibrate_on_read else Mode.raw,
                                 prefer_raw=not args.psana_calibrated,
                                 psana_private_constants=args.psana_private_constants,
                                 psana_handle_shard=args.psana_handle_shard)
        except NoSourceError as e:
            log.error("Rank %d: %s", rank, e)
            return 2
        if args.calibrate_on_read and getattr(source, "calibrated", False):
            log.error("--calibrate_on_read needs raw frames; this psana_wrapper source provides calibrated ones")
            return 2
    if args.start_event:
        if not hasattr(source, "seek"):
            log.error("--start_event: source %s cannot seek", type(source).__name__)
            return 2
        k0 = source.seek(args.start_event)
        log.info("Rank %d: resuming at global event %d (local index %d)", rank, args.start_event, k0)
    mask = load_masks(source, args.uses_bad_pixel_mask, args.manual_mask_path)
    read_cm = resolve_common_mode(args.common_mode, source.consts.spec) \
        if (args.calibrate_on_read and read_mode != Mode.raw) else None
    calibrator = build_calibrator(source, device, mode, mask, args.common_mode)
    # psana-calibrated frames: the shape of the first event (peeked before the ring is built)
    frame_shape = calibrator.out_shape if calibrator else tuple(source.frame_shape)
    dtype = "uint16" if mode == Mode.raw else "float32"
    co_consumer = args.consumer_task != "none"
    frame_bytes = int(np.prod(frame_shape)) * (2 if mode == Mode.raw else 4)

    sess = None
    ep = None
    chunk = max(1, int(args.chunk))
    share = max(1, math.ceil(args.queue_size / size))
    pslots = args.producer_slots if args.producer_slots is not None else max(share, 2 * chunk)
    if args.producer_slots is None and args.route == "spread" and device.type == "cuda":
        from .config import fabric_direct_headroom
        pslots += fabric_direct_headroom(frame_bytes)   # slots kept for direct frames (csrc/engine.h)
    try:
        if args.local or (size == 1 and args.num_consumers == 0):
            if not co_consumer:
                log.error("--local needs --consumer_task (nobody would read the queue)")
                return 2
            ring = FrameRing(frame_shape, torch.float32 if dtype == "float32" else torch.uint16, device,
                             pslots, physical_slots(args.queue_size, frame_bytes, device, args.hbm_fraction, pslots))
            ep = QueueEndpoint(ring)
        else:
            got = initialize_queue(args.ray_address, args.ray_namespace, args.queue_name, args.queue_size, rank,
                                   size, args.num_consumers, frame_shape, dtype, device.type,
                                   extra={"co_consumers": co_consumer,
                                          "panel_shards": {"n_shards": shards,
                                                           "n_panels": source.full_spec.n_panels,
                                                           "detector_name": args.detector_name}
                                          if shards > 1 else None,
                                          "calibrate_on_read": _read_recipe(args, read_mode, read_cm)
                                          if args.calibrate_on_read else None},
                                   timeout_s=args.timeout)
            if got is None:
                return 1
            store, meta = got
            dev_index = device.index if device.type == "cuda" and device.index is not None else -1
            sess = QueueSession(store, args.ray_namespace, args.queue_name, meta,
                                "prosumer" if co_consumer else "producer", device=dev_index,
                                job=f"{args.exp}/{args.run}", rank=rank)
            pslots = physical_slots(pslots, frame_bytes, device, args.hbm_fraction)
            cslots = 0
            if co_consumer:
                cshare = max(1, math.ceil(args.queue_size / max(1, size)))
                cslots = physical_slots(cshare, frame_bytes, device, args.hbm_fraction, pslots)
            ring = FrameRing(frame_shape, torch.float32 if dtype == "float32" else torch.uint16, device, pslots,
                             cslots, shm_name=sess.ring_name() if (co_consumer and device.type == "cpu") else None)
            ep = QueueEndpoint(ring, sess, is_producer=True, is_consumer=co_consumer, route=args.route)
            ep.start()
            log.info("Rank %d: member %d of queue %s/%s (session %d): %d producer slots%s", rank, sess.mid,
                     args.ray_namespace, args.queue_name, meta["session"], pslots,
                     f", {cslots} consumer slots" if co_consumer else "")
        pipe = ProducerPipeline(source, calibrator, ep, rank=rank, chunk=chunk,
                                log_every=1 if logging.getLogger().isEnabledFor(logging.DEBUG) else 0,
                                mask=mask if calibrator is None else None)
        cons_thread = None
        stats = {}
        registry = Registry()
        registry.register("producer", pipe.metrics)
        registry.register("queue", ep.metrics)
        if co_consumer:
            # batch: config.pipeline_shape for the ranks sharing this GPU (mpirun -n 4 on fewer GPUs
            # takes the shared-GPU shape, like bench.py)
            cons = PeakFinderConsumer(ep, frame_shape, PeakFinderParams())
            registry.register("consumer", cons.metrics)

            def consume():
                while True:
                    try:
                        cons.poll(timeout=0.1)
                    except EndOfStream:
                        break
                stats["peaks"] = cons.synchronize()
                stats["consumed"] = cons.frames

            cons_thread = threading.Thread(target=consume, name="co-consumer", daemon=True)
            cons_thread.start()
        reporter = Reporter(registry, rank=rank, interval=args.metrics_interval, json_path=args.metrics_json,
                            prometheus_port=(args.metrics_port + rank) if args.metrics_port else None).start()
        rc = 0
        try:
            n = produce_data(pipe, max_steps=args.max_steps, stop=stop)
            log.info("Rank %d: produced %d frames", rank, n)
            # drain before exit: the frames this rank holds ARE queue items (the reference's detached
            # actor kept them after the producer left, shared_queue.py:35); wait for consumers
            if not ep.join(timeout=args.timeout):
                if ep.failed is not None:
                    log.error("Rank %d: queue fabric failed: %s", rank, ep.failed)
                else:
                    log.error("Rank %d: %d frames were not taken by any consumer within --timeout %.0f s; "
                              "exiting without them", rank, ep.undelivered(), args.timeout)
                rc = 1
            m = ep.metrics()
            if m.get("frames_sent"):
                log.info("Rank %d: fabric: %d frames sent to other processes (%d calibrated straight into the "
                         "consumer's slot, %d of those lost with a consumer that died), %d requeued, %d checksummed",
                         rank, m.get("frames_sent", 0), m.get("frames_direct", 0), m.get("frames_lost_direct", 0),
                         m.get("frames_requeued", 0), m.get("frames_checksummed", 0))
            if cons_thread is not None:
                cons_thread.join()
                log.info("Rank %d: co-located consumer processed %d frames, %d peaks", rank,
                         stats.get("consumed", 0), stats.get("peaks", 0))
        finally:
            reporter.stop(final_sample=args.metrics_interval > 0 or args.metrics_json is not None)
        return rc
    except Exception as e:
        log.error("Rank %d: Unhandled exception in main: %s", rank, e)   # producer.py:163-166
        log.error("Traceback:")
        log.error(traceback.format_exc())
        raise
    finally:
        if ep is not None:
            ep.close(timeout=min(30.0, args.timeout))


if __name__ == "__main__":
    sys.exit(main())
