"""``psana-ray-consumer``: installed consumer entry point (the reference only ships
examples/psana_consumer.py and never installs it, SURVEY R-14 / Q-9).

    psana-ray-consumer [consumer_id] [--queue_name my] [--ray_namespace default] [--task peakfind]

Joins the queue session through :class:`~psana_ray_amd.data_reader.DataReader` (same defaults as
the producer, fixing Q-3), reads ``[rank, idx, data, photon_energy]`` items (4 fields, fixing the
example's 3-field unpack, Q-1) until the explicit end of stream (fixing Q-2), and runs a task:
``print`` (the reference example's behaviour), ``peakfind`` (on-GPU K-07 peak finder over
zero-copy leased batches) or ``none``.  ``--out`` writes the peak lists to an ``.npz``.
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import sys
import time

from .config import (DEFAULT_LOG_LEVEL, DEFAULT_PREFETCH, DEFAULT_QUEUE_NAME, DEFAULT_RAY_ADDRESS,
                     DEFAULT_RAY_NAMESPACE, LOG_LEVELS)

log = logging.getLogger("psana_ray_amd.consumer")


def build_parser():
    ap = argparse.ArgumentParser(description="psana-ray consumer")
    ap.add_argument("consumer_id", nargs="?", type=int, default=None,
                    help="consumer id (examples/psana_consumer.py:51); default: claim the next free id")
    ap.add_argument("--ray_address", type=str, default=DEFAULT_RAY_ADDRESS)
    ap.add_argument("--ray_namespace", type=str, default=DEFAULT_RAY_NAMESPACE)
    ap.add_argument("--queue_name", type=str, default=DEFAULT_QUEUE_NAME)
    ap.add_argument("--device", type=str, default=None)
    ap.add_argument("--task", type=str, default="print", choices=["print", "peakfind", "train", "none"],
                    help="train: online PeakNetLite training from peak-finder labels (trainer.py)")
    ap.add_argument("--lr", type=float, default=1e-3, help="--task train: AdamW learning rate")
    ap.add_argument("--save", type=str, default=None, help="--task train: write the model state_dict here")
    ap.add_argument("--ddp", action="store_true",
                    help="--task train: data-parallel training over the consumer processes of a torchrun launch "
                         "(gradients all-reduced by RCCL on GPUs, gloo on the CPU)")
    ap.add_argument("--batch", type=int, default=None,
                    help="frames per peak-finder / training batch (default: config.pipeline_shape -- 64, or 32 when "
                         "the launch puts more ranks than GPUs on this node)")
    ap.add_argument("--prefetch", type=int, default=None,
                    help=f"read-ahead bound: frames delivered but not read yet + grants outstanding (default "
                         f"max({DEFAULT_PREFETCH}, 2 x --batch)); what a crashed consumer can lose")
    ap.add_argument("--max_frames", type=int, default=None)
    ap.add_argument("--thr_peak", type=float, default=20.0)
    ap.add_argument("--son_min", type=float, default=5.0)
    ap.add_argument("--out", type=str, default=None, help="write peaks (npz) when --task peakfind")
    ap.add_argument("--timeout", type=float, default=300.0)
    ap.add_argument("--metrics_interval", type=float, default=10.0, help="seconds between rate lines; 0 disables")
    ap.add_argument("--metrics_json", type=str, default=None, help="append per-interval metrics as JSON lines")
    ap.add_argument("--log_level", type=str, default=DEFAULT_LOG_LEVEL, choices=LOG_LEVELS)
    return ap


def _init_data_parallel(device) -> int:
    """Join the torchrun group of the training consumers: RCCL ("nccl") on GPUs, gloo on the CPU."""
    import torch
    import torch.distributed as dist

    if "WORLD_SIZE" not in os.environ or "RANK" not in os.environ:
        raise SystemExit("--ddp needs a torchrun launch (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT)")
    dev = torch.device(device)
    if not dist.is_initialized():
        kw = {"device_id": dev} if dev.type == "cuda" else {}
        dist.init_process_group("nccl" if dev.type == "cuda" else "gloo", **kw)
    log.info("data-parallel training: rank %d of %d (%s)", dist.get_rank(), dist.get_world_size(),
             dist.get_backend())
    return dist.get_rank()


def resolve_batch(batch=None) -> int:
    """--batch, else the library's pipeline shape for the ranks sharing this GPU (the producer CLI's
    co-consumer and bench.py resolve the same way)."""
    from .pipeline import resolve_consumer_batch

    return resolve_consumer_batch(batch)


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    logging.basicConfig(level=getattr(logging, args.log_level), format="%(asctime)s - %(levelname)s - %(message)s")
    import numpy as np
    import torch

    from .config import PeakFinderParams
    from .data_reader import DataReader, DataReaderError, EndOfStream

    args.batch = resolve_batch(args.batch)

    stop = {"flag": False}

    def handler(sig, frame):
        print("Ctrl+C pressed. Shutting down...")
        stop["flag"] = True

    signal.signal(signal.SIGINT, handler)
    t0 = time.time()
    n = 0
    peaks_total = 0
    records = []
    from .utils.metrics import Registry, Reporter

    registry = Registry()
    registry.register("consumer", lambda: {"frames_consumed": n, "peaks": peaks_total})
    reporter = None
    with DataReader(args.ray_address, args.queue_name, args.ray_namespace, consumer_id=args.consumer_id,
                    device=args.device, timeout_s=args.timeout,
                    prefetch=args.prefetch or max(DEFAULT_PREFETCH, 2 * args.batch)) as reader:
        cid = reader.consumer_id
        if reader.endpoint is not None:
            registry.register("queue", reader.endpoint.metrics)
        reporter = Reporter(registry, rank=cid if cid is not None else 0, interval=args.metrics_interval,
                            json_path=args.metrics_json).start()
        pf = None
        if args.task == "peakfind":
            from .ops import kernels

            params = PeakFinderParams(thr_peak=args.thr_peak, son_min=args.son_min)
        if args.task == "train":
            if reader.endpoint is None:
                log.error("--task train needs the distributed queue (a producer session)")
                return 2
            from .trainer import OnlinePeakNetTrainer

            ring = reader.endpoint.ring
            shape = reader.calibrator.out_shape if reader.calibrator is not None else ring.frame_shape
            dp_rank = 0
            if args.ddp:
                dp_rank = _init_data_parallel(ring.device)
            trainer = OnlinePeakNetTrainer(shape, ring.device, lr=args.lr,
                                           params=PeakFinderParams(thr_peak=args.thr_peak, son_min=args.son_min),
                                           ddp=args.ddp)
            registry.register("trainer", lambda: {"steps": trainer.steps, "loss": trainer.last_loss})
            try:
                with trainer.join():
                    for batch in reader.batches(args.batch, torch.float32, timeout=1.0):
                        trainer.step(batch.data)
                        n += len(batch)
                        peaks_total = trainer.positives
                        if stop["flag"] or (args.max_frames is not None and n >= args.max_frames):
                            break
            except DataReaderError as e:
                print(f"DataReader error: {e}")
                return 1
            log.info("Consumer %s: %d training steps, last loss %.4f", cid, trainer.steps, trainer.last_loss)
            print(f"Consumer {cid} trained: steps={trainer.steps} frames={n} loss={trainer.last_loss:.4f} "
                  f"params={trainer.param_checksum():.9e}", flush=True)
            if args.save and dp_rank == 0:
                torch.save(trainer.model.state_dict(), args.save)
            if args.ddp:
                import torch.distributed as dist

                dist.destroy_process_group()
        while args.task != "train" and not stop["flag"] and (args.max_frames is None or n < args.max_frames):
            try:
                if args.task == "peakfind" and reader.endpoint is not None:
                    items = reader.read_batch(args.batch, timeout=1.0)
                    if not items:
                        continue
                    meta_items = [(it.rank, it.idx, it.gevt) for it in items]
                    if reader.calibrator is not None:    # raw ring (--calibrate_on_read): calibrate here
                        frames = reader.calibrate(items)
                    else:
                        frames = [it.data for it in items]
                    shape = tuple(frames[0].shape)
                    dev = frames[0].device
                    F = len(items)
                    if dev.type == "cuda":
                        pk = torch.empty((F, params.max_peaks, 8), dtype=torch.float32, device=dev)
                        cnt = torch.zeros(F, dtype=torch.int32, device=dev)
                        sm = torch.zeros((F, 2), dtype=torch.float32, device=dev)
                        kernels.peakfind([frames[i] for i in range(F)], shape, params, pk, cnt, sm)
                        cnt_h = cnt.cpu()
                        for i, it in enumerate(items):
                            k = min(int(cnt_h[i]), params.max_peaks)
                            peaks_total += k
                            if args.out:
                                records.append((*meta_items[i], pk[i, :k].cpu().numpy()))
                    else:
                        from .ops import reference

                        pl, _ = reference.peakfind_reference(torch.stack([frames[i] for i in range(F)]), params)
                        for m, p in zip(meta_items, pl):
                            peaks_total += p.shape[0]
                            if args.out:
                                records.append((*m, p.numpy()))
                    if reader.calibrator is None:
                        for it in items:
                            it.release()
                    n += F
                else:
                    result = reader.read(timeout=1.0)
                    if result is None:
                        print(f"Consumer {cid} waiting for data...")
                        continue
                    rank, idx, data, photon_energy = result
                    if args.task == "print":
                        print(f"Consumer {cid} processed: rank={rank} | idx={idx} | shape={tuple(data.shape)} "
                              f"| photon_energy={photon_energy}")
                    n += 1
            except EndOfStream:
                log.info("Consumer %s: end of stream", cid)
                break
            except DataReaderError as e:
                print(f"DataReader error: {e}")
                print("Queue actor is dead. Exiting...")
                return 1
    if reporter is not None:
        reporter.stop(final_sample=args.metrics_interval > 0 or args.metrics_json is not None)
    dt = time.time() - t0
    log.info("Consumer %s: %d frames in %.2f s (%.1f frames/s), %d peaks", cid, n, dt, n / max(dt, 1e-9), peaks_total)
    if args.out and records:
        counts = np.array([r[3].shape[0] for r in records], dtype=np.int64)
        np.savez(args.out, rank=np.array([r[0] for r in records]), idx=np.array([r[1] for r in records]),
                 gevt=np.array([r[2] for r in records]), counts=counts,
                 peaks=np.concatenate([r[3].reshape(-1, 8) for r in records]).astype(np.float32))
    return 0


def cli(argv=None) -> int:
    """Console entry: startup failures (no store, no queue session, a queue of another frame
    shape) end with one clear line and rc 1 instead of a traceback."""
    try:
        return main(argv)
    except (TimeoutError, ConnectionError, RuntimeError) as e:
        log.error("consumer could not join the queue: %s", e)
        return 1


if __name__ == "__main__":
    sys.exit(cli())
