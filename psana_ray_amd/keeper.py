"""Queue keeper: keeps a queue's frames alive after its producers exit (``psana-ray-keeper``).

Reference behaviour (SURVEY R-11): the shared queue is a *detached* Ray actor
(psana_ray/shared_queue.py:35, ``lifetime="detached"``), so the frames a producer job put into it
outlive the job and a consumer started later still reads them.  In this framework the frames
live in the producers' own HBM pools; a producer that finished waits (bounded by ``--timeout``)
for consumers to take them.  The keeper removes that wait: it is a session member in the
``keeper`` role with a ring of its own, and

  * as a CONSUMER it grants slots to producers that finished producing and still hold
    undelivered frames (state ``draining``), and to LIVE producers whose backlog no other
    consumer has credit for (0.1 s in a row) -- so committed frames move into
    the keeper as they are produced and survive a producer crash, like puts into the detached
    actor; producers route to a keeper only when no real consumer has credit, so it never
    competes with live consumers (``QueueFabric.set_grant_filter`` / ``set_keeper``);
  * every frame it receives goes straight back on offer (``SlotPool.relay_ready``: headers kept)
    and, as a PRODUCER with the ``relay`` policy (never to itself), it delivers them to any
    consumer that attaches, whenever that is;
  * once every other producer of the session is finished and it holds nothing, it posts EOS on
    its links, publishes ``done`` and exits 0 -- consumers then see the end of the stream.

So a producer job drains into the keeper at memory speed and exits; consumers may come minutes
later.  The keeper's ring lives where the session's frames live: host shared memory for a CPU
session, an HBM ring on ``--device cuda:N`` for a GPU session (peer copies over xGMI as for any
consumer).  Memory: 2 x ``--slots`` frames (receive and re-offer budgets).

    psana-ray-keeper --ray_address 127.0.0.1:6379 --queue_name my --slots 512 [--device cuda:7]
"""
from __future__ import annotations

import argparse
import logging
import signal
import sys
import time

from .config import DEFAULT_LOG_LEVEL, DEFAULT_QUEUE_NAME, DEFAULT_RAY_ADDRESS, DEFAULT_RAY_NAMESPACE, LOG_LEVELS

log = logging.getLogger("psana_ray_amd.keeper")


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Keep a psana-ray queue's frames after its producers exit.")
    ap.add_argument("--ray_address", type=str, default=DEFAULT_RAY_ADDRESS)
    ap.add_argument("--ray_namespace", type=str, default=DEFAULT_RAY_NAMESPACE)
    ap.add_argument("--queue_name", type=str, default=DEFAULT_QUEUE_NAME)
    ap.add_argument("--slots", type=int, default=256, help="frames the keeper can hold")
    ap.add_argument("--device", type=str, default=None,
                    help="ring device: cpu for a CPU session; cuda:N for a GPU session (default cuda:0)")
    ap.add_argument("--timeout", type=float, default=300.0, help="seconds to wait for the queue session")
    ap.add_argument("--log_level", type=str, default=DEFAULT_LOG_LEVEL, choices=LOG_LEVELS)
    return ap


def run(args) -> int:
    import torch

    from .parallel.rendezvous import open_store
    from .queue.endpoint import QueueEndpoint
    from .queue.ring import FrameRing
    from .queue.session import QueueSession, wait_meta

    store = open_store(args.ray_address, spawn_if_absent=False, timeout_s=args.timeout)
    meta = wait_meta(store, args.ray_namespace, args.queue_name, args.timeout)
    if meta["device_kind"] == "cuda":
        device = torch.device(args.device or "cuda:0")
        if device.type != "cuda":
            raise SystemExit("psana-ray-keeper: this queue's frames live in HBM; give --device cuda:N")
        torch.cuda.set_device(device)
    else:
        device = torch.device("cpu")
    dtype = {"float32": torch.float32, "uint16": torch.uint16}[meta["dtype"]]
    shape = tuple(meta["frame_shape"])
    sess = QueueSession(store, args.ray_namespace, args.queue_name, meta, "keeper",
                        device=device.index if device.type == "cuda" else -1)
    stop = {"flag": False}
    signal.signal(signal.SIGINT, lambda *_: stop.__setitem__("flag", True))
    signal.signal(signal.SIGTERM, lambda *_: stop.__setitem__("flag", True))
    try:
        n = int(args.slots)
        ring = FrameRing(shape, dtype, device, n, n, shm_name=sess.ring_name() if device.type == "cpu" else None)
        ep = QueueEndpoint(ring, sess, is_producer=True, is_consumer=True, route="relay", keeper=True)
        fab = ep._fabric
        fab.set_grant_filter(True)
        ep.start()
        pool = ring.pool
        log.info("keeper joined queue %s/%s as member %d on %s (%d slots)", args.ray_namespace, args.queue_name,
                 sess.mid, device, n)
        granted = set()
        kept = relayed = 0
        seen_producer = False
        while not stop["flag"]:
            others = {m: i for m, i in sess.producers().items() if i.get("role") != "keeper"}
            seen_producer |= bool(others)
            for mid, info in others.items():
                if mid not in granted and (sess.state(mid) == "draining" or sess.finished(mid)):
                    fab.set_peer_grantable(mid, True)
                    granted.add(mid)
            # received frames go straight back on offer in ONE locked native step bounded by the
            # producer room read under that lock (SlotPool.relay_ready): a frame is never taken out of
            # the receive side without room to re-offer it, however the fabric thread interleaves
            moved = pool.relay_ready(64)
            kept += moved
            if moved == 0:
                time.sleep(0.005 if pool.n_ready() else 0.02)   # nothing received, or no room yet
            if ep.failed is not None:
                raise RuntimeError(f"queue fabric failed: {ep.failed}")
            idle = pool.n_ready() == 0 and pool.n_produced() == 0 and pool.consumer_held() == 0 \
                and pool.producer_held() == 0
            if seen_producer and idle and all(sess.finished(m) for m in others):
                break
        relayed = int(ep.metrics().get("frames_sent", 0))
        ep.finish()
        ep.join(timeout=args.timeout)
        log.info("keeper: %d frames kept, %d delivered; every producer finished -- leaving", kept, relayed)
        print(f"keeper done: kept={kept} delivered={relayed}", flush=True)
        ep.close()
        sess.close("done")
        return 0
    except BaseException:
        sess.close("failed")
        raise


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    logging.basicConfig(level=getattr(logging, args.log_level), format="%(asctime)s - %(levelname)s - %(message)s")
    try:
        return run(args)
    except (TimeoutError, ConnectionError, RuntimeError) as e:
        log.error("keeper: %s", e)
        return 1


if __name__ == "__main__":
    sys.exit(main())
