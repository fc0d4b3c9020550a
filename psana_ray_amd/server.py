"""``psana-ray-server``: standalone rendezvous store (the ``ray start --head`` analog,
README.md:13-16).  Producers and consumers start one themselves (detached, ``--idle_exit``) when
nothing listens at ``--ray_address``; run it explicitly to pin the address or keep it forever.

    psana-ray-server --port 6379
"""
from __future__ import annotations

import argparse
import datetime
import json
import logging
import signal
import sys
import threading
import time

from .config import DEFAULT_STORE_PORT


def _any_member_alive(store, boot: str) -> bool:
    """A queue member registered in this store (psana_ray/_reg/*) whose process still runs."""
    from .ops import _ext

    n = int(store.add("psana_ray/_reg_n", 0))
    C = None
    for i in range(n):
        key = f"psana_ray/_reg/{i}"
        if not store.check([key]):
            continue
        rec = json.loads(store.get(key).decode())
        if rec.get("boot") != boot:
            return True   # a member on another host: cannot check, assume alive
        if C is None:
            C = _ext.load()
        if C.pid_alive(int(rec["pid"])):
            return True
    return False


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=DEFAULT_STORE_PORT)
    ap.add_argument("--idle_exit", type=float, default=0.0,
                    help="exit once no registered queue member has been alive for this many seconds (0: never)")
    ap.add_argument("--log_level", default="INFO")
    a = ap.parse_args(argv)
    logging.basicConfig(level=getattr(logging, a.log_level), format="%(asctime)s - %(levelname)s - %(message)s")
    import torch.distributed as dist

    from .queue.session import boot_id

    store = dist.TCPStore(a.host, a.port, is_master=True, wait_for_workers=False,
                          timeout=datetime.timedelta(seconds=3600))
    logging.info("psana-ray rendezvous store listening on %s:%d (Ctrl+C to stop)", a.host, a.port)
    done = threading.Event()
    signal.signal(signal.SIGINT, lambda *_: done.set())
    signal.signal(signal.SIGTERM, lambda *_: done.set())
    if a.idle_exit > 0:
        boot = boot_id()
        client = dist.TCPStore("127.0.0.1" if a.host in ("0.0.0.0", "") else a.host, a.port, is_master=False,
                               wait_for_workers=False, timeout=datetime.timedelta(seconds=30))
        last_alive = time.time()
        while not done.wait(min(2.0, a.idle_exit / 4)):
            try:
                if _any_member_alive(client, boot):
                    last_alive = time.time()
            except Exception:  # noqa: BLE001
                pass
            if time.time() - last_alive > a.idle_exit:
                logging.info("no live queue member for %.0f s: exiting", a.idle_exit)
                break
        del client
    else:
        done.wait()
    del store
    return 0


if __name__ == "__main__":
    sys.exit(main())
