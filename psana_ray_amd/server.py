"""``psana-ray-server``: standalone rendezvous store (the ``ray start --head`` analog,
README.md:13-16).  Optional: producer rank 0 hosts the store itself when nothing listens at
``--ray_address``; run this when producers and consumers come and go across jobs.

    psana-ray-server --port 6379
"""
from __future__ import annotations

import argparse
import datetime
import logging
import signal
import sys
import threading

from .config import DEFAULT_STORE_PORT


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=DEFAULT_STORE_PORT)
    ap.add_argument("--log_level", default="INFO")
    a = ap.parse_args(argv)
    logging.basicConfig(level=getattr(logging, a.log_level), format="%(asctime)s - %(levelname)s - %(message)s")
    import torch.distributed as dist

    store = dist.TCPStore(a.host, a.port, is_master=True, wait_for_workers=False,
                          timeout=datetime.timedelta(seconds=3600))
    logging.info("psana-ray rendezvous store listening on %s:%d (Ctrl+C to stop)", a.host, a.port)
    done = threading.Event()
    signal.signal(signal.SIGINT, lambda *_: done.set())
    signal.signal(signal.SIGTERM, lambda *_: done.set())
    done.wait()
    del store
    return 0


if __name__ == "__main__":
    sys.exit(main())
