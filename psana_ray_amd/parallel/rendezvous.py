"""Rendezvous store of the shared queue (the Ray head / GCS analog).

Reference behaviour being replaced (SURVEY R-02, C-04, CS-1/CS-5): ``ray start --head`` runs the
cluster head (README.md:13-16); producer rank 0 ``ray.init(address, namespace)`` and looks the
named queue actor up, creating a detached one if missing (psana_ray/producer.py:39-48,
shared_queue.py:33-35), every rank then retries ``ray.get_actor`` 10 x 1 s (producer.py:53-67);
consumers ``ray.init`` + ``ray.get_actor`` (data_reader.py:12-24).

Here the head is a ``torch.distributed.TCPStore`` at the reference's ``--ray_address``
(``auto`` -> ``$PSANA_RAY_ADDRESS`` or ``127.0.0.1:6379``, the Ray head port of README.md:15).
``psana-ray-server`` runs it standalone; when nothing listens at a local address the first member
SPAWNS one as a detached process (``start_new_session``), so the store -- and with it the queue's
membership -- outlives any single producer or consumer job, like the detached Ray actor; the
spawned server exits once no registered member has been alive for ``idle_exit`` seconds.  The
queue itself (sessions, members, links) is :mod:`psana_ray_amd.queue.session`.
"""
from __future__ import annotations

import datetime
import logging
import os
import socket
import subprocess
import sys
import time
from typing import Optional

import torch.distributed as dist

from ..config import resolve_address

log = logging.getLogger(__name__)

LOCAL_HOSTS = ("127.0.0.1", "localhost", "0.0.0.0", "::1")
SPAWNED_IDLE_EXIT_S = 60.0


def _connect_store(host: str, port: int, timeout_s: float):
    return dist.TCPStore(host, port, is_master=False, timeout=datetime.timedelta(seconds=timeout_s),
                         wait_for_workers=False)


def port_open(host: str, port: int, timeout_s: float = 0.5) -> bool:
    try:
        with socket.create_connection((host, port), timeout=timeout_s):
            return True
    except OSError:
        return False


def _is_local(host: str) -> bool:
    return host in LOCAL_HOSTS or host == socket.gethostname()


def spawn_server(host: str, port: int, idle_exit_s: float = SPAWNED_IDLE_EXIT_S) -> subprocess.Popen:
    """Start ``psana-ray-server`` as a detached process (own session: it survives this job)."""
    cmd = [sys.executable, "-m", "psana_ray_amd.server", "--host", host if host != "localhost" else "127.0.0.1",
           "--port", str(port), "--idle_exit", str(idle_exit_s), "--log_level", "WARNING"]
    env = dict(os.environ)
    pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    log.info("no rendezvous store at %s:%d: starting a detached psana-ray-server", host, port)
    return subprocess.Popen(cmd, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                            start_new_session=True, env=env, close_fds=True)


def open_store(address: Optional[str], spawn_if_absent: bool = True, timeout_s: float = 60.0, retries: int = 10,
               retry_delay_s: float = 1.0):
    """Connect to the rendezvous store at ``address``; start a detached server first when nothing
    listens at a local address (``spawn_if_absent``).  Retries like the reference's actor lookup
    (producer.py:56-67) and raises TimeoutError with the address when it stays unreachable."""
    host, port = resolve_address(address)
    last: Optional[BaseException] = None
    spawned = False
    for attempt in range(max(1, retries)):
        if port_open(host, port):
            try:
                return _connect_store(host, port, timeout_s)
            except Exception as e:  # noqa: BLE001
                last = e
        elif spawn_if_absent and not spawned and _is_local(host):
            spawn_server(host, port)
            spawned = True
            t0 = time.time()
            while time.time() - t0 < 15 and not port_open(host, port, 0.2):
                time.sleep(0.05)
            continue
        log.info("Attempt %d/%d to reach the queue store at %s:%d failed. Retrying...", attempt + 1, retries,
                 host, port)   # producer.py:63
        time.sleep(retry_delay_s)
    raise TimeoutError(f"no psana-ray rendezvous store reachable at {host}:{port} "
                       f"(start one with `psana-ray-server --port {port}`)" + (f": {last}" if last else ""))
