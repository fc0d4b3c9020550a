"""Queue-session rendezvous for separately launched producers and consumers.

Reference behaviour being replaced (SURVEY R-02, C-04, CS-1/CS-4):
  * producer rank 0 ``ray.init(address, namespace)`` and looks the named queue actor up, creating a
    detached one if missing (psana_ray/producer.py:39-48, shared_queue.py:33-35);
  * an MPI Barrier, then every rank retries ``ray.get_actor`` 10 x 1 s (producer.py:53-67);
  * consumers ``ray.init`` + ``ray.get_actor(queue_name, namespace)`` (data_reader.py:12-24).

Here the "cluster" is a ``torch.distributed.TCPStore`` at the reference's ``--ray_address``
(``auto`` -> ``$PSANA_RAY_ADDRESS`` or ``127.0.0.1:6379``, the Ray head port of README.md:15).
Producer rank 0 hosts the store unless one is already listening there (``psana-ray-server``, the
``ray start --head`` analog).  A queue is a SESSION keyed by ``(ray_namespace, queue_name)``:
producers publish its metadata (first writer wins: attach-if-exists, Q-5), consumers claim ids
with an atomic counter, and once all ``n_producers + num_consumers`` ranks arrived they form one
process group (gloo control + RCCL/gloo data) through a prefixed view of the store.  Waits are
bounded (``timeout_s``) instead of the reference's unbounded Barrier (Q-7).
"""
from __future__ import annotations

import datetime
import json
import logging
import socket
import time
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist

from ..config import resolve_address

log = logging.getLogger(__name__)


def _connect_store(host: str, port: int, is_master: bool, timeout_s: float):
    return dist.TCPStore(host, port, is_master=is_master, timeout=datetime.timedelta(seconds=timeout_s),
                         wait_for_workers=False)


def port_open(host: str, port: int, timeout_s: float = 0.5) -> bool:
    try:
        with socket.create_connection((host, port), timeout=timeout_s):
            return True
    except OSError:
        return False


def open_store(address: Optional[str], host_if_absent: bool, timeout_s: float = 60.0, retries: int = 10,
               retry_delay_s: float = 1.0):
    """Connect to the rendezvous store; optionally host it if nobody listens there yet."""
    host, port = resolve_address(address)
    last = None
    for attempt in range(max(1, retries)):
        if port_open(host, port):
            try:
                return _connect_store(host, port, False, timeout_s)
            except Exception as e:  # noqa: BLE001
                last = e
        if host_if_absent:
            try:
                st = _connect_store(host, port, True, timeout_s)
                log.info("hosting the psana-ray rendezvous store at %s:%d", host, port)
                return st
            except Exception as e:  # noqa: BLE001 - somebody else won the race
                last = e
        log.info("Attempt %d/%d to reach the queue store at %s:%d failed. Retrying...", attempt + 1, retries,
                 host, port)   # producer.py:63
        time.sleep(retry_delay_s)
    raise TimeoutError(f"Timeout waiting for the queue store at {host}:{port}: {last}")


@dataclass
class SessionMeta:
    queue_size: int
    n_producers: int
    n_consumers: int
    frame_shape: tuple
    dtype: str
    device_kind: str           # "cuda" (RCCL data plane) or "cpu" (gloo)
    session: int = 0
    extra: dict = field(default_factory=dict)

    def to_json(self) -> str:
        d = dict(self.__dict__)
        d["frame_shape"] = list(self.frame_shape)
        return json.dumps(d)

    @classmethod
    def from_json(cls, s) -> "SessionMeta":
        d = json.loads(s)
        d["frame_shape"] = tuple(d["frame_shape"])
        return cls(**d)


@dataclass
class Session:
    store: object
    prefix: str
    meta: SessionMeta
    rank: int            # rank inside the queue world
    world: int
    role: str            # "producer" | "consumer"
    role_index: int      # producer rank / consumer id

    @property
    def producer_ranks(self):
        return list(range(self.meta.n_producers))

    @property
    def consumer_ranks(self):
        return list(range(self.meta.n_producers, self.meta.n_producers + self.meta.n_consumers))


def _key(ns: str, name: str) -> str:
    return f"psana_ray/{ns}/{name}"


def producer_join(store, namespace: str, queue_name: str, producer_rank: int, n_producers: int,
                  meta: SessionMeta, timeout_s: float = 300.0) -> Session:
    """Producer side.  Rank 0 publishes the session metadata (attach-if-exists: an already
    published queue keeps its queue_size, psana_ray/producer.py:43-45); all ranks then wait for
    it, bounded by ``timeout_s``."""
    base = _key(namespace, queue_name)
    if producer_rank == 0:
        if store.check([f"{base}/meta"]) and heartbeat_fresh(store, base):
            raise RuntimeError(f"queue {queue_name!r} in namespace {namespace!r} is in use by a running producer job")
        meta.session = store.add(f"{base}/session_counter", 1)
        store.set(f"{base}/meta", meta.to_json())
        beat(store, base)
        log.info("Rank 0: Shared queue %s created (namespace %s, queue_size=%d, session %d).", queue_name, namespace,
                 meta.queue_size, meta.session)
        got = meta
    else:
        # wait for rank 0's meta of THIS job (a fresh heartbeat distinguishes it from a stale one)
        deadline = time.time() + timeout_s
        while True:
            if store.check([f"{base}/meta"]) and heartbeat_fresh(store, base):
                got = SessionMeta.from_json(store.get(f"{base}/meta").decode())
                break
            if time.time() > deadline:
                raise TimeoutError(f"Rank {producer_rank}: Timeout waiting for shared queue {queue_name!r}")
            time.sleep(0.2)
    if got.n_producers != n_producers:
        raise RuntimeError(f"queue {queue_name!r} was created for {got.n_producers} producers, this job has {n_producers}")
    prefix = f"{base}/s{got.session}"
    store.set(f"{prefix}/producer/{producer_rank}", socket.gethostname())
    return Session(store, prefix, got, producer_rank, got.n_producers + got.n_consumers, "producer", producer_rank)


HEARTBEAT_S = 2.0


def beat(store, base: str):
    store.set(f"{base}/heartbeat", repr(time.time()))


def heartbeat_fresh(store, base: str, max_age_s: float = 5 * HEARTBEAT_S) -> bool:
    try:
        if not store.check([f"{base}/heartbeat"]):
            return False
        return time.time() - float(store.get(f"{base}/heartbeat").decode()) < max_age_s
    except Exception:  # noqa: BLE001
        return False


class Heartbeat:
    """Producer rank 0 keeps its session's heartbeat fresh (liveness for attach/refusal)."""

    def __init__(self, store, namespace: str, queue_name: str):
        import threading

        self.base = _key(namespace, queue_name)
        self.store = store
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True, name="psana-ray-heartbeat")
        self._t.start()

    def _run(self):
        while not self._stop.wait(HEARTBEAT_S):
            try:
                beat(self.store, self.base)
            except Exception:  # noqa: BLE001
                return

    def stop(self):
        self._stop.set()


def consumer_join(store, namespace: str, queue_name: str, consumer_id: Optional[int] = None,
                  timeout_s: float = 300.0) -> Session:
    """Consumer side: wait for the queue's metadata, claim a consumer id (or use the given one)."""
    base = _key(namespace, queue_name)
    deadline = time.time() + timeout_s
    while not (store.check([f"{base}/meta"]) and heartbeat_fresh(store, base)):
        if time.time() > deadline:
            raise TimeoutError(f"queue {queue_name!r} in namespace {namespace!r} did not appear within {timeout_s}s")
        time.sleep(0.2)
    meta = SessionMeta.from_json(store.get(f"{base}/meta").decode())
    prefix = f"{base}/s{meta.session}"
    if consumer_id is None:
        consumer_id = store.add(f"{prefix}/consumer_seq", 1) - 1
    if not 0 <= consumer_id < meta.n_consumers:
        raise RuntimeError(f"consumer id {consumer_id} out of range: the queue expects {meta.n_consumers} consumers "
                           f"(--num_consumers)")
    store.set(f"{prefix}/consumer/{consumer_id}", socket.gethostname())
    rank = meta.n_producers + consumer_id
    return Session(store, prefix, meta, rank, meta.n_producers + meta.n_consumers, "consumer", consumer_id)


def form_world(sess: Session, device, timeout_s: float = 300.0):
    """All ranks of the session form one process group through the prefixed store."""
    from .comm import init_groups

    pstore = dist.PrefixStore(f"{sess.prefix}/pg", sess.store)
    return init_groups(sess.rank, sess.world, device, store=pstore, timeout_s=timeout_s)


def finish_session(sess: Session):
    """Producer rank 0 retires the session so the next job creates a fresh queue."""
    if sess.role == "producer" and sess.role_index == 0:
        try:
            base = _key_from_prefix(sess.prefix)
            sess.store.delete_key(f"{base}/meta")
            sess.store.delete_key(f"{base}/heartbeat")
        except Exception:  # pragma: no cover
            pass


def _key_from_prefix(prefix: str) -> str:
    return prefix.rsplit("/s", 1)[0]
