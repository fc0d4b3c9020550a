"""One process's endpoint of the shared queue (producer and/or consumer roles).

Reference contract being replaced (psana_ray/shared_queue.py, producer.py, data_reader.py):
  * producers ``put([rank, idx, data, photon_energy])``; a full queue returns False and the
    producer backs off (producer.py:98-111) -- here ``acquire()`` hands out an HBM slot of the
    producer's own pool when it has room, blocking on a condition variable instead of sleeping.
    The pool IS the producer's share of the queue: frames wait there until a consumer takes them,
    so producers run with no consumer attached, exactly like puts into the Ray actor;
  * consumers ``get()`` non-blocking, None when empty (data_reader.py:31-37);
  * end of stream was a ``None`` sentinel indistinguishable from "empty" (Q-2) and depended on a
    global MPI Barrier (producer.py:120, hang risk Q-7) -- here every producer posts EOS on each
    of its links once all its frames are delivered; a consumer raises :class:`EndOfStream` when
    every producer of the session finished (or died) and its shard is drained.  No barrier;
  * a dead queue actor raised RayActorError -> DataReaderError (data_reader.py:36-37) -- here the
    queue has no single point of failure: a dead peer only loses what it held; a failure of this
    process's own fabric raises :class:`QueuePeerError`.

Two modes:
  * local (``session=None``): a single process produces and consumes; frames are routed producer
    -> own consumer inside the native pool (zero copy: the calibration kernel already wrote them
    into the consumer's slot);
  * session: the native :class:`QueueFabric` (csrc/fabric.h) runs this process's links -- HIP IPC
    peer writes over xGMI between GPU processes, shared memory between host processes -- and the
    :class:`~psana_ray_amd.queue.session.QueueSession` watcher adds / drops links as members come
    and go.
"""
from __future__ import annotations

import logging
import math
import struct
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from ..ops import _ext
from .ring import FrameRing

log = logging.getLogger(__name__)

# relay: queue keeper; remote_only: every frame crosses to another process while one is linked
POLICIES = {"balanced": 0, "local_first": 1, "spread": 2, "relay": 3, "remote_only": 4}


class QueueError(RuntimeError):
    pass


class QueueClosed(QueueError):
    """The endpoint was closed."""


class QueuePeerError(QueueError):
    """This process's queue fabric failed (the reference's 'Queue actor is dead')."""


class EndOfStream(QueueError):
    """Every producer finished and this consumer's shard is drained."""


def _pe_bits(pe: Optional[float]) -> int:
    return struct.unpack("<q", struct.pack("<d", float("nan") if pe is None else float(pe)))[0]


def _pe_from_bits(b: int) -> Optional[float]:
    v = struct.unpack("<d", struct.pack("<q", int(b)))[0]
    return None if math.isnan(v) else v


@dataclass
class FrameItem:
    """A frame leased from the ring.  ``data`` is a view of the HBM slot: call ``release()``
    (or use ``with``) when done, or ``to_list(copy=True)`` for a reference-style owned item."""

    endpoint: "QueueEndpoint"
    slot: int
    rank: int
    idx: int
    gevt: int
    photon_energy: Optional[float]
    data: torch.Tensor
    _released: bool = False

    def release(self, stream=None):
        if not self._released:
            self._released = True
            self.endpoint.release(self.slot, stream)

    def to_list(self, copy: bool = True):
        """``[rank, idx, data, photon_energy]`` -- the reference item (producer.py:101)."""
        data = self.data.clone() if copy else self.data
        if copy:
            self.release()
        return [self.rank, self.idx, data, self.photon_energy]

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.release()
        return False


class QueueEndpoint:
    def __init__(self, ring: FrameRing, session=None, is_producer: bool = True, is_consumer: bool = True,
                 route: str = "balanced", prefetch: int = 0, keeper: bool = False,
                 copy_engine: Optional[str] = None, copy_workgroups: Optional[int] = None,
                 copy_stream: Optional[str] = None):
        """``prefetch`` (consumer role, fabric mode): at most this many frames noticed-but-not-taken
        plus grants outstanding -- the read-ahead a crashed consumer can lose (0: the ring's free
        slots only).  ``keeper``: this member is a queue keeper (its links are marked so producers
        use it only as the last resort).  ``copy_engine`` / ``copy_workgroups`` (producer role, GPU):
        how frames move into other processes' rings (config.fabric_copy_setting)."""
        if route not in POLICIES:
            raise ValueError(f"unknown routing policy {route!r} ({' | '.join(POLICIES)})")
        self.ring = ring
        self.pool = ring.pool
        self.session = session
        self.is_producer, self.is_consumer = bool(is_producer), bool(is_consumer)
        self.route = route
        self.gpu = ring.device.type == "cuda"
        self._producer_finished = not is_producer
        self._consumer_closed = not is_consumer
        self._views = ring.views                  # per-slot tensor views, built once
        self._slot_bytes = ring.slot_bytes   # the ring's slot stride (>= frame_bytes): what the fabric moves
        self._fabric = None
        self._final: dict = {}
        self._started = False
        self._closed = False
        self._drained_published = False
        if session is None:
            # single process: frames are routed producer -> own consumer inside the native pool
            self.pool.set_auto_route(True)
            self.xport = "local"
            return
        C = _ext.load()
        dev = -1
        if self.gpu:
            dev = ring.device.index if ring.device.index is not None else torch.cuda.current_device()
        self._fabric = C.QueueFabric(self.pool, self._slot_bytes, dev, self.is_producer, self.is_consumer,
                                     POLICIES[route], session.mid)
        self._fabric.set_prefetch(int(prefetch))
        self._fabric.set_keeper(bool(keeper))
        from ..config import FABRIC_COPY_ENGINES, STREAM_KINDS, fabric_copy_setting

        eng, wgs, kind = fabric_copy_setting(copy_engine, copy_workgroups, copy_stream)
        self._fabric.set_copy_engine(FABRIC_COPY_ENGINES[eng], int(wgs), STREAM_KINDS[kind])
        from ..config import fabric_direct, fabric_verify_every

        self._fabric.set_verify_every(fabric_verify_every())
        self._fabric.set_direct(fabric_direct())   # GPU producers with the kernel engine only
        self.copy_engine = (eng, int(wgs), kind)
        if self.is_consumer:
            if self.gpu:
                self._fabric.export_ipc_ring()
            else:
                if ring.shm_name is None:
                    raise ValueError("a host consumer's ring must live in shared memory (FrameRing(shm_name=...))")
                self._fabric.export_host_ring(ring.shm_name)
        self.xport = "fabric"

    # ------------------------------------------------------------------------ membership
    def _on_member(self, mid: int, info: dict):
        from .session import CONSUMER_ROLES, PRODUCER_ROLES

        role = info["role"]
        if self.is_consumer and role in PRODUCER_ROLES:
            self._fabric.add_in_link(mid, self.session.link_name(mid, self.session.mid))
        if self.is_producer and role in CONSUMER_ROLES:
            self._fabric.add_out_link(mid, self.session.link_name(self.session.mid, mid))

    def _on_dead(self, mid: int):
        if self._fabric is not None:
            self._fabric.drop_peer(mid)

    def _on_tick(self):
        # publish "done" as soon as every frame was delivered: consumers end their stream on it
        fab = self._fabric
        if fab is not None and self.is_producer and not self._drained_published and fab.producer_drained:
            self._drained_published = True
            self.session.set_state("done")

    def start(self):
        if self._fabric is not None and not self._started:
            self._started = True
            self._fabric.start()
            self.session.start(self._on_member, self._on_dead, self._on_tick)
        return self

    def set_route(self, route: str):
        """Switch the routing policy of this producer at run time (e.g. bench phases)."""
        if route not in POLICIES:
            raise ValueError(f"unknown routing policy {route!r}")
        self.route = route
        if self._fabric is not None:
            self._fabric.set_policy(POLICIES[route])

    # ------------------------------------------------------------------------ helpers
    def _stream(self, stream) -> int:
        if not self.gpu:
            return 0
        return _ext.stream_handle(stream)

    @property
    def failed(self) -> Optional[BaseException]:
        if self._fabric is None:
            return None
        err = self._fabric.error()
        return RuntimeError(err) if err else None

    def _raise_if_failed(self):
        err = self.failed
        if err is not None:
            raise QueuePeerError(f"shared queue fabric failed: {err}") from err

    # ------------------------------------------------------------------------ producer
    def acquire(self, timeout: Optional[float] = None, stream=None) -> Optional[int]:
        """A free slot for the next calibrated frame, or None on timeout (queue full).
        ``stream`` (default: current) is ordered after the slot's previous readers."""
        self._raise_if_failed()
        if timeout is not None and timeout <= 0:
            s = self.pool.try_acquire_produce()
        else:
            s = self.pool.acquire_produce(-1.0 if timeout is None else float(timeout))
        if s < 0:
            self._raise_if_failed()
            return None
        self.pool.wait_free_on(s, self._stream(stream))
        return s

    def slot_tensor(self, slot: int) -> torch.Tensor:
        return self._views[slot]

    def slot_ptr(self, slot: int) -> int:
        return self.ring.slot_ptrs[slot]

    def commit(self, slot: int, rank: int, idx: int, gevt: int, photon_energy: Optional[float], stream=None):
        C = _ext.load()
        h = C.SlotHeader(int(rank), int(idx), int(gevt), float("nan") if photon_energy is None else float(photon_energy))
        self.pool.commit_produce(slot, h, self._stream(stream))

    def abort(self, slot: int):
        self.pool.abort_produce(slot)

    def finish(self):
        """This process's producer has no more events; its EOS follows once every frame it holds
        was delivered (drain before exit)."""
        if self._producer_finished:
            return
        self._producer_finished = True
        if self._fabric is not None:
            self._fabric.set_producer_finished()
            self.session.set_state("draining")

    @property
    def producer_drained(self) -> bool:
        """Finished, and every frame delivered (with EOS on every link)."""
        if not self.is_producer:
            return True
        if self._fabric is None:
            return self._producer_finished and self.pool.n_produced() == 0
        return bool(self._fabric.producer_drained)

    def undelivered(self) -> int:
        """Frames this producer still holds (not yet taken by any consumer)."""
        return int(self.pool.n_produced())

    # ------------------------------------------------------------------------ consumer
    def get(self, timeout: float = 0.0, stream=None) -> Optional[FrameItem]:
        """Next frame (FIFO within this shard) or None if none arrives within ``timeout``.
        Raises EndOfStream once every producer finished and the shard is drained."""
        s = self.pool.try_get() if timeout <= 0 else self.pool.get(float(timeout))
        if s < 0:
            self._raise_if_failed()
            if self.stream_done and self.pool.n_ready() == 0:
                raise EndOfStream("all producers finished and the queue shard is drained")
            return None
        self.pool.wait_ready_on(s, self._stream(stream))
        if self._fabric is not None:
            self.pool.check_frames([s], self._stream(stream))   # acquire / checksum of a peer-written frame
        h = self.pool.header(s)
        pe = None if math.isnan(h.photon_energy) else h.photon_energy
        return FrameItem(self, s, h.rank, h.idx, h.gevt, pe, self._views[s])

    def get_batch(self, max_n: int, timeout: float = 0.0, stream=None) -> List[int]:
        """Up to ``max_n`` ready slots in ONE native call (waits up to ``timeout`` for the
        first); ``stream`` is ordered after their data.  Release with :meth:`release_batch`.
        Raises EndOfStream like :meth:`get`."""
        slots = self.pool.get_batch(int(max_n), float(timeout), self._stream(stream))
        if not slots:
            self._raise_if_failed()
            if self.stream_done and self.pool.n_ready() == 0:
                raise EndOfStream("all producers finished and the queue shard is drained")
        return slots

    def release_batch(self, slots: Sequence[int], stream=None):
        if slots:
            self.pool.release_batch(list(slots), self._stream(stream))

    def release(self, slot: int, stream=None):
        self.pool.release(slot, self._stream(stream))

    def close_consumer(self):
        """Stop taking frames: producers stop writing into this shard (frames whose copy was in
        flight go back to their producer's FIFO), and every frame that arrived here and was not
        taken is handed back to a live producer for the other consumers (reference: items nobody
        got stay in the actor).  Call it once this process stopped reading.  Frames no live
        producer can take back (all finished) are counted in ``frames_dropped``."""
        if self._consumer_closed:
            return
        self._consumer_closed = True
        if self._fabric is not None:
            self._fabric.set_consumer_closed()

    @property
    def stream_done(self) -> bool:
        """Every producer of the stream finished (or died) and delivered all it will deliver."""
        if self._fabric is None:
            return self._producer_finished and self.pool.n_produced() == 0
        if self.is_producer and not self.producer_drained:
            return False
        sess = self.session
        prods = sess.producers()
        if not prods and not self.is_producer:
            return False   # nobody has produced into this queue yet: keep waiting
        links = {ls.peer: ls for ls in self._fabric.links() if not ls.outgoing}
        for mid in prods:
            if not sess.finished(mid):
                return False
            ls = links.get(mid)
            if ls is not None and ls.attached and not (ls.eos or ls.dead or ls.detached):
                return False
        return True

    def size(self) -> int:
        """Frames ready in this shard (reference Queue.size, shared_queue.py:26-31)."""
        return self.pool.n_ready()

    # ------------------------------------------------------------------------ lifecycle
    def join(self, timeout: Optional[float] = None) -> bool:
        """Producer: wait until every frame this process produced was delivered (drain before
        exit, bounded by ``timeout``).  True when drained."""
        t0 = time.monotonic()
        while not self.producer_drained:
            if self.failed is not None:
                return False
            if timeout is not None and time.monotonic() - t0 > timeout:
                return False
            time.sleep(0.01)
        if self._fabric is not None and self.is_producer and not self._drained_published:
            self._drained_published = True
            self.session.set_state("done")
        return True

    def close(self, timeout: float = 10.0) -> None:
        """Leave the queue: a consumer first makes sure no producer still writes into its ring;
        then the fabric thread stops and the links are detached.  Idempotent."""
        if self._closed or self._fabric is None:
            self._closed = True
            return
        self._closed = True
        fab = self._fabric
        if self.is_consumer:
            self.close_consumer()
            t0 = time.monotonic()
            while not fab.consumer_quiesced and time.monotonic() - t0 < timeout and not fab.error():
                time.sleep(0.005)
        if self.is_producer and self.producer_drained and not self._drained_published:
            self._drained_published = True
            self.session.set_state("done")
        final = "done" if (not self.is_producer or self._drained_published) else "failed"
        self.session.close(final if self.is_producer else "closed")
        self._final = self._counters()
        self._final["verify"] = self.verify_counts()
        fab.request_stop()
        if not fab.join(timeout):
            log.warning("queue fabric thread did not stop within %.0f s", timeout)
            return
        self._fabric = None   # destructor: detach links, close IPC mappings

    # ------------------------------------------------------------------------ observability
    def _counters(self) -> dict:
        if self._fabric is None:
            return dict(self._final)
        st = self._fabric.stats()
        links = self._fabric.links()
        return {"frames_local": st.frames_local, "frames_sent": st.frames_sent, "frames_recv": st.frames_recv,
                "frames_requeued": st.frames_requeued, "bytes_sent": st.bytes_sent, "bytes_recv": st.bytes_recv,
                "batches": st.batches, "grants_given": st.grants_given, "grants_returned": st.grants_returned,
                "grants_reclaimed": st.grants_reclaimed, "peers_dead": st.peers_dead,
                "links_failed": st.links_failed, "frames_returned": st.frames_returned,
                "frames_reclaimed": st.frames_reclaimed, "frames_dropped": st.frames_dropped,
                "returns_rejected": st.returns_rejected, "readahead": st.readahead,
                "links_opened": st.links_opened, "links_live": sum(1 for ls in links if ls.attached and not ls.dead),
                "copy_ms_per_batch": 1e3 * st.copy_s / max(1, st.batches),
                "copy_launches": st.copy_launches, "copy_dev_ms": st.copy_dev_ms,
                "copy_dev_bytes": st.copy_dev_bytes, "taken_local": st.taken_local,
                "taken_remote": st.taken_remote,
                "frames_checksummed": st.frames_checksummed, "frames_corrupted": st.frames_corrupted,
                "frames_direct": st.frames_direct, "frames_lost_direct": st.frames_lost_direct,
                "iterations": st.iterations, "idle_iterations": st.idle_iterations}

    def links(self) -> list:
        return [] if self._fabric is None else list(self._fabric.links())

    def copy_samples(self) -> list:
        """Timed copy dispatches of this producer (newest last): ``(device ms, issue->done ms, bytes,
        frames, links)`` -- device ms is the copy alone, issue->done includes the wait for the
        frames' calibration the copy is ordered after."""
        if self._fabric is None:
            return []
        return [(c.dev_ms, c.issue_to_done_ms, c.bytes, c.frames, c.links) for c in self._fabric.copy_samples()]

    def verify_counts(self) -> dict:
        """End-to-end checks of frames other processes wrote into this consumer's ring (csrc/verify.h):
        frames re-summed and compared with their producer's checksum, mismatches (and the last
        mismatching gevt), and the system-scope acquires issued before reading peer-written frames.
        On a GPU ring, synchronise the streams the frames were read on first for an exact count."""
        if self._fabric is None:
            return dict(self._final.get("verify", {"verified": 0, "mismatched": 0, "last_bad_gevt": -1,
                                                   "acquires": 0}))
        v, m, g, a = self._fabric.verify_counts()
        return {"verified": int(v), "mismatched": int(m), "last_bad_gevt": int(g), "acquires": int(a)}

    def metrics(self) -> dict:
        """Gauges + cumulative counters for utils.metrics."""
        d = {"ready": self.pool.n_ready(), "credits": self.pool.credits(), "held": self.pool.n_produced()}
        d.update(self._counters())
        return d

    def stats(self) -> dict:
        d = self.ring.stats()
        d.update(self._counters())
        d["xport"] = self.xport
        return d
