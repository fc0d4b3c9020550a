"""One rank's endpoint of the sharded shared queue (producer and/or consumer roles).

Reference contract being replaced (psana_ray/shared_queue.py, producer.py, data_reader.py):
  * producers ``put([rank, idx, data, photon_energy])``; a full queue returns False and the
    producer backs off (producer.py:98-111) -- here ``acquire()`` hands out an HBM slot only when
    the producer has budget, blocking on a condition variable instead of sleeping;
  * consumers ``get()`` non-blocking, None when empty (data_reader.py:31-37);
  * end of stream was a ``None`` sentinel indistinguishable from "empty" (Q-2) and depended on a
    global MPI Barrier (producer.py:120, hang risk Q-7) -- here every producer advertises its own
    EOS in the control round once all its frames are routed; a consumer raises
    :class:`EndOfStream` after EOS from every producer and an empty shard.  No barrier.
  * a dead queue actor raised RayActorError -> DataReaderError (data_reader.py:36-37) -- here a
    failed control/data exchange (peer died) raises :class:`QueuePeerError`.

Transport (world > 1, or loopback): rounds of all-gather (offers, credits, headers),
deterministic routing (parallel.routing), then one grouped RCCL send/recv exchange of the frames
on a dedicated stream.  Two drivers of those rounds:
  * ``native`` (default when every rank is on this host): the C++ TransportEngine
    (csrc/xport_engine.h) -- its own thread, control vectors all-gathered through a node-local
    shared-memory segment (microseconds instead of a gloo TCP all-gather), routing and the RCCL
    group issued without Python or the GIL; host pools copy through shared-memory outboxes;
  * ``python``: a Python thread, gloo all-gather, same routing and data plane (multi-host, A/B).
Select with ``xport=`` or ``PSANA_RAY_XPORT``.  World == 1: frames are routed locally (zero copy:
the calibration kernel already wrote them into the consumer's slot).
"""
from __future__ import annotations

import logging
import math
import os
import struct
import threading
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..ops import _ext
from ..utils.tracing import trace_range
from .ring import FrameRing

log = logging.getLogger(__name__)

F_PRODUCER, F_CONSUMER, F_EOS, F_CLOSED, F_FAILED = 1, 2, 4, 8, 16
_POLICY_CODE = {"balanced": 0, "local_first": 1, "spread": 2}
HDR = 4          # fixed words per control vector
PER_OFFER = 4    # rank, idx, gevt, photon-energy bits


class QueueError(RuntimeError):
    pass


class QueueClosed(QueueError):
    """The queue no longer accepts frames (all consumers left, or the endpoint was closed)."""


class QueuePeerError(QueueError):
    """A peer process / the transport failed (the reference's 'Queue actor is dead')."""


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
    def __init__(self, ring: FrameRing, rank: int = 0, world: int = 1, comm=None,
                 producer_ranks: Optional[Sequence[int]] = None, consumer_ranks: Optional[Sequence[int]] = None,
                 route: str = "balanced", max_offer: int = 64, is_producer: bool = True, is_consumer: bool = True,
                 loopback: bool = False, xport: Optional[str] = None):
        self.ring = ring
        self.pool = ring.pool
        self.rank, self.world, self.comm = rank, world, comm
        self.is_producer, self.is_consumer = is_producer, is_consumer
        self.producer_ranks = list(range(world)) if producer_ranks is None else list(producer_ranks)
        self.consumer_ranks = list(range(world)) if consumer_ranks is None else list(consumer_ranks)
        self.route = route
        self.max_offer = max_offer
        # loopback: frames routed to this rank itself still travel through the data exchange
        # (RCCL send/recv to self).  Lets a single GPU run the full multi-GPU transport path.
        self.loopback = bool(loopback)
        if self.loopback and comm is None:
            raise ValueError("loopback transport needs a Comm")
        self.gpu = ring.device.type == "cuda"
        self._lock = threading.Lock()
        self._producer_finished = not is_producer
        self._consumer_closed = not is_consumer
        self._eos_from: set = set()
        self._transport_done = comm is None and False
        self._py_failed: Optional[BaseException] = None
        self._py_consumers_gone = False
        self._round = 0
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self.rounds = 0
        self.round_time_s = 0.0
        self.frames_routed = 0
        if comm is None and world != 1:
            raise ValueError("world > 1 needs a Comm")
        if comm is None:
            # single process: frames are routed producer -> own consumer inside the native pool
            self.pool.set_auto_route(True)
        self._views = list(ring.storage.unbind(0))   # per-slot tensor views, built once
        self._base = int(ring.storage.data_ptr())
        self._slot_bytes = ring.frame_bytes
        self._engine = None
        self._engine_exc: Optional[BaseException] = None
        self.xport = "local" if comm is None else self._pick_xport(xport)
        if self.xport == "native" and not self._make_engine():
            self.xport = "python"

    # ------------------------------------------------------------------------ native transport
    def _pick_xport(self, xport: Optional[str]) -> str:
        x = (xport or os.environ.get("PSANA_RAY_XPORT", "native")).lower()
        if x not in ("native", "python"):
            raise ValueError(f"unknown transport driver {x!r} (native | python)")
        if x == "native" and not getattr(self.comm, "node_local", False):
            log.info("rank %d: ranks span hosts -> python transport driver", self.rank)
            x = "python"
        return x

    def _agree(self, ok: bool) -> bool:
        """All ranks' verdict (min over ranks, on the gloo control group)."""
        if self.world == 1:
            return ok
        import torch.distributed as dist

        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.comm.ctrl_group)
        return bool(t.item())

    def _make_engine(self) -> bool:
        """Set up the shared-memory control segment and the native engine.  Every rank must pick
        the same driver, so a segment that cannot be created or attached anywhere (no /dev/shm,
        size limits, ...) makes ALL ranks fall back to the python driver.  Returns success."""
        C = _ext.load()
        comm = self.comm
        rccl = getattr(comm, "rccl", None)
        tmo = float(os.environ.get("PSANA_RAY_XPORT_TIMEOUT_S", "300"))
        # host pools move frames through per-rank shared-memory outboxes (max_offer slots each)
        box = 0 if rccl is not None else self.max_offer * self._slot_bytes
        name = comm.shm_name()
        words = C.xport_vec_words(self.max_offer)

        def open_segment(create: bool):
            try:
                if os.environ.get("PSANA_RAY_XPORT_TEST_FAIL_RANK") == str(self.rank):
                    raise OSError("injected shared-memory failure (test hook)")
                # attaching happens after rank 0 created the segment: a short wait suffices
                return C.ShmControl(name, create, self.rank, self.world, words, box, tmo if create else 60.0)
            except Exception as e:  # noqa: BLE001
                log.warning("rank %d: shared-memory control segment %s unavailable: %r", self.rank, name, e)
                return None

        ctrl = open_segment(True) if self.rank == 0 else None
        if not self._agree(ctrl is not None or self.rank != 0):
            log.warning("rank %d: native transport unavailable -> python driver", self.rank)
            return False
        if self.rank != 0:
            ctrl = open_segment(False)
        if not self._agree(ctrl is not None):
            log.warning("rank %d: native transport unavailable on some rank -> python driver", self.rank)
            return False
        self._ctrl = ctrl
        dev = self.ring.device.index if self.gpu else -1
        if self.gpu and dev is None:
            dev = torch.cuda.current_device()
        self._engine = C.TransportEngine(self.pool, self._ctrl, rccl, self._base, self._slot_bytes, self.rank,
                                         self.world, self.producer_ranks, self.is_producer, self.is_consumer,
                                         _POLICY_CODE[self.route], self.max_offer, self.loopback,
                                         comm.stream_handle if rccl is not None else 0, dev)
        if self._producer_finished:
            self._engine.set_producer_finished()
        if self._consumer_closed:
            self._engine.set_consumer_closed()
        return True

    @property
    def _failed(self) -> Optional[BaseException]:
        if self._py_failed is not None:
            return self._py_failed
        if self._engine is not None and self._engine_exc is None:
            err = self._engine.error()
            if err:
                self._engine_exc = RuntimeError(err)
        return self._engine_exc

    @property
    def _consumers_gone(self) -> bool:
        if self._engine is not None:
            return bool(self._engine.consumers_gone)
        return self._py_consumers_gone

    # ------------------------------------------------------------------------ helpers
    def _stream(self, stream) -> int:
        if not self.gpu:
            return 0
        return _ext.stream_handle(stream)

    def _raise_if_failed(self):
        if self._failed is not None:
            raise QueuePeerError(f"shared queue transport failed: {self._failed!r}") from self._failed

    # ------------------------------------------------------------------------ producer
    def acquire(self, timeout: Optional[float] = None, stream=None) -> Optional[int]:
        """A free slot for the next calibrated frame, or None on timeout (queue full).
        ``stream`` (default: current) is ordered after the slot's previous readers."""
        self._raise_if_failed()
        if self._consumers_gone:
            raise QueueClosed("no consumer is attached to the queue any more")
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
        return self._base + slot * self._slot_bytes

    def commit(self, slot: int, rank: int, idx: int, gevt: int, photon_energy: Optional[float], stream=None):
        C = _ext.load()
        h = C.SlotHeader(int(rank), int(idx), int(gevt), float("nan") if photon_energy is None else float(photon_energy))
        self.pool.commit_produce(slot, h, self._stream(stream))

    def abort(self, slot: int):
        self.pool.abort_produce(slot)

    def finish(self):
        """This rank's producer has no more events (its EOS is advertised once drained)."""
        self._producer_finished = True
        if self._engine is not None:
            self._engine.set_producer_finished()

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
        self._consumer_closed = True
        if self._engine is not None:
            self._engine.set_consumer_closed()

    @property
    def stream_done(self) -> bool:
        if self.comm is None:
            return self._producer_finished and self.pool.n_produced() == 0
        if self._engine is not None:
            return bool(self._engine.done)
        return self._transport_done

    def size(self) -> int:
        """Frames ready in this shard (reference Queue.size, shared_queue.py:26-31)."""
        return self.pool.n_ready()

    # ------------------------------------------------------------------------ transport rounds
    def _control_vector(self, offers: List[int]) -> np.ndarray:
        v = np.zeros(HDR + PER_OFFER * self.max_offer, dtype=np.int64)
        flags = (F_PRODUCER if self.is_producer else 0) | (F_CONSUMER if self.is_consumer else 0)
        if self._producer_finished and not offers and self.pool.n_produced() == 0:
            flags |= F_EOS
        if self._consumer_closed:
            flags |= F_CLOSED
        credits = 0 if self._consumer_closed else self.pool.credits()
        v[0], v[1], v[2], v[3] = len(offers), credits, flags, self._round
        if offers:
            hs = self.pool.headers(list(offers))          # one native call for the whole offer list
            n = len(hs)
            w = v[HDR:HDR + PER_OFFER * n].reshape(n, PER_OFFER)
            w[:, 0] = [h.rank for h in hs]
            w[:, 1] = [h.idx for h in hs]
            w[:, 2] = [h.gevt for h in hs]
            # photon energy travels as the int64 bit pattern of the float64 (NaN = None)
            w[:, 3] = np.array([h.photon_energy for h in hs], dtype=np.float64).view(np.int64)
        return v

    def step(self) -> int:
        """Run ONE transport round (collective: every rank must call it).  Returns frames moved."""
        if self._engine is not None:
            return int(self._engine.step())
        t0 = time.perf_counter()
        C = _ext.load()
        comm = self.comm
        offers = self.pool.produced(self.max_offer) if self.is_producer else []
        with trace_range("transport.ctrl_allgather"):
            allv = comm.allgather_ctrl(self._control_vector(offers))
        flags = allv[:, 2]
        offer_n = [int(x) for x in allv[:, 0]]
        credits = [int(x) for x in allv[:, 1]]
        for r in range(self.world):
            if flags[r] & F_EOS:
                self._eos_from.add(r)
        consumers_alive = [r for r in range(self.world) if (flags[r] & F_CONSUMER) and not (flags[r] & F_CLOSED)]
        self._py_consumers_gone = len(consumers_alive) == 0
        flat = C.plan_round(offer_n, credits, self._round, _POLICY_CODE[self.route])
        me = self.rank
        sh = comm.stream_handle
        local, send_slots, send_dst, recv_src, recv_hdr = [], [], [], [], []
        n_plan = len(flat) // 3
        for k in range(n_plan):
            p, i, c = flat[3 * k], flat[3 * k + 1], flat[3 * k + 2]
            if p == me and c == me and not self.loopback:
                local.append(offers[i])
                continue
            if p == me:
                send_slots.append(offers[i])
                send_dst.append((c, k))
            if c == me:
                b = HDR + PER_OFFER * i
                row = allv[p]
                pe = _pe_from_bits(row[b + 3])
                recv_src.append((p, k))
                recv_hdr.append(C.SlotHeader(int(row[b]), int(row[b + 1]), int(row[b + 2]),
                                             float("nan") if pe is None else pe))
        for s in local:
            self.pool.route_local(s)
        if getattr(comm, "rccl", None) is not None:
            # GPU: one native call -- slot ordering, ncclGroupStart/Send/Recv/End, completion events
            if send_slots or recv_src:
                comm.round(self.pool, self._base, self._slot_bytes, send_slots, [c for c, _ in send_dst],
                           [p for p, _ in recv_src], recv_hdr)
            if self.rounds % 64 == 0:
                comm.check_async()
        else:
            self.pool.begin_send_batch(send_slots, sh)          # data-ready ordering
            recv_slots = self.pool.begin_recv_batch(len(recv_src), sh) if recv_src else []
            views = self._views
            sends = [(views[s], c, k) for s, (c, k) in zip(send_slots, send_dst)]
            recvs = [(views[s], p, k) for s, (p, k) in zip(recv_slots, recv_src)]
            with trace_range("transport.exchange"):
                comm.exchange(sends, recvs)
            # one event per direction per round (not one per frame)
            self.pool.end_send_batch(send_slots, sh)
            self.pool.end_recv_batch(recv_slots, recv_hdr, sh)
        self._round += 1
        self.rounds += 1
        self.frames_routed += n_plan
        self.round_time_s += time.perf_counter() - t0
        if all(r in self._eos_from for r in self.producer_ranks):
            self._transport_done = True
        return n_plan

    def _loop(self):
        if self.gpu:
            torch.cuda.set_device(self.ring.device)
        idle = 0.0
        try:
            while not self._transport_done:
                moved = self.step()
                if moved == 0:
                    idle = min(2e-3, idle * 2 if idle else 5e-5)
                    time.sleep(idle)
                else:
                    idle = 0.0
        except BaseException as e:  # noqa: BLE001 - surfaced to both roles
            self._py_failed = e
            log.error("rank %d: shared-queue transport failed: %r", self.rank, e)
            try:
                self.comm.abort()   # RCCL: never leave kernels waiting on a dead peer
            except Exception:  # noqa: BLE001
                pass
        finally:
            self.pool.wake_all()

    def start(self):
        if self.comm is None or self._thread is not None:
            return self
        if self._engine is not None:
            if not self._engine.running and not self._engine.done:
                self._engine.start()
            return self
        self._thread = threading.Thread(target=self._loop, name=f"psana-ray-transport-{self.rank}", daemon=True)
        self._thread.start()
        return self

    def join(self, timeout: Optional[float] = None) -> bool:
        if self._engine is not None:
            return bool(self._engine.join(-1.0 if timeout is None else float(timeout)))
        if self._thread is None:
            return True
        self._thread.join(timeout)
        return not self._thread.is_alive()

    def close(self, timeout: float = 10.0) -> None:
        """Stop the transport driver and drop the native engine (it holds references to the RCCL
        communicator and the control segment).  Idempotent; call before ``Comm.close()``."""
        if self._engine is not None:
            _ = self._failed                      # cache a late error before the engine goes
            self._final_counters = self._engine_counters()
            self._engine.request_stop()
            if not self._engine.join(timeout):
                log.warning("rank %d: transport engine did not stop within %.0f s", self.rank, timeout)
                return
            self._engine = None
            self._ctrl = None

    @property
    def failed(self) -> Optional[BaseException]:
        return self._failed

    def _engine_counters(self) -> dict:
        if self._engine is None:
            return dict(getattr(self, "_final_counters", {}))
        st = self._engine.stats()
        return {"rounds": st.rounds, "frames_routed": st.frames_routed, "bytes_sent": st.bytes_sent,
                "bytes_recv": st.bytes_recv, "round_ms": 1e3 * st.round_s / max(1, st.rounds),
                "ctrl_ms": 1e3 * st.ctrl_s / max(1, st.rounds), "idle_rounds": st.idle_rounds,
                "frames_local": st.frames_local}

    def metrics(self) -> dict:
        """Gauges + cumulative counters for utils.metrics."""
        if self._engine is not None or self.xport == "native":
            d = {"ready": self.pool.n_ready(), "credits": self.pool.credits()}
            d.update(self._engine_counters())
            return d
        d = {"ready": self.pool.n_ready(), "credits": self.pool.credits(), "rounds": self.rounds,
             "frames_routed": self.frames_routed if self.comm is not None else self.pool.stats().routed_local}
        if self.comm is not None:
            d.update(bytes_sent=self.comm.bytes_sent, bytes_recv=self.comm.bytes_recv,
                     round_ms=1e3 * self.round_time_s / max(1, self.rounds))
        return d

    def stats(self) -> dict:
        d = self.ring.stats()
        if self._engine is not None or self.xport == "native":
            d.update(self._engine_counters())
            d["xport"] = "native"
            return d
        d.update(rounds=self.rounds, frames_routed=self.frames_routed if self.comm is not None else d["routed_local"],
                 round_ms=1e3 * self.round_time_s / max(1, self.rounds))
        if self.comm is not None:
            d.update(bytes_sent=self.comm.bytes_sent, bytes_recv=self.comm.bytes_recv)
        return d
