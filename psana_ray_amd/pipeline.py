"""Producer and consumer pipelines (the per-rank engines behind the CLIs and ``bench.py``).

Producer (replaces psana_ray/producer.py:78-117, ``produce_data``):
    source events (pinned host pages) --hipMemcpyAsync, side stream--> raw HBM chunk buffers
    --calibration kernels, compute stream--> HBM ring slots --commit--> sharded queue
  * triple-buffered raw chunks: the H2D copy of chunk k+1 overlaps the kernels of chunk k;
    everything is ordered with HIP events, the host never waits for the device except on
    backpressure (no free slot) -- which replaces the reference's sleep-based exponential
    backoff (producer.py:105-111) with a condition-variable wait;
  * masks (bad-pixel via ``create_bad_pixel_mask()``, manual ``.npy``; truthy keeps,
    producer.py:81-82,92-95) are folded into the kernel tables once, not applied per event;
  * frames are written straight into the destination slot (no intermediate copies).

Consumer: drains this rank's shard in batches and runs the on-GPU peak finder (K-07) on a
consumer stream, releasing slots stream-ordered (BASELINE config 5).
"""
from __future__ import annotations

import collections
import logging
import threading
import time
from typing import List, Optional

import numpy as np
import torch

from .config import (CONSUMER_STREAM_KIND, CONSUMER_STREAMS, PRODUCER_STREAM_KIND, STREAM_KINDS, PeakFinderParams,
                     pipeline_shape)
from .models.calibrator import Calibrator
from .ops import _ext, kernels
from .queue.endpoint import EndOfStream, FrameItem, QueueEndpoint
from .utils.tracing import trace_range

log = logging.getLogger(__name__)


def resolve_producer_streams(where: str, compute_streams: Optional[int] = None,
                             ranks_per_gpu: Optional[int] = None) -> int:
    """Producer compute streams: ``compute_streams``, else config.pipeline_shape for raw frames
    ``where`` ("device" / "staged") on a GPU shared by ``ranks_per_gpu`` ranks (None: the launch's,
    parallel.launch.ranks_per_gpu).  ProducerPipeline, the producer CLI and bench.py all use it."""
    if compute_streams is not None:
        return int(compute_streams)
    if ranks_per_gpu is None:
        from .parallel.launch import ranks_per_gpu as _rpg

        ranks_per_gpu = _rpg()
    return pipeline_shape(where, int(ranks_per_gpu))["producer_streams"]


def resolve_consumer_batch(batch: Optional[int] = None, ranks_per_gpu: Optional[int] = None) -> int:
    """Frames per peak-finder launch: ``batch``, else config.pipeline_shape for the ranks sharing
    this GPU (PeakFinderConsumer, the producer's co-consumer, psana-ray-consumer, bench.py)."""
    if batch is not None:
        return int(batch)
    if ranks_per_gpu is None:
        from .parallel.launch import ranks_per_gpu as _rpg

        ranks_per_gpu = _rpg()
    return pipeline_shape("device", int(ranks_per_gpu))["consumer_batch"]


class ProducerPipeline:
    def __init__(self, source, calibrator: Optional[Calibrator], endpoint: QueueEndpoint, rank: int = 0,
                 chunk: int = 32, n_raw_buffers: int = 6, acquire_timeout_s: float = 1.0,
                 log_every: int = 0, copy_workgroups: int = 32, gpu_timing: bool = False,
                 compute_streams: Optional[int] = None, stream_kind: Optional[str] = None,
                 mask: Optional[np.ndarray] = None, n_upload_buffers: int = 3, gap_fill: Optional[bool] = None,
                 ranks_per_gpu: Optional[int] = None):
        """copy_workgroups: host->HBM staging by copy_h2d_kernel with that many workgroups (0 = the
        runtime's hipMemcpyAsync); gpu_timing: event-time each chunk's copy and calibration;
        compute_streams: chunks alternate over that many HIP streams (native engine), so one chunk's
        calibration fills the CUs its predecessor's tail leaves idle; stream_kind: their
        hardware-queue placement (config.STREAM_KINDS).  None: config.pipeline_shape /
        PRODUCER_STREAM_KIND for the source (raw frames already in HBM or staged) and the number of
        ranks sharing this GPU (``ranks_per_gpu``; None: parallel.launch.ranks_per_gpu()).

        gap_fill: image mode, zero the panel gaps of every frame (None: only when the ring was not
        zero-filled at creation -- ``FrameRing.zero_filled`` -- since a zeroed ring's gaps stay 0).

        Sources whose frames arrive calibrated (psana_wrapper without raw access): ``mask`` (truthy
        keeps, producer.py:92-95) is applied on the device after the upload; frames move in
        ``chunk``-frame batches through ``n_upload_buffers`` pinned staging buffers (one H2D copy per
        frame, no host synchronisation except before a staging buffer is refilled)."""
        self.source = source
        self.cal = calibrator
        self.ep = endpoint
        self.rank = rank
        self.chunk = min(chunk, kernels.MAX_FRAMES)
        self.device = endpoint.ring.device
        self.gpu = self.device.type == "cuda"
        self.acquire_timeout_s = acquire_timeout_s
        self.log_every = log_every
        self.frames = 0
        self.full_waits = 0
        self.t_first = None
        self.calibrated_source = getattr(source, "calibrated", False)
        # which calibration runs (metrics "producer.source_path"): the HIP kernels on raw frames,
        # psana's CPU calibration (psana_wrapper fallback), or the fp32 golden model (CPU rehearsal)
        self.source_path = "psana_cpu" if self.calibrated_source else ("raw_hip" if self.gpu else "raw_cpu")
        spec = getattr(source, "spec", None)
        file_source = getattr(source, "reader", None)   # RawFileRun: native RawRunReader
        # file sources: DMA straight out of the registered file mapping when possible
        zero_copy = source.zero_copy_frames() if (self.gpu and not self.calibrated_source
                                                  and hasattr(source, "zero_copy_frames")) else None
        self.zero_copy = zero_copy is not None
        use_engine = self.gpu and not self.calibrated_source and (hasattr(source, "cycled_frames")
                                                                  or file_source is not None)
        if self.gpu and not self.calibrated_source and not use_engine:
            _ext.load()
            self.h2d = torch.cuda.Stream(device=self.device)
            self.compute = torch.cuda.Stream(device=self.device)
            self.raw_bufs = torch.empty((n_raw_buffers, self.chunk, *spec.frame_shape), dtype=torch.uint16,
                                        device=self.device)
            self.buf_free = [torch.cuda.Event() for _ in range(n_raw_buffers)]
            self.buf_used = [False] * n_raw_buffers
            self.h2d_done = [torch.cuda.Event() for _ in range(n_raw_buffers)]
        self._k = 0
        self.mask = None
        if self.calibrated_source:
            self._init_upload(mask, n_upload_buffers)
        # completion log of the Python paths: (frames so far, perf_counter s) at commit -- the CPU
        # calibration is synchronous, so commit == completion (the native engine logs device events)
        self._done_log: List[tuple] = []
        self._inflight = collections.deque()
        self._reuses = hasattr(source, "n_staging")
        self.engine = None
        self.gap_fill = None        # image mode, native engine: kernels zero the panel gaps per frame
        self.stream_config = None   # (compute streams, kind) of the native engine
        if use_engine:
            # native hot loop: no Python (and no GIL) per frame or per chunk
            C = _ext.load()
            ring = endpoint.ring
            dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
            # gevt = event_rank + k * size; a panel-sharded source (source/shard.py) shards events
            # over rank GROUPS, while the headers keep this rank (its panel shard)
            plan = calibrator.plan
            n_gaps = plan.n_gap_runs
            self.gap_fill = bool(n_gaps) and (not ring.zero_filled if gap_fill is None else bool(gap_fill))
            if n_gaps and not self.gap_fill:
                plan.n_gap_runs = 0   # the engine keeps its own copy of the plan
            try:
                self.engine = C.ProducerEngine(ring.pool, ring.frame_bytes, dev_index,
                                               plan, self.chunk, n_raw_buffers,
                                               int(getattr(source, "event_rank", rank)),
                                               int(getattr(source, "size", 1)),
                                               copy_workgroups=int(copy_workgroups), gpu_timing=bool(gpu_timing))
            finally:
                plan.n_gap_runs = n_gaps
            self.engine.set_header_rank(int(rank))
            if zero_copy is not None:
                ptrs, pe = zero_copy
                self._source_map = source._map       # keep the registered mapping alive
                self.engine.set_cycled_source(ptrs, [float("nan") if v is None else float(v) for v in pe])
            elif file_source is not None:
                self.engine.set_file_source(file_source)    # file reads + staging in the native loop
            else:
                ptrs, pe = source.cycled_frames()
                self.engine.set_cycled_source([int(x) for x in ptrs],
                                              [float("nan") if v is None else float(v) for v in pe])
            where = "device" if self.engine.device_resident else "staged"
            n_cs = resolve_producer_streams(where, compute_streams, ranks_per_gpu)
            kind = PRODUCER_STREAM_KIND[where] if stream_kind is None else stream_kind
            self.engine.set_compute_streams(n_cs, STREAM_KINDS[kind])
            self.stream_config = (n_cs, kind)
            fab = getattr(endpoint, "_fabric", None)
            if fab is not None and fab.direct():
                # frames routed to other processes are calibrated straight into their consumer's
                # slot (csrc/fabric.h take_direct); cleared after the engine stopped (_run_engine)
                self.engine.set_fabric(fab)
                from .config import fabric_direct_headroom, fabric_direct_wait_s
                head = fabric_direct_headroom(ring.frame_bytes)   # the byte cap bench / the CLI sized the ring with
                if head > 0 and ring.pool.producer_budget - head >= 2 * self.chunk:
                    self.engine.set_direct_headroom(head, fabric_direct_wait_s())

    # --------------------------------------------------------------------------------
    def _acquire(self, n: int, stream) -> List[int]:
        slots = []
        while len(slots) < n:
            s = self.ep.acquire(timeout=self.acquire_timeout_s, stream=stream)
            if s is None:
                self.full_waits += 1
                if self.full_waits % 50 == 1:
                    log.info("Rank %d: Queue is full, waiting...", self.rank)  # producer.py:106
                continue
            slots.append(s)
        return slots

    def step(self) -> int:
        """Produce up to ``chunk`` frames.  Returns the number produced (0 = source exhausted)."""
        if self.t_first is None:
            self.t_first = time.perf_counter()
        if self.calibrated_source:
            return self._step_calibrated()
        if self._reuses and self.gpu:
            # the source refills pinned staging slots: keep its ring ahead of in-flight copies
            max_inflight = max(1, self.source.n_staging // self.chunk - 1)
            while len(self._inflight) >= max_inflight:
                self._inflight.popleft().synchronize()
        evs = self.source.next_events(self.chunk)
        if not evs:
            return 0
        n = len(evs)
        if self.gpu:
            C = _ext.load()
            b = self._k % len(self.raw_bufs)
            self._k += 1
            buf = self.raw_bufs[b]
            if self.buf_used[b]:
                self.h2d.wait_event(self.buf_free[b])
            self.buf_used[b] = True
            nbytes = evs[0].raw.nbytes
            C.memcpy_h2d_batch([int(buf[i].data_ptr()) for i in range(n)], [int(e.host_ptr) for e in evs], nbytes,
                               int(self.h2d.cuda_stream))
            self.h2d_done[b].record(self.h2d)
            if self._reuses:
                ev = torch.cuda.Event()
                ev.record(self.h2d)
                self._inflight.append(ev)
            slots = self._acquire(n, self.compute)
            self.compute.wait_event(self.h2d_done[b])
            outs = [self.ep.slot_tensor(s) for s in slots]
            self.cal.run([buf[i] for i in range(n)], outs, self.compute)
            self.buf_free[b].record(self.compute)
            for s, e in zip(slots, evs):
                self.ep.commit(s, self.rank, e.idx, e.gevt, e.photon_energy, self.compute)
        else:
            slots = self._acquire(n, None)
            raw = [torch.from_numpy(np.ascontiguousarray(e.raw).view(np.int16)).view(torch.uint16) for e in evs]
            outs = [self.ep.slot_tensor(s) for s in slots]
            self.cal.run(raw, outs)
            for s, e in zip(slots, evs):
                self.ep.commit(s, self.rank, e.idx, e.gevt, e.photon_energy)
        self.frames += n
        if not self.gpu:
            self._done_log.append((self.frames, time.perf_counter()))
        if self.log_every and self.frames % self.log_every < n:
            log.info("Rank %d produced: idx=%d | shape=%s | photon_energy=%s", self.rank, evs[-1].idx,
                     tuple(self.ep.ring.frame_shape), evs[-1].photon_energy)
        return n

    def _init_upload(self, mask, n_bufs: int):
        """Pinned staging for sources that deliver calibrated frames (psana_wrapper fallback path)."""
        shape = tuple(self.ep.ring.frame_shape)
        self._up_shape = shape
        self._up_bufs, self._up_done, self._up_keep = [], [], []
        if mask is not None:
            m = np.asarray(mask).astype(bool)
            if m.shape != shape:
                if m.size != int(np.prod(shape)):
                    raise ValueError(f"mask of shape {m.shape} does not match the frames {shape}")
                m = m.reshape(shape)
            self.mask = torch.from_numpy(~m).to(self.device)   # True = zero this pixel
            # the GPU path masks a whole uploaded chunk in one kernel launch (ops.kernels.mask_frames)
            self._mask_u8 = self.mask.reshape(-1).to(torch.uint8).contiguous() if self.gpu else None
        if self.gpu:
            C = _ext.load()
            nbytes = self.chunk * int(np.prod(shape)) * 4
            for _ in range(max(2, n_bufs)):
                keep = C.PinnedBuffer(nbytes)
                self._up_keep.append(keep)
                self._up_bufs.append(np.frombuffer(keep, dtype=np.float32).reshape(self.chunk, *shape))
                self._up_done.append(None)
            self._up_stream = torch.cuda.Stream(device=self.device)
        self._it = None

    def _step_calibrated(self) -> int:
        """psana path: frames arrive calibrated on the host in the producer's mode.  Up to ``chunk``
        frames are gathered into a pinned staging buffer, copied into their ring slots on a side
        stream (one H2D copy per frame), masked on the device and committed stream-ordered; the host
        waits only before it refills a staging buffer whose copies are still running."""
        if self._it is None:
            self._it = self.source.iter_events(self.source.mode) if hasattr(self.source, "mode") \
                else self.source.iter_events()
            self._idx = int(getattr(self.source, "cursor", 0))
        shape = self._up_shape
        frames, pes = [], []
        for _ in range(self.chunk):
            try:
                data, pe = next(self._it)
            except StopIteration:
                break
            data = np.asarray(data)
            if data.ndim == 2:
                data = data[None]   # producer.py:96-97
            if data.shape != shape:
                raise ValueError(f"psana frame of shape {data.shape}; the queue was built for {shape}")
            frames.append(data)
            pes.append(pe)
        n = len(frames)
        if n == 0:
            return 0
        idx0 = self._idx
        self._idx += n
        if self.gpu:
            C = _ext.load()
            b = self._k % len(self._up_bufs)
            self._k += 1
            if self._up_done[b] is not None:
                self._up_done[b].synchronize()   # this staging buffer's previous copies finished
            buf = self._up_bufs[b]
            for i, f in enumerate(frames):
                np.copyto(buf[i], f, casting="same_kind")
            st = self._up_stream
            slots = self._acquire(n, st)
            C.memcpy_h2d_batch([int(self.ep.slot_ptr(s)) for s in slots], [int(buf[i].ctypes.data) for i in range(n)],
                               int(buf[0].nbytes), int(st.cuda_stream))
            if self.mask is not None:   # np.where(mask, data, 0): one launch for the chunk
                kernels.mask_frames([self.ep.slot_tensor(s) for s in slots], self._mask_u8, st)
            ev = torch.cuda.Event()
            ev.record(st)
            self._up_done[b] = ev
            for i, s in enumerate(slots):
                self.ep.commit(s, self.rank, idx0 + i, self.rank + (idx0 + i) * int(getattr(self.source, "size", 1)),
                               pes[i], st)
        else:
            slots = self._acquire(n, None)
            for i, s in enumerate(slots):
                t = self.ep.slot_tensor(s)
                t.copy_(torch.from_numpy(np.ascontiguousarray(frames[i], dtype=np.float32)).view(t.shape))
                if self.mask is not None:
                    t.masked_fill_(self.mask.view(t.shape), 0.0)
                self.ep.commit(s, self.rank, idx0 + i, self.rank + (idx0 + i) * int(getattr(self.source, "size", 1)),
                               pes[i])
            self._done_log.append((self.frames + n, time.perf_counter()))
        self.frames += n
        return n

    @property
    def produced(self) -> int:
        """Frames whose calibration has COMPLETED (native engine: the chunk's device event; CPU: the
        commit).  ``enqueued`` counts frames committed with kernels possibly still running."""
        return int(self.engine.completed) if self.engine is not None else self.frames

    @property
    def enqueued(self) -> int:
        return int(self.engine.frames) if self.engine is not None else self.frames

    def completion_log(self, since: int = 0):
        """``(first_index, [(frames completed so far, t_seconds), ...])`` -- one entry per completed
        chunk from index ``since`` on, times on the :meth:`clock` of this producer."""
        if self.engine is not None:
            first, v = self.engine.completions(int(since))
            return int(first), [(int(f), ms * 1e-3) for f, ms in v]
        return int(since), list(self._done_log[int(since):])

    def clock(self, stream=None) -> float:
        """Now on the completion log's clock (seconds).  Native engine: device time of an event
        recorded on ``stream`` (default: current) -- the host waits for it, so a consumer stream's
        work issued before is finished at that point."""
        if self.engine is not None:
            h = _ext.stream_handle(stream) if stream is not None else int(torch.cuda.current_stream(self.device).cuda_stream)
            return float(self.engine.mark(h)) * 1e-3
        return time.perf_counter()

    def metrics(self) -> dict:
        """Cumulative counters for utils.metrics (sampled, nothing runs per frame)."""
        d = {"frames_produced": self.produced,
             "full_waits": int(self.engine.full_waits) if self.engine is not None else self.full_waits,
             "source_path": self.source_path}
        if self.engine is not None:
            st, acq, launch, commit, total = self.engine.timing()
            d.update(host_stage_s=st, host_acquire_s=acq, host_launch_s=launch, host_commit_s=commit)
            if self.engine.gpu_timing_enabled:   # gpu_timing=True: event-timed GPU stages
                h2d_ms, h2d_n, cal_ms, cal_n = self.engine.gpu_timing()
                d.update(gpu_h2d_ms_per_chunk=h2d_ms / max(1.0, h2d_n), gpu_calib_ms_per_chunk=cal_ms / max(1.0, cal_n),
                         gpu_chunks_timed=cal_n)
        return d

    def run(self, max_steps: Optional[int] = None, stop=None) -> int:
        """Produce until the source ends, ``max_steps`` events (per rank, Q-6) or ``stop`` is set."""
        if self.engine is not None:
            return self._run_engine(max_steps, stop)
        while not (stop is not None and stop.is_set()):
            if max_steps is not None and self.frames >= max_steps:
                log.info("Rank %d: Reached max_steps %d, terminating", self.rank, max_steps)
                break
            if max_steps is not None:
                self.chunk = max(1, min(self.chunk, max_steps - self.frames))
            if self.step() == 0:
                break
        if self.gpu and not self.calibrated_source:
            self.compute.synchronize()
        if self.gpu and self.calibrated_source:
            self._up_stream.synchronize()
        self.ep.finish()
        return self.frames


    def _run_engine(self, max_steps, stop) -> int:
        n_local = self.source.n_local_events() if hasattr(self.source, "n_local_events") else None
        self.t_first = time.perf_counter()
        k0 = int(getattr(self.source, "cursor", 0))   # resume cursor (source.seek / --start_event)
        self.engine.start(-1 if n_local is None else int(n_local), -1 if max_steps is None else int(max_steps), k0)
        try:
            while not self.engine.join(0.05):
                if (stop is not None and stop.is_set()) or self.ep.failed is not None:
                    self.engine.request_stop()
        finally:
            self.engine.request_stop()
            self.engine.join(-1.0)
            self.engine.set_fabric(None)   # the endpoint may close (and free the fabric) from here on
        err = self.engine.error()
        self.frames = int(self.engine.frames)
        self.full_waits = int(self.engine.full_waits)
        if max_steps is not None and self.frames >= max_steps:
            log.info("Rank %d: Reached max_steps %d, terminating", self.rank, max_steps)
        self.ep.finish()
        if err:
            raise RuntimeError(f"producer engine failed: {err}")
        self.ep._raise_if_failed()
        return self.frames


# Native streams with a hardware-queue placement, per (device, kind): created once (a native pool,
# csrc/streams.h), handed back here when their OWNER is collected and handed out again -- never
# destroyed while the process runs.  Tensors allocated on a stream keep its handle in torch's
# caching allocator after the wrapper is gone, so destroying the native stream could leave the
# allocator a dangling handle; and every CU-masked stream is a hardware queue of its own, so reuse
# also bounds their number.  No weak reference ever points at a torch stream object: torch's stream
# type does not clear weak references when it is freed, and a weakref left behind crashed the
# interpreter's final garbage collection (_PyWeakref_ClearRef, rc 139 after a passing GPU suite).
_STREAM_POOL: dict = {}
_STREAM_POOL_LOCK = threading.Lock()
# handles whose owner is still alive (token -> (key, handles)): at process exit they go back to the
# native pool too, so close_stream_pool() synchronises and destroys every CU-masked queue of ours
# (a PeakFinderConsumer alive at exit left its queues to the runtime's static teardown)
_STREAMS_IN_USE: dict = {}


def _return_streams(key, handles, token=None):
    with _STREAM_POOL_LOCK:
        if token is not None and _STREAMS_IN_USE.pop(token, None) is None:
            return   # already released at exit
        _STREAM_POOL.setdefault(key, []).extend(handles)


def _release_idle_streams(C):
    """Process exit: the idle pooled handles AND those of owners still alive go back to the native
    pool (csrc/streams.h; release synchronises each stream first)."""
    with _STREAM_POOL_LOCK:
        items = [(k, h) for k, hs in _STREAM_POOL.items() for h in hs]
        items += [(k, h) for k, hs in _STREAMS_IN_USE.values() for h in hs]
        _STREAM_POOL.clear()
        _STREAMS_IN_USE.clear()
    for (dev, kind), h in items:
        C.stream_release(dev, kind, h)


def _make_streams(device, n: int, kind: str, owner=None):
    """n torch streams with the given hardware-queue placement (config.STREAM_KINDS), from the
    process-wide pool of native streams (see _STREAM_POOL); they go back to the pool when ``owner``
    (a plain Python object) is collected."""
    if STREAM_KINDS[kind] == 0:
        return [torch.cuda.Stream(device=device) for _ in range(n)]
    import weakref

    C = _ext.load()
    dev = device.index if device.index is not None else torch.cuda.current_device()
    key = (dev, STREAM_KINDS[kind])
    out, handles = [], []
    for _ in range(n):
        with _STREAM_POOL_LOCK:
            free = _STREAM_POOL.setdefault(key, [])
            h = free.pop() if free else None
        if h is None:
            h = int(C.stream_create(dev, STREAM_KINDS[kind]))
        handles.append(h)
        out.append(torch.cuda.ExternalStream(h, device=device))
    if owner is not None:
        token = object()
        with _STREAM_POOL_LOCK:
            _STREAMS_IN_USE[token] = (key, handles)
        fin = weakref.finalize(owner, _return_streams, key, handles, token)
        fin.atexit = False
    return out


class PeakFinderConsumer:
    """Consumer engine: batches of leased slots -> K-07 peak finder -> stream-ordered release.

    GPU: consecutive batches alternate between TWO consumer streams, each with its own peak-finder
    scratch, so one launch's candidate-test tail (every workgroup tests its parked candidates after
    its stream of reads) overlaps the next launch's streaming reads instead of idling HBM."""

    def __init__(self, endpoint: QueueEndpoint, frame_shape, params: Optional[PeakFinderParams] = None,
                 batch: Optional[int] = None, keep_results: bool = False, stream_kind: str = CONSUMER_STREAM_KIND,
                 streams: int = CONSUMER_STREAMS, ranks_per_gpu: Optional[int] = None):
        """batch: frames per peak-finder launch; None -> config.pipeline_shape for the ranks sharing
        this GPU (``ranks_per_gpu``; None: parallel.launch.ranks_per_gpu())."""
        self.ep = endpoint
        self.params = params or PeakFinderParams()
        self.batch = min(resolve_consumer_batch(batch, ranks_per_gpu), kernels.MAX_FRAMES)
        self.device = endpoint.ring.device
        self.gpu = self.device.type == "cuda"
        self.shape = tuple(frame_shape)
        self.frames = 0
        self.peaks_total = 0
        self.keep_results = keep_results
        self.results = []
        if self.gpu:
            self.streams = _make_streams(self.device, int(streams), stream_kind, owner=self)
            self.stream = self.streams[0]
            B = self.batch
            # buffer k % nbuf is reused by launch k + nbuf, on the same stream as k
            self._nbuf = 2 * len(self.streams)
            self.peaks = torch.empty((self._nbuf, B, self.params.max_peaks, 8), dtype=torch.float32, device=self.device)
            # counts [B] int32 and summary [B, 2] f32 of a batch share one row; the peak finder
            # writes them whole from its self-resetting scratch (no per-batch fill)
            self._meta = torch.zeros((self._nbuf, 3 * B), dtype=torch.int32, device=self.device)
            # one scratch block per stream (a block must never serve two launches in flight)
            self._pf_scratch = [torch.zeros(kernels.PF_SCRATCH_WORDS, dtype=torch.int32, device=self.device)
                                for _ in self.streams]
            self.counts = self._meta[:, :B]
            self.summary = self._meta[:, B:].view(torch.float32).view(self._nbuf, B, 2)
            self.count_acc = torch.zeros((), dtype=torch.int64, device=self.device)
            self._b = 0

    def process(self, items: List[FrameItem]):
        n = len(items)
        if n == 0:
            return
        if self.gpu:
            b = self._b % self._nbuf
            k = self._b % len(self.streams)
            st = self.streams[k]
            self._b += 1
            st.wait_stream(torch.cuda.current_stream(self.device))   # the items were leased on it
            with torch.cuda.stream(st):
                kernels.peakfind([it.data for it in items], self.shape, self.params, self.peaks[b, :n],
                                 self.counts[b, :n], self.summary[b, :n], st, total=self.count_acc,
                                 scratch=self._pf_scratch[k])
                if self.keep_results:
                    self.results.append((self.peaks[b, :n].clone(), self.counts[b, :n].clone(),
                                         [(it.rank, it.idx, it.gevt) for it in items]))
            for it in items:
                it.release(st)
        else:
            from .ops import reference

            frames = torch.stack([it.data.reshape(self.shape) for it in items])
            peaks, _summary = reference.peakfind_reference(frames, self.params)
            self.peaks_total += sum(int(p.shape[0]) for p in peaks)
            if self.keep_results:
                self.results.append((peaks, [(it.rank, it.idx, it.gevt) for it in items]))
            for it in items:
                it.release()
        self.frames += n

    def poll(self, timeout: float = 0.05, max_items: Optional[int] = None) -> int:
        """Take up to ``batch`` ready frames (waiting up to ``timeout`` for the first) and process
        them.  Returns frames processed; raises EndOfStream at the end of the stream."""
        n_max = self.batch if max_items is None else max(1, min(self.batch, max_items))
        if not self.gpu:
            items: List[FrameItem] = []
            it = self.ep.get(timeout=timeout)
            if it is None:
                return 0
            items.append(it)
            while len(items) < n_max:
                try:
                    nxt = self.ep.get(timeout=0.0)
                except EndOfStream:
                    break
                if nxt is None:
                    break
                items.append(nxt)
            self.process(items)
            return len(items)
        # GPU: one native call to lease, one kernel launch, one native call to release
        k = self._b % len(self.streams)
        st = self.streams[k]
        slots = self.ep.get_batch(n_max, timeout, st)
        n = len(slots)
        if n == 0:
            return 0
        C = _ext.load()
        b = self._b % self._nbuf
        self._b += 1
        sh = int(st.cuda_stream)
        P, H, W = self.shape
        with trace_range("consumer.peakfind_batch"):
            # one native call: the peak finder on the ring slots with self-resetting outputs (no
            # fill kernel), bumping the on-device running peak total (no per-batch torch ops, no
            # host sync)
            C.peakfind_slots(self.ep.pool, self.ep._slot_bytes, slots, P, H, W, float(self.params.thr_peak),
                             float(self.params.son_min), int(self.params.radius), int(self.params.max_peaks),
                             int(self.peaks[b].data_ptr()), int(self.counts[b].data_ptr()),
                             int(self.summary[b].data_ptr()), int(self.count_acc.data_ptr()), sh,
                             int(self._pf_scratch[k].data_ptr()))
            if self.keep_results:
                hs = self.ep.pool.headers(slots)
                with torch.cuda.stream(st):
                    self.results.append((self.peaks[b, :n].clone(), self.counts[b, :n].clone(),
                                         [(h.rank, h.idx, h.gevt) for h in hs]))
        self.ep.release_batch(slots, st)
        self.frames += n
        return n

    def metrics(self) -> dict:
        return {"frames_consumed": self.frames}

    def sync_streams(self):
        """Host waits for every batch issued so far (both consumer streams)."""
        if self.gpu:
            for st in self.streams:
                st.synchronize()

    def synchronize(self):
        if self.gpu:
            self.sync_streams()
            self.peaks_total = int(self.count_acc.item())
        return self.peaks_total
