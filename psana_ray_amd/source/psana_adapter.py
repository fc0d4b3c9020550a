"""Adapter over the real ``psana_wrapper`` (E-01), used when it is importable.

The reference constructs ``PsanaWrapperSmd(exp=..., run=..., detector_name=...)`` and iterates
``iter_events(mode=ImageRetrievalMode.calib|image)`` -> ``(data, photon_energy)``, with an
optional ``create_bad_pixel_mask()`` (psana_ray/producer.py:11,81,88,150-159).  psana shards the
run over the MPI ranks itself (SMD mode, P-01), so each rank's wrapper yields that rank's events.

Two ways frames enter the GPU pipeline:

* **raw** (preferred, ``source_path = "raw_hip"``): raw uint16 frames go through pinned staging and
  the producer calibrates them with the gfx950 kernels (K-01..K-05: gain decode, pedestal, gain,
  common mode, masks, geometry) -- the same path as the synthetic and file sources; psana's CPU
  calibration never runs.  It needs raw frames AND the run's calibration constants, probed by
  attribute (nothing is fetched, nothing guessed over a network):
    raw frames  1. the wrapper's own ``ImageRetrievalMode.raw`` through ``iter_events`` -- the
                   preferred path: it keeps the wrapper's SMD sharding and its photon energies;
                2. else the psana detector handle the wrapper holds (``det`` / ``detector`` / ...):
                   psana2 ``det.raw.raw(evt)`` or psana1 ``det.raw(evt)``, over the events of the
                   run it holds (``run.events()`` / ``ds.events()``; photon energy from a wrapper
                   ``get_photon_energy(evt)`` when it has one).  That loop bypasses the wrapper, so
                   it is sharded EXPLICITLY: rank r of size keeps the loop's events i with
                   i % size == r (``handle_shard="explicit"``, the default), unless the operator
                   says psana already shards it (``--psana_handle_shard psana``); the path taken is
                   logged and reported as ``raw_via``;
    constants   1. an adapter hook ``calib_constants()`` on the wrapper (mapping below), else
                2. the detector handle's PUBLIC psana1 accessors ``det.pedestals(run)``,
                   ``gain(run)``, ``status(run)``, ``gain_config(run)``, ``indexes_xy(run)``, else
                3. only when the operator opts in (``--psana_private_constants``): psana2's private
                   ``det.raw._pedestals()``, ``_gain()`` (ADU/keV), ``_status()``, ``_gain_config()``,
                   ``_pixel_coord_indexes()`` (names that may change between psana releases);
                   without the opt-in the source falls back to psana's CPU calibration with a
                   WARNING that names the flag.
                An ePix10ka's per-pixel gain configuration must come with constants read from a
                detector handle: without it the gain range each pixel auto-switches through is
                unknown, so the source falls back to psana's CPU calibration instead of guessing.
                Only the ``calib_constants()`` hook may omit it (documented default: AHL).
* **calibrated** (fallback, ``source_path = "psana_cpu"``, logged once at WARNING): frames arrive
  calibrated by psana in the requested mode and are uploaded in pinned batches (one H2D copy per
  frame of a chunk, no per-frame synchronisation); masks are applied by one kernel per chunk.

``calib_constants()`` mapping -- ``pedestals`` [G, P, H, W] (ADU), ``gains`` [G, P, H, W] (ADU per
keV), optional ``status`` [P, H, W] or [G, P, H, W] (non-zero = bad), ``gain_config`` [P, H, W]
(epix10ka: 0..4 = FH FM FL AHL AML; default AHL), ``pix_rows`` / ``pix_cols`` [P, H, W] (image-mode
pixel indices; default: the framework's geometry of the detector).
The detector must be one the framework knows (``models/detector.py``) with matching shapes.

Neither psana nor psana_wrapper exists in this environment: parity with real
psana is unpinned; the contract is pinned by a stub ``psana_wrapper`` module in
``tests/stubs/`` (tests/test_psana_wrapper.py).
"""
from __future__ import annotations

import itertools
import logging
from typing import Iterator, List, Optional, Tuple

import numpy as np

from ..models.detector import Mode
from .errors import NoSourceError

log = logging.getLogger(__name__)


_DET_ATTRS = ("det", "detector", "psana_det", "psana_detector", "_det", "_detector")
_EVENT_ATTRS = ("run", "psana_run", "_run", "ds", "datasource", "_ds")
_PE_ATTRS = ("get_photon_energy", "photon_energy", "_photon_energy")
_warned_cpu = False


def _find_detector(wrapper):
    """(attribute name, psana detector handle) the wrapper holds, or (None, None): a handle is an
    object with a ``raw`` member (psana2: an object with ``raw(evt)``; psana1: a method)."""
    for a in _DET_ATTRS:
        d = getattr(wrapper, a, None)
        if d is not None and getattr(d, "raw", None) is not None:
            return a, d
    return None, None


def _raw_accessor(det):
    """evt -> raw frame of a detector handle: psana2 ``det.raw.raw``, psana1 ``det.raw``."""
    r = getattr(det, "raw", None)
    if r is not None and callable(getattr(r, "raw", None)):
        return r.raw
    return r if callable(r) else None


def _find_events(wrapper):
    """The run's event iterator factory the wrapper holds (``run.events`` / ``ds.events``)."""
    for a in _EVENT_ATTRS:
        o = getattr(wrapper, a, None)
        if o is not None and callable(getattr(o, "events", None)):
            return o.events
    return None


def _call(fn, *alts):
    """fn(), else fn(alt) for the first alternative argument it accepts (psana1 accessors take the
    run or an event)."""
    try:
        return fn()
    except TypeError:
        if not alts:
            raise
    err = None
    for a in alts:
        try:
            return fn(a)
        except TypeError as e:
            err = e
    raise err


PRIVATE_FLAG = "--psana_private_constants"


def _constants_from_detector(det, run: int, private_ok: bool = False):
    """The calib_constants() mapping from a psana detector handle, or (None, why).  psana1's public
    accessors are used as is; psana2's private ones (``det.raw._pedestals`` ...) only when
    ``private_ok`` (the operator's opt-in)."""
    r = getattr(det, "raw", None)
    if hasattr(det, "pedestals") and callable(getattr(det, "pedestals")):   # psana1 Detector (public API)
        acc = {"pedestals": "pedestals", "gains": "gain", "status": "status", "coords": "indexes_xy",
               "gain_config": "gain_config"}
        obj, style = det, "psana1"
    elif r is not None and hasattr(r, "_pedestals"):      # psana2 AreaDetector (det.raw._* : private)
        if not private_ok:
            return None, (f"the psana2 detector handle exposes its constants only through private accessors "
                          f"(det.raw._pedestals / _gain / _status); pass {PRIVATE_FLAG} to use them")
        acc = {"pedestals": "_pedestals", "gains": "_gain", "status": "_status", "coords": "_pixel_coord_indexes",
               "gain_config": "_gain_config"}
        obj, style = r, "psana2"
    else:
        return None, "the psana detector handle exposes no calibration constants"
    out = {}
    for key in ("pedestals", "gains"):
        fn = getattr(obj, acc[key], None)
        v = _call(fn, run) if callable(fn) else None
        if v is None:
            return None, f"the {style} detector handle gives no {key} ({acc[key]})"
        out[key] = np.asarray(v)
    for key in ("status", "gain_config"):
        fn = getattr(obj, acc[key], None)
        if callable(fn):
            v = _call(fn, run)
            if v is not None:
                out[key] = np.asarray(v)
    fn = getattr(obj, acc["coords"], None)
    if callable(fn):
        rc = _call(fn, run)
        if rc is not None and len(rc) >= 2:
            out["pix_rows"], out["pix_cols"] = np.asarray(rc[0]), np.asarray(rc[1])
    return out, style


def psana_available() -> bool:
    try:
        import psana_wrapper  # noqa: F401

        return True
    except Exception:
        return False


def _normalise(data: np.ndarray) -> np.ndarray:
    """The reference's ndim fix-up (producer.py:96-97): 2-D frames become (1, H, W)."""
    data = np.asarray(data)
    return data[None] if data.ndim == 2 else data


class RawUnavailable(NoSourceError):
    """Raw frames were requested (``--mode raw`` / ``calibrate_on_read``) from a psana_wrapper that
    cannot provide them; a :class:`~psana_ray_amd.source.NoSourceError` too (the CLI's clean exit 2)."""


class PsanaWrapperSource:
    """``(exp, run, detector_name)`` through psana_wrapper, for one producer rank.

    ``mode`` is the retrieval mode the producer serves (image by default, producer.py:156-159).
    After construction ``calibrated`` tells which path applies: False -> ``spec`` / ``consts`` /
    ``geometry`` describe the raw frames ``next_events`` stages; True -> ``frame_shape`` is the shape
    of the calibrated frames ``iter_events`` yields (peeked from the first event)."""

    def __init__(self, exp: str, run: int, detector_name: str, mode: Mode = Mode.image, rank: int = 0,
                 size: int = 1, pinned: bool = False, prefer_raw: bool = True, staging: int = 128,
                 n_events: Optional[int] = None, private_constants: bool = False, handle_shard: str = "explicit"):
        import psana_wrapper  # type: ignore

        self.exp, self.run, self.detector_name = exp, int(run), detector_name
        self.rank, self.size = int(rank), int(size)
        self.mode = Mode(mode)
        self.n_events = n_events
        if handle_shard not in ("explicit", "psana"):
            raise ValueError(f"handle_shard must be 'explicit' or 'psana', not {handle_shard!r}")
        self.private_constants = bool(private_constants)
        self.handle_shard = handle_shard
        self._modes = psana_wrapper.ImageRetrievalMode
        self.wrapper = psana_wrapper.PsanaWrapperSmd(exp=exp, run=run, detector_name=detector_name)
        self._skip = 0
        self._cursor = 0
        self._it = None
        self._peeked: Optional[Tuple[np.ndarray, Optional[float]]] = None
        self.geometry = None
        self.consts = None
        self.raw_via = self.constants_via = None
        self._raw_fn = self._events_fn = self._pe_fn = None
        why = self._try_raw(prefer_raw)
        self.calibrated = why is not None
        self.source_path = "psana_cpu" if self.calibrated else "raw_hip"
        if self.calibrated:
            if self.mode == Mode.raw:
                raise RawUnavailable(f"psana_wrapper source {exp}/{run}/{detector_name}: raw mode requested but {why}")
            global _warned_cpu
            if not _warned_cpu and prefer_raw:
                log.warning("psana_wrapper %s/%d/%s: the HIP calibration kernels cannot run (%s); psana calibrates on "
                            "the CPU and its %s frames are uploaded in pinned batches", exp, run, detector_name, why,
                            self.mode.value)
                _warned_cpu = True
            else:
                log.info("psana_wrapper %s/%d/%s: psana-calibrated %s frames uploaded in pinned batches (%s)", exp, run,
                         detector_name, self.mode.value, why)
            first = self._peek()
            if first is None:
                raise NoSourceError(f"psana_wrapper source {exp}/{run}/{detector_name}: the run has no events")
            self.frame_shape = tuple(_normalise(first[0]).shape)
            self.frame_dtype = np.float32
        else:
            log.info("psana_wrapper %s/%d/%s: RAW frames (%s) calibrated on the GPU with constants from the %s "
                     "(HIP kernels, %s mode)", exp, run, detector_name, self.raw_via, self.constants_via, self.mode.value)
            self.frame_shape = tuple(self.spec.frame_shape)
            if pinned:
                from ..ops import _ext

                self._buf = _ext.load().PinnedBuffer(staging * self.spec.raw_frame_bytes)
                self.staging = np.frombuffer(self._buf, dtype=np.uint16).reshape(staging, *self.spec.frame_shape)
            else:
                self.staging = np.empty((staging, *self.spec.frame_shape), np.uint16)
            self.n_staging = staging
            self._slot = 0

    # ---- capability probe ------------------------------------------------------------------
    def _try_raw(self, prefer_raw: bool) -> Optional[str]:
        """Set up the raw path; returns None when it applies, else why not."""
        if not prefer_raw:
            return "raw path disabled (--psana_calibrated)"
        det_attr, det = _find_detector(self.wrapper)
        # raw frames: the wrapper's raw retrieval mode, else the detector handle over the run's events
        if hasattr(self._modes, "raw"):
            self.raw_via = "iter_events(raw)"
        elif det is not None and _raw_accessor(det) is not None and _find_events(self.wrapper) is not None:
            # the run's own event loop bypasses the wrapper's SMD sharding: shard it here unless the
            # operator says psana already does
            shard = f"every {self.size}th event from {self.rank}" if (self.handle_shard == "explicit"
                                                                     and self.size > 1) else "as psana yields them"
            self.raw_via = f"{det_attr}.raw(evt) over the run's events ({shard})"
            self._raw_fn = _raw_accessor(det)
            self._events_fn = _find_events(self.wrapper)
            self._pe_fn = next((getattr(self.wrapper, a) for a in _PE_ATTRS if callable(getattr(self.wrapper, a, None))),
                               None)
        else:
            return ("the wrapper has no ImageRetrievalMode.raw and no psana detector handle with raw frames and a "
                    "run event loop")
        # calibration constants: the adapter hook, else the detector handle's accessors
        hook = getattr(self.wrapper, "calib_constants", None)
        if callable(hook):
            c = hook()
            self.constants_via = "calib_constants() hook"
        elif det is not None:
            c, style = _constants_from_detector(det, self.run, self.private_constants)
            if c is None:
                return style
            self.constants_via = f"{style} detector handle ({det_attr})"
        else:
            return "no calibration constants: no calib_constants() hook and no psana detector handle"
        from ..models.constants import EPIX_CM_GAINS, JUNGFRAU_CM_GAINS, CalibConstants
        from ..models.detector import get_detector
        from ..models.geometry import Geometry, make_geometry

        try:
            spec = get_detector(self.detector_name)
        except KeyError:
            return f"detector {self.detector_name!r} has no kernel description"
        ped = np.ascontiguousarray(c["pedestals"], dtype=np.float32)
        gains = np.ascontiguousarray(c["gains"], dtype=np.float32)
        want = (spec.n_gains, *spec.frame_shape)
        if ped.shape != want or gains.shape != want:
            return f"constants {ped.shape} / {gains.shape} do not match {spec.name} {want}"
        status = np.asarray(c.get("status", np.zeros(spec.frame_shape, np.uint8)))
        if status.ndim == len(spec.frame_shape) + 1:   # per gain mode (psana2 _status()): bad in any
            status = (status != 0).any(axis=0)
        status = status.astype(np.uint8)
        cfg = c.get("gain_config")
        if spec.kind == "epix10ka":
            if cfg is None and not callable(hook):
                # a fixed-gain or AML run would select the wrong pedestal / gain range
                # under an AHL guess -- psana's own CPU calibration knows the configuration
                return (f"the {self.constants_via} gives no per-pixel gain configuration for the ePix10ka "
                        f"(needed to decode its gain ranges)")
            if cfg is None:
                log.warning("psana_wrapper %s: calib_constants() gives no per-pixel gain configuration; assuming "
                            "AHL (auto high-to-low) for every pixel (the hook's documented default)",
                            self.detector_name)
            cfg = np.full(spec.frame_shape, 3, np.uint8) if cfg is None else \
                np.asarray(cfg).astype(np.uint8).reshape(spec.frame_shape)
        cmg = {"epix10ka": EPIX_CM_GAINS, "jungfrau": JUNGFRAU_CM_GAINS}.get(spec.kind, (0,))
        self.spec = spec
        self.consts = CalibConstants(spec, ped, gains, status.reshape(spec.frame_shape), cfg, tuple(cmg))
        rows, cols = c.get("pix_rows"), c.get("pix_cols")
        if rows is not None and cols is not None:
            rows = np.asarray(rows, np.int32).reshape(spec.frame_shape)
            cols = np.asarray(cols, np.int32).reshape(spec.frame_shape)
            self.geometry = Geometry(spec, (int(rows.max()) + 1, int(cols.max()) + 1), rows, cols)
        else:
            self.geometry = make_geometry(spec)
        return None

    # ---- reference surface -----------------------------------------------------------------
    def create_bad_pixel_mask(self) -> np.ndarray:
        return np.asarray(self.wrapper.create_bad_pixel_mask())

    def seek(self, start_event: int) -> int:
        """Skip this rank's first ``start_event`` events (psana shards inside its SMD reader, so the
        skip is rank-local: ``--start_event`` resumes each rank at the same local position)."""
        if self._it is not None and self._cursor:
            raise RuntimeError("PsanaWrapperSource.seek after events were read")
        self._skip = max(0, int(start_event))
        self._cursor = self._skip
        self._it = None
        self._peeked = None
        if self.calibrated and self._peek() is None:
            log.warning("psana_wrapper source: nothing left after --start_event %d", start_event)
        return self._skip

    @property
    def cursor(self) -> int:
        return self._cursor

    def _raw_from_handle(self):
        """(raw frame, photon energy) per event of the run through the psana detector handle; with
        explicit sharding this rank keeps the loop's events i with i % size == rank."""
        explicit = self.handle_shard == "explicit" and self.size > 1
        for i, evt in enumerate(self._events_fn()):
            if explicit and i % self.size != self.rank:
                continue
            data = self._raw_fn(evt)
            if data is None:   # the detector is not in this event (psana returns None)
                continue
            pe = self._pe_fn(evt) if self._pe_fn is not None else None
            yield data, pe

    def _events(self):
        if self._it is None:
            if not self.calibrated and self._raw_fn is not None:
                it = self._raw_from_handle()
            else:
                m = getattr(self._modes, "raw" if not self.calibrated else
                            ("calib" if self.mode == Mode.calib else "image"))
                it = iter(self.wrapper.iter_events(mode=m))
            # --num_events: this rank's events after --start_event (it was ignored)
            stop = None if self.n_events is None else self._skip + int(self.n_events)
            self._it = itertools.islice(it, self._skip, stop) if (self._skip or stop is not None) else it
        return self._it

    def _peek(self):
        if self._peeked is None:
            try:
                self._peeked = next(self._events())
            except StopIteration:
                return None
        return self._peeked

    def _next(self):
        if self._peeked is not None:
            ev, self._peeked = self._peeked, None
            return ev
        return next(self._events())

    def n_local_events(self) -> Optional[int]:
        return None   # psana's SMD reader decides; the stream ends when the iterator does

    def iter_events(self, mode: Optional[Mode] = None) -> Iterator[Tuple[np.ndarray, Optional[float]]]:
        """Calibrated path: ``(data, photon_energy)`` in ``self.mode`` (the producer's requested mode;
        a different ``mode`` argument is an error -- the source was opened for one mode)."""
        if mode is not None and Mode(mode.value if hasattr(mode, "value") else mode) != self.mode:
            raise ValueError(f"source opened for {self.mode.value} mode, asked for {mode}")
        while True:
            try:
                data, pe = self._next()
            except StopIteration:
                return
            self._cursor += 1
            yield data, pe

    def next_events(self, n: int) -> List:
        """Raw path: up to ``n`` raw events staged into the (pinned) staging ring.  ``gevt`` is the
        nominal ``rank + idx * size`` (psana's SMD batches do not expose a global index)."""
        from .synthetic import RawEvent

        out = []
        n = min(n, self.n_staging)
        for _ in range(n):
            try:
                data, pe = self._next()
            except StopIteration:
                break
            s = self._slot
            self._slot = (self._slot + 1) % self.n_staging
            frame = np.asarray(data)
            if frame.shape != self.spec.frame_shape:
                frame = frame.reshape(self.spec.frame_shape)
            np.copyto(self.staging[s], frame, casting="unsafe")
            k = self._cursor
            self._cursor += 1
            out.append(RawEvent(self.rank + k * self.size, k, self.staging[s], self.staging[s].ctypes.data,
                                None if pe is None else float(pe)))
        return out
