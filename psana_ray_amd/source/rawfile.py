"""Raw-run files: the on-disk event format read by the native ``RawRunReader`` (C++ thread pool).

Stands in for psana's XTC2 reader (the reference's events come from psana via
``PsanaWrapperSmd``, psana_ray/producer.py:150-154).  Fixed-size records make event ``i``
addressable at ``header_bytes + i * record_bytes`` so every producer rank reads its shard
(``i % size == rank``, P-01) with positional reads straight into pinned staging buffers.

Layout (little endian): a 4096-byte file header ``PRAWRUN1`` (see csrc/runtime.h) followed by
records ``[i64 gevt, f64 photon_energy, i64 timestamp, i64 reserved, raw frame bytes]``.
"""
from __future__ import annotations

import logging
import os
import struct
from pathlib import Path
from typing import List, Optional

import numpy as np

from ..models.constants import CalibConstants, run_seed
from ..models.detector import DetectorSpec, get_detector
from .synthetic import RawEvent, generate_raw

log = logging.getLogger(__name__)

HEADER_BYTES = 4096
RECORD_HEADER = 32


def run_path(data_dir: str, exp: str, run: int, detector: str) -> Path:
    return Path(data_dir) / exp / f"r{run:04d}" / f"{detector}.praw"


def write_run(path, spec: DetectorSpec, frames: np.ndarray, photon_energy: np.ndarray, first_gevt: int = 0):
    """Write frames [n, P, H, W] uint16 as a raw-run file."""
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    n = frames.shape[0]
    frame_bytes = spec.raw_frame_bytes
    rec = RECORD_HEADER + frame_bytes
    hdr = bytearray(HEADER_BYTES)
    shape = list(spec.frame_shape) + [0] * (4 - len(spec.frame_shape))
    struct.pack_into("<8sII64sII4QII2Q", hdr, 0, b"PRAWRUN1", 1, HEADER_BYTES,
                     spec.name.encode()[:63], len(spec.frame_shape), 0, *shape, 2, 0, n, rec)
    with open(path, "wb") as f:
        f.write(hdr)
        for i in range(n):
            f.write(struct.pack("<qdqq", first_gevt + i, float(photon_energy[i]), i, 0))
            f.write(np.ascontiguousarray(frames[i], dtype=np.uint16).tobytes())


def make_synthetic_run(data_dir: str, exp: str, run: int, detector: str, n_events: int, chunk: int = 16) -> Path:
    """Materialise a synthetic run on disk (``psana-ray-mkrun``)."""
    spec = get_detector(detector)
    consts = CalibConstants.random(spec, seed=run_seed(exp, run, spec.name))
    path = run_path(data_dir, exp, run, spec.name)
    frames_all, pe_all = [], []
    for a in range(0, n_events, chunk):
        fr, pe = generate_raw(consts, min(chunk, n_events - a), seed=run_seed(exp, run, spec.name) + 7 + a)
        frames_all.append(fr)
        pe_all.append(pe)
    write_run(path, spec, np.concatenate(frames_all), np.concatenate(pe_all))
    return path


ENV_ZEROCOPY = "PSANA_RAY_FILE_ZEROCOPY"


def _mem_available() -> int:
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 0


def zero_copy_wanted(nbytes: int) -> bool:
    """``PSANA_RAY_FILE_ZEROCOPY``: 1 = always map + register the run file, 0 = never (pread into
    pinned staging), auto (default) = when the file fits in min(64 GiB, 25 % of available RAM):
    registration pins every page of the file for the whole run."""
    mode = os.environ.get(ENV_ZEROCOPY, "auto").lower()
    if mode in ("0", "off", "false"):
        return False
    if mode in ("1", "on", "true"):
        return True
    return nbytes <= min(64 << 30, _mem_available() // 4)


class RawFileRun:
    """Event source over a raw-run file, read by the native thread-pool reader into pinned
    staging buffers (ring of ``staging`` frames; callers must not reuse a staged frame before
    its H2D copy completed -- the producer pipeline waits on the copy event)."""

    def __init__(self, path, detector_name: str, exp: str = "file", run: int = 0, rank: int = 0, size: int = 1,
                 staging: int = 64, n_threads: int = 16, pinned: bool = True, n_events: Optional[int] = None,
                 reader=None):
        from ..ops import _ext

        C = _ext.load()
        self.spec = get_detector(detector_name)
        self.exp, self.run = exp, run
        self.path = str(path)
        # reader: a prebuilt native reader (e.g. index mode over an XTC2 bigdata file)
        self.reader = C.RawRunReader(str(path), n_threads) if reader is None else reader
        if self.reader.frame_bytes != self.spec.raw_frame_bytes:
            raise ValueError(f"{path}: frame size {self.reader.frame_bytes} != {self.spec.name} raw frame")
        self.rank, self.size = rank, size
        total = self.reader.n_events if n_events is None else min(n_events, self.reader.n_events)
        self.n_events = total
        self.consts = CalibConstants.random(self.spec, seed=run_seed(exp, run, self.spec.name))
        nbytes = staging * self.spec.raw_frame_bytes
        if pinned:
            self._buf = C.PinnedBuffer(nbytes)
            self.staging = np.frombuffer(self._buf, dtype=np.uint16).reshape(staging, *self.spec.frame_shape)
        else:
            self.staging = np.empty((staging, *self.spec.frame_shape), np.uint16)
        self.n_staging = staging
        self._cursor = 0
        self._slot = 0
        self._map = None
        # per-event (payload offset, gevt, photon energy) when the reader is index-based (XTC2)
        self.index = None

    def create_bad_pixel_mask(self) -> np.ndarray:
        return self.consts.create_bad_pixel_mask()

    def _event_table(self):
        """(payload offsets, gevts, photon energies) of every event in the file."""
        if self.index is not None:
            return self.index
        import ctypes

        r = self.reader
        n = self.n_events
        raw = np.ctypeslib.as_array((ctypes.c_uint8 * (r.header_bytes + n * r.record_bytes)).from_address(self._map.ptr))
        recs = raw[r.header_bytes:].reshape(n, r.record_bytes)[:, :RECORD_HEADER].copy()
        gevt = recs[:, :8].view(np.int64)[:, 0]
        pe = recs[:, 8:16].view(np.float64)[:, 0]
        off = r.header_bytes + np.arange(n, dtype=np.int64) * r.record_bytes + RECORD_HEADER
        return off, gevt, pe

    def zero_copy_frames(self):
        """Host pointers (into the registered file mapping) + photon energies of this rank's
        events, for the producer engine's copy-from-source path: the DMA engines read the payloads
        straight out of the page cache (no pread into staging).  None when disabled / unsuitable."""
        from ..ops import _ext

        try:
            if self._map is None:
                if not zero_copy_wanted(os.path.getsize(self.path)):
                    return None
                self._map = _ext.load().MappedFile(self.path, True)
            off, gevt, pe = (np.asarray(x) for x in self._event_table())
        except Exception as e:  # noqa: BLE001 - fall back to the pread path
            log.warning("zero-copy mapping of %s unavailable (%r): pread staging", self.path, e)
            self._map = None
            return None
        local = np.arange(self.rank, self.n_events, self.size, dtype=np.int64)
        if not np.array_equal(gevt[local], local):
            return None      # event ids are not positions: the engine derives gevt from the position
        ptrs = [int(self._map.ptr + int(o)) for o in off[local]]
        pes = [None if np.isnan(v) else float(v) for v in pe[local]]
        return ptrs, pes

    def n_local_events(self) -> int:
        return max(0, (self.n_events - self.rank + self.size - 1) // self.size)

    def seek(self, start_event: int) -> int:
        """Resume at global event ``start_event`` (see synthetic.first_local_event)."""
        from .synthetic import first_local_event

        self._cursor = first_local_event(start_event, self.rank, self.size)
        return self._cursor

    @property
    def cursor(self) -> int:
        return self._cursor

    def next_events(self, n: int) -> List[RawEvent]:
        n = min(n, self.n_local_events() - self._cursor, self.n_staging)
        if n <= 0:
            return []
        ks = list(range(self._cursor, self._cursor + n))
        gevts = [self.rank + k * self.size for k in ks]
        slots = [(self._slot + i) % self.n_staging for i in range(n)]
        ptrs = [self.staging[s].ctypes.data for s in slots]
        meta = self.reader.read(gevts, ptrs)
        self._cursor += n
        self._slot = (self._slot + n) % self.n_staging
        return [RawEvent(int(m[0]), k, self.staging[s], p, None if np.isnan(m[1]) else float(m[1]))
                for k, s, p, m in zip(ks, slots, ptrs, meta)]
