"""XTC2-style runs: writer, pure-Python walker, and the event source over the native scanner.

The reference reads events through psana's XTC2 reader in small-data (SMD) mode --
``PsanaWrapperSmd(exp, run, detector_name)`` (psana_ray/producer.py:11,150-154; SURVEY E-01):
a small per-stream ``.smd.xtc2`` file lists every L1Accept with the offset and size of its
datagram in the big ``.xtc2`` file, and MPI ranks split the events (P-01).  This module writes and
reads that two-file layout:

* :func:`write_xtc2_run` / :func:`make_synthetic_xtc2_run` (``psana-ray-mkrun --format xtc2``)
  emit Configure / BeginRun / BeginStep / Enable, one L1Accept per frame, then Disable / EndStep /
  EndRun into ``<data_dir>/<exp>/xtc/<exp>-r<run>-s000-c000.xtc2`` and the matching smalldata file.
* :func:`open_xtc2_run` scans the smalldata file ONCE in C++ (``csrc/xtc2.cpp``) into a per-event
  table, then reads each event's raw array with the native pread thread pool straight into pinned
  staging pages (the same path as the producer engine's file source).
* :func:`walk` / :func:`scan_py` are an independent pure-Python reader (tests cross-check the two).

Container layout: see ``csrc/xtc2.h``.  The structure (Dgram -> Xtc tree, Names in Configure,
ShapesData = Shapes + Data in L1Accept, smdinfo offsets) follows LCLS-II xtcdata; byte-exactness
with psana's files is not pinned (no psana and no XTC2 fixture offline).
"""
from __future__ import annotations

import math
import struct
from pathlib import Path
from typing import Dict, Iterator, List, Optional, Tuple

import numpy as np

from ..models.constants import CalibConstants, run_seed
from ..models.detector import get_detector

# TransitionId (env bits 24..27)
CONFIGURE, BEGINRUN, ENDRUN, BEGINSTEP, ENDSTEP, ENABLE, DISABLE, L1ACCEPT = 2, 4, 5, 6, 7, 8, 9, 12
# TypeId::Type
PARENT, SHAPESDATA, SHAPES, DATA, NAMES = 0, 1, 2, 3, 4
# Name::DataType
UINT8, UINT16, UINT32, UINT64, INT8, INT16, INT32, INT64, FLOAT, DOUBLE, CHARSTR = range(11)
_NP = {UINT8: np.uint8, UINT16: np.uint16, UINT32: np.uint32, UINT64: np.uint64, INT8: np.int8, INT16: np.int16,
       INT32: np.int32, INT64: np.int64, FLOAT: np.float32, DOUBLE: np.float64, CHARSTR: np.uint8}
MAX_RANK = 5
NAME_BYTES = 256
DGRAM_HEADER = 24
XTC_HEADER = 12
TYPE_VERSION = 1

# NamesId values (node << 8 | index) used by the writer
DET_ID, EBEAM_ID, SMDINFO_ID = (1 << 8) | 0, (1 << 8) | 1, (1 << 8) | 2


def xtc2_paths(data_dir, exp: str, run: int, stream: int = 0) -> Tuple[Path, Path]:
    """(bigdata, smalldata) paths of one stream of a run, psana's directory convention."""
    base = Path(data_dir) / exp / "xtc"
    stem = f"{exp}-r{run:04d}-s{stream:03d}-c000"
    return base / f"{stem}.xtc2", base / "smalldata" / f"{stem}.smd.xtc2"


def _pad4(n: int) -> int:
    return (n + 3) & ~3


def _xtc(src: int, typ: int, payload: bytes) -> bytes:
    body = payload + b"\0" * (_pad4(len(payload)) - len(payload))
    return struct.pack("<IHHI", src, 0, (TYPE_VERSION << 8) | typ, XTC_HEADER + len(body)) + body


def _dgram(service: int, ts: int, children: bytes) -> bytes:
    env = (service & 0xF) << 24
    return struct.pack("<III", ts & 0xFFFFFFFF, ts >> 32, env) + \
        struct.pack("<IHHI", 0, 0, (TYPE_VERSION << 8) | PARENT, XTC_HEADER + len(children)) + children


def _names(src: int, det: str, det_type: str, alg: str, names: List[Tuple[str, int, int]], segment: int = 0) -> bytes:
    def s(x):
        return x.encode()[:NAME_BYTES - 1].ljust(NAME_BYTES, b"\0")
    head = s(det) + s(det_type) + s(f"{det}_{segment}") + s(alg) + struct.pack("<IIII", 0x020000, segment,
                                                                              len(names), 0)
    body = b"".join(s(n) + struct.pack("<II", t, r) for n, t, r in names)
    return _xtc(src, NAMES, head + body)


def _shapes_data(src: int, arrays: List[np.ndarray]) -> bytes:
    shapes = b""
    data = []
    for a in arrays:
        sh = list(a.shape) + [0] * (MAX_RANK - a.ndim)
        shapes += struct.pack("<5I", *sh)
        b = np.ascontiguousarray(a).tobytes()
        data.append(b + b"\0" * (_pad4(len(b)) - len(b)))
    return _xtc(src, SHAPESDATA, _xtc(0, SHAPES, shapes) + _xtc(0, DATA, b"".join(data)))


class Xtc2Writer:
    """Writes one stream of an XTC2-style run (bigdata + smalldata) for one detector array."""

    def __init__(self, big_path, smd_path, det_name: str, det_type: str, dtype=np.uint16, ndim: int = 3,
                 t0_sec: int = 1_700_000_000):
        self.big_path, self.smd_path = Path(big_path), Path(smd_path)
        self.big_path.parent.mkdir(parents=True, exist_ok=True)
        self.smd_path.parent.mkdir(parents=True, exist_ok=True)
        self.big = open(self.big_path, "wb")
        self.smd = open(self.smd_path, "wb")
        self.t0 = t0_sec
        self.n = 0
        self.dtype = np.dtype(dtype)
        dt = {np.dtype(v): k for k, v in _NP.items() if k != CHARSTR}[np.dtype(dtype)]
        cfg = (_names(DET_ID, det_name, det_type, "raw", [("raw", dt, ndim)]) +
               _names(EBEAM_ID, "ebeam", "ebeam", "raw", [("ebeamPhotonEnergy", DOUBLE, 0)]) +
               _names(SMDINFO_ID, "smdinfo", "smdinfo", "offsetAlg", [("intOffset", UINT64, 0),
                                                                      ("intDgramSize", UINT64, 0)]))
        for svc in (CONFIGURE, BEGINRUN, BEGINSTEP, ENABLE):
            self._both(_dgram(svc, self._ts(), cfg if svc == CONFIGURE else b""))

    def _ts(self) -> int:
        # 120 Hz event clock
        ns = self.n * 8_333_333
        return ((self.t0 + ns // 1_000_000_000) << 32) | (ns % 1_000_000_000)

    def _both(self, dg: bytes):
        self.big.write(dg)
        self.smd.write(dg)

    def add_event(self, raw: np.ndarray, photon_energy: Optional[float]):
        ts = self._ts()
        kids = _shapes_data(DET_ID, [np.ascontiguousarray(raw, dtype=self.dtype)])
        if photon_energy is not None:
            kids += _shapes_data(EBEAM_ID, [np.array(photon_energy, dtype=np.float64)])
        dg = _dgram(L1ACCEPT, ts, kids)
        off = self.big.tell()
        self.big.write(dg)
        small = _shapes_data(SMDINFO_ID, [np.array(off, np.uint64), np.array(len(dg), np.uint64)])
        if photon_energy is not None:     # small data rides in the smd file too (psana's SMD mode)
            small += _shapes_data(EBEAM_ID, [np.array(photon_energy, dtype=np.float64)])
        self.smd.write(_dgram(L1ACCEPT, ts, small))
        self.n += 1

    def close(self):
        if self.big.closed:
            return
        for svc in (DISABLE, ENDSTEP, ENDRUN):
            self._both(_dgram(svc, self._ts(), b""))
        self.big.close()
        self.smd.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def write_xtc2_run(data_dir, exp: str, run: int, det_name: str, frames: np.ndarray, photon_energy,
                   det_type: Optional[str] = None) -> Tuple[Path, Path]:
    spec = get_detector(det_name)
    big, smd = xtc2_paths(data_dir, exp, run)
    with Xtc2Writer(big, smd, spec.name, det_type or spec.kind, ndim=frames.ndim - 1) as w:
        for i in range(frames.shape[0]):
            pe = None if photon_energy is None or math.isnan(float(photon_energy[i])) else float(photon_energy[i])
            w.add_event(frames[i], pe)
    return big, smd


def make_synthetic_xtc2_run(data_dir, exp: str, run: int, detector: str, n_events: int,
                            chunk: int = 16) -> Tuple[Path, Path]:
    """Materialise a synthetic run as XTC2-style files (``psana-ray-mkrun --format xtc2``)."""
    from .synthetic import generate_raw

    spec = get_detector(detector)
    consts = CalibConstants.random(spec, seed=run_seed(exp, run, spec.name))
    big, smd = xtc2_paths(data_dir, exp, run)
    with Xtc2Writer(big, smd, spec.name, spec.kind, ndim=len(spec.frame_shape)) as w:
        for a in range(0, n_events, chunk):
            fr, pe = generate_raw(consts, min(chunk, n_events - a), seed=run_seed(exp, run, spec.name) + 7 + a)
            for i in range(fr.shape[0]):
                w.add_event(fr[i], float(pe[i]))
    return big, smd


# ----------------------------------------------------------------------------- pure-Python reader
def walk(path) -> Iterator[Tuple[int, int, int, int, bytes]]:
    """Yields (offset, size, service, timestamp, body) per datagram of an XTC2-style file."""
    buf = Path(path).read_bytes()
    pos = 0
    while pos < len(buf):
        nsec, sec, env = struct.unpack_from("<III", buf, pos)
        _, _, _, extent = struct.unpack_from("<IHHI", buf, pos + 12)
        size = DGRAM_HEADER - XTC_HEADER + extent
        if extent < XTC_HEADER or pos + size > len(buf):
            raise ValueError(f"{path}: corrupt datagram at {pos}")
        yield pos, size, (env >> 24) & 0xF, (sec << 32) | nsec, buf[pos + DGRAM_HEADER:pos + size]
        pos += size


def _children(body: bytes, base: int = 0):
    p = 0
    while p < len(body):
        src, _, contains, extent = struct.unpack_from("<IHHI", body, p)
        if extent < XTC_HEADER or p + extent > len(body):
            raise ValueError("corrupt xtc child")
        yield src, contains & 0xFF, body[p + XTC_HEADER:p + extent], base + p + XTC_HEADER
        p += _pad4(extent)


def _parse_names(payload: bytes):
    cs = lambda b: b.split(b"\0", 1)[0].decode()  # noqa: E731
    det, det_type, alg = cs(payload[:256]), cs(payload[256:512]), cs(payload[768:1024])
    n = struct.unpack_from("<I", payload, 1024 + 8)[0]
    names = []
    for i in range(n):
        q = 1040 + i * (NAME_BYTES + 8)
        names.append((cs(payload[q:q + NAME_BYTES]),) + struct.unpack_from("<II", payload, q + NAME_BYTES))
    return det, det_type, alg, names


def _parse_shapes_data(payload: bytes, names, base: int):
    shapes = data = None
    for _, typ, body, off in _children(payload, base):
        if typ == SHAPES:
            shapes = body
        elif typ == DATA:
            data, data_off = body, off
    out = {}
    o = 0
    for i, (nm, t, rank) in enumerate(names):
        sh = struct.unpack_from("<5I", shapes, i * 20)[:rank]
        dt = np.dtype(_NP[t])
        nb = int(np.prod(sh, dtype=np.int64)) * dt.itemsize if rank else dt.itemsize
        out[nm] = (np.frombuffer(data, dtype=dt, count=nb // dt.itemsize, offset=o).reshape(sh), data_off + o)
        o += _pad4(nb)
    return out


def scan_py(smd_path, big_path, det_name: str, array_name: str = "raw") -> Dict[str, list]:
    """Pure-Python equivalent of the native scan (tests): per-event payload offsets etc."""
    names: Dict[int, tuple] = {}
    res = {"payload_off": [], "timestamp": [], "photon_energy": [], "shape": None, "frames": []}
    big = Path(big_path).read_bytes()
    for _, _, svc, ts, body in walk(smd_path):
        if svc == CONFIGURE:
            for src, typ, payload, _ in _children(body):
                if typ == NAMES:
                    names[src] = _parse_names(payload)
        elif svc == L1ACCEPT:
            pe = float("nan")
            off = size = None
            for src, typ, payload, _ in _children(body):
                det = names[src]
                vals = _parse_shapes_data(payload, det[3], 0)
                if det[0] == "smdinfo":
                    off = int(vals["intOffset"][0].reshape(-1)[0])
                    size = int(vals["intDgramSize"][0].reshape(-1)[0])
                elif det[0] == "ebeam":
                    pe = float(vals["ebeamPhotonEnergy"][0].reshape(-1)[0])
            dg = big[off:off + size]
            for src, typ, payload, poff in _children(dg[DGRAM_HEADER:], DGRAM_HEADER):
                if names[src][0] == det_name:
                    arr, aoff = _parse_shapes_data(payload, names[src][3], poff)[array_name]
                    res["payload_off"].append(off + aoff)
                    res["shape"] = list(arr.shape)
                    res["frames"].append(arr)
            res["timestamp"].append(ts)
            res["photon_energy"].append(pe)
    return res


# ----------------------------------------------------------------------------- event source
def find_xtc2_run(data_dir, exp: str, run: int) -> Optional[Tuple[Path, Path]]:
    big, smd = xtc2_paths(data_dir, exp, run)
    return (big, smd) if big.exists() and smd.exists() else None


def open_xtc2_run(data_dir, exp: str, run: int, detector_name: str, **kw):
    """:class:`~psana_ray_amd.source.rawfile.RawFileRun` over an XTC2-style run: the native scan
    builds the event index, RawRunReader (index mode) preads raw arrays into pinned staging."""
    from ..ops import _ext
    from .rawfile import RawFileRun

    C = _ext.load()
    big, smd = xtc2_paths(data_dir, exp, run)
    spec = get_detector(detector_name)
    ix = C.xtc2_scan(str(smd), str(big), spec.name, "raw")
    if list(ix.shape) != list(spec.frame_shape) or ix.dtype != UINT16:
        raise ValueError(f"{big}: raw array {list(ix.shape)} (type {ix.dtype}) is not a {spec.name} uint16 frame")
    n_threads = int(kw.pop("n_threads", 16))
    reader = C.RawRunReader(str(big), n_threads, list(ix.payload_off), list(ix.gevt), list(ix.photon_energy),
                            int(ix.frame_bytes))
    src = RawFileRun(big, detector_name, exp=exp, run=run, reader=reader, **kw)
    src.index = (np.asarray(ix.payload_off, dtype=np.int64), np.asarray(ix.gevt, dtype=np.int64),
                 np.asarray(ix.photon_energy, dtype=np.float64))
    src.timestamps = np.asarray(ix.timestamp, dtype=np.int64)
    src.transitions = list(ix.transitions)
    return src
