"""XTC2-style runs (bigdata + smalldata index, psana's SMD layout): writer, native scanner vs the
independent pure-Python walker, sharded reads through the native index-mode reader, source
selection, corruption handling, and (GPU) the producer engine fed from an XTC2 run.

Parity note: the container structure follows LCLS-II xtcdata, but no psana / XTC2 fixture exists
offline, so byte-exactness with psana-written files is "parity unpinned"; these tests pin our own
writer <-> reader contract."""
import math
import os
import subprocess
import sys
import threading

import numpy as np
import pytest
import torch

from psana_ray_amd.models import CalibConstants, get_detector
from psana_ray_amd.source import generate_raw, open_source, write_xtc2_run, xtc2_paths
from psana_ray_amd.source import xtc2 as X


def _run(tmp_path, det="tiny_epix", n=9, nan_at=(4,)):
    spec = get_detector(det)
    c = CalibConstants.random(spec, seed=1)
    frames, pe = generate_raw(c, n, seed=2)
    pe = np.asarray(pe, dtype=np.float64).copy()
    for i in nan_at:
        pe[i] = np.nan
    big, smd = write_xtc2_run(str(tmp_path), "expX", 3, det, frames, pe)
    return spec, np.asarray(frames), pe, big, smd


def test_native_scan_matches_python_walker(native, tmp_path):
    spec, frames, pe, big, smd = _run(tmp_path)
    ix = native.xtc2_scan(str(smd), str(big), spec.name, "raw")
    py = X.scan_py(smd, big, spec.name)
    assert list(ix.shape) == list(spec.frame_shape) == py["shape"]
    assert ix.frame_bytes == spec.raw_frame_bytes and ix.dtype == X.UINT16
    assert list(ix.payload_off) == py["payload_off"]
    assert list(ix.timestamp) == py["timestamp"]
    assert list(ix.gevt) == list(range(len(frames)))
    for a, b in zip(ix.photon_energy, py["photon_energy"]):
        assert (math.isnan(a) and math.isnan(b)) or a == b
    assert math.isnan(ix.photon_energy[4]) and ix.photon_energy[0] == pe[0]
    for i, f in enumerate(py["frames"]):
        np.testing.assert_array_equal(f, frames[i])
    t = list(ix.transitions)
    assert t[X.L1ACCEPT] == len(frames)
    assert all(t[s] == 1 for s in (X.CONFIGURE, X.BEGINRUN, X.BEGINSTEP, X.ENABLE, X.DISABLE, X.ENDSTEP, X.ENDRUN))
    # raw arrays are 4-byte aligned inside their datagrams (pinned-page preads stay aligned)
    assert all(o % 4 == 0 for o in ix.payload_off)


def test_sharded_reads_through_index(native, tmp_path):
    spec, frames, pe, big, smd = _run(tmp_path)
    got = []
    for rank in range(2):
        src = X.open_xtc2_run(str(tmp_path), "expX", 3, spec.name, rank=rank, size=2, staging=4, pinned=False)
        assert src.reader.indexed and src.n_events == len(frames)
        while True:
            evs = src.next_events(3)
            if not evs:
                break
            for e in evs:
                assert e.gevt % 2 == rank
                np.testing.assert_array_equal(e.raw, frames[e.gevt])
                assert (e.photon_energy is None) == (e.gevt == 4)
                if e.photon_energy is not None:
                    assert e.photon_energy == pe[e.gevt]
                got.append(e.gevt)
    assert sorted(got) == list(range(len(frames)))


def test_open_source_prefers_xtc2(native, tmp_path, monkeypatch):
    spec, frames, pe, big, smd = _run(tmp_path, det="tiny_plain", n=3, nan_at=())
    monkeypatch.setenv("PSANA_RAY_DATA", str(tmp_path))
    src = open_source("expX", 3, "tiny_plain", pinned=False)
    assert src.reader.indexed and src.n_events == 3
    assert list(src.transitions)[X.L1ACCEPT] == 3
    assert np.all(np.diff(src.timestamps) > 0)


def test_variable_size_datagrams_are_walked(native, tmp_path):
    """Events without an ebeam record are shorter: their layout is found by walking their heads."""
    spec, frames, pe, big, smd = _run(tmp_path, nan_at=(1, 2, 6))
    ix = native.xtc2_scan(str(smd), str(big), spec.name, "raw")
    assert ix.walked >= 2
    py = X.scan_py(smd, big, spec.name)
    assert list(ix.payload_off) == py["payload_off"]


def test_full_size_frames_head_walk(native, tmp_path):
    """epix10k2M datagrams (4.3 MB) are larger than the scanner's head window: the raw array is
    located from the datagram's head only."""
    X.make_synthetic_xtc2_run(str(tmp_path), "e", 1, "epix10k2M", n_events=2, chunk=2)
    big, smd = xtc2_paths(tmp_path, "e", 1)
    ix = native.xtc2_scan(str(smd), str(big), "epix10k2M", "raw")
    py = X.scan_py(smd, big, "epix10k2M")
    assert list(ix.payload_off) == py["payload_off"] and list(ix.shape) == [16, 352, 384]
    src = X.open_xtc2_run(str(tmp_path), "e", 1, "epix10k2M", pinned=False)
    for e in src.next_events(2):
        np.testing.assert_array_equal(e.raw, py["frames"][e.gevt])


def test_corrupt_or_mismatched_files_raise(native, tmp_path):
    spec, frames, pe, big, smd = _run(tmp_path)
    with pytest.raises(RuntimeError, match="not configured"):
        native.xtc2_scan(str(smd), str(big), "jungfrau16M", "raw")
    data = smd.read_bytes()
    bad = tmp_path / "trunc.smd.xtc2"
    bad.write_bytes(data[:-7])
    with pytest.raises(RuntimeError, match="xtc2"):
        native.xtc2_scan(str(bad), str(big), spec.name, "raw")
    short = tmp_path / "short.xtc2"
    short.write_bytes(big.read_bytes()[: len(big.read_bytes()) // 2])
    with pytest.raises(RuntimeError, match="past the end"):
        native.xtc2_scan(str(smd), str(short), spec.name, "raw")
    with pytest.raises(RuntimeError, match="not configured"):
        X.open_xtc2_run(str(tmp_path), "expX", 3, "tiny_plain")


def test_mkrun_cli_xtc2(native, tmp_path):
    r = subprocess.run([sys.executable, "-m", "psana_ray_amd.mkrun", "--data_dir", str(tmp_path), "--exp", "e1",
                        "--run", "5", "--detector_name", "tiny_epix", "--num_events", "6"],
                       capture_output=True, text=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr
    big, smd = xtc2_paths(tmp_path, "e1", 5)
    assert big.exists() and smd.exists() and str(big) in r.stdout
    src = X.open_xtc2_run(str(tmp_path), "e1", 5, "tiny_epix", pinned=False)
    assert src.n_events == 6


def test_zero_copy_event_pointers(native, tmp_path):
    """The zero-copy file path hands the engine pointers into the file mapping: check they address
    exactly each local event's raw array (CPU: plain mmap, no HIP registration)."""
    import ctypes

    from psana_ray_amd.source import RawFileRun, write_run

    spec, frames, pe, big, smd = _run(tmp_path, nan_at=(4,))
    praw = tmp_path / "r.praw"
    write_run(praw, spec, frames, pe)
    for src in (X.open_xtc2_run(str(tmp_path), "expX", 3, spec.name, rank=1, size=2, pinned=False),
                RawFileRun(praw, spec.name, rank=1, size=2, pinned=False)):
        src._map = native.MappedFile(src.path, False)
        ptrs, pes = src.zero_copy_frames()
        local = list(range(1, len(frames), 2))
        assert len(ptrs) == len(local) == src.n_local_events()
        for p, g, v in zip(ptrs, local, pes):
            got = np.frombuffer((ctypes.c_uint8 * spec.raw_frame_bytes).from_address(p), dtype=np.uint16)
            np.testing.assert_array_equal(got.reshape(frames[g].shape), frames[g])
            assert (v is None) == (g == 4) and (v is None or v == pe[g])


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", ["0", "1"])
def test_xtc2_source_native_engine(cuda_device, tmp_path, monkeypatch, zero_copy):
    """XTC2 run -> native scan -> producer engine (pread pool into pinned staging, or DMA out of
    the registered file mapping; H2D, calib + common mode) -> queue: every event once, exact vs
    the golden model."""
    monkeypatch.setenv("PSANA_RAY_FILE_ZEROCOPY", zero_copy)
    from psana_ray_amd.config import CommonModeParams
    from psana_ray_amd.models import Calibrator, Mode
    from psana_ray_amd.ops import reference
    from psana_ray_amd.pipeline import ProducerPipeline
    from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint

    X.make_synthetic_xtc2_run(str(tmp_path), "exp", 9, "epix10k2M", n_events=40, chunk=16)
    src = X.open_xtc2_run(str(tmp_path), "exp", 9, "epix10k2M")
    ref = X.scan_py(*reversed(xtc2_paths(tmp_path, "exp", 9)), "epix10k2M")
    cal = Calibrator(src.consts, cuda_device, Mode.calib, common_mode=CommonModeParams())
    ring = FrameRing(cal.out_shape, cal.out_dtype, cuda_device, 40, 24)
    ep = QueueEndpoint(ring)
    prod = ProducerPipeline(src, cal, ep, chunk=8)
    assert prod.engine is not None, "XTC2 sources must run on the native engine"
    assert prod.zero_copy == (zero_copy == "1")
    t = threading.Thread(target=prod.run)
    t.start()
    seen = {}
    while True:
        try:
            it = ep.get(timeout=0.5)
        except EndOfStream:
            break
        if it is None:
            continue
        with it:
            got = it.data.clone()
            gevt, pe = it.gevt, it.photon_energy
        torch.cuda.synchronize()
        raw = torch.from_numpy(ref["frames"][gevt].astype(np.int32))[None]
        exp = reference.calibrate_reference(raw, src.consts, None, cal.cm)[0]
        assert torch.equal(got.cpu(), exp), f"event {gevt}"
        assert pe == ref["photon_energy"][gevt]
        seen[gevt] = seen.get(gevt, 0) + 1
    t.join()
    assert sorted(seen) == list(range(40)) and all(v == 1 for v in seen.values())
