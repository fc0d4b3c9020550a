"""End-to-end single-GPU pipeline: pinned host raw -> H2D -> HIP calib -> HBM ring -> consumer."""
import threading

import numpy as np
import pytest
import torch

from psana_ray_amd.config import CommonModeParams, PeakFinderParams
from psana_ray_amd.models import Calibrator, Mode
from psana_ray_amd.ops import reference
from psana_ray_amd.pipeline import PeakFinderConsumer, ProducerPipeline
from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint
from psana_ray_amd.source import SyntheticRun

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cm,copy_kernel", [(None, 32), ("default", 32), ("default", 0)])
def test_local_pipeline_frames_exact(cuda_device, cm, copy_kernel):
    """copy_kernel: staging copies by copy_h2d_kernel (csrc/gather.hip, default 32 workgroups) or
    by hipMemcpyAsync (0)."""
    n_events = 50
    src = SyntheticRun("synthetic", 3, "epix10k2M", n_events=n_events, pool_frames=8, pinned=True,
                       gen_device="cuda")
    cmp = CommonModeParams.parse(cm)
    cal = Calibrator(src.consts, cuda_device, Mode.calib, common_mode=cmp)
    ring = FrameRing(cal.out_shape, cal.out_dtype, cuda_device, 16, 12)   # small ring: backpressure
    ep = QueueEndpoint(ring)
    prod = ProducerPipeline(src, cal, ep, chunk=8, copy_workgroups=copy_kernel)
    t = threading.Thread(target=prod.run)
    t.start()
    ref = reference.calibrate_reference(torch.from_numpy(src.pool.astype(np.int32)), src.consts, None, cal.cm)
    seen = []
    while True:
        try:
            it = ep.get(timeout=0.5)
        except EndOfStream:
            break
        if it is None:
            continue
        with it:
            got = it.data.clone()
        torch.cuda.synchronize()
        assert torch.equal(got.cpu(), ref[it.idx % 8]), f"frame idx {it.idx} corrupted"
        assert it.gevt == it.idx and it.rank == 0
        assert it.photon_energy == pytest.approx(float(src.pool_pe[it.idx % 8]))
        seen.append(it.idx)
    t.join()
    assert sorted(seen) == list(range(n_events))
    assert seen == sorted(seen), "FIFO order within a shard"
    st = ep.stats()
    assert st["produce_full"] > 0, "the small ring should have exercised backpressure"
    assert prod.engine is not None, "the native producer engine must run on a GPU"
    span, single, by_kernel = prod.engine.copy_stats()
    assert span + single > 0
    assert (by_kernel == span + single) if copy_kernel != 0 else by_kernel == 0


@pytest.mark.parametrize("kind", ["shared", "dedicated"])
def test_peakfinder_consumer_counts(cuda_device, kind):
    """Peak totals of a producer -> consumer run equal the golden model's, with ordinary streams
    and with streams that own their hardware queues (producer and consumer sides)."""
    src = SyntheticRun("synthetic", 4, "epix10k2M", n_events=40, pool_frames=4, pinned=True, gen_device="cuda")
    cal = Calibrator(src.consts, cuda_device, Mode.calib)
    ring = FrameRing(cal.out_shape, cal.out_dtype, cuda_device, 16, 32)
    ep = QueueEndpoint(ring)
    prod = ProducerPipeline(src, cal, ep, chunk=16, compute_streams=2, stream_kind=kind)
    params = PeakFinderParams()
    cons = PeakFinderConsumer(ep, cal.out_shape, params, batch=16, stream_kind=kind)
    t = threading.Thread(target=prod.run)
    t.start()
    n = 0
    while True:
        try:
            n += cons.poll(0.5)
        except EndOfStream:
            break
    t.join()
    total = cons.synchronize()
    assert n == 40
    frames = reference.calibrate_reference(torch.from_numpy(src.pool.astype(np.int32)), src.consts)
    ref_peaks, _ = reference.peakfind_reference(frames, params)
    expect = sum(ref_peaks[i % 4].shape[0] for i in range(40))
    assert total == expect


def test_device_resident_source_calibrates_in_place(cuda_device):
    """Frames already in HBM: the native engine calibrates them in place (no staging copy) and the
    results are identical to the golden model."""
    src = SyntheticRun("synthetic", 5, "epix10k2M", n_events=40, pool_frames=8, pinned=False, gen_device="cuda")
    dev_pool = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16).to(cuda_device)

    class DevSource:
        spec = src.spec
        size = 1
        calibrated = False
        consts = src.consts

        def cycled_frames(self):
            return [int(dev_pool[j].data_ptr()) for j in range(dev_pool.shape[0])], [9.5] * dev_pool.shape[0]

        def n_local_events(self):
            return 40

    cal = Calibrator(src.consts, cuda_device, Mode.calib, common_mode=CommonModeParams())
    ring = FrameRing(cal.out_shape, cal.out_dtype, cuda_device, 16, 64)
    ep = QueueEndpoint(ring)
    prod = ProducerPipeline(DevSource(), cal, ep, chunk=8)
    assert prod.engine is not None and prod.engine.device_resident
    prod.run()
    ref = reference.calibrate_reference(torch.from_numpy(src.pool.astype(np.int32)), src.consts, None, cal.cm)
    n = 0
    while True:
        try:
            it = ep.get(timeout=0.5)
        except EndOfStream:
            break
        if it is None:
            continue
        with it:
            got = it.data.clone()
        torch.cuda.synchronize()
        assert torch.equal(got.cpu(), ref[it.idx % 8]), f"frame {it.idx}"
        n += 1
    assert n == 40
    assert prod.engine.timing()[0] < 1e-3, "no staging copies expected for a device-resident source"


@pytest.mark.parametrize("zero_copy", ["0", "1"])
def test_file_source_native_engine(cuda_device, tmp_path, monkeypatch, zero_copy):
    """Raw-run file -> native producer engine (pread thread pool into pinned staging, or DMA
    straight out of the registered file mapping; H2D, calib + common mode) -> queue: every event
    once, exact vs the golden model, gevt / photon energy from the file records, resume cursor
    honoured."""
    from psana_ray_amd.source import RawFileRun, make_synthetic_run

    monkeypatch.setenv("PSANA_RAY_FILE_ZEROCOPY", zero_copy)
    path = make_synthetic_run(str(tmp_path), "exp", 7, "epix10k2M", n_events=70, chunk=16)
    src = RawFileRun(path, "epix10k2M", exp="exp", run=7, rank=0, size=1)
    src.seek(5)
    cal = Calibrator(src.consts, cuda_device, Mode.calib, common_mode=CommonModeParams())
    ring = FrameRing(cal.out_shape, cal.out_dtype, cuda_device, 40, 24)   # small ring: backpressure
    ep = QueueEndpoint(ring)
    prod = ProducerPipeline(src, cal, ep, chunk=8)
    assert prod.engine is not None, "file sources must run on the native engine"
    assert prod.zero_copy == (zero_copy == "1")
    t = threading.Thread(target=prod.run)
    t.start()
    ref_src = RawFileRun(path, "epix10k2M", exp="exp", run=7, rank=0, size=1, pinned=False)
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
        ev = ref_src.staging[0]
        meta = ref_src.reader.read([gevt], [int(ev.ctypes.data)])
        exp = reference.calibrate_reference(torch.from_numpy(ev.astype(np.int32))[None], src.consts, None, cal.cm)[0]
        assert torch.equal(got.cpu(), exp), f"event {gevt}"
        assert meta[0][0] == gevt and (pe is None or abs(pe - meta[0][1]) < 1e-9)
        seen[gevt] = seen.get(gevt, 0) + 1
    t.join()
    assert sorted(seen) == list(range(5, 70)) and all(v == 1 for v in seen.values())


def test_engine_gpu_stage_timing(cuda_device):
    """gpu_timing=True: the engine event-times every chunk's H2D copy and calibration."""
    src = SyntheticRun("synthetic", 6, "epix10k2M", n_events=96, pool_frames=8, pinned=True, gen_device="cuda")
    cal = Calibrator(src.consts, cuda_device, Mode.calib, common_mode=CommonModeParams())
    ring = FrameRing(cal.out_shape, cal.out_dtype, cuda_device, 64, 128)
    ep = QueueEndpoint(ring)
    prod = ProducerPipeline(src, cal, ep, chunk=16, gpu_timing=True)
    assert prod.engine.gpu_timing_enabled
    prod.run()
    h2d_ms, h2d_n, cal_ms, cal_n = prod.engine.gpu_timing()
    assert h2d_n == 6 and cal_n == 6, (h2d_n, cal_n)
    assert h2d_ms > 0 and cal_ms > 0
    m = prod.metrics()
    assert m["gpu_chunks_timed"] == 6 and m["gpu_h2d_ms_per_chunk"] > 0
