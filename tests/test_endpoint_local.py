"""Single-process shared queue (world == 1) on the CPU: producer pipeline -> ring -> consumer."""
import threading

import numpy as np
import pytest
import torch

from psana_ray_amd.config import CommonModeParams
from psana_ray_amd.models import Calibrator, Mode
from psana_ray_amd.ops import reference
from psana_ray_amd.pipeline import ProducerPipeline
from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint
from psana_ray_amd.source import SyntheticRun


@pytest.mark.parametrize("mode", [Mode.calib, Mode.image, Mode.raw])
def test_local_stream_exactly_once_and_eos(native, mode):
    src = SyntheticRun("synthetic", 1, "tiny_epix", n_events=23, pool_frames=5, gen_device="cpu")
    cal = Calibrator(src.consts, "cpu", mode, common_mode=CommonModeParams() if mode == Mode.calib else None)
    ring = FrameRing(cal.out_shape, cal.out_dtype, "cpu", 4, 3)
    ep = QueueEndpoint(ring)
    prod = ProducerPipeline(src, cal, ep, chunk=4)
    t = threading.Thread(target=prod.run)
    t.start()
    seen = []
    pool_raw = torch.from_numpy(src.pool.astype(np.int32))
    while True:
        try:
            it = ep.get(timeout=0.2)
        except EndOfStream:
            break
        if it is None:
            continue
        rank, idx, data, pe = it.to_list(copy=True)
        assert data.shape == tuple(cal.out_shape)
        assert data.dim() >= 3                                    # R-06 ndim >= 3
        if mode == Mode.calib:
            exp = reference.calibrate_reference(pool_raw[idx % 5][None], src.consts, None, cal.cm)[0]
            assert torch.equal(data, exp)
        seen.append(idx)
    t.join(10)
    assert seen == list(range(23))
    with pytest.raises(EndOfStream):
        ep.get()


def test_max_steps_is_per_rank(native):
    src = SyntheticRun("synthetic", 1, "tiny_plain", n_events=None, pool_frames=2, gen_device="cpu")
    cal = Calibrator(src.consts, "cpu", Mode.calib)
    ep = QueueEndpoint(FrameRing(cal.out_shape, cal.out_dtype, "cpu", 4, 64))
    n = ProducerPipeline(src, cal, ep, chunk=4).run(max_steps=10)
    assert n == 10 and ep.size() == 10


def test_backpressure_blocks_until_consumed(native):
    src = SyntheticRun("synthetic", 1, "tiny_plain", n_events=12, pool_frames=2, gen_device="cpu")
    cal = Calibrator(src.consts, "cpu", Mode.calib)
    ep = QueueEndpoint(FrameRing(cal.out_shape, cal.out_dtype, "cpu", 2, 2))
    prod = ProducerPipeline(src, cal, ep, chunk=2, acquire_timeout_s=0.05)
    t = threading.Thread(target=prod.run)
    t.start()
    t.join(0.5)
    assert t.is_alive(), "producer must block while the queue is full"
    got = 0
    while True:
        try:
            it = ep.get(timeout=0.2)
        except EndOfStream:
            break
        if it is not None:
            it.release()
            got += 1
    t.join(5)
    assert got == 12 and prod.full_waits > 0


def test_ring_slots_are_256_byte_strided_for_odd_frames(native):
    """a 9 x 17 float32 image is 612 B; its ring slots start 256-B aligned (768-B stride)
    so the 16-B-vector kernels and the fabric's copy kernel can use every slot."""
    import torch

    from psana_ray_amd.queue import FrameRing

    ring = FrameRing((1, 9, 17), torch.float32, torch.device("cpu"), 3, 4)
    assert ring.frame_bytes == 612 and ring.slot_bytes == 768
    ptrs = ring.slot_ptrs
    assert all(b - a == 768 for a, b in zip(ptrs, ptrs[1:]))
    assert all(p % 16 == 0 for p in ptrs)
    for i in range(ring.n_slots):
        v = ring.slot(i)
        assert v.shape == (1, 9, 17) and v.is_contiguous() and v.data_ptr() == ptrs[i]
    for i in range(ring.n_slots):   # host ring memory is not zero-initialised
        ring.slot(i).fill_(0.0)
    ring.slot(1).fill_(7.0)
    assert float(ring.slot(0).sum()) == 0.0 and float(ring.slot(2).sum()) == 0.0
