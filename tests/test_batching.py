"""Batches for PyTorch consumers (batching.py): leased slots -> one contiguous tensor + metadata,
slots released (the ring recycles), bf16 conversion, DataReader.batches on the in-process queue,
and (GPU) the single-launch gather kernel vs torch."""
import math
import threading

import numpy as np
import pytest
import torch

from psana_ray_amd.batching import FrameBatch, collate_items
from psana_ray_amd.models import Calibrator, Mode
from psana_ray_amd.pipeline import ProducerPipeline
from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint
from psana_ray_amd.source import SyntheticRun


def _stream_batches(device, dtype, n_events=19, batch=4, consumer_slots=5):
    src = SyntheticRun("synthetic", 3, "tiny_epix", n_events=n_events, pool_frames=4,
                       gen_device="cpu" if device == "cpu" else "cuda", pinned=device != "cpu")
    cal = Calibrator(src.consts, device, Mode.calib)
    ring = FrameRing(cal.out_shape, cal.out_dtype, device, 8, consumer_slots)
    ep = QueueEndpoint(ring)
    prod = ProducerPipeline(src, cal, ep, chunk=4)
    t = threading.Thread(target=prod.run)
    t.start()
    out, pending, refs = [], [], {}
    while True:
        try:
            it = ep.get(timeout=0.2)
        except EndOfStream:
            break
        if it is None:
            continue
        refs[it.idx] = it.data.detach().clone().float().cpu()
        pending.append(it)
        if len(pending) == batch:
            out.append(collate_items(pending, dtype))
            pending = []
    if pending:
        out.append(collate_items(pending, dtype))
    t.join(30)
    return out, refs, ring


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_collate_cpu_ring_recycles(native, dtype):
    # 5 consumer slots, 19 events, batches of 4: completes only if collated slots are released
    batches, refs, ring = _stream_batches("cpu", dtype)
    assert sum(len(b) for b in batches) == 19 and all(isinstance(b, FrameBatch) for b in batches)
    seen = []
    for b in batches:
        assert b.data.dtype == dtype and b.data.shape[1:] == next(iter(refs.values())).shape
        for i in range(len(b)):
            k = int(b.idx[i])
            assert torch.equal(b.data[i].float(), refs[k].to(dtype).float())
            assert int(b.gevt[i]) == k and int(b.rank[i]) == 0
            seen.append(k)
    assert seen == list(range(19))
    items = list(batches[0].items())
    assert len(items) == len(batches[0]) and items[0][1] == int(batches[0].idx[0])


def test_reader_batches_in_process_queue(native):
    from psana_ray_amd.data_reader import DataReader
    from psana_ray_amd.queue.cpu_queue import create_queue, drop_queue

    drop_queue("bq", "bns")
    q = create_queue("bq", "bns", maxsize=64)
    for i in range(10):
        assert q.put([0, i, np.full((2, 4, 8), i, np.float32), None if i == 3 else 9.5])
    with DataReader(queue_name="bq", ray_namespace="bns") as r:
        bs = list(r.batches(4, timeout=0.2))
    drop_queue("bq", "bns")
    assert [len(b) for b in bs] == [4, 4, 2]
    assert [int(x) for b in bs for x in b.idx] == list(range(10))
    assert math.isnan(float(bs[0].photon_energy[3])) and float(bs[0].photon_energy[0]) == 9.5
    assert float(bs[2].data[1].mean()) == 9.0


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gather_kernel_matches_torch(native, cuda_device, dtype):
    from psana_ray_amd.ops import kernels

    g = torch.Generator(device="cuda").manual_seed(0)
    frames = [torch.randn((16, 352, 384), device=cuda_device, generator=g) * 100 for _ in range(37)]
    frames[5][0, 0, :4] = torch.tensor([float("nan"), float("inf"), -0.0, 1e-40])
    out = torch.empty((37, 16, 352, 384), dtype=dtype, device=cuda_device)
    kernels.gather_frames(frames, out)
    ref = torch.stack(frames).to(dtype)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16 if dtype == torch.bfloat16 else torch.int32),
                       ref.view(torch.int16 if dtype == torch.bfloat16 else torch.int32)), "bitwise mismatch"
    with pytest.raises(ValueError):
        kernels.gather_frames(frames[:2], out[:3])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_collate_gpu_ring_recycles(native, cuda_device, dtype):
    batches, refs, ring = _stream_batches("cuda", dtype)
    assert sum(len(b) for b in batches) == 19
    for b in batches:
        assert b.data.device.type == "cuda" and b.data.dtype == dtype
        for i in range(len(b)):
            assert torch.equal(b.data[i].float().cpu(), refs[int(b.idx[i])].to(dtype).float())
