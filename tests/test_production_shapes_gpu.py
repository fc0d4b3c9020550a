"""The shipped launch shapes under bit-exact test.

The producer launches 64 epix10k2M frames per kernel (bench.py --chunk, producer.py --chunk), and
the common-mode kernel's tile -> frame mapping depends on the frame count of the launch
(csrc/common_mode.hip, cm_coords), so the production count (64) and an odd one (37) are checked
in calib and in image mode, bitwise (int32 views: -0 vs +0 and NaN payloads count) against the
fp32 golden model (every event calibrated, masked and shaped, psana_ray/producer.py:88-97).  The
golden model runs on the GPU through plain PyTorch ops (sort-based medians, the same formulas
as on the CPU).  Plus: the end-to-end pipeline at chunk 64 with the default ring, and a peak-finder
batch whose workgroups park more candidates than fit in LDS (csrc/peakfind.hip, kPfCandCap)."""
import threading

import numpy as np
import pytest
import torch

from psana_ray_amd.config import PRODUCER_STREAM_KIND, PRODUCER_STREAMS, CommonModeParams, PeakFinderParams
from psana_ray_amd.models import CalibConstants, Calibrator, Mode, get_detector
from psana_ray_amd.ops import kernels, reference
from psana_ray_amd.source import generate_raw

pytestmark = pytest.mark.gpu


def _bitwise(a: torch.Tensor, b: torch.Tensor, what: str):
    a, b = a.contiguous(), b.to(a.device).contiguous()
    assert a.shape == b.shape, (a.shape, b.shape)
    ai, bi = a.view(torch.int32), b.view(torch.int32)
    bad = int((ai != bi).sum())
    if bad:
        d = (a - b).abs()
        d = d[~torch.isnan(d)]
        raise AssertionError(f"{what}: {bad} words differ (max |diff| {float(d.max()) if d.numel() else 0})")


@pytest.mark.parametrize("mode", ["calib", "image"])
@pytest.mark.parametrize("nframes", [64, 37])
def test_common_mode_production_launch_bitwise(cuda_device, mode, nframes):
    spec = get_detector("epix10k2M")
    consts = CalibConstants.random(spec, seed=31, gain_config="mixed", bad_fraction=0.02)
    raw, _ = generate_raw(consts, nframes, seed=32)
    raw = torch.from_numpy(raw.view(np.int16)).view(torch.uint16).to(cuda_device)
    mask = (np.random.default_rng(33).random(spec.frame_shape) > 0.05).astype(np.uint8) if mode == "calib" else None
    cm = CommonModeParams.parse("default")
    cal = Calibrator(consts, cuda_device, Mode(mode), mask=mask, common_mode=cm)
    out = torch.full((nframes, *cal.out_shape), float("nan"), device=cuda_device)
    cal.run([raw[i] for i in range(nframes)], [out[i] for i in range(nframes)])   # ONE launch (<= 64)
    torch.cuda.synchronize()
    for f0 in range(0, nframes, 16):   # golden model in slices (memory of the sort-based medians)
        r = raw[f0:f0 + 16].to(torch.int32)
        ref = reference.calibrate_reference(r, consts, mask, cal.cm)
        if mode == "image":
            geo = cal.geometry
            ref = reference.assemble_reference(ref, geo.rows, geo.cols, geo.image_shape)
        _bitwise(out[f0:f0 + 16], ref, f"{mode} cm, {nframes}-frame launch, frames {f0}..")
        del ref


@pytest.mark.parametrize("chunk,streams,kind", [(64, None, None), (16, 3, "dedicated"), (64, 1, "shared"),
                                               (32, 2, "high")])
def test_pipeline_exact_at_production_chunk(cuda_device, chunk, streams, kind):
    """The producer engine at its shipped chunk (64) with bench.py's default ring sizes: every frame
    of 200 events bit-exact, FIFO, with the sustained-rate completion log covering all of them --
    with the shipped compute streams, chunks spread over 3 streams with their own hardware queues,
    one ordinary stream, and two high-priority streams."""
    from psana_ray_amd.pipeline import ProducerPipeline
    from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint
    from psana_ray_amd.source import SyntheticRun

    n_events, batch = 200, 32
    src = SyntheticRun("synthetic", 5, "epix10k2M", n_events=n_events, pool_frames=8, pinned=True,
                       gen_device="cuda")
    cal = Calibrator(src.consts, cuda_device, Mode.calib, common_mode=CommonModeParams())
    ring = FrameRing(cal.out_shape, cal.out_dtype, cuda_device, 4 * chunk + batch, 400)
    ep = QueueEndpoint(ring)
    prod = ProducerPipeline(src, cal, ep, chunk=chunk, compute_streams=streams, stream_kind=kind)
    assert prod.chunk == chunk and prod.engine is not None
    assert prod.engine.compute_streams == (streams or PRODUCER_STREAMS["staged"])
    assert prod.stream_config == (streams or PRODUCER_STREAMS["staged"], kind or PRODUCER_STREAM_KIND["staged"])
    t = threading.Thread(target=prod.run)
    t.start()
    ref = reference.calibrate_reference(torch.from_numpy(src.pool.astype(np.int32)).to(cuda_device), src.consts, None,
                                        cal.cm)
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
        _bitwise(got, ref[it.idx % 8], f"frame {it.idx}")
        seen.append(it.idx)
    t.join()
    assert seen == list(range(n_events))
    _, log = prod.completion_log(0)
    assert log[-1][0] == n_events and len(log) == (n_events + chunk - 1) // chunk
    assert all(b[1] >= a[1] for a, b in zip(log, log[1:])), "completions out of order"


def _sorted_peaks(p):
    p = p.cpu()
    q = p[:, :3].to(torch.int64)
    return p[torch.argsort(q[:, 0] * 100_000_000 + q[:, 1] * 10_000 + q[:, 2])]


@pytest.mark.parametrize("quantile,floor,F", [(0.70, 512, 2), (0.50, 1200, 6)])
def test_peakfind_candidate_overflow(cuda_device, quantile, floor, F):
    """Candidates above thr_peak at ~30 % / ~50 % of the pixels: every workgroup parks more than
    kPfCandCap (512) of them in LDS and the rest go to its spill list in the scratch block
    (kPfSpillCap, 4096); with 6 frames at 50 % each workgroup's range (>= 4 x 4096 pixels of the 768
    resident workgroups, > 1200 candidates each) holds > 4608, past both, so the in-stream test
    path runs too.  The
    peak list still matches the golden model exactly (positions / values; intensities to fp32
    summation order)."""
    spec = get_detector("epix10k2M")
    consts = CalibConstants.random(spec, seed=8, gain_config="AHL")
    raw, _ = generate_raw(consts, F, seed=9)
    frames = reference.calibrate_reference(torch.from_numpy(raw.astype(np.int32)), consts, None, None)
    thr = float(torch.quantile(frames[0].flatten()[::97], quantile))
    params = PeakFinderParams(thr_peak=thr, son_min=0.0, radius=1, max_peaks=400_000)
    above = (frames > thr).reshape(F, -1).float()
    per_range = above.reshape(F, -1, 4096).sum(-1)
    assert float(per_range.min()) > floor, "test data too weak: some 4096-pixel range stays under the cap"
    d = frames.to(cuda_device).contiguous()
    peaks = torch.zeros((F, params.max_peaks, 8), dtype=torch.float32, device=cuda_device)
    counts = torch.zeros(F, dtype=torch.int32, device=cuda_device)
    summary = torch.zeros((F, 2), dtype=torch.float32, device=cuda_device)
    scr = torch.zeros(kernels.PF_SCRATCH_WORDS, dtype=torch.int32, device=cuda_device)
    kernels.peakfind([d[i] for i in range(F)], spec.frame_shape, params, peaks, counts, summary, scratch=scr)
    torch.cuda.synchronize()
    ref_peaks, ref_summary = reference.peakfind_reference(frames, params)
    for f in range(F):
        n = int(counts[f])
        assert n == ref_peaks[f].shape[0] and n < params.max_peaks, (n, ref_peaks[f].shape[0])
        got, exp = _sorted_peaks(peaks[f, :n]), _sorted_peaks(ref_peaks[f])
        assert torch.equal(got[:, :4], exp[:, :4])
        assert torch.allclose(got[:, 4:], exp[:, 4:], rtol=1e-4, atol=1e-3)
    assert torch.equal(summary[:, 0].cpu(), ref_summary[:, 0])
    assert int(scr[:256].abs().sum()) == 0   # the counters reset themselves (the spill lists need not)


def _keys(p):
    q = p[:, :3].to(torch.int64).cpu()
    return set((q[:, 0] * 100_000_000 + q[:, 1] * 10_000 + q[:, 2]).tolist())


@pytest.mark.parametrize("radius", [1, 2])
def test_peakfind_hit_rich_past_max_peaks(cuda_device, radius):
    """A hit-rich batch (10 % of the pixels above threshold: several candidate rounds per workgroup,
    ~100k peaks per frame) with max_peaks = 2048: counts are exact, and the 2048 records written per
    frame are distinct peaks of the golden model with its values (slots are reserved once per
    workgroup and frame; rounds past round 0 are re-tested only while their frame's reserved range
    reaches below max_peaks)."""
    spec = get_detector("epix10k2M")
    consts = CalibConstants.random(spec, seed=8, gain_config="AHL")
    raw, _ = generate_raw(consts, 2, seed=9)
    frames = reference.calibrate_reference(torch.from_numpy(raw.astype(np.int32)), consts, None, None)
    thr = float(torch.quantile(frames[0].flatten()[::97], 0.90))
    params = PeakFinderParams(thr_peak=thr, son_min=0.0, radius=radius, max_peaks=2048)
    F = frames.shape[0]
    d = frames.to(cuda_device).contiguous()
    peaks = torch.zeros((F, params.max_peaks, 8), dtype=torch.float32, device=cuda_device)
    counts = torch.zeros(F, dtype=torch.int32, device=cuda_device)
    summary = torch.zeros((F, 2), dtype=torch.float32, device=cuda_device)
    total = torch.zeros((), dtype=torch.int64, device=cuda_device)
    scr = torch.zeros(kernels.PF_SCRATCH_WORDS, dtype=torch.int32, device=cuda_device)
    kernels.peakfind([d[i] for i in range(F)], spec.frame_shape, params, peaks, counts, summary, total=total,
                     scratch=scr)
    torch.cuda.synchronize()
    ref_peaks, _ = reference.peakfind_reference(frames, PeakFinderParams(thr_peak=thr, son_min=0.0, radius=radius,
                                                                         max_peaks=1 << 30))
    assert int(total) == F * params.max_peaks
    for f in range(F):
        n = int(counts[f])
        assert n == ref_peaks[f].shape[0] and n > 8 * params.max_peaks, (n, ref_peaks[f].shape[0])
        got = _sorted_peaks(peaks[f])
        keys = _keys(got)
        assert len(keys) == params.max_peaks, "records written twice or left empty"
        ref = ref_peaks[f]
        q = ref[:, :3].to(torch.int64)
        rk = q[:, 0] * 100_000_000 + q[:, 1] * 10_000 + q[:, 2]
        sel = torch.isin(rk, torch.tensor(sorted(keys), dtype=torch.int64))
        assert int(sel.sum()) == params.max_peaks, "a written record is not a golden-model peak"
        exp = _sorted_peaks(ref[sel])
        assert torch.equal(got[:, :4], exp[:, :4])
        assert torch.allclose(got[:, 4:], exp[:, 4:], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("gap_fill", [None, True])
def test_image_pipeline_zero_filled_ring_exact(cuda_device, gap_fill):
    """Image mode through the producer engine at chunk 64 with a small ring (every slot reused
    several times): the ring starts zero-filled, so by default the kernels skip the per-frame gap
    fill (the gaps of every slot stay 0); with and without the skip every assembled frame is
    bit-exact against the golden assembly, gaps included."""
    from psana_ray_amd.pipeline import ProducerPipeline
    from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint
    from psana_ray_amd.source import SyntheticRun

    n_events, chunk = 320, 64
    src = SyntheticRun("synthetic", 5, "epix10k2M", n_events=n_events, pool_frames=8, pinned=True,
                       gen_device="cuda")
    cal = Calibrator(src.consts, cuda_device, Mode.image, common_mode=CommonModeParams())
    assert cal.plan.n_gap_runs > 0
    ring = FrameRing(cal.out_shape, cal.out_dtype, cuda_device, 2 * chunk, 32)
    assert ring.zero_filled
    ep = QueueEndpoint(ring)
    prod = ProducerPipeline(src, cal, ep, chunk=chunk, gap_fill=gap_fill)
    assert prod.gap_fill == (gap_fill is True)
    assert cal.plan.n_gap_runs > 0                  # the calibrator's own plan is untouched
    t = threading.Thread(target=prod.run)
    t.start()
    geo = cal.geometry
    ref = reference.calibrate_reference(torch.from_numpy(src.pool.astype(np.int32)).to(cuda_device), src.consts,
                                        None, cal.cm)
    ref = reference.assemble_reference(ref, geo.rows, geo.cols, geo.image_shape, None)
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
        _bitwise(got.view(-1), ref[it.idx % 8].reshape(-1), f"image frame {it.idx}")
        seen.append(it.idx)
    t.join()
    assert seen == list(range(n_events))
