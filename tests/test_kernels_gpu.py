"""HIP kernels vs the fp32 PyTorch golden models (ops.reference) on a real MI355X."""
import numpy as np
import pytest
import torch

from psana_ray_amd.config import CommonModeParams, PeakFinderParams
from psana_ray_amd.models import CalibConstants, Calibrator, Mode, get_detector, make_geometry
from psana_ray_amd.models.detector import DetectorSpec, register
from psana_ray_amd.ops import kernels, reference
from psana_ray_amd.source import generate_raw

pytestmark = pytest.mark.gpu

# ASIC shapes that route the common-mode launcher (csrc/common_mode.hip, launch_calib_cm) to each
# of its kernels: epix10k2M -> 176x48 compile-time net kernel, jungfrau -> 256x128 compile-time
# net kernel, tiny_epix -> 8-column-bank net kernel (runtime shape), cm_epix174 -> 48-column-bank
# net kernel (runtime shape), cm_epix44 / cm_jf64 / tiny_jungfrau -> generic bitonic kernel
register(DetectorSpec("cm_epix174", "epix10ka", 2, 174, 96, 174, 96, 48, 100.0, panel_gap_px=2))
register(DetectorSpec("cm_epix44", "epix10ka", 2, 88, 96, 44, 48, 16, 100.0, panel_gap_px=2))
register(DetectorSpec("cm_jf64", "jungfrau", 1, 128, 128, 64, 64, 32, 75.0, panel_gap_px=2))


def _setup(det, n, seed=0, gain_config="mixed"):
    spec = get_detector(det)
    consts = CalibConstants.random(spec, seed=seed, gain_config=gain_config, bad_fraction=0.02)
    raw, _ = generate_raw(consts, n, seed=seed + 1)
    return spec, consts, torch.from_numpy(raw.view(np.int16)).view(torch.uint16)


def _mask(spec, seed=3):
    rng = np.random.default_rng(seed)
    return (rng.random(spec.frame_shape) > 0.05).astype(np.uint8)


def _assert_equal(a, b, what):
    """Bit-exact: float outputs compare as int32 words, so -0 vs +0 (the reference masks with
    np.where(mask, data, 0) -> +0) and NaN payloads count."""
    a, b = a.cpu().contiguous(), b.cpu().contiguous()
    diff = (a - b).abs().max().item()
    if a.dtype == torch.float32 and b.dtype == torch.float32:
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), \
            f"{what}: max |diff| = {diff}, {int((a.view(torch.int32) != b.view(torch.int32)).sum())} words differ"
    else:
        assert torch.equal(a, b), f"{what}: max |diff| = {diff}"


@pytest.mark.parametrize("det", ["tiny_epix", "tiny_jungfrau", "tiny_plain", "epix10k2M", "jungfrau4M"])
@pytest.mark.parametrize("masked", [False, True])
def test_calib_basic_bitwise(cuda_device, det, masked):
    n = 3 if det in ("epix10k2M", "jungfrau4M") else 37   # 37 > 32 exercises launch chunking
    spec, consts, raw = _setup(det, n)
    mask = _mask(spec) if masked else None
    cal = Calibrator(consts, cuda_device, Mode.calib, mask=mask)
    out = cal(raw.to(cuda_device))
    torch.cuda.synchronize()
    ref = reference.calibrate_reference(raw.to(torch.int32), consts, mask)
    _assert_equal(out, ref, f"calib {det}")


@pytest.mark.parametrize("det", ["tiny_epix", "epix10k2M", "jungfrau05M", "cm_epix174", "cm_epix44", "cm_jf64",
                                 "tiny_jungfrau"])
@pytest.mark.parametrize("flags", [1, 2, 3])
def test_common_mode_bitwise(cuda_device, det, flags):
    n = 2 if det in ("epix10k2M", "jungfrau05M") else 5
    spec, consts, raw = _setup(det, n, seed=11, gain_config="mixed")
    cm = CommonModeParams(flags=flags, thr=30.0, maxcorr=50.0, npix_min=5)
    mask = _mask(spec)
    cal = Calibrator(consts, cuda_device, Mode.calib, mask=mask, common_mode=cm)
    out = cal(raw.to(cuda_device))
    torch.cuda.synchronize()
    ref = reference.calibrate_reference(raw.to(torch.int32), consts, mask, cal.cm)
    base = reference.calibrate_reference(raw.to(torch.int32), consts, mask, None)
    assert (ref - base).abs().max() > 0, "common mode changed nothing: test data too weak"
    _assert_equal(out, ref, f"cm{flags} {det}")


@pytest.mark.parametrize("det", ["epix10k2M", "jungfrau4M", "tiny_epix"])
def test_common_mode_switched_and_unswitched_waves_bitwise(cuda_device, det):
    """The decode / store phases take a wave-uniform fast path for items with no gain-switched pixel
    (PR_CM_BASE_FAST) and the general path otherwise: frames whose left half has a gain-switch bit on
    ~7 % of the pixels (every wave there takes the general path) and whose right half has none (every
    wave takes the fast path), Jungfrau also with its invalid gain code, bitwise against the golden."""
    spec = get_detector(det)
    consts = CalibConstants.random(spec, seed=9, gain_config="mixed", bad_fraction=0.02)
    n = 2
    raw, _ = generate_raw(consts, n, seed=4)
    raw = raw.astype(np.int32)
    rng = np.random.default_rng(2)
    P, H, W = spec.frame_shape
    left = np.zeros((n, P, H, W), bool)
    left[..., : W // 2] = True
    sw = left & (rng.random((n, P, H, W)) < 0.07)
    raw = np.where(sw, (raw & 0x3FFF) | (1 << 14), raw & 0x3FFF if spec.kind != "plain" else raw)
    if spec.kind == "jungfrau":   # some gain code 3 (G2) and code 2 (invalid) pixels in the left half too
        g2 = left & (rng.random((n, P, H, W)) < 0.02)
        bad = left & (rng.random((n, P, H, W)) < 0.01)
        raw = np.where(g2, raw | (3 << 14), raw)
        raw = np.where(bad, (raw & 0x3FFF) | (2 << 14), raw)
    raw = torch.from_numpy(raw.astype(np.uint16).view(np.int16)).view(torch.uint16)
    cm = CommonModeParams(flags=3, thr=30.0, maxcorr=50.0, npix_min=5)
    mask = _mask(spec)
    cal = Calibrator(consts, cuda_device, Mode.calib, mask=mask, common_mode=cm)
    out = cal(raw.to(cuda_device))
    torch.cuda.synchronize()
    ref = reference.calibrate_reference(raw.to(torch.int32), consts, mask, cal.cm)
    _assert_equal(out, ref, f"switched / unswitched waves {det}")


@pytest.mark.parametrize("det", ["epix10k2M", "jungfrau05M"])
@pytest.mark.parametrize("peds", ["random", "zeros_and_negative"])
def test_common_mode_signed_pedestals_match_bit_planes(cuda_device, det, peds, monkeypatch):
    """The production kernels read the CM eligibility from the pedestal sign bits
    (config.CM_SIGNED_PEDESTALS, CalibConstants.cm_signed_pedestals) instead of bit-planes: both
    encodings bitwise equal to each other and to the golden, with gain-switched pixels; a table with
    +0 / -0 pedestals still encodes, one negative pedestal falls back to the planes."""
    from psana_ray_amd import config
    spec, consts, raw = _setup(det, 3, seed=21, gain_config="mixed")   # odd: a one-frame tail workgroup
    r = raw.view(torch.int16).numpy().astype(np.int32) & 0xFFFF
    rng = np.random.default_rng(8)
    sw = rng.random(r.shape) < 0.03
    r = np.where(sw, (r & 0x3FFF) | (1 << 14), r)
    raw = torch.from_numpy(r.astype(np.uint16).view(np.int16)).view(torch.uint16)
    if peds == "zeros_and_negative":
        consts.pedestals[..., :3, :5] = 0.0
        consts.pedestals[..., 3:5, :5] = -0.0
    cm = CommonModeParams(flags=3, thr=30.0, maxcorr=50.0, npix_min=5)
    mask = _mask(spec)
    outs = {}
    for signed in (True, False):
        monkeypatch.setattr(config, "CM_SIGNED_PEDESTALS", signed)
        cal = Calibrator(consts, cuda_device, Mode.calib, mask=mask, common_mode=cm)
        assert (cal.ped_sg is not None) == signed   # both production kernels read them
        outs[signed] = cal(raw.to(cuda_device))
    torch.cuda.synchronize()
    ref = reference.calibrate_reference(raw.to(torch.int32), consts, mask, cal.cm)
    _assert_equal(outs[True], outs[False], f"signed vs planes {det} {peds}")
    _assert_equal(outs[True], ref, f"signed {det} {peds}")
    if peds == "zeros_and_negative":   # one negative pedestal: the sign cannot carry eligibility
        monkeypatch.setattr(config, "CM_SIGNED_PEDESTALS", True)
        consts.pedestals[(slice(None),) + (0,) * (consts.pedestals.ndim - 1)] = -1.0   # every gain range
        cal = Calibrator(consts, cuda_device, Mode.calib, mask=mask, common_mode=cm)
        assert cal.ped_sg is None
        out = cal(raw.to(cuda_device))
        torch.cuda.synchronize()
        _assert_equal(out, reference.calibrate_reference(raw.to(torch.int32), consts, mask, cal.cm),
                      f"negative pedestal fallback {det}")


def test_common_mode_even_odd_and_empty_segments(cuda_device):
    """Hand-built tile: even/odd participant counts, all-masked rows, |median| > maxcorr."""
    spec = get_detector("tiny_epix")
    consts = CalibConstants.random(spec, seed=5, gain_config="FH", bad_fraction=0.0)
    consts.pedestals[:] = 0.0
    consts.gains[:] = 1.0
    rng = np.random.default_rng(0)
    adu = rng.integers(0, 40, size=(4, *spec.frame_shape)).astype(np.uint16)
    adu[0, 0, 0, :8] = 1000           # bank fully above threshold -> no correction
    adu[1, 0, 3, 8:16] = 200          # |median| > maxcorr -> skipped
    raw = torch.from_numpy(adu.view(np.int16)).view(torch.uint16)
    mask = np.ones(spec.frame_shape, np.uint8)
    mask[0, 5, :] = 0                 # fully masked row
    mask[1, :, 7] = 0                 # masked column
    mask[0, 6, 1::2] = 0              # even/odd counts per bank
    cm = CommonModeParams(flags=3, thr=100.0, maxcorr=60.0, npix_min=3)
    cal = Calibrator(consts, cuda_device, Mode.calib, mask=mask, common_mode=cm)
    out = cal(raw.to(cuda_device))
    torch.cuda.synchronize()
    ref = reference.calibrate_reference(raw.to(torch.int32), consts, mask, cal.cm)
    _assert_equal(out, ref, "cm edge cases")


@pytest.mark.parametrize("det,cm", [("tiny_epix", None), ("tiny_epix", "3,30,50,5"), ("epix10k2M", None),
                                    ("epix10k2M", "default"), ("tiny_jungfrau", None), ("tiny_jungfrau", "default"),
                                    ("jungfrau05M", None), ("jungfrau05M", "default"), ("tiny_plain", None)])
def test_image_mode_matches_scatter(cuda_device, det, cm):
    """Without common mode: the LDS-tiled fused calibration + assembly; with common mode the CM
    kernel writes the image from its LDS tiles (gaps zero-filled).  Outputs start as NaN so
    unwritten (gap) pixels show up."""
    n = 2 if det in ("epix10k2M", "jungfrau05M") else 37   # 37 > 32: launch chunking
    spec, consts, raw = _setup(det, n, seed=21)
    cmp = CommonModeParams.parse(cm)
    cal = Calibrator(consts, cuda_device, Mode.image, common_mode=cmp)
    assert cal.tile_map is not None
    assert (cal.plan.mode == 5) == (cm is not None)
    out = torch.full((n, *cal.out_shape), float("nan"), device=cuda_device)
    raw = raw.to(cuda_device)
    cal.run([raw[i] for i in range(n)], [out[i] for i in range(n)])
    torch.cuda.synchronize()
    geo = cal.geometry
    calib = reference.calibrate_reference(raw.to(torch.int32), consts, None, cal.cm)
    ref = reference.assemble_reference(calib, geo.rows, geo.cols, geo.image_shape)
    assert out.shape == (n, 1, *geo.image_shape)
    _assert_equal(out, ref, f"image {det}")


@pytest.mark.parametrize("det,cm", [("tiny_epix", None), ("tiny_epix", "3,30,50,5"), ("epix10k2M", None),
                                    ("epix10k2M", "default")])
def test_image_mask_applied_after_assembly(cuda_device, det, cm):
    """Image-shaped masks: folded into the tile codes (no common mode) or into the fused plan's
    gain factors (common mode; eligibility unchanged, the reference masks after assembly)."""
    spec, consts, raw = _setup(det, 3, seed=4)
    geo = make_geometry(spec)
    imask = (np.random.default_rng(1).random(geo.image_shape) > 0.3).astype(np.uint8)
    cal = Calibrator(consts, cuda_device, Mode.image, mask=imask, common_mode=CommonModeParams.parse(cm))
    out = cal(raw.to(cuda_device))
    torch.cuda.synchronize()
    calib = reference.calibrate_reference(raw.to(torch.int32), consts, None, cal.cm)
    ref = reference.assemble_reference(calib, geo.rows, geo.cols, geo.image_shape, imask)
    _assert_equal(out, ref, "image mask")


def _sorted_peaks(p):
    p = p.cpu()
    if p.numel() == 0:
        return p
    q = p[:, :3].to(torch.int64)
    key = q[:, 0] * 100_000_000 + q[:, 1] * 10_000 + q[:, 2]
    return p[torch.argsort(key)]


@pytest.mark.parametrize("scratch", [False, True])
@pytest.mark.parametrize("radius", [1, 2])
@pytest.mark.parametrize("det", ["tiny_epix", "tiny_plain", "epix10k2M", "jungfrau05M"])
def test_peakfind_vs_reference(cuda_device, det, radius, scratch):
    """scratch: the self-resetting outputs (no zeroing before the call); run twice with the same
    scratch and garbage in counts / summary to show the last workgroup writes them whole and
    re-zeroes the scratch."""
    spec, consts, raw = _setup(det, 3, seed=8, gain_config="AHL")
    frames = reference.calibrate_reference(raw.to(torch.int32), consts, None, None)
    params = PeakFinderParams(thr_peak=15.0, son_min=4.0, radius=radius, max_peaks=4096)
    F = frames.shape[0]
    d = frames.to(cuda_device).contiguous()
    peaks = torch.zeros((F, params.max_peaks, 8), dtype=torch.float32, device=cuda_device)
    counts = torch.zeros(F, dtype=torch.int32, device=cuda_device)
    summary = torch.zeros((F, 2), dtype=torch.float32, device=cuda_device)
    total = torch.zeros((), dtype=torch.int64, device=cuda_device)
    scr = torch.zeros(kernels.PF_SCRATCH_WORDS, dtype=torch.int32, device=cuda_device) if scratch else None
    for _ in range(2 if scratch else 1):
        counts.fill_(12345)
        summary.fill_(-7.0)
        kernels.peakfind([d[i] for i in range(F)], spec.frame_shape, params, peaks, counts, summary, total=total,
                         scratch=scr)
    torch.cuda.synchronize()
    ref_peaks, ref_summary = reference.peakfind_reference(frames, params)
    if scratch:
        assert int(scr[:256].abs().sum()) == 0, "scratch counters not re-zeroed by the last workgroup"
    assert int(total) == (2 if scratch else 1) * sum(min(int(c), params.max_peaks) for c in counts.cpu())
    for f in range(F):
        n = int(counts[f])
        assert n == ref_peaks[f].shape[0], f"frame {f}: {n} peaks vs reference {ref_peaks[f].shape[0]}"
        assert n > 0 or det == "tiny_plain"
        got = _sorted_peaks(peaks[f, :n])
        exp = _sorted_peaks(ref_peaks[f])
        assert torch.equal(got[:, :4], exp[:, :4])
        assert torch.allclose(got[:, 4:], exp[:, 4:], rtol=1e-4, atol=1e-3)
    assert torch.equal(summary[:, 0].cpu(), ref_summary[:, 0])
    assert torch.allclose(summary[:, 1].cpu(), ref_summary[:, 1], rtol=1e-4)


@pytest.mark.parametrize("scratch", [False, True])
def test_peakfind_total_counts_only_written_records(cuda_device, scratch):
    """max_peaks below the frames' peak counts: counts report every accepted peak, the running
    total only the records written (min(count, max_peaks) per frame) -- per peak without a scratch
    block, in one atomic per launch from the last workgroup with one."""
    spec, consts, raw = _setup("jungfrau05M", 5, seed=8, gain_config="AHL")
    frames = reference.calibrate_reference(raw.to(torch.int32), consts, None, None)
    params = PeakFinderParams(thr_peak=15.0, son_min=4.0, radius=1, max_peaks=3)
    ref_peaks, _ = reference.peakfind_reference(frames, PeakFinderParams(thr_peak=15.0, son_min=4.0, radius=1))
    F = frames.shape[0]
    assert all(p.shape[0] > params.max_peaks for p in ref_peaks), "fixture must overflow max_peaks"
    d = frames.to(cuda_device).contiguous()
    peaks = torch.zeros((F, params.max_peaks, 8), dtype=torch.float32, device=cuda_device)
    counts = torch.zeros(F, dtype=torch.int32, device=cuda_device)
    summary = torch.zeros((F, 2), dtype=torch.float32, device=cuda_device)
    total = torch.full((), 5, dtype=torch.int64, device=cuda_device)
    scr = torch.zeros(kernels.PF_SCRATCH_WORDS, dtype=torch.int32, device=cuda_device) if scratch else None
    for _ in range(3):
        kernels.peakfind([d[i] for i in range(F)], spec.frame_shape, params, peaks, counts, summary, total=total,
                         scratch=scr)
    torch.cuda.synchronize()
    assert [int(c) for c in counts.cpu()] == [p.shape[0] for p in ref_peaks]
    assert int(total) == 5 + 3 * F * params.max_peaks
    for f in range(F):   # the written records: distinct golden-model peaks
        got = peaks[f].cpu()
        ref = {tuple(r[:4].tolist()) for r in ref_peaks[f]}
        rows = {tuple(r[:4].tolist()) for r in got}
        assert len(rows) == params.max_peaks and rows <= ref


@pytest.mark.parametrize("det,F", [("tiny_epix", kernels.MAX_FRAMES), ("jungfrau05M", 7)])
def test_peakfind_full_batch(cuda_device, det, F):
    """A whole launch (64 frames) and an odd frame count: the balanced grid's contiguous chunk
    ranges cross frame boundaries at arbitrary points; every frame's statistics and records must
    still match the golden model."""
    spec, consts, raw = _setup(det, F, seed=11, gain_config="AHL")
    frames = reference.calibrate_reference(raw.to(torch.int32), consts, None, None)
    params = PeakFinderParams(thr_peak=15.0, son_min=4.0, radius=1, max_peaks=4096)
    d = frames.to(cuda_device).contiguous()
    peaks = torch.zeros((F, params.max_peaks, 8), dtype=torch.float32, device=cuda_device)
    counts = torch.zeros(F, dtype=torch.int32, device=cuda_device)
    summary = torch.zeros((F, 2), dtype=torch.float32, device=cuda_device)
    scr = torch.zeros(kernels.PF_SCRATCH_WORDS, dtype=torch.int32, device=cuda_device)
    kernels.peakfind([d[i] for i in range(F)], spec.frame_shape, params, peaks, counts, summary, scratch=scr)
    torch.cuda.synchronize()
    ref_peaks, ref_summary = reference.peakfind_reference(frames, params)
    assert int(scr[:256].abs().sum()) == 0   # counters (the spill lists need not be zero)
    for f in range(F):
        n = int(counts[f])
        assert n == ref_peaks[f].shape[0], f"frame {f}: {n} peaks vs reference {ref_peaks[f].shape[0]}"
        assert torch.equal(_sorted_peaks(peaks[f, :n])[:, :4], _sorted_peaks(ref_peaks[f])[:, :4])
    assert torch.equal(summary[:, 0].cpu(), ref_summary[:, 0])
    assert torch.allclose(summary[:, 1].cpu(), ref_summary[:, 1], rtol=1e-4)


def test_kernel_rejects_bad_shapes(cuda_device):
    spec, consts, raw = _setup("tiny_epix", 1)
    cal = Calibrator(consts, cuda_device, Mode.calib)
    bad_out = torch.empty(10, device=cuda_device)
    with pytest.raises(ValueError):
        kernels.calib_basic([raw[0].to(cuda_device)], [bad_out], cal.ped, cal.gf, spec.kernel_kind)
    with pytest.raises(ValueError):
        kernels.calib_basic([raw[0]], [torch.empty(spec.npix)], cal.ped, cal.gf, spec.kernel_kind)


@pytest.mark.parametrize("det", ["cm_epix44", "cm_jf64", "tiny_jungfrau"])
def test_common_mode_generic_kernel_bitwise(cuda_device, det):
    """Shapes without a compile-time network run the generic whole-wave bitonic kernel (any tile
    size): exact as well, with a frame mask and mixed gain configuration."""
    spec, consts, raw = _setup(det, 2, seed=13, gain_config="mixed")
    cm = CommonModeParams(flags=3, thr=30.0, maxcorr=50.0, npix_min=5)
    mask = _mask(spec)
    cal = Calibrator(consts, cuda_device, Mode.calib, mask=mask, common_mode=cm)
    out = cal(raw.to(cuda_device))
    torch.cuda.synchronize()
    ref = reference.calibrate_reference(raw.to(torch.int32), consts, mask, cal.cm)
    _assert_equal(out, ref, f"generic cm {det}")


@pytest.mark.parametrize("wgs", [1, 7, 128, 4096])
def test_copy_runs_kernel_bitwise(cuda_device, native, wgs):
    """The queue fabric's batched copy (csrc/gather.hip copy_runs_kernel): many runs of different
    lengths (a 16-B word up to several 16-KB chunks, not chunk multiples) in ONE launch, with grids
    smaller and larger than the chunk count -- every byte lands once, nothing outside the runs is
    touched."""
    g = torch.Generator(device="cpu").manual_seed(5)
    sizes = [16, 48, 16384, 16400, 65536 + 32, 3 * 16384 - 16, 1 << 20, 8650752]
    srcs = [torch.randint(-2 ** 31, 2 ** 31 - 1, (n // 4,), generator=g, dtype=torch.int32).to(cuda_device)
            for n in sizes]
    dst = torch.full((sum(n // 4 for n in sizes) + 64,), -7, dtype=torch.int32, device=cuda_device)
    offs, o = [], 16
    for n in sizes:
        offs.append(o)
        o += n // 4
    grid = native.copy_runs([int(s.data_ptr()) for s in srcs], [int(dst[a:].data_ptr()) for a in offs], sizes,
                            wgs, 0)
    torch.cuda.synchronize()
    assert 1 <= grid <= wgs
    for s, a in zip(srcs, offs):
        assert torch.equal(dst[a:a + s.numel()], s)
    assert int((dst[:16] != -7).sum()) == 0 and int((dst[o:] != -7).sum()) == 0


@pytest.mark.parametrize("shape,n", [((16, 352, 384), 40), ((1, 9, 17), 3), ((1, 5, 7), 70)])
def test_mask_frames_kernel_matches_where(cuda_device, shape, n):
    """psana-calibrated upload path: one mask_frames launch per <= 64 frames equals
    np.where(mask, data, 0) (psana_ray/producer.py:92-95) bit for bit, 4-pixel body and scalar tail."""
    from psana_ray_amd.queue.ring import slot_stride

    g = torch.Generator().manual_seed(5)
    data = torch.randn((n, *shape), generator=g).to(cuda_device)
    keep = torch.rand(shape, generator=g) > 0.3
    zero = (~keep).reshape(-1).to(torch.uint8).to(cuda_device)
    ref = torch.where(keep.to(cuda_device), data, torch.zeros_like(data))
    # frames in ring-like slots: 256-B aligned starts whatever the frame size (FrameRing.slot_bytes)
    fb = data[0].numel() * 4
    sb = slot_stride(fb)
    buf = torch.zeros(n * sb, dtype=torch.uint8, device=cuda_device)
    frames = [buf[i * sb:i * sb + fb].view(torch.float32).view(shape) for i in range(n)]
    for i in range(n):
        frames[i].copy_(data[i])
    kernels.mask_frames(frames, zero)
    torch.cuda.synchronize()
    _assert_equal(torch.stack(frames), ref, f"mask_frames {shape}")
