"""Golden-model (ops.reference) semantics on CPU: gain decode, masks, common mode, assembly."""
import numpy as np
import pytest
import torch

from psana_ray_amd.config import CommonModeParams, PeakFinderParams
from psana_ray_amd.models import (EPIX10K2M, CalibConstants, Calibrator, Mode, get_detector, list_detectors,
                                  make_geometry)
from psana_ray_amd.ops import reference
from psana_ray_amd.source import generate_raw


def _raw(det, n=2, seed=0, cfg="mixed"):
    spec = get_detector(det)
    c = CalibConstants.random(spec, seed=seed, gain_config=cfg)
    r, pe = generate_raw(c, n, seed=seed + 1)
    return spec, c, torch.from_numpy(r.astype(np.int32))


def test_epix_gain_decode_bit14():
    spec, c, _ = _raw("tiny_epix", cfg="AHL")
    raw = torch.zeros((1, *spec.frame_shape), dtype=torch.int32)
    raw[..., 0, 0] = 100                   # high gain -> AHL_H (3)
    raw[..., 0, 1] = 100 | (1 << 14)       # switched -> AHL_L (5)
    adu, g, valid = reference.decode_gain(raw, c)
    assert int(g[0, 0, 0, 0]) == 3 and int(g[0, 0, 0, 1]) == 5
    assert int(adu[0, 0, 0, 1]) == 100 and bool(valid.all())


def test_jungfrau_gain_bits():
    spec, c, _ = _raw("tiny_jungfrau")
    raw = torch.zeros((1, *spec.frame_shape), dtype=torch.int32)
    for k, gb in enumerate((0, 1, 2, 3)):
        raw[0, 0, 0, k] = 50 | (gb << 14)
    adu, g, valid = reference.decode_gain(raw, c)
    assert g[0, 0, 0, :4].tolist()[:2] == [0, 1] and int(g[0, 0, 0, 3]) == 2
    assert valid[0, 0, 0, :4].tolist() == [True, True, False, True]
    out = reference.calibrate_reference(raw, c)
    assert float(out[0, 0, 0, 2]) == 0.0   # invalid gain bits -> 0


def test_calibration_formula_and_mask_truthy_keeps():
    spec, c, raw = _raw("tiny_epix", n=1)
    mask = np.ones(spec.frame_shape, np.uint8)
    mask[0, 0, :5] = 0
    out = reference.calibrate_reference(raw, c, mask)
    adu, g, _ = reference.decode_gain(raw, c)
    ped = np.take_along_axis(c.pedestals, g[0].numpy()[None], 0)[0]
    gain = np.take_along_axis(c.gains, g[0].numpy()[None], 0)[0]
    exp = (adu[0].numpy().astype(np.float32) - ped) * (np.float32(1) / gain)
    exp = np.where(mask.astype(bool), exp, 0)
    np.testing.assert_array_equal(out[0].numpy(), exp.astype(np.float32))
    assert (out[0, 0, 0, :5] == 0).all()


def test_common_mode_removes_row_offsets():
    spec = get_detector("tiny_epix")
    c = CalibConstants.random(spec, seed=2, gain_config="FH", bad_fraction=0.0)
    rng = np.random.default_rng(0)
    offs = rng.normal(0, 8, size=(spec.n_panels, spec.panel_rows, spec.panel_cols // spec.bank_cols))
    adu = c.pedestals[0] + np.repeat(offs, spec.bank_cols, axis=2) + rng.normal(0, 0.5, spec.frame_shape)
    raw = torch.from_numpy(np.round(adu).astype(np.int32))[None]
    base = reference.calibrate_reference(raw, c)
    cm = reference.calibrate_reference(raw, c, None, CommonModeParams(flags=1, thr=50, maxcorr=100, npix_min=3,
                                                                       bank_cols=spec.bank_cols))
    assert float((cm * c.gains[0]).std()) < 0.3 * float((base * c.gains[0]).std())


def test_masked_median_numpy_semantics():
    x = torch.tensor([[3.0, 1.0, 2.0, 10.0], [4.0, 4.0, 1.0, 2.0]])
    m = torch.tensor([[True, True, True, False], [True, True, True, True]])
    med, cnt = reference.masked_median(x, m, dim=-1)
    assert med.squeeze(-1).tolist() == [2.0, 3.0]
    assert cnt.squeeze(-1).tolist() == [3, 4]


def test_geometry_unique_and_epix_image_size():
    for det in list_detectors():
        geo = make_geometry(get_detector(det))
        idx = geo.index_map()
        assert (idx >= 0).sum() == geo.spec.npix
    geo = make_geometry(EPIX10K2M)
    assert 1500 <= geo.image_shape[0] <= 1800   # "H,W ~ 1.7k" (SURVEY K-05)


def test_gap_fill_table_covers_exactly_the_gaps():
    """The fused CM -> image kernel zeroes the image through this table: aligned 16-B chunks
    first (entry >= 0, a multiple of 4), single elements after (entry = -1 - element); together
    they must cover every gap element once and no panel pixel."""
    for det in list_detectors():
        geo = make_geometry(get_detector(det))
        gap = geo.index_map().ravel() < 0
        t = geo.gap_fill_table()
        assert t.dtype == np.int32
        nch = int((t >= 0).sum())
        assert (t[:nch] >= 0).all() and (t[nch:] < 0).all(), "chunks must precede singles"
        ch, si = t[:nch], -1 - t[nch:]
        assert (ch % 4 == 0).all()
        hits = np.zeros(gap.size, np.int32)
        for k in range(4):
            np.add.at(hits, ch + k, 1)
        np.add.at(hits, si, 1)
        assert np.array_equal(hits, gap.astype(np.int32)), det


def test_cpu_calibrator_image_mode_shape():
    spec, c, raw = _raw("tiny_epix", n=2)
    cal = Calibrator(c, "cpu", Mode.image)
    out = cal(torch.from_numpy(raw.numpy().astype(np.uint16).view(np.int16)).view(torch.uint16))
    assert out.shape == (2, 1, *cal.geometry.image_shape)
    assert out.dtype == torch.float32


def test_peakfind_reference_finds_planted_peak():
    frames = torch.zeros((1, 1, 32, 32))
    frames[0, 0, 10, 12] = 100.0
    frames[0, 0, 10, 13] = 50.0
    peaks, summ = reference.peakfind_reference(frames, PeakFinderParams(thr_peak=20, son_min=0.0, radius=1))
    assert peaks[0].shape[0] == 1
    assert peaks[0][0, :3].tolist() == [0.0, 10.0, 12.0]
    assert summ[0].tolist() == [2.0, 150.0]


def test_commonmode_parse():
    assert CommonModeParams.parse("off") is None
    cm = CommonModeParams.parse("1,20,inf,7,24")
    assert cm.flags == 1 and cm.thr == 20 and cm.maxcorr == float("inf") and cm.npix_min == 7 and cm.bank_cols == 24


def _emulate_tiles(frame: np.ndarray, tm):
    """numpy model of csrc/image.hip's use of a TileMap (stage box with pitch w+1, then codes)."""
    from psana_ray_amd.models.geometry import TILE_H, TILE_W

    himg, wimg = tm.image_shape
    out = np.zeros(himg * wimg, np.float32)
    flat = frame.ravel()
    codes = tm.codes.reshape(himg, wimg)
    for t in range(tm.n_tiles):
        ty, tx = divmod(t, tm.tiles_x)
        ys = slice(ty * TILE_H, min(himg, (ty + 1) * TILE_H))
        xs = slice(tx * TILE_W, min(wimg, (tx + 1) * TILE_W))
        cd = codes[ys, xs]
        p, r0, c0, h, w = tm.tiles[t, :5]
        stage = np.zeros(h * (w + 1) + 1, np.float32)
        if p >= 0:
            box = np.zeros((h, w + 1), np.float32)
            box[:, :w] = frame[p, r0:r0 + h, c0:c0 + w]
            stage[:h * (w + 1)] = box.ravel()
        v = np.zeros(cd.shape, np.float32)
        v[cd >= 0] = stage[cd[cd >= 0]]
        v[cd <= -2] = flat[-(cd[cd <= -2].astype(np.int64) + 2)]
        out.reshape(himg, wimg)[ys, xs] = v
    return out.reshape(himg, wimg)


@pytest.mark.parametrize("det", ["tiny_epix", "epix10k2M", "tiny_jungfrau"])
@pytest.mark.parametrize("masked", [False, True])
def test_tile_map_reproduces_assembly(det, masked):
    from psana_ray_amd.models import get_detector, make_geometry
    from psana_ray_amd.models.geometry import build_tile_map

    spec = get_detector(det)
    geo = make_geometry(spec)
    rng = np.random.default_rng(1)
    frame = rng.normal(size=spec.frame_shape).astype(np.float32)
    mask = (rng.random(geo.image_shape) > 0.1).astype(np.uint8) if masked else None
    tm = build_tile_map(geo.index_map(), spec, geo.image_shape, mask)
    assert tm.staged_px + tm.direct_px == (spec.npix if mask is None else int((geo.index_map().reshape(geo.image_shape)[mask > 0] >= 0).sum()))
    ref = reference.assemble_reference(torch.from_numpy(frame)[None], geo.rows, geo.cols, geo.image_shape,
                                       mask)[0, 0].numpy()
    np.testing.assert_array_equal(_emulate_tiles(frame, tm), ref)


def test_cm_quad_lane_algorithm_emulation():
    """The 4-lanes-per-column median of csrc/common_mode.hip (CQ = 4), emulated lane by lane in
    numpy, equals np.median on random columns (ties, empty / tiny / odd-sized columns)."""
    import importlib.util
    import os

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "cm_quad_emulation.py")
    spec = importlib.util.spec_from_file_location("cm_quad_emulation", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.run(trials=600, seed=3) == 0


@pytest.mark.parametrize("det", ["epix10k2M", "jungfrau05M", "tiny_epix"])
def test_cm_signed_pedestals_encode_eligibility(det):
    """CalibConstants.cm_signed_pedestals: |table| is the pedestal table, the sign bit is set exactly
    where device_tables' eligibility planes have a 0 bit, -0.0 pedestals encode like +0.0, and a
    negative pedestal makes the encoding unavailable (None)."""
    spec = get_detector(det)
    consts = CalibConstants.random(spec, seed=4, gain_config="mixed", bad_fraction=0.05)
    consts.pedestals[..., 0, :4] = -0.0
    ped, _, planes = consts.device_tables(None)
    sg = consts.cm_signed_pedestals(ped)
    assert sg is not None and sg.dtype == np.float32 and sg.shape == ped.shape
    np.testing.assert_array_equal(np.abs(sg), np.where(ped == 0, np.float32(0), ped))
    nc = ped.shape[0]
    stride = {1: 1, 2: 2, 3: 4}[nc]
    pl = planes.reshape(-1, stride)
    for c in range(nc):
        elig = ((pl[:, c][:, None] >> np.arange(8)) & 1).astype(bool).reshape(-1)
        np.testing.assert_array_equal(~np.signbit(sg[c]), elig)
    assert 0 < np.signbit(sg).mean() < 1
    ped[0, 7] = -1.0
    assert consts.cm_signed_pedestals(ped) is None
