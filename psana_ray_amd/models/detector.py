"""Detector models: geometry/gain-family descriptions of the detectors psana-ray streams.

The reference streams whatever ``psana_wrapper.PsanaWrapperSmd(exp, run, detector_name)``
yields (psana_ray/producer.py:150-154); its README example is ``--detector_name epix10k2M``
(README.md:20).  Frames are ``(panels, H, W)`` in calib mode and ``(H, W)`` -> ``(1, H, W)`` in
image mode (producer.py:96-97).  These specs carry the shapes and gain families the HIP kernels
need (documented domain knowledge, parameters not verified facts).
"""
from __future__ import annotations

import enum
from dataclasses import dataclass
from typing import Dict


class Mode(enum.Enum):
    """psana_wrapper.ImageRetrievalMode equivalent (E-02): raw, calib, image."""

    raw = "raw"
    calib = "calib"
    image = "image"


ImageRetrievalMode = Mode  # reference spelling (psana_ray/producer.py:11,156-159)


# epix10ka gain-range indices (psana order): FH, FM, FL, AHL-H, AML-M, AHL-L, AML-L
EPIX_GAIN_NAMES = ("FH", "FM", "FL", "AHL_H", "AML_M", "AHL_L", "AML_L")
# per-pixel gain configuration (from detector config bits) -> candidate gain index for
# data bit 14 == 0 / == 1
EPIX_CONFIG_NAMES = ("FH", "FM", "FL", "AHL", "AML")
EPIX_CAND_A = (0, 1, 2, 3, 4)
EPIX_CAND_B = (0, 1, 2, 5, 6)
JUNGFRAU_GAIN_NAMES = ("G0", "G1", "G2")


@dataclass(frozen=True)
class DetectorSpec:
    name: str
    kind: str            # "epix10ka" | "jungfrau" | "plain"
    n_panels: int
    panel_rows: int
    panel_cols: int
    asic_rows: int
    asic_cols: int
    bank_cols: int       # common-mode bank width (epix10ka: 384 / 8 = 48)
    pixel_size_um: float
    panel_gap_px: int = 10

    @property
    def n_gains(self) -> int:
        return {"epix10ka": 7, "jungfrau": 3, "plain": 1}[self.kind]

    @property
    def n_candidates(self) -> int:
        """Gain tables the kernels see per pixel (epix: bit14 pair, jungfrau: G0/G1/G2)."""
        return {"epix10ka": 2, "jungfrau": 3, "plain": 1}[self.kind]

    @property
    def kernel_kind(self) -> int:
        return {"epix10ka": 0, "jungfrau": 1, "plain": 2}[self.kind]

    @property
    def frame_shape(self):
        return (self.n_panels, self.panel_rows, self.panel_cols)

    @property
    def npix(self) -> int:
        return self.n_panels * self.panel_rows * self.panel_cols

    @property
    def raw_frame_bytes(self) -> int:
        return self.npix * 2

    @property
    def calib_frame_bytes(self) -> int:
        return self.npix * 4

    @property
    def n_asics(self) -> int:
        return self.n_panels * (self.panel_rows // self.asic_rows) * (self.panel_cols // self.asic_cols)

    @property
    def panel_pixels(self) -> int:
        return self.panel_rows * self.panel_cols

    def panel_subset(self, lo: int, hi: int) -> "DetectorSpec":
        """The detector made of panels ``[lo, hi)``: same ASIC/bank geometry and gain family, so
        every per-ASIC kernel (calibration, common mode) runs unchanged on a panel shard."""
        if not 0 <= lo < hi <= self.n_panels:
            raise ValueError(f"panel range [{lo}, {hi}) outside the {self.n_panels} panels of {self.name}")
        if (lo, hi) == (0, self.n_panels):
            return self
        return DetectorSpec(f"{self.name}[{lo}:{hi}]", self.kind, hi - lo, self.panel_rows, self.panel_cols,
                            self.asic_rows, self.asic_cols, self.bank_cols, self.pixel_size_um, self.panel_gap_px)


def panel_shard_range(n_panels: int, shard: int, n_shards: int):
    """Panels ``[lo, hi)`` of shard ``shard`` when a frame is split over ``n_shards`` ranks.  Shards
    are equal (the queue carries one frame shape per session), so ``n_shards`` must divide the
    panel count."""
    if n_shards < 1 or n_panels % n_shards:
        raise ValueError(f"--panel_shards {n_shards} must divide the detector's {n_panels} panels")
    if not 0 <= shard < n_shards:
        raise ValueError(f"panel shard {shard} outside [0, {n_shards})")
    per = n_panels // n_shards
    return shard * per, (shard + 1) * per


_REGISTRY: Dict[str, DetectorSpec] = {}


def register(spec: DetectorSpec, *aliases: str) -> DetectorSpec:
    for key in (spec.name, *aliases):
        _REGISTRY[key.lower()] = spec
    return spec


EPIX10K2M = register(
    DetectorSpec("epix10k2M", "epix10ka", 16, 352, 384, 176, 192, 48, 100.0),
    "epix10ka2m", "epix10k2m", "epix10ka_2m")
EPIX10KA = register(DetectorSpec("epix10ka", "epix10ka", 1, 352, 384, 176, 192, 48, 100.0), "epix10ka_1panel")
JUNGFRAU16M = register(DetectorSpec("jungfrau16M", "jungfrau", 32, 512, 1024, 256, 256, 64, 75.0), "jungfrau16m")
JUNGFRAU4M = register(DetectorSpec("jungfrau4M", "jungfrau", 8, 512, 1024, 256, 256, 64, 75.0), "jungfrau4m")
JUNGFRAU05M = register(DetectorSpec("jungfrau05M", "jungfrau", 1, 512, 1024, 256, 256, 64, 75.0), "jungfrau05m")
# BASELINE config 1: synthetic 256x256 float-like frames without gain switching
PLAIN256 = register(DetectorSpec("plain256", "plain", 1, 256, 256, 128, 128, 32, 100.0), "synthetic256")
# small detectors for CPU tests (same kernels, same code paths)
TINY_EPIX = register(DetectorSpec("tiny_epix", "epix10ka", 2, 32, 48, 16, 24, 8, 100.0, panel_gap_px=2))
TINY_JUNGFRAU = register(DetectorSpec("tiny_jungfrau", "jungfrau", 2, 16, 32, 8, 16, 8, 75.0, panel_gap_px=2))
TINY_PLAIN = register(DetectorSpec("tiny_plain", "plain", 1, 16, 16, 8, 8, 8, 100.0, panel_gap_px=2))
# image frames of 9 x 17 pixels = 612 B, not a multiple of 16 B (like the psana raw path's
# pix_rows.max() + 1 geometries): ring slots are padded to 256 B (queue/ring.py SLOT_ALIGN)
TINY_ODD = register(DetectorSpec("tiny_odd", "plain", 2, 9, 8, 9, 8, 8, 100.0, panel_gap_px=1))


def get_detector(name: str) -> DetectorSpec:
    try:
        return _REGISTRY[name.lower()]
    except KeyError:
        raise KeyError(f"unknown detector {name!r}; known: {sorted(set(s.name for s in _REGISTRY.values()))}")


def list_detectors():
    return sorted(set(s.name for s in _REGISTRY.values()))
