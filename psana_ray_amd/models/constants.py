"""Per-run calibration constants (pedestals, gains, status, gain configuration).

psana reads these from its calibration database for ``(exp, run, detector)``; psana-ray reaches
them only implicitly through ``iter_events(mode)`` (psana_ray/producer.py:88) and
``create_bad_pixel_mask()`` (:81).  Offline there is no calibration DB, so constants are
random-initialised with physically plausible magnitudes (BASELINE.json: "random-init calibration
constants"), deterministically from a seed derived from ``(exp, run, detector)``.

``device_tables`` packs them into the kernel layout: per candidate gain table ``c`` and pixel
``p`` -> pedestal ``ped[c, p]`` and gain factor ``gf[c, p] = mask[p] / gain[g(c, p)]``, plus a
per-pixel flag byte (bit0 output mask, bit1+c common-mode eligible for candidate c).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from .detector import EPIX_CAND_A, EPIX_CAND_B, DetectorSpec

# nominal gains (ADU per keV) and pedestal levels (ADU); domain values, not psana facts
_EPIX_GAIN = (16.4, 5.47, 0.164, 16.4, 5.47, 0.164, 0.164)
_EPIX_PED = (2500.0, 2500.0, 1800.0, 2500.0, 2500.0, 1800.0, 1800.0)
_JF_GAIN = (41.0, -1.5, -0.11)
_JF_PED = (3000.0, 14500.0, 15000.0)
# default common-mode gain set: high / medium gains (epix: FH, FM, AHL-H, AML-M; jungfrau: G0)
EPIX_CM_GAINS = (0, 1, 3, 4)
JUNGFRAU_CM_GAINS = (0,)


def run_seed(exp: str, run: int, detector: str) -> int:
    h = hashlib.sha256(f"{exp}/{run}/{detector}".encode()).digest()
    return int.from_bytes(h[:4], "little")


@dataclass
class CalibConstants:
    spec: DetectorSpec
    pedestals: np.ndarray           # [G, P, H, W] float32
    gains: np.ndarray               # [G, P, H, W] float32 (ADU / keV)
    status: np.ndarray              # [P, H, W] uint8, nonzero = bad pixel
    gain_config: Optional[np.ndarray] = None   # epix: [P, H, W] uint8 in 0..4 (FH FM FL AHL AML)
    cm_gains: Sequence[int] = field(default_factory=tuple)

    @classmethod
    def random(cls, spec: DetectorSpec, seed: int = 0, bad_fraction: float = 0.005,
               gain_config: str = "AHL") -> "CalibConstants":
        """Random-init constants.  ``gain_config``: one of FH FM FL AHL AML or ``"mixed"``."""
        rng = np.random.default_rng(seed)
        shape = spec.frame_shape
        G = spec.n_gains
        if spec.kind == "epix10ka":
            gain0, ped0, cmg = _EPIX_GAIN, _EPIX_PED, EPIX_CM_GAINS
            ped_sd = 150.0
        elif spec.kind == "jungfrau":
            gain0, ped0, cmg = _JF_GAIN, _JF_PED, JUNGFRAU_CM_GAINS
            ped_sd = 200.0
        else:
            gain0, ped0, cmg = (1.0,), (100.0,), (0,)
            ped_sd = 5.0
        ped = np.empty((G, *shape), np.float32)
        gains = np.empty((G, *shape), np.float32)
        for g in range(G):
            ped[g] = (ped0[g] + ped_sd * rng.standard_normal(shape)).astype(np.float32)
            gains[g] = (gain0[g] * (1.0 + 0.03 * rng.standard_normal(shape))).astype(np.float32)
        status = (rng.random(shape) < bad_fraction).astype(np.uint8)
        cfg = None
        if spec.kind == "epix10ka":
            names = ("FH", "FM", "FL", "AHL", "AML")
            if gain_config == "mixed":
                cfg = rng.integers(0, 5, size=shape, dtype=np.uint8)
            else:
                cfg = np.full(shape, names.index(gain_config), np.uint8)
        return cls(spec, ped, gains, status, cfg, tuple(cmg))

    def panel_subset(self, lo: int, hi: int) -> "CalibConstants":
        """Constants of panels ``[lo, hi)`` (views; a panel shard of the frame, SURVEY P-04)."""
        spec = self.spec.panel_subset(lo, hi)
        if spec is self.spec:
            return self
        return CalibConstants(spec, self.pedestals[:, lo:hi], self.gains[:, lo:hi], self.status[lo:hi],
                              None if self.gain_config is None else self.gain_config[lo:hi], tuple(self.cm_gains))

    # ------------------------------------------------------------------------------------
    def create_bad_pixel_mask(self) -> np.ndarray:
        """psana_wrapper.create_bad_pixel_mask() equivalent (producer.py:81): truthy = good."""
        return (self.status == 0).astype(np.uint8)

    def candidate_gain_index(self) -> np.ndarray:
        """[NC, P, H, W] gain-range index of each kernel candidate table."""
        s = self.spec
        if s.kind == "epix10ka":
            a = np.asarray(EPIX_CAND_A, np.int64)[self.gain_config]
            b = np.asarray(EPIX_CAND_B, np.int64)[self.gain_config]
            return np.stack([a, b])
        if s.kind == "jungfrau":
            return np.stack([np.full(s.frame_shape, g, np.int64) for g in range(3)])
        return np.zeros((1, *s.frame_shape), np.int64)

    def device_tables(self, mask: Optional[np.ndarray] = None):
        """Kernel tables: ``ped [NC, npix]``, ``gf [NC, npix]`` (mask folded) and the common-mode
        eligibility bit-planes ``elig [npix / 8, S]`` (uint8, S = 1, 2 or 4 for 1, 2 or 3 candidate
        tables): bit j of byte k of group g is set when pixel 8g + j is CM-eligible (status good,
        gain in the CM set; the output mask does not enter) if it decodes to candidate k
        (csrc/common_mode.hip cm_decode8).

        ``mask`` is the combined output mask (bad-pixel & manual, truthy = keep) in frame shape;
        None keeps every pixel (the reference applies masks only when asked, producer.py:92-95).
        """
        s = self.spec
        cand = self.candidate_gain_index()                     # [NC, P, H, W]
        ped = np.take_along_axis(self.pedestals, cand, axis=0)  # [NC, P, H, W]
        gain = np.take_along_axis(self.gains, cand, axis=0)
        keep = np.ones(s.frame_shape, bool) if mask is None else np.asarray(mask).astype(bool)
        keep = np.broadcast_to(keep, s.frame_shape)
        gf = np.where(keep[None], np.float32(1.0) / gain, np.float32(0.0)).astype(np.float32)
        status_good = self.status == 0
        cm_set = np.zeros(max(s.n_gains, 1), bool)
        cm_set[list(self.cm_gains)] = True
        npix = s.npix
        if npix % 8:
            raise ValueError("common-mode tables need a multiple of 8 pixels per frame")
        nc = cand.shape[0]
        stride = {1: 1, 2: 2, 3: 4}[nc]
        planes = np.zeros((npix // 8, stride), np.uint8)
        weights = (1 << np.arange(8)).astype(np.uint16)
        for c in range(nc):
            # common-mode eligibility ignores the output mask: the reference applies masks to psana's
            # calibrated frames afterwards (producer.py:92-95), so they never change the median
            elig = (status_good & cm_set[cand[c]]).reshape(npix // 8, 8)
            planes[:, c] = (elig.astype(np.uint16) * weights).sum(axis=1).astype(np.uint8)
        return (np.ascontiguousarray(ped.reshape(-1, npix)),
                np.ascontiguousarray(gf.reshape(-1, npix)),
                np.ascontiguousarray(planes.reshape(-1)))

    def cm_eligibility(self) -> np.ndarray:
        """[NC, npix] bool: pixel p is common-mode eligible when it decodes to candidate c (status
        good and the candidate's gain range in the CM set) -- the bits of ``device_tables``' planes."""
        s = self.spec
        cand = self.candidate_gain_index()
        cm_set = np.zeros(max(s.n_gains, 1), bool)
        cm_set[list(self.cm_gains)] = True
        return (((self.status == 0)[None] & cm_set[cand])).reshape(cand.shape[0], s.npix)

    def cm_signed_pedestals(self, ped: np.ndarray) -> Optional[np.ndarray]:
        """The common-mode kernel's pedestal tables with the eligibility in the sign bits: ``ped[c, p]``
        where pixel p is eligible for candidate c, ``-ped[c, p]`` elsewhere (csrc/common_mode.hip
        cm_decode8 SG: v = ADU - |p|, eligible = sign clear).  ``ped`` is ``device_tables``' [NC,
        npix] table.  -0.0 pedestals become +0.0 first (ADU - 0 is the same either way); None when a
        pedestal is negative or NaN, which the sign cannot carry (the kernel then loads bit-planes)."""
        p = np.asarray(ped, np.float32)
        if not np.all(p >= 0):          # also catches NaN
            return None
        p = np.where(p == 0, np.float32(0.0), p).astype(np.float32)   # -0.0 -> +0.0
        sg = np.where(self.cm_eligibility(), p, -p).astype(np.float32)
        return np.ascontiguousarray(sg)
