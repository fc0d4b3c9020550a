"""Stub of the external ``psana_wrapper`` package (SURVEY E-01), for tests only.

It has the surface psana-ray uses -- ``PsanaWrapperSmd(exp, run, detector_name)``,
``.iter_events(mode)`` -> ``(data, photon_energy)``, ``.create_bad_pixel_mask()`` and
``ImageRetrievalMode`` (psana_ray/producer.py:11,81,88,150-159) -- plus the adapter hook
``calib_constants()`` (psana_ray_amd/source/psana_adapter.py).  Behind it sits the framework's
synthetic detector; "psana's" calibrated / image frames are the fp32 golden model of the same raw
frames, so a test can compare what reaches a consumer with what this stub says psana produces.

Knobs (environment):
  PSANA_STUB_RAW=0        no ImageRetrievalMode.raw / no calib_constants() / no detector handle
                          (psana-calibrated path)
  PSANA_STUB_STYLE=...    how raw frames and constants can be reached (the adapter's probes):
                          hook (default): ImageRetrievalMode.raw + the calib_constants() hook;
                          psana2: ImageRetrievalMode.raw, constants only on a psana2-style detector
                            handle ``wrapper.det`` (det.raw._pedestals() / _gain() / per-gain
                            _status() / _pixel_coord_indexes());
                          psana2_events: no raw retrieval mode at all -- raw frames through
                            ``wrapper.det.raw.raw(evt)`` over ``wrapper.run.events()``, photon
                            energy from ``wrapper.get_photon_energy(evt)``;
                          psana1: no raw retrieval mode; a psana1-style handle ``wrapper.detector``
                            (detector.raw(evt), pedestals(run), gain(run), status(run)) over
                            ``wrapper.ds.events()``
  PSANA_STUB_EVENTS=N     events in the run (default 24)
  PSANA_STUB_GAINCFG=...  the ePix10ka per-pixel gain configuration (AHL default, "mixed": random
                          FH/FM/FL/AHL/AML per pixel)
  PSANA_STUB_NO_GAINCFG=1 the detector handles expose no gain-configuration accessor
  PSANA_STUB_HANDLE_SHARDED=1  the handle styles' run / DataSource event loop yields only this
                          rank's events (default: every event of the run -- the loop bypasses the
                          wrapper's SMD sharding, so the adapter shards it explicitly)
  PSANA_STUB_CM=text      common mode "psana" applies (default: "default"; "off" disables)
SMD sharding: the rank / size come from the same launcher variables the producer reads, and rank
r yields global events r, r + size, ... (psana's SMD mode distributes events over MPI ranks).
"""
from __future__ import annotations

import enum
import os

import numpy as np

RAW_OK = os.environ.get("PSANA_STUB_RAW", "1") != "0"
STYLE = os.environ.get("PSANA_STUB_STYLE", "hook") if RAW_OK else "none"

if STYLE in ("hook", "psana2"):
    class ImageRetrievalMode(enum.Enum):
        raw = "raw"
        calib = "calib"
        image = "image"
else:
    class ImageRetrievalMode(enum.Enum):
        calib = "calib"
        image = "image"


def _rank_size():
    from psana_ray_amd.parallel.launch import detect

    li = detect()
    return li.rank, li.size


class PsanaWrapperSmd:
    def __init__(self, exp, run, detector_name):
        from psana_ray_amd.source.synthetic import SyntheticRun

        self.exp, self.run, self.detector_name = exp, int(run), detector_name
        self.runnum = int(run)
        self.rank, self.size = _rank_size()
        self.n_events = int(os.environ.get("PSANA_STUB_EVENTS", "24"))
        # one generator for the whole run (seeded by exp/run), sharded like SMD mode
        self._syn = SyntheticRun(exp, run, detector_name, rank=0, size=1, pool_frames=8, gen_device="cpu",
                                 gain_config=os.environ.get("PSANA_STUB_GAINCFG", "AHL"))
        self.consts = self._syn.consts
        if STYLE in ("psana2", "psana2_events"):
            self.det = _Psana2Det(self)
        if STYLE == "psana2_events":
            self.run_obj = _Run(self)
            self.run = self.run_obj          # psana2: the wrapper holds the run (``run.events()``)
        if STYLE == "psana1":
            self.detector = _Psana1Det(self)
            self.ds = _Run(self)             # psana1: the DataSource (``ds.events()``)

    def get_photon_energy(self, evt):
        return self.photon_energy(evt.gevt)

    # ---- reference surface -------------------------------------------------------------------
    def create_bad_pixel_mask(self):
        return self.consts.create_bad_pixel_mask()

    def raw_frame(self, gevt: int) -> np.ndarray:
        return self._syn.pool[gevt % self._syn.pool_frames]

    def photon_energy(self, gevt: int):
        return None if gevt % 5 == 4 else float(self._syn.pool_pe[gevt % self._syn.pool_frames])

    def local_events(self):
        return range(self.rank, self.n_events, self.size)

    def iter_events(self, mode):
        name = mode.value if hasattr(mode, "value") else str(mode)
        for g in self.local_events():
            if name == "raw":
                yield self.raw_frame(g).copy(), self.photon_energy(g)
            else:
                yield expected_frame(self, g, name), self.photon_energy(g)

    # ---- adapter hook: the run's calibration constants ---------------------------------------
    if STYLE == "hook":
        def calib_constants(self):
            c = self.consts
            return {"pedestals": c.pedestals, "gains": c.gains, "status": c.status, "gain_config": c.gain_config}


class _Evt:
    def __init__(self, gevt):
        self.gevt = gevt


class _Run:
    """psana2 run / psana1 DataSource: this rank's events (SMD sharding)."""

    def __init__(self, w):
        self._w = w

    def events(self):
        sharded = os.environ.get("PSANA_STUB_HANDLE_SHARDED", "0") == "1"
        for g in (self._w.local_events() if sharded else range(self._w.n_events)):
            yield _Evt(g)


class _Psana2Raw:
    """psana2 ``det.raw``: raw(evt) and the run's constants (per gain mode, as psana2 keeps them)."""

    def __init__(self, w):
        self._w = w

    def raw(self, evt):
        return self._w.raw_frame(evt.gevt).copy()

    def _pedestals(self):
        return self._w.consts.pedestals

    def _gain(self):
        return self._w.consts.gains

    def _status(self):
        st = self._w.consts.status
        return np.broadcast_to(st, (self._w.consts.pedestals.shape[0], *st.shape)).copy()

    if os.environ.get("PSANA_STUB_NO_GAINCFG", "0") != "1":
        def _gain_config(self):
            return self._w.consts.gain_config

    def _pixel_coord_indexes(self):
        from psana_ray_amd.models.geometry import make_geometry

        g = make_geometry(self._w.consts.spec)
        return g.rows, g.cols


class _Psana2Det:
    def __init__(self, w):
        self.raw = _Psana2Raw(w)


class _Psana1Det:
    """psana1 ``Detector``: raw(evt) and constants that take the run number."""

    def __init__(self, w):
        self._w = w

    def raw(self, evt):
        return self._w.raw_frame(evt.gevt).copy()

    def pedestals(self, run):
        assert run == self._w.runnum, "psana1 constants are looked up by run number"
        return self._w.consts.pedestals

    def gain(self, run):
        return self._w.consts.gains

    def status(self, run):
        return self._w.consts.status

    if os.environ.get("PSANA_STUB_NO_GAINCFG", "0") != "1":
        def gain_config(self, run):
            return self._w.consts.gain_config


def stub_common_mode():
    from psana_ray_amd.config import CommonModeParams

    return CommonModeParams.parse(os.environ.get("PSANA_STUB_CM", "default"))


def expected_frame(w: PsanaWrapperSmd, gevt: int, mode: str, mask=None) -> np.ndarray:
    """What "psana" returns for event ``gevt`` in ``mode`` (calib: (P, H, W); image: 2-D), with an
    optional output mask applied like the reference (np.where(mask, data, 0), producer.py:92-95)."""
    import torch

    from psana_ray_amd.models.calibrator import Calibrator
    from psana_ray_amd.models.detector import Mode

    cm = stub_common_mode()
    if cm is not None and cm.bank_cols is None:
        cm.bank_cols = w.consts.spec.bank_cols
    cal = Calibrator(w.consts, "cpu", Mode(mode), mask=mask, common_mode=cm)
    out = cal(torch.from_numpy(w.raw_frame(gevt).astype(np.int32)).to(torch.uint16)[None])[0].numpy()
    return out[0] if mode == "image" else out
