"""Synthetic detector event source (stands in for psana_wrapper.PsanaWrapperSmd, E-01).

The reference iterates ``PsanaWrapperSmd(exp, run, detector_name).iter_events(mode)`` ->
``(data, photon_energy)`` (psana_ray/producer.py:88,150-154) and builds a bad-pixel mask with
``create_bad_pixel_mask()`` (:81).  Offline there is no psana / XTC2 data, so this source
produces raw detector frames with realistic structure:

* per-pixel pedestals and gains from :class:`CalibConstants` (random-init, seeded by run),
* Bragg-like spots (Gaussian, log-normal amplitudes) on a diffuse Poisson background,
* per-event common-mode offsets (per ASIC row-bank and per column) and read noise,
* gain switching (epix10ka auto-ranging bit 14, Jungfrau G0/G1/G2 bits) for bright pixels,
* a per-event photon energy (None-able).

Raw frames are generated ONCE into a pool (pinned host memory for GPU pipelines) and cycled
(SURVEY H-5: the host cannot generate 10^4 frames/s).  Events are sharded over producer ranks
round-robin: global event ``g`` belongs to rank ``g % size`` (P-01).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Iterator, List, Optional

import numpy as np
import torch

from ..models.constants import CalibConstants, run_seed
from ..models.detector import DetectorSpec, Mode, get_detector


@dataclass
class RawEvent:
    gevt: int              # global event id
    idx: int               # rank-local index (the reference's idx, producer.py:88)
    raw: np.ndarray        # uint16 frame-shaped view (pinned host memory when staged)
    host_ptr: int          # address of raw (for hipMemcpyAsync)
    photon_energy: Optional[float]


def generate_raw(consts: CalibConstants, n: int, seed: int, device="cpu", spots=(30, 80),
                 cm_sigma=6.0, noise_sigma=3.0, bkg_photons=0.02):
    """n raw frames [n, P, H, W] uint16 plus photon energies [n] (eV)."""
    spec = consts.spec
    g = torch.Generator(device=device).manual_seed(seed)
    P, H, W = spec.frame_shape
    dev = torch.device(device)
    pe_ev = 9500.0 + 50.0 * torch.randn(n, generator=g, device=dev)
    out = torch.empty((n, P, H, W), dtype=torch.int32, device=dev)
    ped = torch.as_tensor(consts.pedestals, device=dev)
    gain = torch.as_tensor(consts.gains, device=dev)
    cfg = None if consts.gain_config is None else torch.as_tensor(consts.gain_config.astype(np.int64), device=dev)
    R, C, L = spec.asic_rows, spec.asic_cols, spec.bank_cols
    for i in range(n):
        e_kev = float(pe_ev[i]) / 1000.0
        lam = torch.full((P, H, W), bkg_photons, device=dev)
        photons = torch.poisson(lam, generator=g)
        ns = int(torch.randint(spots[0], spots[1] + 1, (1,), generator=g, device=dev))
        if ns > 0:
            pp = torch.randint(0, P, (ns,), generator=g, device=dev)
            rr = torch.randint(2, max(3, H - 2), (ns,), generator=g, device=dev)
            cc = torch.randint(2, max(3, W - 2), (ns,), generator=g, device=dev)
            amp = torch.exp(torch.randn(ns, generator=g, device=dev) * 1.2 + math.log(60.0))
            sig = 0.7 + 0.5 * torch.rand(ns, generator=g, device=dev)
            dy, dx = torch.meshgrid(torch.arange(-2, 3, device=dev), torch.arange(-2, 3, device=dev), indexing="ij")
            wgt = torch.exp(-(dy[None] ** 2 + dx[None] ** 2) / (2 * sig[:, None, None] ** 2))
            wgt = wgt / wgt.sum(dim=(1, 2), keepdim=True) * amp[:, None, None]
            r_idx = (rr[:, None, None] + dy[None]).clamp(0, H - 1)
            c_idx = (cc[:, None, None] + dx[None]).clamp(0, W - 1)
            p_idx = pp[:, None, None].expand_as(r_idx)
            photons.index_put_((p_idx.reshape(-1), r_idx.reshape(-1), c_idx.reshape(-1)),
                               torch.round(wgt).reshape(-1), accumulate=True)
        sig_kev = photons * e_kev
        noise = noise_sigma * torch.randn((P, H, W), generator=g, device=dev)
        cm_rows = cm_sigma * torch.randn((P, H, W // L), generator=g, device=dev)
        cm_cols = 0.5 * cm_sigma * torch.randn((P, 1, W), generator=g, device=dev)
        cm = cm_rows.repeat_interleave(L, dim=2) + cm_cols
        if spec.kind == "epix10ka":
            ga = torch.as_tensor((0, 1, 2, 3, 4), device=dev)[cfg]
            gb = torch.as_tensor((0, 1, 2, 5, 6), device=dev)[cfg]
            adu_a = torch.gather(ped, 0, ga[None]).squeeze(0) + sig_kev * torch.gather(gain, 0, ga[None]).squeeze(0)
            adu_b = torch.gather(ped, 0, gb[None]).squeeze(0) + sig_kev * torch.gather(gain, 0, gb[None]).squeeze(0)
            switch = (cfg >= 3) & (adu_a > 12000.0)
            adu = torch.where(switch, adu_b, adu_a + cm) + noise
            adu = adu.round().clamp(0, 16383).to(torch.int32)
            out[i] = adu | (switch.to(torch.int32) << 14)
        elif spec.kind == "jungfrau":
            a0 = ped[0] + sig_kev * gain[0]
            a1 = ped[1] + sig_kev * gain[1]
            a2 = ped[2] + sig_kev * gain[2]
            use1 = a0 > 15000.0
            use2 = use1 & (a1 < 1000.0)
            adu = torch.where(use2, a2, torch.where(use1, a1, a0)) + noise
            adu = adu.round().clamp(0, 16383).to(torch.int32)
            gbits = torch.where(use2, torch.full_like(adu, 3), use1.to(torch.int32))
            out[i] = adu | (gbits << 14)
        else:
            adu = ped[0] + sig_kev * gain[0] + cm + noise
            out[i] = adu.round().clamp(0, 65535).to(torch.int32)
    return out.to(torch.int32).cpu().numpy().astype(np.uint16), (pe_ev.cpu().numpy()).astype(np.float64)


def first_local_event(start_event: int, rank: int, size: int) -> int:
    """First rank-local index k with global id ``rank + k * size >= start_event`` (round-robin
    sharding, P-01)."""
    return max(0, -(-(int(start_event) - rank) // size))


class SyntheticRun:
    """psana_wrapper-like source for ``(exp, run, detector_name)`` (``--exp synthetic`` or no psana)."""

    def __init__(self, exp: str, run: int, detector_name: str, rank: int = 0, size: int = 1,
                 n_events: Optional[int] = None, pool_frames: int = 32, seed: Optional[int] = None,
                 gain_config: str = "AHL", pinned: bool = False, gen_device: Optional[str] = None,
                 photon_energy_none: bool = False):
        self.exp, self.run, self.detector_name = exp, run, detector_name
        self.spec: DetectorSpec = get_detector(detector_name)
        self.rank, self.size = rank, size
        self.n_events = n_events
        base = run_seed(exp, run, self.spec.name) if seed is None else seed
        self.consts = CalibConstants.random(self.spec, seed=base, gain_config=gain_config)
        if gen_device is None:
            gen_device = "cuda" if torch.cuda.is_available() else "cpu"
        frames, pe = generate_raw(self.consts, pool_frames, seed=base + 1 + rank, device=gen_device)
        self.pool_frames = pool_frames
        self._pinned = None
        if pinned:
            from ..ops import _ext

            C = _ext.load()
            self._pinned = C.PinnedBuffer(frames.nbytes)
            self.pool = np.frombuffer(self._pinned, dtype=np.uint16).reshape(frames.shape)
            self.pool[...] = frames
        else:
            self.pool = frames
        self.pool_pe = pe  # eV, like psana's beam-energy detector
        self.photon_energy_none = photon_energy_none
        self._cursor = 0

    # ---- reference surface -------------------------------------------------------------
    def create_bad_pixel_mask(self) -> np.ndarray:
        return self.consts.create_bad_pixel_mask()

    def n_local_events(self) -> Optional[int]:
        if self.n_events is None:
            return None
        return max(0, (self.n_events - self.rank + self.size - 1) // self.size)

    def seek(self, start_event: int) -> int:
        """Resume at global event ``start_event``: this rank's next event is its first one with
        ``gevt >= start_event``.  Returns that rank-local index."""
        self._cursor = first_local_event(start_event, self.rank, self.size)
        return self._cursor

    @property
    def cursor(self) -> int:
        return self._cursor

    def cycled_frames(self):
        """(host pointers, photon energies) of the cycled pool for the native producer engine:
        rank-local event k reads pool[k % pool_frames] (the same mapping as ``next_events``)."""
        pe = [None if self.photon_energy_none else float(v) for v in self.pool_pe]
        return [int(self.pool[j].ctypes.data) for j in range(self.pool_frames)], pe

    def next_events(self, n: int) -> List[RawEvent]:
        """Up to n raw events of this rank's shard (fewer at the end of a finite run)."""
        evs: List[RawEvent] = []
        lim = self.n_local_events()
        for _ in range(n):
            k = self._cursor
            if lim is not None and k >= lim:
                break
            j = k % self.pool_frames
            raw = self.pool[j]
            pe = None if self.photon_energy_none else float(self.pool_pe[j])
            evs.append(RawEvent(self.rank + k * self.size, k, raw, raw.ctypes.data, pe))
            self._cursor += 1
        return evs

    def iter_raw(self) -> Iterator[RawEvent]:
        while True:
            evs = self.next_events(1)
            if not evs:
                return
            yield evs[0]

    def iter_events(self, mode=Mode.calib):
        """Reference-compatible CPU iterator: ``(data ndarray, photon_energy)`` per event,
        calibrated with the fp32 golden model (no GPU; psana_wrapper semantics)."""
        from ..models.calibrator import Calibrator

        mode = Mode(mode.value if hasattr(mode, "value") else mode)
        cal = Calibrator(self.consts, "cpu", mode)
        for ev in self.iter_raw():
            out = cal(torch.from_numpy(ev.raw.astype(np.int32)).to(torch.uint16)[None])[0].numpy()
            if mode == Mode.image:
                out = out[0]   # psana image mode returns 2-D (the reference re-adds the axis)
            yield out, ev.photon_energy
