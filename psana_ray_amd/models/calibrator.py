"""The calibration "model": raw detector frames -> frames in the requested retrieval mode.

This is the work psana does inside ``PsanaWrapperSmd.iter_events(mode)`` for psana-ray
(psana_ray/producer.py:88, mode from ``--calib`` at :156-159) plus the reference's own masking
(:92-95) and ndim fix-up (:96-97), re-designed as gfx950 kernels writing straight into the
destination buffers (HBM ring slots):

  mode=raw    raw u16 frames, untouched                         -> (P, H, W) uint16
  mode=calib  K-01..K-04 (+K-03 common mode if enabled)         -> (P, H, W) float32
  mode=image  the above + K-05 geometry assembly                -> (1, Himg, Wimg) float32

On a CUDA(HIP) device the HIP kernels are mandatory (no silent PyTorch fallback); on
``device="cpu"`` the fp32 golden model (ops.reference) is the explicit compute path.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import config
from ..config import CommonModeParams
from ..ops import kernels, reference
from .constants import CalibConstants
from .detector import Mode
from .geometry import Geometry, build_tile_map, make_geometry


class Calibrator:
    def __init__(self, consts: CalibConstants, device, mode: Mode = Mode.calib,
                 mask: Optional[np.ndarray] = None, common_mode: Optional[CommonModeParams] = None,
                 geometry: Optional[Geometry] = None):
        self.consts = consts
        self.spec = consts.spec
        self.device = torch.device(device)
        self.mode = Mode(mode) if not isinstance(mode, Mode) else mode
        self.cm = common_mode
        if self.cm is not None and self.cm.bank_cols is None:
            self.cm = CommonModeParams(self.cm.flags, self.cm.thr, self.cm.maxcorr, self.cm.npix_min,
                                       self.spec.bank_cols)
        spec = self.spec
        # masks: frame-shaped masks fold into the tables; image-shaped ones apply at assembly
        self.geometry = geometry
        frame_mask, image_mask = None, None
        if mask is not None:
            m = np.asarray(mask)
            if m.size == spec.npix:
                frame_mask = m.reshape(spec.frame_shape).astype(bool)
            else:
                if self.mode != Mode.image:
                    raise ValueError(f"mask of shape {m.shape} does not match frame shape {spec.frame_shape}")
                image_mask = m
        self.frame_mask = frame_mask
        if self.mode == Mode.image:
            self.geometry = geometry or make_geometry(spec)
            if image_mask is not None and image_mask.size != int(np.prod(self.geometry.image_shape)):
                raise ValueError(f"image mask of shape {image_mask.shape} does not match image {self.geometry.image_shape}")
        self.image_mask = image_mask

        self._gpu = self.device.type == "cuda"
        ped, gf, elig = consts.device_tables(frame_mask)
        self.plan = None
        if self._gpu:
            C = kernels._ext.load()  # fail loudly on a GPU box without the extension
            self.ped = torch.from_numpy(ped).to(self.device)
            self.gf = torch.from_numpy(gf).to(self.device)
            self.elig = torch.from_numpy(elig).to(self.device)
            # pedestals carrying the CM eligibility in their sign bits (None: some pedestal < 0), for
            # the production kernels that read them (the launcher's predicate, _C.cm_signed_shape)
            self.ped_sg = None
            sg_shape = self.cm is not None and bool(C.cm_signed_shape(spec.kernel_kind, spec.asic_rows, spec.asic_cols,
                                                                      int(self.cm.bank_cols)))
            if common_mode is not None and config.CM_SIGNED_PEDESTALS and sg_shape:
                sg = consts.cm_signed_pedestals(ped)
                if sg is not None:
                    self.ped_sg = torch.from_numpy(sg).to(self.device)
            self.idx = None
            self.omask = None
            self.tile_map = None
            if self.mode == Mode.image:
                imap = self.geometry.index_map()
                self.idx = torch.from_numpy(imap).to(self.device)
                kernels._validate_index_map(self.idx, spec.npix, "Calibrator")
                # LDS-tiled assembly (csrc/image.hip); the image mask folds into its codes
                tm = build_tile_map(imap, spec, self.geometry.image_shape, image_mask)
                self.tile_map = tm
                self._tiles = torch.from_numpy(tm.tiles).to(self.device)
                self._codes = torch.from_numpy(tm.codes).to(self.device)
                self.omask = None if image_mask is None else \
                    torch.from_numpy(np.asarray(image_mask).astype(np.uint8).ravel()).to(self.device)
            if self.cm is not None:
                if C.cm_tile_cols(spec.asic_rows, spec.asic_cols, int(self.cm.bank_cols), 0, spec.kernel_kind) == 0:
                    raise ValueError(f"common mode: no full-height stripe of the {spec.asic_rows}x{spec.asic_cols} "
                                     f"ASIC (bank {self.cm.bank_cols}) fits in 160 KiB of LDS")
            self.plan = self._make_plan(C)
        self._out_frame_bytes = self.out_frame_bytes

    # ------------------------------------------------------------------------------------
    @property
    def out_shape(self):
        if self.mode == Mode.image:
            return (1, *self.geometry.image_shape)
        return self.spec.frame_shape

    @property
    def out_dtype(self):
        return torch.uint16 if self.mode == Mode.raw else torch.float32

    @property
    def out_frame_bytes(self) -> int:
        return int(np.prod(self.out_shape)) * (2 if self.mode == Mode.raw else 4)

    def run(self, raw: Sequence[torch.Tensor], out: Sequence[torch.Tensor], stream=None) -> None:
        """Calibrate ``raw[i]`` (uint16, frame shape) into ``out[i]`` (``out_shape``) on ``stream``."""
        if len(raw) != len(out):
            raise ValueError("raw/out length mismatch")
        if not raw:
            return
        if not self._gpu:
            self._run_reference(raw, out)
            return
        # cheap per-tensor checks (this runs per batch on the host; keep it well under a kernel's time)
        npix, ofb, odt = self.spec.npix, self._out_frame_bytes, self.out_dtype
        di = self.device.index if self.device.index is not None else torch.cuda.current_device()
        for r in raw:
            if r.dtype is not torch.uint16 or r.numel() != npix or not r.is_contiguous() or r.get_device() != di:
                raise ValueError("Calibrator.run: raw frames must be contiguous uint16 frames on the calibrator device")
        for o in out:
            if o.dtype is not odt or o.numel() * o.element_size() != ofb or not o.is_contiguous() or \
                    o.get_device() != di or o.data_ptr() % 16:
                raise ValueError("Calibrator.run: outputs must be contiguous, 16-B aligned frames of out_shape")
        self.run_ptrs([int(r.data_ptr()) for r in raw], [int(o.data_ptr()) for o in out], stream)

    def run_ptrs(self, raw_ptrs, out_ptrs, stream=None) -> None:
        """Pointer-level entry (buffers already validated by the caller, e.g. ring slots)."""
        from ..ops import _ext

        _ext.load().run_calib_plan(self.plan, list(raw_ptrs), list(out_ptrs), _ext.stream_handle(stream))

    def _make_plan(self, C):
        spec = self.spec
        p = C.CalibPlan()
        p.kind = spec.kernel_kind
        p.npix = spec.npix
        p.ped, p.gf, p.elig = int(self.ped.data_ptr()), int(self.gf.data_ptr()), int(self.elig.data_ptr())
        p.ped_sg = 0 if self.ped_sg is None else int(self.ped_sg.data_ptr())
        p.n_panels, p.panel_rows, p.panel_cols = spec.n_panels, spec.panel_rows, spec.panel_cols
        p.asic_rows, p.asic_cols = spec.asic_rows, spec.asic_cols
        p.raw_frame_bytes = spec.raw_frame_bytes
        p.out_frame_bytes = self.out_frame_bytes
        if self.cm is not None:
            p.use_cm = 1
            p.thr, p.maxcorr = float(self.cm.thr), float(self.cm.maxcorr)
            p.npix_min, p.cm_flags, p.bank_cols = int(self.cm.npix_min), int(self.cm.flags), int(self.cm.bank_cols)
        if self.mode == Mode.raw:
            p.mode = 0
        elif self.mode == Mode.calib:
            p.mode = 2 if self.cm is not None else 1
        else:
            p.idx, p.nout = int(self.idx.data_ptr()), int(self.idx.numel())
            if self.tile_map is not None:
                tm = self.tile_map
                p.use_tiles = 1
                p.tiles, p.codes = int(self._tiles.data_ptr()), int(self._codes.data_ptr())
                p.n_tiles, p.tiles_x = tm.n_tiles, tm.tiles_x
                p.img_h, p.img_w = tm.image_shape
            place = self.geometry.panel_placement() if self.cm is not None else None
            if self.cm is None and (self.omask is None or self.tile_map is not None):
                p.mode = 3
            elif place is not None:
                # common mode writes the assembled image from its LDS tiles (no scratch round trip);
                # the same kernel zeroes the gaps between panels (gap table).  Every panel pixel lands on exactly
                # one image pixel, so the image mask folds into this plan's gain factors (the
                # common-mode eligibility is unchanged: the reference masks after assembly)
                p.mode = 5
                self._img_desc = torch.from_numpy(place.ravel().copy()).to(self.device)
                self._gap_runs = torch.from_numpy(self.geometry.gap_fill_table()).to(self.device)
                p.img_desc, p.gap_runs = int(self._img_desc.data_ptr()), int(self._gap_runs.data_ptr())
                p.n_gap_runs = int(self._gap_runs.numel())
                if self.image_mask is not None:
                    imap = self.geometry.index_map().ravel()
                    keep = np.ones(spec.npix, dtype=np.float32)
                    hit = imap >= 0
                    keep[imap[hit]] = (np.asarray(self.image_mask).ravel()[hit] != 0).astype(np.float32)
                    self._gf_img = (self.gf.view(-1, spec.npix) * torch.from_numpy(keep).to(self.device)).contiguous()
                    p.gf = int(self._gf_img.data_ptr())
            else:
                p.mode = 4
                self._scratch = torch.empty((kernels.MAX_FRAMES, *spec.frame_shape), dtype=torch.float32,
                                            device=self.device)
                p.scratch = int(self._scratch.data_ptr())
                p.omask = 0 if self.omask is None else int(self.omask.data_ptr())
        return p

    def _run_reference(self, raw, out):
        if self.mode == Mode.raw:
            for r, o in zip(raw, out):
                o.copy_(r.view(o.shape))
            return
        batch = torch.stack([r.view(self.spec.frame_shape) for r in raw])
        cal = reference.calibrate_reference(batch, self.consts, self.frame_mask, self.cm)
        if self.mode == Mode.image:
            cal = reference.assemble_reference(cal, self.geometry.rows, self.geometry.cols,
                                               self.geometry.image_shape, self.image_mask)
        for i, o in enumerate(out):
            o.copy_(cal[i].view(o.shape))

    def __call__(self, raw: torch.Tensor, stream=None) -> torch.Tensor:
        """Convenience: [F, P, H, W] (or [P, H, W]) uint16 -> newly allocated output batch."""
        if raw.dim() == 3:
            raw = raw.unsqueeze(0)
        out = torch.empty((raw.shape[0], *self.out_shape), dtype=self.out_dtype, device=raw.device)
        self.run([raw[i] for i in range(raw.shape[0])], [out[i] for i in range(raw.shape[0])], stream)
        return out


