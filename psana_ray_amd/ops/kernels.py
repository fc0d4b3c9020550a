"""Validated torch-facing wrappers of the gfx950 HIP kernels (K-01..K-05, K-07).

Every wrapper checks device / dtype / shape / contiguity / alignment on the host BEFORE the
launch (a mis-shaped launch of a hand-written kernel can fault the GPU), splits batches into
launches of at most ``MAX_FRAMES`` frames, and launches on the given torch stream.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from . import _ext

MAX_FRAMES = 64
# int32 words of the peak finder's self-resetting scratch (csrc/peakfind.hip PfScratch)
# peak-finder scratch block per consumer stream (csrc/kernels.h kPfScratchBytes): self-resetting
# counters (1 KiB header) + every workgroup's candidate spill list for hit-rich frames (16 MiB)
PF_SCRATCH_WORDS = (1024 + 4096 * 1024 * 4) // 4


def _ptr(t: torch.Tensor) -> int:
    return int(t.data_ptr())


def _check_frames(frames: Sequence[torch.Tensor], dtype, numel: int, device, what: str):
    for t in frames:
        if t.device != device:
            raise ValueError(f"{what}: tensor on {t.device}, expected {device}")
        if t.dtype != dtype:
            raise ValueError(f"{what}: dtype {t.dtype}, expected {dtype}")
        if t.numel() != numel:
            raise ValueError(f"{what}: {t.numel()} elements, expected {numel}")
        if not t.is_contiguous():
            raise ValueError(f"{what}: tensor must be contiguous")
        if t.data_ptr() % 16:
            raise ValueError(f"{what}: tensor must be 16-byte aligned")


def _validate_index_map(idx: torch.Tensor, npix: int, what: str):
    """One-time (cached on the tensor) host check that the gather map stays inside the frame."""
    if getattr(idx, "_pr_checked_npix", None) == npix:
        return
    if idx.dtype != torch.int32 or not idx.is_contiguous() or idx.data_ptr() % 16:
        raise ValueError(f"{what}: idx must be a contiguous, 16-B aligned int32 tensor")
    if idx.numel() and (int(idx.max()) >= npix or int(idx.min()) < -1):
        raise ValueError(f"{what}: index map points outside the frame")
    idx._pr_checked_npix = npix


def _chunks(n: int):
    for i in range(0, n, MAX_FRAMES):
        yield i, min(n, i + MAX_FRAMES)


def calib_basic(raw: Sequence[torch.Tensor], out: Sequence[torch.Tensor], ped: torch.Tensor, gf: torch.Tensor,
                kind: int, stream: Optional[torch.cuda.Stream] = None):
    C = _ext.load()
    npix = ped.shape[1]
    dev = ped.device
    _check_frames(raw, torch.uint16, npix, dev, "calib_basic raw")
    _check_frames(out, torch.float32, npix, dev, "calib_basic out")
    if len(raw) != len(out):
        raise ValueError("calib_basic: raw/out length mismatch")
    s = _ext.stream_handle(stream)
    for a, b in _chunks(len(raw)):
        C.calib_basic([_ptr(t) for t in raw[a:b]], [_ptr(t) for t in out[a:b]], _ptr(ped), _ptr(gf), npix, kind, s)


def calib_image(raw, out, ped, gf, kind, idx: torch.Tensor, stream=None):
    C = _ext.load()
    npix = ped.shape[1]
    dev = ped.device
    nout = idx.numel()
    _check_frames(raw, torch.uint16, npix, dev, "calib_image raw")
    _check_frames(out, torch.float32, nout, dev, "calib_image out")
    if idx.device != dev:
        raise ValueError("calib_image: idx must be on the kernel device")
    _validate_index_map(idx, npix, "calib_image")
    s = _ext.stream_handle(stream)
    for a, b in _chunks(len(raw)):
        C.calib_image([_ptr(t) for t in raw[a:b]], [_ptr(t) for t in out[a:b]], _ptr(ped), _ptr(gf), npix, kind,
                      _ptr(idx), nout, s)


def calib_cm(raw, out, ped, gf, elig, kind, spec, cm, stream=None, ped_sg=None):
    """``ped_sg``: optional signed pedestal tables (CalibConstants.cm_signed_pedestals); the production
    shapes then read the eligibility from their sign bits instead of ``elig``."""
    C = _ext.load()
    npix = ped.shape[1]
    dev = ped.device
    _check_frames(raw, torch.uint16, npix, dev, "calib_cm raw")
    _check_frames(out, torch.float32, npix, dev, "calib_cm out")
    stride = {1: 1, 2: 2, 3: 4}[ped.shape[0]]
    if elig.dtype != torch.uint8 or elig.numel() != (npix // 8) * stride:
        raise ValueError("calib_cm: elig must be the uint8 eligibility bit-planes [npix / 8, stride] "
                         "(CalibConstants.device_tables)")
    if ped_sg is not None and (ped_sg.dtype != torch.float32 or ped_sg.shape != ped.shape or ped_sg.device != dev
                               or not ped_sg.is_contiguous()):
        raise ValueError("calib_cm: ped_sg must be a contiguous float32 table shaped like ped on its device")
    bank = cm.bank_cols or spec.bank_cols
    if C.cm_tile_cols(spec.asic_rows, spec.asic_cols, int(bank), 0, int(kind)) == 0:
        raise ValueError(f"common mode: no full-height stripe of the {spec.asic_rows}x{spec.asic_cols} ASIC "
                         f"(bank {bank}) fits in 160 KiB of LDS")
    s = _ext.stream_handle(stream)
    for a, b in _chunks(len(raw)):
        C.calib_cm([_ptr(t) for t in raw[a:b]], [_ptr(t) for t in out[a:b]], _ptr(ped), _ptr(gf), _ptr(elig), kind,
                   spec.n_panels, spec.panel_rows, spec.panel_cols, spec.asic_rows, spec.asic_cols,
                   float(cm.thr), float(cm.maxcorr), int(cm.npix_min), int(cm.flags), int(bank), s,
                   0 if ped_sg is None else _ptr(ped_sg))


def assemble(frames, out, idx: torch.Tensor, npix: int, omask: Optional[torch.Tensor] = None, stream=None):
    C = _ext.load()
    dev = idx.device
    nout = idx.numel()
    _check_frames(frames, torch.float32, npix, dev, "assemble in")
    _check_frames(out, torch.float32, nout, dev, "assemble out")
    _validate_index_map(idx, npix, "assemble")
    if omask is not None and (omask.dtype != torch.uint8 or omask.numel() != nout or omask.device != dev):
        raise ValueError("assemble: omask must be uint8[nout] on the kernel device")
    s = _ext.stream_handle(stream)
    for a, b in _chunks(len(frames)):
        C.assemble([_ptr(t) for t in frames[a:b]], [_ptr(t) for t in out[a:b]], _ptr(idx), nout,
                   0 if omask is None else _ptr(omask), s)


def peakfind(frames: Sequence[torch.Tensor], shape, params, peaks: torch.Tensor, counts: torch.Tensor,
             summary: torch.Tensor, stream=None, total: Optional[torch.Tensor] = None,
             scratch: Optional[torch.Tensor] = None):
    """frames: F tensors of ``shape`` = (P, H, W) f32.  Outputs: peaks [F, max_peaks, 8] f32,
    counts [F] int32, summary [F, 2] f32.  ``total`` (int64 scalar on the device, optional) is
    incremented by the number of peak records written.

    ``scratch``: a zero-initialised int32 tensor of PF_SCRATCH_WORDS on the frames' device, reused
    by every call on one stream.  The kernel then accumulates there and its last workgroup writes
    counts / summary whole and re-zeroes the scratch -- no fill kernel per call.  Without it, counts
    and summary are zeroed here on the stream first."""
    C = _ext.load()
    P, H, W = shape
    F = len(frames)
    if F == 0:
        return
    dev = frames[0].device
    _check_frames(frames, torch.float32, P * H * W, dev, "peakfind in")
    if peaks.shape != (F, params.max_peaks, 8) or peaks.dtype != torch.float32:
        raise ValueError("peakfind: peaks must be float32 [F, max_peaks, 8]")
    if counts.shape != (F,) or counts.dtype != torch.int32:
        raise ValueError("peakfind: counts must be int32 [F]")
    if summary.shape != (F, 2) or summary.dtype != torch.float32:
        raise ValueError("peakfind: summary must be float32 [F, 2]")
    if params.radius not in (1, 2):
        raise ValueError("peakfind: radius must be 1 or 2")
    if total is not None and (total.dtype != torch.int64 or total.numel() != 1 or total.device != dev):
        raise ValueError("peakfind: total must be an int64 scalar on the frames' device")
    if C.PF_SCRATCH_BYTES != 4 * PF_SCRATCH_WORDS:   # the kernel's spill lists would overrun the block
        raise RuntimeError(f"peakfind: PF_SCRATCH_WORDS {PF_SCRATCH_WORDS} disagrees with the extension's "
                           f"kPfScratchBytes {C.PF_SCRATCH_BYTES}")
    if scratch is not None and (scratch.dtype != torch.int32 or scratch.numel() < PF_SCRATCH_WORDS
                                or scratch.device != dev or not scratch.is_contiguous()):
        raise ValueError(f"peakfind: scratch must be a contiguous int32 [{PF_SCRATCH_WORDS}] tensor on the frames' device")
    s = _ext.stream_handle(stream)
    if scratch is None:
        with torch.cuda.stream(stream) if stream is not None else torch.cuda.stream(torch.cuda.current_stream()):
            counts.zero_()
            summary.zero_()
    for a, b in _chunks(F):
        C.peakfind([_ptr(t) for t in frames[a:b]], P, H, W, float(params.thr_peak), float(params.son_min),
                   int(params.radius), int(params.max_peaks), _ptr(peaks[a]), _ptr(counts[a:]), _ptr(summary[a]), s,
                   0 if total is None else _ptr(total), 0 if scratch is None else _ptr(scratch))


def mask_frames(frames: Sequence[torch.Tensor], zero: torch.Tensor, stream=None):
    """In place, ``np.where(mask, data, 0)`` (psana_ray/producer.py:92-95) over F float32 frames:
    pixel i of every frame becomes 0 where ``zero[i]`` (uint8, 1 = masked) is non-zero.  ONE launch
    per 64 frames (csrc/gather.hip mask_frames_kernel) -- the psana-calibrated upload path."""
    C = _ext.load()
    if not frames:
        return
    dev = frames[0].device
    n = frames[0].numel()
    _check_frames(frames, torch.float32, n, dev, "mask_frames")
    if zero.dtype != torch.uint8 or zero.numel() != n or zero.device != dev or not zero.is_contiguous() \
            or _ptr(zero) % 4:
        raise ValueError(f"mask_frames: zero must be a contiguous, 4-B aligned uint8 [{n}] tensor on {dev}")
    s = _ext.stream_handle(stream)
    for a, b in _chunks(len(frames)):
        C.mask_frames([_ptr(t) for t in frames[a:b]], _ptr(zero), n, s)


def gather_frames(frames: Sequence[torch.Tensor], out, stream=None):
    """Copy F leased f32 frames (scattered ring slots) into ``out``: a contiguous batch [F, ...]
    or a list of F contiguous destination tensors (e.g. the panel ranges of assembled frames);
    float32 or bfloat16 (converted on the fly, round-to-nearest-even).  ONE launch per 32 frames
    (csrc/gather.hip)."""
    C = _ext.load()
    F = len(frames)
    if F == 0:
        return out
    dev = frames[0].device
    n = frames[0].numel()
    _check_frames(frames, torch.float32, n, dev, "gather_frames in")
    outs = list(out) if isinstance(out, (list, tuple)) else None
    if outs is None:
        if out.device != dev or out.dtype not in (torch.float32, torch.bfloat16) or not out.is_contiguous():
            raise ValueError("gather_frames: out must be a contiguous float32/bfloat16 tensor on the frames' device")
        if out.shape[0] != F or out[0].numel() != n:
            raise ValueError(f"gather_frames: out shape {tuple(out.shape)} does not hold {F} frames of {n} elements")
        odt = out.dtype
        outs = [out[i] for i in range(F)]
    else:
        if len(outs) != F:
            raise ValueError(f"gather_frames: {len(outs)} destinations for {F} frames")
        odt = outs[0].dtype
        if odt not in (torch.float32, torch.bfloat16):
            raise ValueError("gather_frames: destinations must be float32/bfloat16")
        _check_frames(outs, odt, n, dev, "gather_frames out")
    if n % 4 or any(o.data_ptr() % 16 for o in outs):
        raise ValueError("gather_frames: frames must be multiples of 4 elements, destinations 16-B aligned")
    bf16 = odt == torch.bfloat16
    s = _ext.stream_handle(stream)
    for a, b in _chunks(F):
        C.gather_frames([_ptr(t) for t in frames[a:b]], [_ptr(o) for o in outs[a:b]], n, bf16, s)
    return out
