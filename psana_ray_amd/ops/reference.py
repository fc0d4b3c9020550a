"""Pure-PyTorch fp32 golden models of every numeric op (K-01 .. K-07).

These are the oracles the HIP kernels are tested against and the
explicit compute path of ``device="cpu"`` pipelines (BASELINE config 1 runs without a GPU).  They
are written from the documented formulas and the *unpacked* constants (pedestals/gains per gain
range, gain configuration, status), not from the kernel's packed tables, so a packing bug is
caught too.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from ..config import CommonModeParams, PeakFinderParams
from ..models.constants import CalibConstants
from ..models.detector import EPIX_CAND_A, EPIX_CAND_B


def decode_gain(raw: torch.Tensor, consts: CalibConstants):
    """K-01: per-pixel ADU, gain-range index and validity from raw u16 frames [F, P, H, W]."""
    s = consts.spec
    r = raw.to(torch.int32)
    if s.kind == "epix10ka":
        adu = r & 0x3FFF
        bit = (r >> 14) & 1
        cfg = torch.as_tensor(consts.gain_config.astype(np.int64), device=raw.device)
        a = torch.as_tensor(EPIX_CAND_A, device=raw.device)[cfg]
        b = torch.as_tensor(EPIX_CAND_B, device=raw.device)[cfg]
        g = torch.where(bit.bool(), b, a)
        valid = torch.ones_like(adu, dtype=torch.bool)
    elif s.kind == "jungfrau":
        adu = r & 0x3FFF
        gb = r >> 14
        g = torch.where(gb == 3, torch.full_like(gb, 2), gb & 1).to(torch.int64)
        valid = gb != 2
    else:
        adu = r
        g = torch.zeros_like(r, dtype=torch.int64)
        valid = torch.ones_like(r, dtype=torch.bool)
    return adu, g.to(torch.int64), valid


def _take(table: np.ndarray, g: torch.Tensor) -> torch.Tensor:
    t = torch.as_tensor(table, device=g.device)            # [G, P, H, W]
    F = g.shape[0]
    tt = t.unsqueeze(0).expand(F, *t.shape)                 # [F, G, P, H, W]
    return torch.gather(tt, 1, g.unsqueeze(1)).squeeze(1)


def masked_median(x: torch.Tensor, m: torch.Tensor, dim: int):
    """numpy-semantics median of x over ``dim`` restricted to m; returns (median, count)."""
    xs = torch.where(m, x, torch.full_like(x, float("inf"))).sort(dim=dim).values
    cnt = m.sum(dim=dim, keepdim=True)
    i0 = ((cnt - 1) // 2).clamp(min=0)
    i1 = (cnt // 2).clamp(min=0, max=x.shape[dim] - 1)
    a = torch.gather(xs, dim, i0)
    b = torch.gather(xs, dim, i1)
    return (a + b) * 0.5, cnt


def common_mode_reference(v: torch.Tensor, elig: torch.Tensor, consts: CalibConstants,
                          cm: CommonModeParams) -> torch.Tensor:
    """K-03 on pre-gain values v [F, P, H, W]: rows-by-bank then columns, per ASIC."""
    s = consts.spec
    F, P, H, W = v.shape
    R, C = s.asic_rows, s.asic_cols
    L = cm.bank_cols or s.bank_cols

    def to_tiles(x):
        return x.reshape(F, P, H // R, R, W // C, C).permute(0, 1, 2, 4, 3, 5).contiguous()

    def from_tiles(x):
        return x.permute(0, 1, 2, 4, 3, 5).reshape(F, P, H, W)

    t = to_tiles(v)
    e = to_tiles(elig)
    if cm.flags & 1:
        tb = t.reshape(*t.shape[:-1], C // L, L)
        eb = e.reshape(*e.shape[:-1], C // L, L)
        med, cnt = masked_median(tb, eb & (tb.abs() < cm.thr), dim=-1)
        ok = (cnt >= max(cm.npix_min, 1)) & (med.abs() <= cm.maxcorr)
        tb = torch.where(eb & ok, tb - med, tb)
        t = tb.reshape(t.shape)
    if cm.flags & 2:
        med, cnt = masked_median(t, e & (t.abs() < cm.thr), dim=-2)
        ok = (cnt >= max(cm.npix_min, 1)) & (med.abs() <= cm.maxcorr)
        t = torch.where(e & ok, t - med, t)
    return from_tiles(t)


def calibrate_reference(raw: torch.Tensor, consts: CalibConstants, mask: Optional[np.ndarray] = None,
                        cm: Optional[CommonModeParams] = None) -> torch.Tensor:
    """K-01..K-04: raw u16 [F, P, H, W] -> calibrated f32 [F, P, H, W] (keV), masked (truthy keeps)."""
    s = consts.spec
    if raw.dim() == 3:
        raw = raw.unsqueeze(0)
    adu, g, valid = decode_gain(raw, consts)
    ped = _take(consts.pedestals, g)
    gain = _take(consts.gains, g)
    v = adu.to(torch.float32) - ped
    keep = torch.ones(s.frame_shape, dtype=torch.bool, device=raw.device) if mask is None else \
        torch.as_tensor(np.asarray(mask).astype(bool), device=raw.device).expand(s.frame_shape)
    if cm is not None:
        cm_set = torch.zeros(max(s.n_gains, 1), dtype=torch.bool, device=raw.device)
        cm_set[list(consts.cm_gains)] = True
        status_good = torch.as_tensor(consts.status == 0, device=raw.device)
        # the output mask does NOT enter the estimate: the reference masks psana's calibrated frames
        # afterwards (np.where(mask, data, 0), psana_ray/producer.py:92-95), psana's common mode sees
        # only its own status constants
        elig = valid & status_good & cm_set[g]
        v = common_mode_reference(v, elig, consts, cm)
    gf = 1.0 / gain                      # float32, same rounding as the packed device table
    out = v * gf
    out = torch.where(valid, out, torch.zeros_like(out))
    out = torch.where(keep, out, torch.zeros_like(out))   # np.where(mask, data, 0) (producer.py:92-95)
    return out


def assemble_reference(frames: torch.Tensor, rows: np.ndarray, cols: np.ndarray, image_shape,
                       image_mask: Optional[np.ndarray] = None) -> torch.Tensor:
    """K-05 as a SCATTER from per-pixel image coordinates: [F, P, H, W] -> [F, 1, Himg, Wimg]."""
    F = frames.shape[0]
    himg, wimg = image_shape
    out = torch.zeros(F, himg * wimg, dtype=frames.dtype, device=frames.device)
    dst = torch.as_tensor((rows.astype(np.int64) * wimg + cols).ravel(), device=frames.device)
    out[:, dst] = frames.reshape(F, -1)
    if image_mask is not None:
        out = torch.where(torch.as_tensor(np.asarray(image_mask).astype(bool).ravel(), device=out.device),
                          out, torch.zeros_like(out))
    return out.reshape(F, 1, himg, wimg)


def peakfind_reference(frames: torch.Tensor, p: PeakFinderParams):
    """K-07 golden: per frame, an [n, 8] float tensor (panel,row,col,value,intensity,bkg,noise,snr)
    sorted by (panel,row,col), plus the [F, 2] summary (n pixels above thr, their sum)."""
    if frames.dim() == 3:
        frames = frames.unsqueeze(0)
    F, P, H, W = frames.shape
    R = p.radius
    h = R + 2
    x = frames.to(torch.float32)
    xp = torch.full((F, P, H + 2 * h, W + 2 * h), float("nan"), dtype=torch.float32, device=x.device)
    xp[:, :, h:h + H, h:h + W] = x

    def sh(dy, dx):
        return xp[:, :, h + dy:h + dy + H, h + dx:h + dx + W]

    above = x > p.thr_peak
    summary = torch.stack([above.sum(dim=(1, 2, 3)).to(torch.float32),
                           torch.where(above, x, torch.zeros_like(x)).sum(dim=(1, 2, 3))], dim=1)
    is_max = above.clone()
    for dy in range(-R, R + 1):
        for dx in range(-R, R + 1):
            if dy == 0 and dx == 0:
                continue
            n = sh(dy, dx)
            before = dy < 0 or (dy == 0 and dx < 0)
            okn = (x > n) if before else (x >= n)
            is_max &= okn | torch.isnan(n)
    s = torch.zeros_like(x)
    s2 = torch.zeros_like(x)
    nr = torch.zeros_like(x)
    for dy in range(-h, h + 1):
        for dx in range(-h, h + 1):
            if max(abs(dy), abs(dx)) <= R:
                continue
            n = sh(dy, dx)
            ok = ~torch.isnan(n)
            n0 = torch.where(ok, n, torch.zeros_like(n))
            s += n0
            s2 += n0 * n0
            nr += ok.to(torch.float32)
    bkg = torch.where(nr > 0, s / nr.clamp(min=1), torch.zeros_like(s))
    var = torch.where(nr > 0, (s2 / nr.clamp(min=1) - bkg * bkg).clamp(min=0), torch.zeros_like(s))
    noise = var.sqrt()
    snr = (x - bkg) / noise.clamp(min=1e-6)
    inten = torch.zeros_like(x)
    for dy in range(-R, R + 1):
        for dx in range(-R, R + 1):
            n = sh(dy, dx)
            inten += torch.where(torch.isnan(n), torch.zeros_like(n), n - bkg)
    keep = is_max & (snr >= p.son_min)
    peaks: List[torch.Tensor] = []
    for f in range(F):
        idx = keep[f].nonzero()
        pk, r, c = idx[:, 0], idx[:, 1], idx[:, 2]
        rec = torch.stack([pk.float(), r.float(), c.float(), x[f, pk, r, c], inten[f, pk, r, c],
                           bkg[f, pk, r, c], noise[f, pk, r, c], snr[f, pk, r, c]], dim=1)
        peaks.append(rec)
    return peaks, summary
