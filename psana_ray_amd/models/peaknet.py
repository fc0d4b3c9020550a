"""A small peak-segmentation network trained online from the stream ("PyTorch Task" consumer).

The reference's architecture figure ends in a "PyTorch Task" consumer and its package
description names PeakNet (setup.py:11, SURVEY Q-15): frames from the queue feed a network that
segments Bragg peaks.  This is that consumer's model, sized for streaming: panels are the batch
(epix10k2M: 16 panels of 352x384 per frame), a 2-level U-Net of 3x3 convolutions (MIOpen on
gfx950) run in bf16 autocast, and per-pixel peak labels come from the on-GPU peak finder (K-07)
over the same frames -- the usual way PeakNet-style models are bootstrapped from a classical
finder, here without leaving the GPU.
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F


def _block(cin: int, cout: int) -> nn.Sequential:
    return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout), nn.ReLU(inplace=True),
                         nn.Conv2d(cout, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


class PeakNetLite(nn.Module):
    """2-level U-Net: [N, 1, H, W] panel images -> [N, 1, H, W] peak logits (H, W divisible by 4)."""

    def __init__(self, width: int = 16):
        super().__init__()
        w = width
        self.enc1, self.enc2, self.mid = _block(1, w), _block(w, 2 * w), _block(2 * w, 4 * w)
        self.up2, self.dec2 = nn.ConvTranspose2d(4 * w, 2 * w, 2, stride=2), _block(4 * w, 2 * w)
        self.up1, self.dec1 = nn.ConvTranspose2d(2 * w, w, 2, stride=2), _block(2 * w, w)
        self.head = nn.Conv2d(w, 1, 1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        e1 = self.enc1(x)
        e2 = self.enc2(F.max_pool2d(e1, 2))
        m = self.mid(F.max_pool2d(e2, 2))
        d2 = self.dec2(torch.cat([self.up2(m), e2], 1))
        d1 = self.dec1(torch.cat([self.up1(d2), e1], 1))
        return self.head(d1)


def normalize_panels(frames: torch.Tensor) -> torch.Tensor:
    """[B, P, H, W] calibrated keV-scale frames -> [B*P, 1, H, W] inputs (log-compressed)."""
    x = frames.reshape(-1, 1, *frames.shape[-2:]).float()
    return torch.sign(x) * torch.log1p(x.abs())


def peak_masks(peaks: torch.Tensor, counts: torch.Tensor, shape: Sequence[int], radius: int = 1) -> torch.Tensor:
    """Peak-finder records -> per-pixel targets [B*P, 1, H, W] (1 within ``radius`` of a peak).

    ``peaks`` [B, max_peaks, 8] (panel, row, col, ...) and ``counts`` [B] as written by
    :func:`psana_ray_amd.ops.kernels.peakfind` (or the golden model's lists, padded)."""
    B = peaks.shape[0]
    P, H, W = shape
    mask = torch.zeros((B * P, 1, H, W), dtype=torch.float32, device=peaks.device)
    n = counts.clamp(max=peaks.shape[1]).to(torch.int64)
    valid = torch.arange(peaks.shape[1], device=peaks.device)[None, :] < n[:, None]
    b, k = valid.nonzero(as_tuple=True)
    if b.numel() == 0:
        return mask
    rec = peaks[b, k]
    img = b * P + rec[:, 0].long()
    r, c = rec[:, 1].long(), rec[:, 2].long()
    for dy in range(-radius, radius + 1):
        for dx in range(-radius, radius + 1):
            rr, cc = (r + dy).clamp(0, H - 1), (c + dx).clamp(0, W - 1)
            mask[img, 0, rr, cc] = 1.0
    return mask
