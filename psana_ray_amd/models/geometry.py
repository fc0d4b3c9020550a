"""Panel geometry and the image-assembly index map (K-05).

psana assembles calibrated panels into a 2-D image in image mode (the reference's default mode,
psana_ray/producer.py:22,156-159; SURVEY E-03 / Appendix B).  Without psana geometry files the
framework builds a synthetic but realistic layout: each panel is placed by an integer
90-degree rotation + translation (epix10k2M: four 2x2-panel quads in a pinwheel), so every
panel pixel lands on exactly one image pixel and scatter == gather exactly.

The GPU kernel consumes the inverse map (image pixel -> flat source pixel, -1 for gaps), a
deterministic, atomics-free gather.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from .detector import DetectorSpec


def _rotate(rr: np.ndarray, cc: np.ndarray, h: int, w: int, k: int):
    """Rotate pixel coordinates of an h x w block by k*90 degrees; returns (rows, cols, h', w')."""
    k %= 4
    if k == 0:
        return rr, cc, h, w
    if k == 1:
        return (w - 1 - cc), rr, w, h
    if k == 2:
        return (h - 1 - rr), (w - 1 - cc), h, w
    return cc, (h - 1 - rr), w, h


@dataclass
class Geometry:
    spec: DetectorSpec
    image_shape: tuple
    rows: np.ndarray  # [P, H, W] int32 image row of each panel pixel
    cols: np.ndarray  # [P, H, W] int32 image col

    def index_map(self) -> np.ndarray:
        """Flat gather map of the image: source flat pixel index or -1 (gap)."""
        himg, wimg = self.image_shape
        idx = np.full(himg * wimg, -1, dtype=np.int32)
        dst = (self.rows.astype(np.int64) * wimg + self.cols).ravel()
        idx[dst] = np.arange(self.spec.npix, dtype=np.int32)
        return idx

    def panel_placement(self):
        """``[P, 3]`` int32 (base, step per panel row, step per panel column) such that pixel
        ``(y, x)`` of panel ``p`` lands at flat image element ``base + y*sy + x*sx``, or None when a
        panel is not placed by an integer rotation + translation (then the fused common-mode image
        kernel does not apply and the two-pass path is used)."""
        himg, wimg = self.image_shape
        P, H, W = self.rows.shape
        out = np.zeros((P, 3), np.int64)
        yy, xx = np.meshgrid(np.arange(H, dtype=np.int64), np.arange(W, dtype=np.int64), indexing="ij")
        for p in range(P):
            idx = self.rows[p].astype(np.int64) * wimg + self.cols[p]
            b = int(idx[0, 0])
            sy = int(idx[1, 0] - b) if H > 1 else wimg
            sx = int(idx[0, 1] - b) if W > 1 else 1
            if sorted((abs(sy), abs(sx))) != sorted((1, wimg)) or not np.array_equal(idx, b + yy * sy + xx * sx):
                return None
            out[p] = (b, sy, sx)
        if himg * wimg >= 2 ** 31:
            return None
        return out.astype(np.int32)

    def gap_runs(self, max_len: int = 1024) -> np.ndarray:
        """``[n, 2]`` int32 (start, length) runs of flat image elements no panel pixel covers,
        split to at most ``max_len`` elements (one GPU wave zero-fills one run)."""
        gap = (self.index_map() < 0).astype(np.int8)
        d = np.diff(np.concatenate([[0], gap, [0]]))
        starts, ends = np.where(d == 1)[0], np.where(d == -1)[0]
        runs = []
        for a, e in zip(starts.tolist(), ends.tolist()):
            for s0 in range(a, e, max_len):
                runs.append((s0, min(max_len, e - s0)))
        return np.asarray(runs, np.int32).reshape(-1, 2)

    def gap_fill_table(self) -> np.ndarray:
        """int32 gap table of the fused common-mode -> image kernel (csrc/common_mode.hip, ImgOut):
        the image elements no panel pixel covers, as aligned 16-B chunks first (entry = first
        element, a multiple of 4: all four elements are gaps) and the remaining gap elements after
        them (entry = -1 - element)."""
        gap = self.index_map() < 0
        n = gap.size
        n4 = n // 4
        full = gap[: 4 * n4].reshape(n4, 4).all(axis=1)
        chunks = 4 * np.nonzero(full)[0]
        single = gap.copy()
        single[: 4 * n4] &= ~np.repeat(full, 4)
        singles = np.nonzero(single)[0]
        return np.concatenate([chunks, -1 - singles]).astype(np.int32)

    def pixel_coords_um(self):
        """(x, y) pixel-centre coordinates in micrometres (psana-style geometry output)."""
        ps = self.spec.pixel_size_um
        return self.cols * ps, self.rows * ps


def _panel_grid(spec: DetectorSpec, gap: int):
    """Generic layout: panels on a near-square grid, no rotation."""
    P, H, W = spec.frame_shape
    ncol = int(math.ceil(math.sqrt(P)))
    nrow = int(math.ceil(P / ncol))
    rr, cc = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    rows = np.empty((P, H, W), np.int32)
    cols = np.empty((P, H, W), np.int32)
    for p in range(P):
        gr, gc = divmod(p, ncol)
        rows[p] = rr + gr * (H + gap)
        cols[p] = cc + gc * (W + gap)
    return rows, cols, (nrow * (H + gap) - gap, ncol * (W + gap) - gap)


def _epix_quads(spec: DetectorSpec, gap: int):
    """epix10k2M-like: 4 quads of 2x2 panels, quad q rotated by q*90 deg (pinwheel)."""
    P, H, W = spec.frame_shape
    assert P == 16
    QH, QW = 2 * H + gap, 2 * W + gap
    cell = max(QH, QW) + 2 * gap
    rr, cc = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    rows = np.empty((P, H, W), np.int32)
    cols = np.empty((P, H, W), np.int32)
    cell_of_quad = [(0, 0), (0, 1), (1, 1), (1, 0)]  # clockwise around the beam
    for p in range(P):
        q, i = divmod(p, 4)
        qr, qc = divmod(i, 2)
        yr = rr + qr * (H + gap)
        xc = cc + qc * (W + gap)
        yr, xc, qh, qw = _rotate(yr, xc, QH, QW, q)
        cy, cx = cell_of_quad[q]
        oy = cy * cell + (cell - qh) // 2
        ox = cx * cell + (cell - qw) // 2
        rows[p] = yr + oy
        cols[p] = xc + ox
    return rows, cols, (2 * cell, 2 * cell)


def make_geometry(spec: DetectorSpec) -> Geometry:
    gap = spec.panel_gap_px
    if spec.kind == "epix10ka" and spec.n_panels == 16:
        rows, cols, shape = _epix_quads(spec, gap)
    else:
        rows, cols, shape = _panel_grid(spec, gap)
    geo = Geometry(spec, tuple(int(s) for s in shape), rows, cols)
    flat = rows.astype(np.int64) * shape[1] + cols
    assert np.unique(flat).size == spec.npix, "geometry maps two pixels onto one image pixel"
    assert rows.min() >= 0 and cols.min() >= 0 and rows.max() < shape[0] and cols.max() < shape[1]
    return geo


# ------------------------------------------------------------------------------------------
# Tiled assembly map for csrc/image.hip (LDS-staged gather)
TILE_H, TILE_W, TILE_STAGE, TILE_LDS = 32, 64, 2048, 2176


@dataclass
class TileMap:
    """Per-tile staging boxes + per-output-pixel codes (see csrc/image.hip).

    tiles[t] = (panel, r0, c0, h, w, 0, 0, 0): source box staged for output tile t (panel -1:
    nothing staged); codes[o] >= 0 is the LDS word of output pixel o (row pitch w+1), -1 a gap or
    masked pixel, <= -2 the source pixel ``-(code+2)`` read directly."""

    image_shape: tuple
    tiles: np.ndarray      # int32 [n_tiles, 8]
    codes: np.ndarray      # int32 [img_h * img_w]
    tiles_x: int
    staged_px: int
    direct_px: int

    @property
    def n_tiles(self) -> int:
        return int(self.tiles.shape[0])


def build_tile_map(index_map: np.ndarray, spec: DetectorSpec, image_shape, image_mask=None,
                   th: int = TILE_H, tw: int = TILE_W) -> TileMap:
    """Cut the image into th x tw tiles; per tile, stage the bounding box of the dominant panel's
    source pixels when it fits (<= TILE_STAGE pixels, padded rows <= TILE_LDS words)."""
    P, H, W = spec.frame_shape
    himg, wimg = (int(image_shape[0]), int(image_shape[1]))
    idx = np.asarray(index_map, dtype=np.int64).reshape(himg, wimg).copy()
    if image_mask is not None:
        m = np.asarray(image_mask).reshape(himg, wimg)
        idx[m == 0] = -1                       # masked pixels become gaps: output 0
    nty, ntx = -(-himg // th), -(-wimg // tw)
    tiles = np.zeros((nty * ntx, 8), dtype=np.int32)
    codes = np.full((himg, wimg), -1, dtype=np.int64)
    staged = direct = 0
    ppix = H * W
    for ty in range(nty):
        for tx in range(ntx):
            t = ty * ntx + tx
            ys, xs = slice(ty * th, min(himg, (ty + 1) * th)), slice(tx * tw, min(wimg, (tx + 1) * tw))
            sub = idx[ys, xs]
            valid = sub >= 0
            tiles[t, 0] = -1
            if not valid.any():
                continue
            pan = np.where(valid, sub // ppix, -1)
            dom = int(np.bincount(pan[valid]).argmax())
            sel = pan == dom
            rem = sub[sel] % ppix
            r, c = rem // W, rem % W
            r0, c0 = int(r.min()), int(c.min())
            bh, bw = int(r.max()) - r0 + 1, int(c.max()) - c0 + 1
            csub = codes[ys, xs]
            if bh * bw <= TILE_STAGE and bh * (bw + 1) <= TILE_LDS:
                tiles[t, :5] = (dom, r0, c0, bh, bw)
                csub[sel] = (r - r0) * (bw + 1) + (c - c0)
                other = valid & ~sel
                staged += int(sel.sum())
            else:
                other = valid
            csub[other] = -2 - sub[other]
            direct += int(other.sum())
    if codes.min() < -(2 ** 31):
        raise ValueError("tile map: source index out of int32 range")
    return TileMap((himg, wimg), tiles, codes.astype(np.int32).ravel(), ntx, staged, direct)
