"""Panel sharding: one detector frame split over several producer ranks (SURVEY P-04 / §5.7).

The reference moves whole frames only: every rank ships complete ``(panels, H, W)`` arrays
through the Ray object store (psana_ray/producer.py:88-101).  For Jungfrau-16M-scale frames
(32 x 512 x 1024: 33.5 MB raw, 67 MB calibrated) the frame itself is the "long context": one
rank's PCIe link needs 0.6 ms to stage it, and one consumer shard holds it whole.  With
``--panel_shards G`` the producer ranks form groups of G; the ranks of a group walk the SAME
events (events are sharded over groups, P-01) and each stages, calibrates and queues only its
``n_panels / G`` panels:

* the H2D copy per rank is 1/G of the frame (G PCIe links per frame instead of one),
* calibration and common mode are per ASIC, so a panel subset is calibrated by the unchanged
  kernels on a sub-detector (:meth:`DetectorSpec.panel_subset`) -- bit-identical to the
  corresponding panels of the whole-frame result,
* every queue item is one panel shard: its header keeps the producer rank (shard = rank % G)
  and the global event id; :class:`~psana_ray_amd.batching.ShardAssembler` regroups shards
  into whole frames when a consumer wants them (one gather launch per batch).

:class:`PanelShardSource` wraps any raw event source (synthetic, raw-run file, XTC2) opened
with the GROUP as its rank; calibrated sources (real psana) are sliced on the host.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from ..models.detector import Mode, panel_shard_range
from .synthetic import RawEvent


def shard_layout(rank: int, size: int, n_shards: int):
    """(group, n_groups, shard) of ``rank`` when ``size`` ranks split frames ``n_shards`` ways."""
    if n_shards < 1 or size % n_shards:
        raise ValueError(f"--panel_shards {n_shards} must divide the number of producer ranks ({size})")
    return rank // n_shards, size // n_shards, rank % n_shards


class PanelShardSource:
    """Panels ``[lo, hi)`` of every event of ``inner`` (which shards events over rank groups)."""

    def __init__(self, inner, shard: int, n_shards: int):
        self.inner = inner
        full = inner.spec
        self.n_shards, self.shard = int(n_shards), int(shard)
        self.lo, self.hi = panel_shard_range(full.n_panels, self.shard, self.n_shards)
        self.full_spec = full
        self.spec = full.panel_subset(self.lo, self.hi)
        self.consts = inner.consts.panel_subset(self.lo, self.hi) if hasattr(inner, "consts") else None
        self._off = self.lo * full.panel_pixels * 2          # byte offset of the shard in a raw frame
        self.exp, self.run = getattr(inner, "exp", None), getattr(inner, "run", None)
        self.detector_name = getattr(inner, "detector_name", full.name)
        self.event_rank = int(getattr(inner, "rank", 0))     # the group: gevt = group + k * n_groups
        self.rank = self.event_rank
        self.size = int(getattr(inner, "size", 1))
        self.calibrated = bool(getattr(inner, "calibrated", False))
        # expose exactly the capabilities of the wrapped source (the pipeline probes with hasattr)
        if hasattr(inner, "cycled_frames"):
            self.cycled_frames = self._cycled_frames
        if hasattr(inner, "zero_copy_frames"):
            self.zero_copy_frames = self._zero_copy_frames
        if hasattr(inner, "n_staging"):
            self.n_staging = inner.n_staging
        if hasattr(inner, "seek"):
            self.seek = inner.seek
        # NOTE: no `reader` attribute: the native pread path stages whole records; shards of a
        # file source use the zero-copy mapping or the Python staging path

    # ---- reference surface -------------------------------------------------------------
    def create_bad_pixel_mask(self) -> np.ndarray:
        return np.asarray(self.inner.create_bad_pixel_mask())[self.lo:self.hi]

    def n_local_events(self) -> Optional[int]:
        f = getattr(self.inner, "n_local_events", None)
        return f() if f is not None else None

    @property
    def cursor(self) -> int:
        return int(getattr(self.inner, "cursor", 0))

    @property
    def _map(self):
        return getattr(self.inner, "_map", None)

    def _shift(self, ptrs):
        return [int(p) + self._off for p in ptrs]

    def _cycled_frames(self):
        ptrs, pe = self.inner.cycled_frames()
        return self._shift(ptrs), pe

    def _zero_copy_frames(self):
        z = self.inner.zero_copy_frames()
        if z is None:
            return None
        ptrs, pe = z
        return self._shift(ptrs), pe

    def next_events(self, n: int) -> List[RawEvent]:
        return [RawEvent(e.gevt, e.idx, e.raw[self.lo:self.hi], int(e.host_ptr) + self._off, e.photon_energy)
                for e in self.inner.next_events(n)]

    def iter_events(self, mode=Mode.calib):
        mode = Mode(mode.value if hasattr(mode, "value") else mode)
        if mode == Mode.image:
            raise ValueError("panel shards carry per-panel data: use --calib (or raw); image assembly needs "
                             "every panel of the frame")
        for data, pe in self.inner.iter_events(mode):
            yield np.asarray(data)[self.lo:self.hi], pe
