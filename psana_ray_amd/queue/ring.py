"""HBM frame ring: one rank's shard of the shared queue (storage tensor + native SlotPool).

Replaces the reference's ``deque(maxlen=maxsize)`` inside the Ray actor
(psana_ray/shared_queue.py:6-7).  Slots are preallocated once in device memory (HBM3E) and
recycled, so steady-state streaming performs no allocation; frames are written in place by the
calibration kernels (local producer) or by RCCL receives (remote producer).  The slot state
machine, per-slot HIP events and blocking waits live in C++ (``_C.SlotPool``).

Capacity (SURVEY H-8): ``queue_size`` is the LOGICAL bound of the whole queue (the reference
never preallocates); physical slots per shard = min(share of queue_size, what fits in
``hbm_fraction`` of free device memory).  E.g. Jungfrau-16M f32 frames (67 MB) fit ~3.8k slots
in 288 GB, so queue_size=400000 is honoured as a bound, not as storage.
"""
from __future__ import annotations

import logging
import math
from typing import Optional, Tuple

import torch

from ..ops import _ext

log = logging.getLogger(__name__)


def physical_slots(logical_share: int, frame_bytes: int, device: torch.device, hbm_fraction: float,
                   reserve_slots: int = 0) -> int:
    """Slots that honour ``logical_share`` but fit in ``hbm_fraction`` of free memory."""
    if device.type != "cuda":
        return max(1, logical_share)
    free, _total = torch.cuda.mem_get_info(device)
    fit = int(free * hbm_fraction) // max(1, frame_bytes) - reserve_slots
    if fit < 1:
        raise MemoryError(f"not even one {frame_bytes}-byte frame slot fits in device memory")
    if fit < logical_share:
        log.warning("queue share %d slots capped to %d by HBM (%.1f GB free x %.2f)", logical_share, fit,
                    free / 1e9, hbm_fraction)
    return max(1, min(logical_share, fit))


class FrameRing:
    def __init__(self, frame_shape: Tuple[int, ...], dtype: torch.dtype, device, producer_slots: int,
                 consumer_slots: int):
        C = _ext.load()
        self.device = torch.device(device)
        self.frame_shape = tuple(frame_shape)
        self.dtype = dtype
        n = producer_slots + consumer_slots
        if n <= 0:
            raise ValueError("ring needs at least one slot")
        self.storage = torch.empty((n, *self.frame_shape), dtype=dtype, device=self.device)
        dev_index = -1
        if self.device.type == "cuda":
            dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.pool = C.SlotPool(producer_slots, consumer_slots, dev_index)
        self.frame_bytes = int(math.prod(self.frame_shape)) * self.storage.element_size()

    @property
    def n_slots(self) -> int:
        return self.pool.n_slots

    def slot(self, i: int) -> torch.Tensor:
        return self.storage[i]

    def stats(self) -> dict:
        s = self.pool.stats()
        return dict(produced=s.produced, routed_local=s.routed_local, sent=s.sent, received=s.received,
                    got=s.got, released=s.released, produce_full=s.produce_full,
                    ready=self.pool.n_ready(), consumer_held=self.pool.consumer_held(),
                    producer_held=self.pool.producer_held())
