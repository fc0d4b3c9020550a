"""HBM frame ring: one rank's shard of the shared queue (storage tensor + native SlotPool).

Replaces the reference's ``deque(maxlen=maxsize)`` inside the Ray actor
(psana_ray/shared_queue.py:6-7).  Slots are preallocated once in device memory (HBM3E) and
recycled, so steady-state streaming performs no allocation; frames are written in place by the
calibration kernels (local producer) or by a remote producer's peer copy into a granted slot
(queue fabric, csrc/fabric.cpp).  The slot state
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
    fit = int(free * hbm_fraction) // max(1, slot_stride(frame_bytes)) - reserve_slots
    if fit < 1:
        raise MemoryError(f"not even one {frame_bytes}-byte frame slot fits in device memory")
    if fit < logical_share:
        log.warning("queue share %d slots capped to %d by HBM (%.1f GB free x %.2f)", logical_share, fit,
                    free / 1e9, hbm_fraction)
    return max(1, min(logical_share, fit))


SEGMENT_BYTES = 1 << 30   # HBM rings are built from allocations of at most 1 GiB (HIP IPC limit, see below)
# Slot stride alignment: every slot starts on a 256-B boundary whatever the frame size (the kernels
# and the fabric's copy kernel move 16-B words; an assembled image of H * W pixels with H * W not a
# multiple of 4 -- psana's pix_rows.max() + 1 geometries -- would otherwise misalign every other slot).
SLOT_ALIGN = 256


def slot_stride(frame_bytes: int) -> int:
    return -(-int(frame_bytes) // SLOT_ALIGN) * SLOT_ALIGN


class FrameRing:
    """``producer_slots + consumer_slots`` frame slots plus their native :class:`SlotPool`.

    HBM rings are NOT one tensor: they are made of segments of at most ``SEGMENT_BYTES``, each its
    own ``hipMalloc`` (``_C.DeviceBuffer``, wrapped zero-copy with DLPack).  A consumer exports
    every segment to producer processes as a HIP IPC handle, and opening the handle of an
    allocation above 2 GiB hangs on this ROCm stack (profiles/r2/ipc_attach.md: 2.08 GB attaches in
    0.2 ms, 2.16 GB never returns).  The pool knows every slot's address (``slot_ptrs``), so
    kernels, copies and the fabric never assume one contiguous ring.  Host rings are one region:
    named shared memory when producer processes must write into them (``shm_name``)."""

    def __init__(self, frame_shape: Tuple[int, ...], dtype: torch.dtype, device, producer_slots: int,
                 consumer_slots: int, shm_name: Optional[str] = None, segment_bytes: int = SEGMENT_BYTES):
        C = _ext.load()
        self.device = torch.device(device)
        self.frame_shape = tuple(frame_shape)
        self.dtype = dtype
        n = producer_slots + consumer_slots
        if n <= 0:
            raise ValueError("ring needs at least one slot")
        esz = torch.empty((), dtype=dtype).element_size()
        self.frame_bytes = int(math.prod(self.frame_shape)) * esz
        # slot stride (SLOT_ALIGN): the frame is a prefix of its slot; the fabric moves whole slots
        self.slot_bytes = slot_stride(self.frame_bytes)
        sb = self.slot_bytes
        self.shm_name = shm_name if self.device.type == "cpu" else None
        self._region = None
        self._buffers = []
        self.segments = []     # (flat uint8 tensor [k * slot_bytes], first slot, k)
        dev_index = -1
        if self.device.type == "cpu":
            if self.shm_name is not None:
                # a host consumer's shard lives in named shared memory so producer processes write into it
                self._region = C.ShmRegion(self.shm_name, n * sb, True)
                flat = torch.frombuffer(self._region, dtype=torch.uint8)
            else:
                flat = torch.empty(n * sb, dtype=torch.uint8)
            self.segments.append((flat, 0, n))
        else:
            dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
            per = max(1, int(segment_bytes) // sb)
            for first in range(0, n, per):
                k = min(per, n - first)
                buf = C.DeviceBuffer(k * sb, dev_index)
                self._buffers.append(buf)
                self.segments.append((torch.from_dlpack(buf), first, k))
        # HBM rings start zeroed: slots only ever receive whole frames of the session's shape, so
        # pixels no kernel writes (the panel gaps of an assembled image) stay 0 in every slot and the
        # producer engine skips their per-frame fill (``zero_filled``; ProducerPipeline)
        self.zero_filled = False
        if self.device.type == "cuda":
            for t, _, _ in self.segments:
                t.zero_()
            torch.cuda.synchronize(self.device)
            self.zero_filled = True
        fb = self.frame_bytes
        self.views = [t[j * sb:j * sb + fb].view(dtype).view(self.frame_shape)
                      for t, _, k in self.segments for j in range(k)]
        self.slot_ptrs = [int(v.data_ptr()) for v in self.views]
        self.pool = C.SlotPool(producer_slots, consumer_slots, dev_index)
        self.pool.set_slot_ptrs(self.slot_ptrs)

    @property
    def n_slots(self) -> int:
        return self.pool.n_slots

    @property
    def nbytes(self) -> int:
        return self.n_slots * self.slot_bytes

    def slot(self, i: int) -> torch.Tensor:
        return self.views[i]

    def stats(self) -> dict:
        s = self.pool.stats()
        return dict(produced=s.produced, routed_local=s.routed_local, sent=s.sent, received=s.received,
                    got=s.got, released=s.released, produce_full=s.produce_full,
                    ready=self.pool.n_ready(), consumer_held=self.pool.consumer_held(),
                    producer_held=self.pool.producer_held())
