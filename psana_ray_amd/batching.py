"""Batches for PyTorch consumers: leased queue frames -> one contiguous tensor (+ metadata).

The reference's consumer gets one frame per actor RPC (psana_ray/data_reader.py:35) and its
architecture figure feeds a "PyTorch Task" (PeakNet, setup.py:11).  A training or inference step
wants ``[B, *frame]`` on the GPU: :func:`collate_items` gathers B leased HBM slots with ONE HIP
launch (csrc/gather.hip; bf16 conversion fused), then releases the slots stream-ordered, so the
ring is recycled while the step runs.  :class:`FrameStream` wraps a :class:`DataReader` as a
``torch.utils.data.IterableDataset`` (use ``DataLoader(stream, batch_size=None)``).
:class:`ShardAssembler` regroups the panel shards of ``--panel_shards`` producers into whole frames.
"""
from __future__ import annotations

import collections
import math
from dataclasses import dataclass
from typing import Callable, Iterator, List, Optional

import torch

from .ops import kernels


@dataclass
class FrameBatch:
    data: torch.Tensor            # [n, *frame_shape] on the consumer's device
    rank: torch.Tensor            # int64 [n]: producer rank (reference item field 0)
    idx: torch.Tensor             # int64 [n]: rank-local event index (field 1)
    gevt: torch.Tensor            # int64 [n]: global event id
    photon_energy: torch.Tensor   # float64 [n]: NaN where the event had none (field 3 = None)

    def __len__(self) -> int:
        return int(self.data.shape[0])

    def items(self):
        """Reference-style ``[rank, idx, data, photon_energy]`` items (views into ``data``)."""
        for i in range(len(self)):
            pe = float(self.photon_energy[i])
            yield [int(self.rank[i]), int(self.idx[i]), self.data[i], None if math.isnan(pe) else pe]


def _meta(items) -> dict:
    def col(f, dt):
        return torch.tensor([f(it) for it in items], dtype=dt)
    return dict(rank=col(lambda it: it.rank, torch.int64), idx=col(lambda it: it.idx, torch.int64),
                gevt=col(lambda it: it.gevt, torch.int64),
                photon_energy=col(lambda it: float("nan") if it.photon_energy is None else it.photon_energy,
                                  torch.float64))


def collate_items(items: List, dtype: torch.dtype = torch.float32, stream=None, release: bool = True,
                  calibrate: Optional[Callable] = None) -> FrameBatch:
    """Gather leased :class:`~psana_ray_amd.queue.endpoint.FrameItem` s into a new batch tensor.
    ``calibrate(items) -> [n, ...] f32`` handles raw (``--calibrate_on_read``) rings."""
    meta = _meta(items)
    if calibrate is not None:
        data = calibrate(items)            # releases the raw slots itself
        data = data if data.dtype == dtype else data.to(dtype)
        return FrameBatch(data=data, **meta)
    frames = [it.data for it in items]
    shape = tuple(frames[0].shape)
    dev = frames[0].device
    out = torch.empty((len(frames), *shape), dtype=dtype, device=dev)
    if dev.type == "cuda" and frames[0].dtype == torch.float32:
        kernels.gather_frames(frames, out, stream)
    else:                                  # host rings (CPU queues / tests) or raw u16 frames
        torch.stack(frames, out=out) if frames[0].dtype == dtype else out.copy_(torch.stack(frames))
    if release:
        for it in items:
            it.release(stream)             # slot reusable once the gather on `stream` ran
    return FrameBatch(data=out, **meta)


class FrameStream(torch.utils.data.IterableDataset):
    """``IterableDataset`` of :class:`FrameBatch` es read from a queue session.

    ``reader_kwargs`` go to :class:`~psana_ray_amd.data_reader.DataReader`; the reader connects
    lazily in ``__iter__`` (so the dataset can be built before the producers start) and closes
    at the end of the stream.  Single-process iteration only (one reader per consumer rank)."""

    def __init__(self, batch_size: int = 16, dtype: torch.dtype = torch.float32, max_batches: Optional[int] = None,
                 timeout: float = 1.0, drop_last: bool = False, **reader_kwargs):
        super().__init__()
        self.batch_size, self.dtype, self.max_batches = batch_size, dtype, max_batches
        self.timeout, self.drop_last = timeout, drop_last
        self.reader_kwargs = reader_kwargs

    def __iter__(self) -> Iterator[FrameBatch]:
        from .data_reader import DataReader

        with DataReader(**self.reader_kwargs) as reader:
            for k, b in enumerate(reader.batches(self.batch_size, self.dtype, self.timeout, self.drop_last)):
                if self.max_batches is not None and k >= self.max_batches:
                    break
                yield b


@dataclass
class AssembledFrame:
    gevt: int                     # global event id (shared by every shard of the event)
    data: torch.Tensor            # [n_panels, H, W]: the whole frame
    photon_energy: Optional[float]


class ShardAssembler:
    """Regroup panel shards (``--panel_shards G`` producers, source/shard.py) into whole frames.

    Shard ``s = item.rank % G`` of event ``item.gevt`` holds panels ``[s*P/G, (s+1)*P/G)``.  Every
    :meth:`add` copies its shards into their events' pending frames with ONE gather launch
    (csrc/gather.hip, destinations = panel ranges of the frames) and releases the ring slots at
    once, so incomplete events never pin queue slots.  Complete frames are returned in arrival
    order.  A consumer sees every shard of an event when it is the only consumer (or the shards
    are routed to it); ``max_pending`` bounds the frames waiting for missing shards."""

    def __init__(self, n_shards: int, shard_shape, device=None, dtype: torch.dtype = torch.float32,
                 max_pending: int = 256):
        if n_shards < 1:
            raise ValueError("n_shards must be >= 1")
        self.n_shards = int(n_shards)
        self.shard_shape = tuple(int(x) for x in shard_shape)
        self.frame_shape = (self.shard_shape[0] * self.n_shards, *self.shard_shape[1:])
        self.device = None if device is None else torch.device(device)
        self.dtype = dtype
        self.max_pending = int(max_pending)
        self._pending: "collections.OrderedDict[int, list]" = collections.OrderedDict()
        self._full = (1 << self.n_shards) - 1

    @property
    def pending(self) -> int:
        return len(self._pending)

    def add(self, items: List, stream=None) -> List[AssembledFrame]:
        if not items:
            return []
        per = self.shard_shape[0]
        srcs, dsts = [], []
        for it in items:
            if tuple(it.data.shape) != self.shard_shape:
                raise ValueError(f"shard of shape {tuple(it.data.shape)}, expected {self.shard_shape}")
            s = int(it.rank) % self.n_shards
            e = self._pending.get(int(it.gevt))
            if e is None:
                if len(self._pending) >= self.max_pending:
                    raise RuntimeError(f"{len(self._pending)} events wait for missing panel shards: are the "
                                       f"shards routed to another consumer?")
                dev = self.device or it.data.device
                e = [torch.empty(self.frame_shape, dtype=self.dtype, device=dev), 0, it.photon_energy]
                self._pending[int(it.gevt)] = e
            if e[1] >> s & 1:
                raise ValueError(f"duplicate shard {s} of event {it.gevt}")
            e[1] |= 1 << s
            srcs.append(it.data)
            dsts.append(e[0][s * per:(s + 1) * per])
        if srcs[0].device.type == "cuda" and srcs[0].dtype == torch.float32 and \
                all(d.device == srcs[0].device for d in dsts):
            kernels.gather_frames(srcs, dsts, stream)
        else:
            for a, d in zip(srcs, dsts):
                d.copy_(a, non_blocking=True)
        for it in items:
            it.release(stream)
        done = [g for g, e in self._pending.items() if e[1] == self._full]
        return [AssembledFrame(g, *self._pop(g)) for g in done]

    def _pop(self, g):
        e = self._pending.pop(g)
        return e[0], e[2]
