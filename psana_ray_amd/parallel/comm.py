"""Communication backends of the sharded shared queue.

Two process groups over the SAME ranks (one process per GPU):
  * control group -- gloo on the CPU: one small all-gather per transport round carries every
    rank's (offers, credits, flags, frame headers).  Keeping it off the GPU means a round's
    routing never waits behind the previous round's frame transfers.
  * data group    -- ``nccl`` (= RCCL over xGMI on MI355X) for HBM frames, or gloo for host
    frames (CPU tests / BASELINE config 1 over processes).  Frames move with grouped
    ``isend``/``irecv`` (``batch_isend_irecv`` -> one ncclGroupStart/End per round) issued on a
    dedicated HIP stream; completion is stream-ordered (no host sync).

This replaces the reference's data plane -- a synchronous Ray actor RPC per frame through the
object store (psana_ray/producer.py:101, data_reader.py:35; C-01/C-03) -- and its MPI control
plane (Barriers at producer.py:53,120; C-05/C-06).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist


class Comm:
    def __init__(self, rank: int, world: int, ctrl_group, data_group, device: torch.device):
        self.rank = rank
        self.world = world
        self.ctrl_group = ctrl_group
        self.data_group = data_group
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.device) if self.gpu else None
        self.bytes_sent = 0
        self.bytes_recv = 0

    def allgather_ctrl(self, vec: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(np.ascontiguousarray(vec, dtype=np.int64))
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.ctrl_group)
        return torch.stack(out).numpy()

    def exchange(self, sends: Sequence[Tuple[torch.Tensor, int, int]], recvs: Sequence[Tuple[torch.Tensor, int, int]]):
        """Issue all (tensor, peer, tag) sends and receives of a round as one group.

        GPU: ops are enqueued on ``self.stream``; on return that stream is ordered after their
        completion (``work.wait()`` is a stream dependency for NCCL), so callers record events
        on ``self.stream``.  CPU/gloo: returns after completion."""
        self.bytes_sent += sum(t.numel() * t.element_size() for t, _, _ in sends)
        self.bytes_recv += sum(t.numel() * t.element_size() for t, _, _ in recvs)
        if not self.gpu:
            # gloo has no send-to-self: loopback pairs (matched in order, like RCCL) are copies
            own_s = [t for t, peer, _ in sends if peer == self.rank]
            own_r = [t for t, peer, _ in recvs if peer == self.rank]
            if len(own_s) != len(own_r):
                raise RuntimeError("loopback exchange: unmatched self send/recv")
            for a, b in zip(own_s, own_r):
                b.copy_(a)
            sends = [x for x in sends if x[1] != self.rank]
            recvs = [x for x in recvs if x[1] != self.rank]
        ops = [dist.P2POp(dist.isend, t, peer, group=self.data_group, tag=tag) for t, peer, tag in sends]
        ops += [dist.P2POp(dist.irecv, t, peer, group=self.data_group, tag=tag) for t, peer, tag in recvs]
        if not ops:
            return
        if self.gpu:
            with torch.cuda.stream(self.stream):
                works = dist.batch_isend_irecv(ops)
                for w in works:
                    w.wait()
        else:
            works = dist.batch_isend_irecv(ops)
            for w in works:
                w.wait()

    @property
    def stream_handle(self) -> int:
        return int(self.stream.cuda_stream) if self.gpu else 0


def init_groups(rank: int, world: int, device, store=None, master_addr: Optional[str] = None,
                master_port: Optional[int] = None, timeout_s: float = 600.0):
    """Create (or reuse) the default process group and the control/data groups.

    GPU device -> default group ``nccl`` (bound to the device: eager communicator init) plus a
    gloo control group; CPU -> gloo for both.  Returns a :class:`Comm`.
    """
    import datetime

    device = torch.device(device)
    gpu = device.type == "cuda"
    tmo = datetime.timedelta(seconds=timeout_s)
    if not dist.is_initialized():
        kw = dict(rank=rank, world_size=world, timeout=tmo)
        if store is not None:
            kw["store"] = store
        elif master_addr is not None:
            kw["init_method"] = f"tcp://{master_addr}:{master_port}"
        if gpu:
            torch.cuda.set_device(device)
            dist.init_process_group("nccl", device_id=device, **kw)
        else:
            dist.init_process_group("gloo", **kw)
    if gpu:
        data = dist.group.WORLD
        ctrl = dist.new_group(backend="gloo", timeout=tmo)
        # first collective on the data group involves every rank (batch_isend_irecv requirement)
        t = torch.ones(1, device=device)
        dist.all_reduce(t, group=data)
        torch.cuda.synchronize(device)
    else:
        data = dist.group.WORLD
        ctrl = dist.new_group(backend="gloo", timeout=tmo)
    return Comm(rank, world, ctrl, data, device)
