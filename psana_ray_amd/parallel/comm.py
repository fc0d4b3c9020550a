"""Communication backends of the sharded shared queue.

Two planes over the SAME ranks (one process per GPU):
  * control -- a gloo process group on the CPU: one small all-gather per transport round carries
    every rank's (offers, credits, flags, frame headers).  Keeping it off the GPU means a round's
    routing never waits behind the previous round's frame transfers.
  * data    -- on GPUs a native RCCL communicator (csrc/transport.cpp; id broadcast over the
    control group): a round's frames move as ONE ncclGroupStart/End of ncclSend/ncclRecv on a
    dedicated HIP stream, slot bookkeeping and event ordering included, in a single native call
    with the GIL released (the first version used torch ``batch_isend_irecv``: ~1 torch P2POp
    per frame in Python capped a round at ~10k frames/s).  On the CPU (tests / BASELINE config 1
    over processes) gloo ``isend``/``irecv`` of host tensors.

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
    def __init__(self, rank: int, world: int, ctrl_group, data_group, device: torch.device, rccl=None,
                 node_local: bool = False, token: str = "", owns_default_group: bool = False):
        self.rank = rank
        # True when init_groups created the default process group: only then may the owner of this
        # Comm destroy it (reference quirk Q-13: DataReader.close() shut Ray down even when the
        # caller had initialised it, psana_ray/data_reader.py:26-29)
        self.owns_default_group = bool(owns_default_group)
        self.world = world
        # every rank on this host: the native transport engine (csrc/xport_engine.h) can run the
        # control plane through shared memory instead of gloo
        self.node_local = bool(node_local)
        self.token = token
        self._n_shm = 0
        self.ctrl_group = ctrl_group
        self.data_group = data_group
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.rccl = rccl
        self.stream = torch.cuda.Stream(device=self.device) if self.gpu else None
        self._bytes_sent = 0
        self._bytes_recv = 0

    @property
    def bytes_sent(self) -> int:
        return int(self.rccl.bytes_sent) if self.rccl is not None else self._bytes_sent

    @property
    def bytes_recv(self) -> int:
        return int(self.rccl.bytes_recv) if self.rccl is not None else self._bytes_recv

    def round(self, pool, ring_base: int, slot_bytes: int, send_slots, send_peers, recv_peers, recv_headers):
        """GPU: one fused native transport round (see csrc/transport.h).  Returns the recv slots."""
        return self.rccl.round(pool, ring_base, slot_bytes, send_slots, send_peers, recv_peers, recv_headers,
                               self.stream_handle)

    def shm_name(self) -> str:
        """A fresh node-local segment name, identical on every rank (endpoints are created in the
        same order on every rank of a session)."""
        self._n_shm += 1
        return f"/psray-{self.token}-{self._n_shm}"

    def check_async(self) -> None:
        if self.rccl is not None:
            err = self.rccl.async_error()
            if err:
                raise RuntimeError(f"RCCL asynchronous error: {err}")

    def abort(self) -> None:
        """Drop the data communicator without waiting for peers (after a failure)."""
        if self.rccl is not None:
            self.rccl.abort()

    def close(self) -> None:
        if self.rccl is not None:
            r, self.rccl = self.rccl, None
            del r   # ncclCommDestroy (waits for this rank's outstanding work only)

    def allgather_ctrl(self, vec: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(np.ascontiguousarray(vec, dtype=np.int64))
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.ctrl_group)
        return torch.stack(out).numpy()

    def exchange(self, sends: Sequence[Tuple[torch.Tensor, int, int]], recvs: Sequence[Tuple[torch.Tensor, int, int]]):
        """Issue all (tensor, peer, tag) sends and receives of a round as one group.

        GPU (RCCL): enqueued on ``self.stream``; callers order their events after that stream.
        All tensors of one call must have the same byte size.  CPU/gloo: returns after completion."""
        if self.rccl is not None:
            nb = {t.numel() * t.element_size() for t, _, _ in list(sends) + list(recvs)}
            if not nb:
                return
            if len(nb) != 1:
                raise ValueError("RCCL exchange: all messages of a round must have the same size")
            self.rccl.exchange([int(t.data_ptr()) for t, _, _ in sends], [int(p) for _, p, _ in sends],
                               [int(t.data_ptr()) for t, _, _ in recvs], [int(p) for _, p, _ in recvs],
                               nb.pop(), self.stream_handle)
            return
        self._bytes_sent += sum(t.numel() * t.element_size() for t, _, _ in sends)
        self._bytes_recv += sum(t.numel() * t.element_size() for t, _, _ in recvs)
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
        works = dist.batch_isend_irecv(ops)
        for w in works:
            w.wait()

    @property
    def stream_handle(self) -> int:
        return int(self.stream.cuda_stream) if self.gpu else 0


def init_groups(rank: int, world: int, device, store=None, master_addr: Optional[str] = None,
                master_port: Optional[int] = None, timeout_s: float = 600.0):
    """Create (or reuse) the default gloo process group (control plane) and, on a GPU, the native
    RCCL communicator of the data plane.  Returns a :class:`Comm`."""
    import datetime

    device = torch.device(device)
    gpu = device.type == "cuda"
    tmo = datetime.timedelta(seconds=timeout_s)
    if gpu:
        torch.cuda.set_device(device)
    owns = not dist.is_initialized()
    if not owns and (dist.get_rank(), dist.get_world_size()) != (rank, world):
        raise RuntimeError(f"an existing default process group (rank {dist.get_rank()} of {dist.get_world_size()}) "
                           f"does not match the queue world (rank {rank} of {world})")
    if owns:
        kw = dict(rank=rank, world_size=world, timeout=tmo)
        if store is not None:
            kw["store"] = store
        elif master_addr is not None:
            kw["init_method"] = f"tcp://{master_addr}:{master_port}"
        dist.init_process_group("gloo", **kw)
    ctrl = dist.new_group(backend="gloo", timeout=tmo)
    # node locality + a session token for shared-memory names (one small exchange at startup)
    import socket
    import uuid

    here = [socket.gethostname(), _boot_id()]
    hosts = [None] * world
    dist.all_gather_object(hosts, here, group=ctrl)
    tok = [uuid.uuid4().hex[:12] if rank == 0 else None]
    dist.broadcast_object_list(tok, src=0, group=ctrl)
    node_local = all(h == here for h in hosts)
    rccl = None
    if gpu:
        from ..ops import _ext

        C = _ext.load()
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            uid = torch.frombuffer(bytearray(C.rccl_unique_id()), dtype=torch.uint8).clone()
        dist.broadcast(uid, src=0, group=ctrl)
        dev_index = device.index if device.index is not None else torch.cuda.current_device()
        rccl = C.RcclTransport(bytes(uid.numpy().tobytes()), rank, world, dev_index)
    return Comm(rank, world, ctrl, dist.group.WORLD, device, rccl=rccl, node_local=node_local, token=tok[0],
                owns_default_group=owns)


def _boot_id() -> str:
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            return f.read().strip()
    except OSError:
        return ""
