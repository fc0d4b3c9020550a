"""Shared-queue API parity module (reference: psana_ray/shared_queue.py).

* :class:`Queue` / :func:`create_queue` -- the reference's bounded queue contract, in process
  (``put`` -> bool backpressure, non-blocking ``get`` -> item or None, ``size``); BASELINE config 1.
* The distributed queue of a producer job is the sharded HBM ring
  (:class:`~psana_ray_amd.queue.endpoint.QueueEndpoint`): created by ``psana-ray-producer`` rank 0
  at the rendezvous store and read through :class:`~psana_ray_amd.data_reader.DataReader`.
"""
from .queue.cpu_queue import Queue, create_queue, drop_queue, get_queue
from .queue.endpoint import EndOfStream, QueueClosed, QueueEndpoint, QueuePeerError
from .queue.ring import FrameRing

__all__ = ["Queue", "create_queue", "get_queue", "drop_queue", "QueueEndpoint", "FrameRing", "EndOfStream",
           "QueueClosed", "QueuePeerError"]
