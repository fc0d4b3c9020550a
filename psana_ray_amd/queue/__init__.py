"""Shared-queue implementations: in-process CPU queue (reference semantics) and the sharded
HBM ring endpoint."""
from .cpu_queue import Queue, create_queue, drop_queue, get_queue
from .endpoint import (EndOfStream, FrameItem, QueueClosed, QueueEndpoint, QueueError, QueuePeerError)
from .ring import FrameRing, physical_slots

__all__ = ["Queue", "create_queue", "get_queue", "drop_queue", "EndOfStream", "FrameItem", "QueueClosed",
           "QueueEndpoint", "QueueError", "QueuePeerError", "FrameRing", "physical_slots"]
