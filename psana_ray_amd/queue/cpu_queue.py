"""In-process bounded queue with the exact semantics of the reference's Ray actor ``Queue``.

Reference: psana_ray/shared_queue.py:4-31 -- ``deque(maxlen=maxsize)``; ``put`` appends only while
``len < maxlen`` and returns True, else False (backpressure, NOT drop-oldest, Q-4); ``get`` is
non-blocking ``popleft`` or None; ``size`` returns the length; every method swallows errors
(prints, returns False / None / 0).  ``create_queue`` (:33-38) creates a named queue in a
namespace; here the name registry is process-local and attach-if-exists (Q-5, the reference's
``ray.get_actor`` reuse at psana_ray/producer.py:43-45).

This is BASELINE config 1's queue (synthetic 256x256 frames, 1 producer + 1 consumer, no GPU)
and the unit-test model of the queue contract.  Unlike the single-threaded actor it is safe for
concurrent threads (a lock guards the deque) and it optionally supports an explicit
end-of-stream marker distinct from "empty" (fixes Q-2).
"""
from __future__ import annotations

import threading
from collections import deque
from typing import Any, Dict, Optional, Tuple

from ..config import DEFAULT_QUEUE_SIZE


class Queue:
    def __init__(self, maxsize: int = DEFAULT_QUEUE_SIZE):
        self.items: deque = deque(maxlen=maxsize)
        self._lock = threading.Lock()
        self._not_empty = threading.Condition(self._lock)
        self._not_full = threading.Condition(self._lock)

    @property
    def maxsize(self) -> int:
        return self.items.maxlen

    def put(self, item: Any) -> bool:
        try:
            with self._lock:
                if len(self.items) < self.items.maxlen:
                    self.items.append(item)
                    self._not_empty.notify()
                    return True
                return False
        except Exception as e:  # reference: print + False (shared_queue.py:15-17)
            print(f"Error in put: {e}")
            return False

    def get(self, timeout: Optional[float] = None) -> Any:
        """Non-blocking by default (None when empty, shared_queue.py:19-24); ``timeout`` > 0
        waits up to that long for an item (event-driven, replaces the consumer's 1 s poll)."""
        try:
            with self._lock:
                if not self.items and timeout:
                    self._not_empty.wait_for(lambda: bool(self.items), timeout=timeout)
                if not self.items:
                    return None
                item = self.items.popleft()
                self._not_full.notify()
                return item
        except Exception as e:
            print(f"Error in get: {e}")
            return None

    def wait_not_full(self, timeout: Optional[float] = None) -> bool:
        """Block until a ``put`` could succeed (event-driven replacement of the producer's
        exponential backoff, producer.py:105-111).  Returns False on timeout."""
        with self._lock:
            return self._not_full.wait_for(lambda: len(self.items) < self.items.maxlen, timeout=timeout)

    def size(self) -> int:
        try:
            with self._lock:
                return len(self.items)
        except Exception as e:
            print(f"Error in size: {e}")
            return 0


_REGISTRY: Dict[Tuple[str, str], Queue] = {}
_REG_LOCK = threading.Lock()


def create_queue(queue_name: str = "shared_queue", ray_namespace: str = "default",
                 maxsize: int = DEFAULT_QUEUE_SIZE) -> Optional[Queue]:
    """Create (or attach to) the named in-process queue; None on error (shared_queue.py:33-38).
    The reference's function defaults are kept: ``'shared_queue'`` / ``'default'`` / 100."""
    try:
        with _REG_LOCK:
            key = (ray_namespace, queue_name)
            q = _REGISTRY.get(key)
            if q is None:
                q = _REGISTRY[key] = Queue(maxsize=maxsize)
            return q
    except Exception as e:
        print(f"Error creating queue '{queue_name}' in namespace '{ray_namespace}': {e}")
        return None


def get_queue(queue_name: str, ray_namespace: str) -> Queue:
    """``ray.get_actor`` analog: raises ValueError when the queue does not exist."""
    with _REG_LOCK:
        q = _REGISTRY.get((ray_namespace, queue_name))
    if q is None:
        raise ValueError(f"queue {queue_name!r} not found in namespace {ray_namespace!r}")
    return q


def drop_queue(queue_name: str, ray_namespace: str) -> None:
    with _REG_LOCK:
        _REGISTRY.pop((ray_namespace, queue_name), None)
