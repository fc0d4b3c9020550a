"""roctx ranges from Python (consumer batches) next to the native ones
(``producer.chunk`` / ``producer.stage_h2d`` / ``producer.acquire`` / ``producer.launch_calib``,
csrc/engine.cpp).  View them with ``rocprofv3 --marker-trace --kernel-trace -- python ...``.

The reference has no tracing; ranges cost one native call each and are skipped
entirely when the roctx library is absent or ``PSANA_RAY_ROCTX=0``.
"""
from __future__ import annotations

import contextlib

_C = None
_ON = None


def _api():
    global _C, _ON
    if _ON is None:
        try:
            from ..ops import _ext

            _C = _ext.load(build_if_missing=False)
            _ON = bool(_C.roctx_enabled())
        except Exception:  # noqa: BLE001 - tracing is optional
            _C, _ON = None, False
    return _C if _ON else None


def enabled() -> bool:
    return _api() is not None


@contextlib.contextmanager
def trace_range(name: str):
    c = _api()
    if c is None:
        yield
        return
    c.roctx_push(name)
    try:
        yield
    finally:
        c.roctx_pop()


def mark(name: str) -> None:
    c = _api()
    if c is not None:
        c.roctx_mark(name)
