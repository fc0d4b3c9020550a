"""Optional adapter over the real ``psana_wrapper`` (E-01), used only when it is importable.

The reference constructs ``PsanaWrapperSmd(exp=..., run=..., detector_name=...)`` and iterates
``iter_events(mode=ImageRetrievalMode.calib|image)`` (psana_ray/producer.py:150-159).  psana
calibrates on the CPU, so frames from this source are already calibrated: the producer
uploads them (pinned -> hipMemcpyAsync) and skips the HIP calibration kernels.  Neither psana
nor psana_wrapper exists in this environment: this path is import-gated and
its parity is unpinned.
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import numpy as np

from ..models.detector import Mode


def psana_available() -> bool:
    try:
        import psana_wrapper  # noqa: F401

        return True
    except Exception:
        return False


class PsanaWrapperSource:
    calibrated = True

    def __init__(self, exp: str, run: int, detector_name: str):
        from psana_wrapper import ImageRetrievalMode, PsanaWrapperSmd  # type: ignore

        self._mode_enum = ImageRetrievalMode
        self.wrapper = PsanaWrapperSmd(exp=exp, run=run, detector_name=detector_name)

    def create_bad_pixel_mask(self) -> np.ndarray:
        return self.wrapper.create_bad_pixel_mask()

    def seek(self, start_event: int) -> int:
        """Skip this rank's first ``start_event`` events (psana shards inside its SMD reader)."""
        self._skip = max(0, int(start_event))
        return self._skip

    def iter_events(self, mode: Mode) -> Iterator[Tuple[np.ndarray, Optional[float]]]:
        import itertools

        m = self._mode_enum.calib if Mode(mode) == Mode.calib else self._mode_enum.image
        return itertools.islice(self.wrapper.iter_events(mode=m), getattr(self, "_skip", 0), None)
