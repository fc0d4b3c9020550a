"""Event sources: synthetic detector, raw-run files (native reader), optional psana adapter."""
from __future__ import annotations

import os
from typing import Optional

from .errors import NoSourceError
from .psana_adapter import PsanaWrapperSource, RawUnavailable, psana_available
from .rawfile import RawFileRun, make_synthetic_run, run_path, write_run
from .synthetic import RawEvent, SyntheticRun, generate_raw
from .xtc2 import find_xtc2_run, make_synthetic_xtc2_run, open_xtc2_run, write_xtc2_run, xtc2_paths

ENV_DATA_DIR = "PSANA_RAY_DATA"


SYNTHETIC_EXPS = ("synthetic",)


def open_source(exp: str, run: int, detector_name: str, rank: int = 0, size: int = 1,
                n_events: Optional[int] = None, pinned: bool = False, pool_frames: int = 32,
                data_dir: Optional[str] = None, mode=None, prefer_raw: bool = True,
                psana_private_constants: bool = False, psana_handle_shard: str = "explicit", **kw):
    """Pick the event source for ``(exp, run, detector_name)``:

    1. an XTC2-style run ``$PSANA_RAY_DATA/<exp>/xtc/<exp>-r<run>-s000-c000.xtc2`` (+ its
       smalldata index) if it exists;
    2. a raw-run file ``$PSANA_RAY_DATA/<exp>/r<run>/<detector>.praw`` if it exists;
    3. the synthetic detector for ``--exp synthetic``;
    4. the real psana_wrapper (``mode``: the retrieval mode the producer serves; raw frames into
       the HIP kernels when the wrapper can provide them, see source/psana_adapter.py).

    Anything else raises :class:`NoSourceError` -- a real experiment name never silently turns
    into synthetic frames.
    """
    from ..models.detector import Mode

    data_dir = data_dir or os.environ.get(ENV_DATA_DIR)
    if data_dir and find_xtc2_run(data_dir, exp, run) is not None:
        return open_xtc2_run(data_dir, exp, run, detector_name, rank=rank, size=size, pinned=pinned,
                             n_events=n_events)
    if data_dir:
        p = run_path(data_dir, exp, run, detector_name)
        if p.exists():
            return RawFileRun(p, detector_name, exp=exp, run=run, rank=rank, size=size, pinned=pinned,
                              n_events=n_events)
    if exp in SYNTHETIC_EXPS:
        return SyntheticRun(exp, run, detector_name, rank=rank, size=size, n_events=n_events,
                            pool_frames=pool_frames, pinned=pinned, **kw)
    if psana_available():
        return PsanaWrapperSource(exp, run, detector_name, mode=Mode.image if mode is None else Mode(mode),
                                  rank=rank, size=size, pinned=pinned, prefer_raw=prefer_raw, n_events=n_events,
                                  private_constants=psana_private_constants, handle_shard=psana_handle_shard)
    where = f" and no run file under {data_dir}" if data_dir else f" and ${ENV_DATA_DIR} is not set"
    raise NoSourceError(f"no event source for exp={exp!r} run={run} detector={detector_name!r}: psana_wrapper is "
                        f"not importable{where}.  Use --exp synthetic for the synthetic detector "
                        f"(random-init constants), or psana-ray-mkrun to write a run file.")


__all__ = ["NoSourceError", "RawUnavailable", "SYNTHETIC_EXPS", "RawEvent", "SyntheticRun", "RawFileRun", "PsanaWrapperSource", "open_source", "generate_raw",
           "write_run", "make_synthetic_run", "run_path", "psana_available", "find_xtc2_run", "open_xtc2_run",
           "write_xtc2_run", "make_synthetic_xtc2_run", "xtc2_paths"]
