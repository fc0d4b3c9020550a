"""Loader for the native extension ``psana_ray_amd._C`` (HIP kernels + host runtime).

torch is imported first so the process has exactly one HIP runtime: torch ships
``libamdhip64.so.7`` and the extension links against the same soname (rpath to torch/lib).
If the extension is missing and ``hipcc`` is available it is built in-tree on first use; on a
GPU box a missing/failed extension raises -- GPU ops never silently fall back to PyTorch.
"""
from __future__ import annotations

import atexit
import importlib
import os
import threading
import weakref

import torch  # noqa: F401  (must precede the extension: one HIP runtime per process)

_lock = threading.Lock()
_mod = None
_err = None


def load(build_if_missing: bool = True):
    global _mod, _err
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            if build_if_missing and os.environ.get("PSANA_RAY_AMD_NO_BUILD") != "1":
                from .. import _build

                _build.build()
            mod = importlib.import_module("psana_ray_amd._C")
            # at exit: Python threads that drive native objects (queue-session watchers) stop first,
            # then every native thread (queue fabric, producer engines) -- all before the
            # interpreter and the HIP runtime tear down (csrc/lifecycle.h)
            atexit.register(_shutdown, mod)
            _mod = mod
            return _mod
        except Exception as e:  # pragma: no cover - surfaced to the caller
            _err = e
            raise RuntimeError(f"psana_ray_amd native extension unavailable: {e}") from e


_exit_hooks: "weakref.WeakSet" = None


def on_exit(obj) -> None:
    """Call ``obj.stop_at_exit()`` at process exit, before the native threads halt (weakly held:
    an object collected earlier is forgotten)."""
    global _exit_hooks
    with _lock:
        if _exit_hooks is None:
            _exit_hooks = weakref.WeakSet()
        _exit_hooks.add(obj)


def _shutdown(mod) -> None:
    mod.install_segv_trace()   # diagnostic (PSANA_RAY_AMD_SEGV_TRACE=1): after test runners restored theirs
    for obj in list(_exit_hooks or ()):
        try:
            obj.stop_at_exit()
        except Exception:  # noqa: BLE001 - best effort at exit
            pass
    mod.halt_native_threads()
    # pooled dedicated streams: Python's idle handles back to the native pool, then the pool is
    # destroyed (no queue of ours is left for the runtime's static teardown)
    try:
        from .. import pipeline

        pipeline._release_idle_streams(mod)
    except Exception:  # noqa: BLE001 - best effort at exit
        pass
    mod.close_stream_pool()


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


def stream_handle(stream=None) -> int:
    """Raw hipStream_t of a torch stream (default: the current stream of the current device)."""
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)
