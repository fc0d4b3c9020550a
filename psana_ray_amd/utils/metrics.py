"""Counters, rates and a periodic summary for producers / consumers / the queue fabric.

Reference parity (SURVEY §5 "Metrics / logging / observability"): psana-ray only has
``--log_level`` (psana_ray/producer.py:31-32,135-136), a per-event INFO line (:103) and a
full-queue INFO line (:106); ``Queue.size()`` exists but is unused (shared_queue.py:26-31).
At 10^4 frames/s a per-event log line IS the bottleneck, so here:

  * components expose cumulative counters as plain callables (``register(name, fn)``); the hot
    paths (native producer engine, slot pool, queue fabric) already count, so nothing extra runs
    per frame;
  * a :class:`Reporter` thread samples every source every ``interval`` seconds, derives rates
    from the deltas, logs ONE summary line per interval and optionally appends a JSON line to
    a file (for benchmarks) and/or publishes Prometheus gauges (``prometheus_client``, if
    installed) on an HTTP port.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from typing import Callable, Dict, Optional

log = logging.getLogger("psana_ray_amd.metrics")

Source = Callable[[], Dict[str, float]]

# counters whose per-interval delta is reported as a rate (everything else is a gauge)
RATE_KEYS = ("frames", "frames_produced", "frames_consumed", "frames_routed", "bytes_sent", "bytes_recv",
             "peaks", "rounds", "full_waits")


def sustained_rate(log_entries, t0: float, t1: float):
    """Sustained production rate inside the window ``(t0, t1]`` from a completion log.

    ``log_entries``: ``[(frames completed so far, completion time), ...]`` in completion order (one
    entry per chunk; ``ProducerPipeline.completion_log``).  Frames of chunks that completed at or
    before ``t0`` -- already READY when the window opened -- are excluded; the rate runs from the
    last completion at or before ``t0`` to the last completion at or before ``t1``, i.e. between
    two chunk completions, so a window never gains or loses a fraction of a chunk.

    Returns ``(frames completed inside the window, frames / s or None when fewer than one
    completion on each side of t0)``."""
    before = None
    last = None
    for f, t in log_entries:
        if t <= t0:
            before = (f, t)
        elif t <= t1:
            last = (f, t)
        else:
            break
    if before is None or last is None:
        return (0 if last is None else last[0] - (before[0] if before else 0)), None
    frames = last[0] - before[0]
    dt = last[1] - before[1]
    return frames, (frames / dt if dt > 0 else None)


class Registry:
    def __init__(self):
        self._lock = threading.Lock()
        self._sources: Dict[str, Source] = {}

    def register(self, name: str, fn: Source) -> None:
        with self._lock:
            self._sources[name] = fn

    def unregister(self, name: str) -> None:
        with self._lock:
            self._sources.pop(name, None)

    def snapshot(self) -> Dict[str, float]:
        """Flat ``{"source.key": value}`` of every numeric value every source reports now."""
        with self._lock:
            items = list(self._sources.items())
        out: Dict[str, float] = {}
        for name, fn in items:
            try:
                d = fn() or {}
            except Exception as e:  # noqa: BLE001 - a dying component must not kill the reporter
                out[f"{name}.error"] = 1.0
                log.debug("metrics source %s failed: %r", name, e)
                continue
            for k, v in d.items():
                if isinstance(v, bool):
                    v = int(v)
                if isinstance(v, (int, float)):
                    out[f"{name}.{k}"] = float(v)
                elif isinstance(v, str):   # a label (e.g. producer.source_path): JSON as is, Prometheus as info
                    out[f"{name}.{k}"] = v
        return out


def rates(prev: Dict[str, float], cur: Dict[str, float], dt: float) -> Dict[str, float]:
    """Per-second rates of the counter keys between two snapshots."""
    r = {}
    if dt <= 0:
        return r
    for k, v in cur.items():
        if k.rsplit(".", 1)[-1] in RATE_KEYS and k in prev:
            r[k + "_per_s"] = (v - prev[k]) / dt
    return r


def summary_line(rank: int, cur: Dict[str, float], rate: Dict[str, float]) -> str:
    parts = [f"rank {rank}"]
    for k in sorted(rate):
        if k.endswith("bytes_sent_per_s") or k.endswith("bytes_recv_per_s"):
            parts.append(f"{k[:-6]}={rate[k] / 1e9:.2f} GB/s")
        else:
            parts.append(f"{k}={rate[k]:,.1f}")
    for k in sorted(cur):
        leaf = k.rsplit(".", 1)[-1]
        if leaf in ("ready", "credits", "depth", "producing", "leased", "free"):
            parts.append(f"{k}={int(cur[k])}")
    return " | ".join(parts)


class Reporter:
    """Samples a :class:`Registry` periodically; logs / dumps / exports."""

    def __init__(self, registry: Registry, rank: int = 0, interval: float = 10.0,
                 json_path: Optional[str] = None, prometheus_port: Optional[int] = None,
                 level: int = logging.INFO):
        self.registry = registry
        self.rank = rank
        self.interval = float(interval)
        self.json_path = json_path
        self.level = level
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._prev: Optional[Dict[str, float]] = None
        self._t_prev = 0.0
        self._gauges = {}
        self._prom = None
        if prometheus_port:
            try:
                import prometheus_client

                prometheus_client.start_http_server(int(prometheus_port))
                self._prom = prometheus_client
            except Exception as e:  # noqa: BLE001
                log.warning("prometheus exporter unavailable: %r", e)

    def sample(self) -> Dict[str, float]:
        """Take one sample now: returns the snapshot merged with rates since the last one."""
        now = time.monotonic()
        cur = self.registry.snapshot()
        r = rates(self._prev, cur, now - self._t_prev) if self._prev is not None else {}
        self._prev, self._t_prev = cur, now
        rec = dict(cur)
        rec.update(r)
        if r:
            log.log(self.level, "%s", summary_line(self.rank, cur, r))
        if self.json_path:
            with open(self.json_path, "a") as f:
                f.write(json.dumps({"t": time.time(), "rank": self.rank, **rec}) + "\n")
        if self._prom is not None:
            for k, v in rec.items():
                name = "psana_ray_" + k.replace(".", "_").replace("-", "_")
                if isinstance(v, str):   # info-style gauge: the label carries the value
                    name += "_info"
                    g = self._gauges.get(name)
                    if g is None:
                        g = self._gauges[name] = self._prom.Gauge(name, k, ["rank", "value"])
                    g.labels(rank=str(self.rank), value=v).set(1)
                    continue
                g = self._gauges.get(name)
                if g is None:
                    g = self._gauges[name] = self._prom.Gauge(name, k, ["rank"])
                g.labels(rank=str(self.rank)).set(v)
        return rec

    def _loop(self):
        self.sample()
        while not self._stop.wait(self.interval):
            self.sample()

    def start(self) -> "Reporter":
        if self.interval > 0 and self._thread is None:
            self._thread = threading.Thread(target=self._loop, name="psana-ray-metrics", daemon=True)
            self._thread.start()
        return self

    def stop(self, final_sample: bool = True) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None
        if final_sample:
            self.sample()


_default = Registry()


def default_registry() -> Registry:
    return _default
