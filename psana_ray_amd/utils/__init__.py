"""Observability helpers: roctx ranges (tracing) and sampled counters / rates (metrics)."""
from .metrics import Registry, Reporter, default_registry
from .tracing import mark, trace_range

__all__ = ["Registry", "Reporter", "default_registry", "mark", "trace_range"]
