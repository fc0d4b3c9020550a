"""Multi-GPU plumbing: launch-env detection, rendezvous, RCCL/gloo comm, routing."""
from .comm import Comm, init_groups
from .routing import POLICIES, plan_round

__all__ = ["Comm", "init_groups", "plan_round", "POLICIES"]
