"""Multi-process plumbing: launch-env detection (mpirun / torchrun / Slurm) and the rendezvous
store.  Queue membership and links: :mod:`psana_ray_amd.queue.session`, ``csrc/fabric.h``."""
from .launch import detect, device_for
from .rendezvous import open_store, port_open

__all__ = ["detect", "device_for", "open_store", "port_open"]
