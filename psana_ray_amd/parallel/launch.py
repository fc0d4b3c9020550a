"""Launch-environment detection: one process per GPU, started by mpirun/mpiexec, torchrun or Slurm.

The reference is launched as ``mpirun -n 4 psana-ray-producer ...`` and reads its rank from
``mpi4py`` (psana_ray/producer.py:13,138-140).  mpi4py is not required here: rank / size / local
rank come from the launcher's environment (MPICH/Hydra ``PMI_*``/``MPI_LOCALRANKID``, Open MPI
``OMPI_COMM_WORLD_*``, torchrun ``RANK``/``WORLD_SIZE``/``LOCAL_RANK``, Slurm ``SLURM_*``).
"""
from __future__ import annotations

import logging
import os
from dataclasses import dataclass
from typing import Optional

log = logging.getLogger(__name__)

_RANK = ("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "PMIX_RANK", "SLURM_PROCID")
_SIZE = ("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS")
_LOCAL = ("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "PMI_LOCAL_RANK", "SLURM_LOCALID")
_LOCAL_SIZE = ("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", "PMI_LOCAL_SIZE",
               "SLURM_NTASKS_PER_NODE")


def _first_int(names, default: Optional[int] = None) -> Optional[int]:
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            try:
                return int(v)
            except ValueError:
                continue
    return default


@dataclass
class LaunchInfo:
    rank: int
    size: int
    local_rank: int
    launcher: str
    local_size: int = 1   # ranks of this launch on this node

    @property
    def distributed(self) -> bool:
        return self.size > 1


def detect() -> LaunchInfo:
    rank = _first_int(_RANK, 0)
    size = _first_int(_SIZE, 1)
    local = _first_int(_LOCAL, None)
    if local is None:
        local = rank
    if "OMPI_COMM_WORLD_RANK" in os.environ:
        launcher = "openmpi"
    elif "PMI_RANK" in os.environ:
        launcher = "mpich"
    elif "TORCHELASTIC_RUN_ID" in os.environ or "RANK" in os.environ:
        launcher = "torchrun"
    elif "SLURM_PROCID" in os.environ:
        launcher = "slurm"
    else:
        launcher = "single"
    local_size = _first_int(_LOCAL_SIZE, None)
    if local_size is None:
        # no launcher told how many of its ranks share this node: assume one (the
        # global size would make a multi-node PMI launch take the shared-GPU pipeline shape).
        # torchrun, Open MPI, MPICH/Hydra and bench.py's self-launch all set a local size.
        local_size = 1
    return LaunchInfo(rank, size, local, launcher, max(1, local_size))


def ranks_per_gpu(n_gpus: Optional[int] = None, local_size: Optional[int] = None) -> int:
    """How many ranks of this launch share one GPU of this node: ceil(local ranks / GPUs) (1 on a
    node with a GPU per rank; `mpirun -n 4` on a one-GPU box: 4).  ``n_gpus`` default: the visible
    GPUs (counting them does not initialise the HIP runtime); 1 without a GPU."""
    if local_size is None:
        local_size = detect().local_size
    if n_gpus is None:
        import torch

        n_gpus = torch.cuda.device_count()
    share = max(1, -(-int(local_size) // max(1, int(n_gpus))))
    log.debug("ranks per GPU: %d (%d local ranks on %d GPU(s))", share, int(local_size), int(n_gpus))
    return share


def device_for(local_rank: int, requested: Optional[str] = None):
    """``cuda:<local_rank mod #GPUs>`` when a GPU exists (or ``requested``), else ``cpu``."""
    import torch

    if requested and requested != "auto":
        return torch.device(requested)
    n = torch.cuda.device_count()
    if n > 0:
        return torch.device(f"cuda:{local_rank % n}")
    return torch.device("cpu")


def bind_numa_to_device(device) -> Optional[int]:
    """Pin this process to the CPUs of the GPU's NUMA node, so pinned staging pages are
    allocated node-local to the GPU's PCIe root (host->device copies cross no socket link)."""
    import torch

    if os.environ.get("PSANA_RAY_NUMA_BIND", "1") == "0":
        return None
    try:
        if torch.device(device).type != "cuda":
            return None
        props = torch.cuda.get_device_properties(device)
        bus = getattr(props, "pci_bus_id", None)
        domain = getattr(props, "pci_domain_id", 0)
        dev_id = getattr(props, "pci_device_id", None)
        if bus is None or dev_id is None:
            return None
        path = f"/sys/bus/pci/devices/{domain:04x}:{bus:02x}:{dev_id:02x}.0/numa_node"
        node = int(open(path).read().strip())
        if node < 0:
            return None
        cpus = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
        cpuset = set()
        for part in cpus.split(","):
            a, _, b = part.partition("-")
            cpuset.update(range(int(a), int(b or a) + 1))
        allowed = os.sched_getaffinity(0)
        target = cpuset & allowed
        if target:
            os.sched_setaffinity(0, target)
            return node
    except Exception:
        return None
    return None
