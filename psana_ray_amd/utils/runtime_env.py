"""Process-level ROCm runtime settings that must be chosen before the HIP runtime initialises.

Host -> HBM staging copies (the producer's ``hipMemcpyAsync`` of pinned raw frames) can run on the
SDMA copy engines (ROCr default) or as blit kernels on the compute units (``HSA_ENABLE_SDMA=0``).
Both reach the same isolated PCIe rate (57 GB/s, ``bench/h2d.py``), but inside the pipeline --
copies interleaved with calibration / peak-finder kernels and cross-stream events -- the blit path
sustains 12.7k vs 12.2k epix10k2M frames/s on the same box (``tools/gpu_sdma_ab.sh``,
profiles/bench_ab_r1.md).  ROCr reads the variable once, at ``hsa_init`` (the first HIP call of
the process), so this must run before anything touches ``torch.cuda``.
"""
from __future__ import annotations

import os

COPY_ENGINES = ("blit", "sdma")


def select_copy_engine(engine: str = "blit") -> str:
    """Choose the copy engine for this process (an explicit ``HSA_ENABLE_SDMA`` wins).  Returns
    the engine in effect."""
    if engine not in COPY_ENGINES:
        raise ValueError(f"copy engine {engine!r}: choose from {COPY_ENGINES}")
    os.environ.setdefault("HSA_ENABLE_SDMA", "0" if engine == "blit" else "1")
    return "blit" if os.environ["HSA_ENABLE_SDMA"] == "0" else "sdma"
