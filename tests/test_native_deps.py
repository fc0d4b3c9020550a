"""ABI hygiene of the native extension (round-1 verdict item: RCCL header / library skew).

The queue's data plane no longer uses RCCL (HIP IPC peer copies, csrc/fabric.cpp), so the
extension must not link librccl at all: the only RCCL in a process is the one torch.distributed
loads for the data-parallel trainer (its own, self-consistent build).  The HIP runtime it links is
the image's (ROCm 7.x)."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_extension_links_no_rccl(native):
    sos = glob.glob(os.path.join(ROOT, "psana_ray_amd", "_C*.so"))
    assert sos, "extension not built in-tree"
    if shutil.which("readelf") is None:
        pytest.skip("readelf not available")
    out = subprocess.run(["readelf", "-d", sos[0]], capture_output=True, text=True, check=True).stdout
    needed = [l.split("[")[1].rstrip("]") for l in out.splitlines() if "(NEEDED)" in l]
    assert not any("rccl" in n or "nccl" in n for n in needed), needed
    assert any(n.startswith("libamdhip64.so") for n in needed), needed
