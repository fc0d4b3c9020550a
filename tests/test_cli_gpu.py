"""The installed producer entry point on one GPU (single-process queue + co-located peak finder)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_producer_local_gpu_peakfind(cuda_device):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-m", "psana_ray_amd.producer", "--exp", "synthetic", "--run", "1",
                        "--detector_name", "epix10k2M", "--calib", "--num_events", "300", "--local",
                        "--consumer_task", "peakfind", "--common_mode", "default", "--uses_bad_pixel_mask",
                        "--queue_size", "64"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "produced 300 frames" in r.stderr
    assert "co-located consumer processed 300 frames" in r.stderr


def test_producer_local_gpu_image_mode(cuda_device):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-m", "psana_ray_amd.producer", "--exp", "synthetic", "--run", "2",
                        "--detector_name", "epix10k2M", "--num_events", "64", "--local", "--consumer_task",
                        "peakfind", "--queue_size", "32"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "co-located consumer processed 64 frames" in r.stderr
