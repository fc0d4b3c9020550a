"""The multi-GPU transport path on ONE device (loopback: frames routed to self still go through
the control round and the grouped send/recv exchange).

On the GPU this runs RCCL send/recv to self on the comm stream with the slot pool's HIP events --
the exact code the 2/4/8-GPU runs use (RCCL refuses two ranks on one GPU, so this is the only
way to exercise it on a 1-GPU box)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1")


# native = C++ TransportEngine (shared-memory control plane), python = gloo-driven rounds
XPORTS = ["native", "python"]


def _run(args, timeout, xport="native"):
    return subprocess.run([sys.executable] + args, cwd=ROOT, env=dict(ENV, PSANA_RAY_XPORT=xport),
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("xport", XPORTS)
def test_loopback_integrity_cpu(xport):
    r = _run(["tests/_loopback_worker.py", "cpu", "150"], 120, xport)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "LOOPBACK_OK 150" in r.stdout and f"xport={xport}" in r.stdout


@pytest.mark.parametrize("xport", XPORTS)
def test_bench_loopback_cpu(xport):
    r = _run(["bench.py", "--device", "cpu", "--detector", "tiny_epix", "--steps", "3", "--warmup", "1",
              "--batch", "4", "--loopback"], 300, xport)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["config"]["loopback"] is True
    assert res["extra"]["bytes_sent_rank0"] > 0
    assert res["extra"]["transport_driver"] == xport


@pytest.mark.gpu
@pytest.mark.parametrize("xport", XPORTS)
def test_loopback_integrity_rccl(native, xport):
    r = _run(["tests/_loopback_worker.py", "cuda:0", "300"], 300, xport)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "LOOPBACK_OK 300" in r.stdout and "native=True" in r.stdout and f"xport={xport}" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("xport", XPORTS)
def test_bench_loopback_rccl(native, xport):
    """Full producer engine -> transport (native engine or python thread) -> RCCL -> peak-finder
    consumer on one GPU."""
    r = _run(["bench.py", "--steps", "20", "--warmup", "5", "--loopback"], 420, xport)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["value"] > 0 and res["extra"]["bytes_sent_rank0"] > 0
    assert res["extra"]["transport_driver"] == xport
    print(json.dumps(res))
