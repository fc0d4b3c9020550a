"""bench.py's multi-rank flow (timing, barriers, drain, EOS, teardown) rehearsed on the CPU with
torch.distributed.run + gloo and a tiny detector -- the same code path the driver's 8-GPU run uses
with RCCL."""
import json
import os
import random
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("nproc,route,producers", [(2, "balanced", 0), (4, "spread", 0), (4, "balanced", 2)])
def test_bench_multirank_cpu(native, nproc, route, producers):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    port = random.randint(30000, 45000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--steps", "4", "--warmup", "2", "--batch", "4", "--detector", "tiny_epix",
           "--device", "cpu", "--queue-size", "16", "--chunk", "4", "--route", route,
           "--producers", str(producers)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == nproc and d["steps"] == 4 and d["value"] > 0
    assert d["config"]["global_batch"] == 4 * nproc
    assert d["extra"]["bytes_sent_rank0"] > 0, "frames must cross ranks through the transport"
    assert d["config"]["producer_ranks"] == (producers or nproc)
