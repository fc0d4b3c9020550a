"""End-to-end frame checks of the queue fabric (csrc/verify.h): producers attach a content
checksum to every N-th frame they send to another process, consumers re-sum it from their own ring
and count matches / mismatches; a frame damaged in transit makes bench.py exit 4 (VERDICT r5 next
#2).  CPU rehearsal: host rings in shared memory, the same fabric code and the same hash as the GPU
kernel (tests/test_kernels_gpu.py checks host == device)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(nproc, extra_env, steps=4):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.update(extra_env)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--steps", str(steps), "--warmup",
           "2", "--batch", "4", "--detector", "tiny_epix", "--device", "cpu", "--queue-size", str(16 * nproc),
           "--chunk", "4"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd="/tmp")
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, (json.loads(lines[0]) if lines else None)


def test_checksum_host_matches_reference(native):
    """The host checksum equals an independent numpy implementation of the documented hash."""
    C = native
    rng = np.random.default_rng(3)
    for nbytes in (16, 4096, 12288, 1000):
        a = rng.integers(0, 256, nbytes, dtype=np.uint8)
        M = (1 << 64) - 1
        s = 0
        pad = np.zeros((nbytes + 15) // 16 * 16, np.uint8)
        pad[:nbytes] = a
        w = pad.view("<u8").reshape(-1, 2)
        for q, (lo, hi) in enumerate(w.tolist()):
            h = ((lo ^ (((q + 1) * 0x9E3779B97F4A7C15) & M)) * 0xBF58476D1CE4E5B9) & M
            h = (h + hi * 0x94D049BB133111EB) & M
            h ^= h >> 31
            h = (h * 0xD6E8FEB86659FD93) & M
            h ^= h >> 32
            s = (s + h) & M
        assert C.frame_checksum_host(int(a.ctypes.data), nbytes) == s
        # a one-byte change or a swap of two 16-B words changes it
        if nbytes >= 32:
            b = a.copy()
            b[5] ^= 1
            assert C.frame_checksum_host(int(b.ctypes.data), nbytes) != s
            c = a.copy()
            c[:16], c[16:32] = a[16:32].copy(), a[:16].copy()
            if not np.array_equal(a[:16], a[16:32]):
                assert C.frame_checksum_host(int(c.ctypes.data), nbytes) != s


def test_cross_process_frames_verified_cpu(native):
    """2 ranks, every frame checksummed: the consumers verify frames and find no mismatch."""
    r, d = _run_bench(2, {"PSANA_RAY_AMD_VERIFY_EVERY": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    fc = d["extra"]["frame_checks"]
    assert fc["verify_every"] == 1
    assert fc["frames_verified"] > 0 and fc["frames_mismatched"] == 0, fc
    assert sum(fc["checksummed_sent_per_rank"]) >= fc["frames_verified"] > 0
    assert all(a > 0 for a in fc["acquires_per_rank"]), fc
    x = d["extra"]["xgmi_phase"]
    assert x["frames_verified"] == fc["frames_verified"] and x["frames_mismatched"] == 0


def test_corrupted_frame_fails_the_run_cpu(native):
    """Fault injection: every 3rd frame a producer sends is damaged in the consumer's ring after
    its copy.  The consumers catch it and bench.py exits 4 after printing its line."""
    r, d = _run_bench(2, {"PSANA_RAY_AMD_VERIFY_EVERY": "1", "PSANA_RAY_AMD_FAULT_CORRUPT": "3"})
    assert r.returncode == 4, (r.returncode, r.stderr[-3000:])
    fc = d["extra"]["frame_checks"]
    assert sum(fc["corrupted_injected_per_rank"]) > 0
    assert fc["frames_mismatched"] > 0, fc
    assert any(g >= 0 for g in fc["last_bad_gevt_per_rank"]), fc
    assert "differ from what their producer sent" in r.stderr


@pytest.mark.gpu
def test_checksum_device_matches_host(native, cuda_device):
    """gfx950 checksum kernel == host checksum (bitwise), for frame sizes of the real detectors and
    a small one; the device compare mode counts a match and a damaged frame as a mismatch."""
    import torch

    C = native
    dev = cuda_device
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    for nbytes in (16 * 1024, 8650752, 12288 + 16 * 7):
        frames = [torch.randint(-2**31, 2**31 - 1, (nbytes // 4,), dtype=torch.int32, device=dev) for _ in range(3)]
        v = C.FrameVerifier(dev.index, nbytes)
        base = v.checksum_async([int(f.data_ptr()) for f in frames], sh)
        stream.synchronize()
        got = [v.result(base + i) for i in range(3)]
        host = [f.cpu().numpy() for f in frames]   # kept alive while the host checksum reads them
        want = [C.checksum_tag(C.frame_checksum_host(int(h.ctypes.data), nbytes)) for h in host]
        assert got == want
        # consumer mode: frame 1 damaged after its checksum was taken
        frames[1][nbytes // 8] ^= 1
        v.acquire(sh)
        v.verify([int(f.data_ptr()) for f in frames], got, [10, 11, 12], sh)
        stream.synchronize()
        ok, bad, last, acq = v.counts()
        assert (ok, bad, last, acq) == (2, 1, 11, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("direct", ["1", "0"])
def test_two_ranks_one_gpu_frames_verified(native, direct):
    """bench.py --gpus 2 (self-launched, two processes on the box's GPU, device-resident raw frames):
    the route=remote_only window moves every frame between processes through HIP IPC -- calibrated
    straight into the consumer's slot (direct) or copied by copy_runs_kernel -- and the consumers
    verify every 4th frame's checksum bitwise."""
    r, d = _run_gpu_bench(2, {"PSANA_RAY_AMD_VERIFY_EVERY": "4", "PSANA_RAY_AMD_FABRIC_DIRECT": direct})
    assert r.returncode == 0, r.stderr[-3000:]
    assert d["n_gpus"] == 1 and d["n_ranks"] == 2
    fc, x = d["extra"]["frame_checks"], d["extra"]["xgmi_phase"]
    assert fc["frames_verified"] > 0 and fc["frames_mismatched"] == 0, fc
    assert x["cross_gpu_fraction"] >= 0.9
    if direct == "1":
        # direct headroom (engine.h): the producers wait for grants rather than queue copies, so
        # most routed frames are calibrated straight into the consumer's slot (92-98 % measured)
        assert x["direct_headroom_slots"] > 0, x
        assert sum(x["frames_direct_per_rank"]) >= 0.6 * sum(x["frames_sent_per_rank"]), x
    else:
        assert sum(x["frames_direct_per_rank"]) == 0, x


def _run_gpu_bench(nproc, extra_env):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.update(extra_env)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--steps", "20", "--warmup", "3",
           "--source", "device", "--gate-max-s", "3"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=200, cwd="/tmp")
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, (json.loads(lines[0]) if lines else None)


@pytest.mark.gpu
def test_plain_store_mask_is_bitwise_equal(native, cuda_device):
    """Frames calibrated for ANOTHER process's ring (direct grants) use plain stores instead of the
    streaming ones (CmParams plain_mask): the epix10k2M common-mode kernel's output is bit-identical
    either way, for a mixed mask over a 64-frame launch."""
    import numpy as np
    import torch

    from psana_ray_amd.models.calibrator import Calibrator
    from psana_ray_amd.models.detector import Mode
    from psana_ray_amd.config import resolve_common_mode
    from psana_ray_amd.source import SyntheticRun

    C = native
    dev = cuda_device
    src = SyntheticRun("synthetic", 0, "epix10k2M", pool_frames=8, gen_device="cuda")
    cal = Calibrator(src.consts, dev, Mode.calib, common_mode=resolve_common_mode("auto", src.consts.spec))
    raw = torch.from_numpy(src.pool.view(np.int16)).view(torch.uint16).to(dev)
    n = 64
    ins = [int(raw[i % raw.shape[0]].data_ptr()) for i in range(n)]
    a = torch.empty((n, *cal.out_shape), dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    s = torch.cuda.current_stream(dev)
    C.run_calib_plan(cal.plan, ins, [int(a[i].data_ptr()) for i in range(n)], s.cuda_stream)
    C.run_calib_plan(cal.plan, ins, [int(b[i].data_ptr()) for i in range(n)], s.cuda_stream,
                     [1 if i % 3 else 0 for i in range(n)])
    s.synchronize()
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))
