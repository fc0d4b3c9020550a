"""Panel sharding (SURVEY P-04 / §5.7, source/shard.py): a frame's panels split over a group of
producer ranks.  Shard calibration (incl. common mode) must equal the matching panels of the
whole-frame calibration, the shard source must hand out the right raw spans / event ids, the
ShardAssembler must rebuild whole frames, and the CLI path (2 producer processes, 1 consumer)
must deliver every event exactly once as whole frames equal to the golden model."""
import os
import random
import subprocess
import sys

import numpy as np
import pytest
import torch

from psana_ray_amd.batching import ShardAssembler
from psana_ray_amd.config import CommonModeParams
from psana_ray_amd.models import Calibrator, Mode
from psana_ray_amd.models.detector import get_detector, panel_shard_range
from psana_ray_amd.source import SyntheticRun
from psana_ray_amd.source.shard import PanelShardSource, shard_layout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_ranges_and_layout():
    assert [panel_shard_range(32, s, 4) for s in range(4)] == [(0, 8), (8, 16), (16, 24), (24, 32)]
    with pytest.raises(ValueError):
        panel_shard_range(16, 0, 3)
    assert [shard_layout(r, 8, 2) for r in range(4)] == [(0, 4, 0), (0, 4, 1), (1, 4, 0), (1, 4, 1)]
    with pytest.raises(ValueError):
        shard_layout(0, 6, 4)
    sub = get_detector("jungfrau16M").panel_subset(8, 16)
    assert sub.frame_shape == (8, 512, 1024) and sub.kind == "jungfrau" and sub.asic_rows == 256


@pytest.mark.parametrize("det", ["tiny_epix", "tiny_jungfrau"])
def test_shard_calibration_equals_slice_of_full(det):
    src = SyntheticRun("synthetic", 5, det, n_events=4, pool_frames=4, gen_device="cpu")
    cm = CommonModeParams.parse("default")
    mask = src.create_bad_pixel_mask()
    full = Calibrator(src.consts, "cpu", Mode.calib, mask=mask, common_mode=cm)
    raw = torch.from_numpy(src.pool.astype(np.int32)).to(torch.uint16)
    ref = full(raw)
    P = src.spec.n_panels
    for s in range(2):
        sh = PanelShardSource(SyntheticRun("synthetic", 5, det, n_events=4, pool_frames=4, gen_device="cpu"), s, 2)
        cal = Calibrator(sh.consts, "cpu", Mode.calib, mask=sh.create_bad_pixel_mask(), common_mode=cm)
        lo, hi = sh.lo, sh.hi
        assert (lo, hi) == (s * P // 2, (s + 1) * P // 2) and cal.out_shape == (P // 2, *src.spec.frame_shape[1:])
        got = cal(raw[:, lo:hi].contiguous())
        assert torch.equal(got, ref[:, lo:hi])


def test_shard_source_events_and_pointers():
    inner = SyntheticRun("synthetic", 2, "tiny_epix", rank=1, size=3, n_events=20, pool_frames=4, gen_device="cpu")
    sh = PanelShardSource(inner, 1, 2)
    pb = inner.spec.panel_pixels * 2
    evs = sh.next_events(3)
    assert [e.gevt for e in evs] == [1, 4, 7] and [e.idx for e in evs] == [0, 1, 2]
    for e in evs:
        assert e.raw.shape == (1, 32, 48) and e.raw.flags["C_CONTIGUOUS"]
        assert e.host_ptr == e.raw.ctypes.data and np.array_equal(e.raw, inner.pool[e.idx % 4][1:2])
    ptrs, _ = sh.cycled_frames()
    iptrs, _ = inner.cycled_frames()
    assert ptrs == [p + pb for p in iptrs]
    assert sh.event_rank == 1 and sh.size == 3 and sh.n_local_events() == inner.n_local_events()
    assert sh.create_bad_pixel_mask().shape == (1, 32, 48)


class _Item:
    def __init__(self, rank, gevt, data, pe=9.5):
        self.rank, self.gevt, self.data, self.photon_energy = rank, gevt, data, pe
        self.released = False

    def release(self, stream=None):
        self.released = True


def test_shard_assembler_regroups_out_of_order():
    G, per = 4, 2
    frames = {g: torch.randn(G * per, 5, 8) for g in range(6)}
    items = [_Item(r, g, frames[g][(r % G) * per:(r % G + 1) * per].clone()) for g in frames for r in range(G)]
    random.Random(0).shuffle(items)
    asm = ShardAssembler(G, (per, 5, 8))
    out = []
    for i in range(0, len(items), 5):
        out += asm.add(items[i:i + 5])
    assert sorted(f.gevt for f in out) == list(range(6)) and asm.pending == 0
    for f in out:
        assert torch.equal(f.data, frames[f.gevt]) and f.photon_energy == 9.5
    assert all(it.released for it in items)
    with pytest.raises(ValueError):
        asm.add([_Item(0, 0, torch.zeros(per, 5, 8)), _Item(4, 0, torch.zeros(per, 5, 8))])   # shard 0 twice


def _env(extra=None):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.update(extra or {})
    return env


def run_sharded_session(device: str, n_prod: int = 2, shards: int = 2, n_events: int = 10, det: str = "tiny_epix"):
    port = random.randint(30000, 45000)
    addr = f"127.0.0.1:{port}"
    prods = [subprocess.Popen(
        [sys.executable, "-m", "psana_ray_amd.producer", "--exp", "synthetic", "--run", "6", "--detector_name", det,
         "--calib", "--num_events", str(n_events), "--ray_address", addr, "--num_consumers", "1", "--queue_size", "6",
         "--device", device, "--uses_bad_pixel_mask", "--common_mode", "default", "--panel_shards", str(shards),
         "--timeout", "60"],
        env=_env({"RANK": str(r), "WORLD_SIZE": str(n_prod), "LOCAL_RANK": "0"}), stdout=subprocess.PIPE,
        stderr=subprocess.STDOUT, text=True) for r in range(n_prod)]
    cons = subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_shard_consumer.py"), addr,
                             str(n_prod // shards), det, "6", device],
                            env=_env(), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    outs = []
    try:
        for p in prods + [cons]:
            out, _ = p.communicate(timeout=180)
            outs.append((p.returncode, out))
    finally:
        for p in prods + [cons]:
            if p.poll() is None:
                p.kill()
    for rc, out in outs:
        assert rc == 0, out[-3000:]
    return outs[-1][1]


def test_panel_sharded_cli_cpu(native):
    out = run_sharded_session("cpu")
    assert "SHARD_OK 10 20 G=2" in out, out[-2000:]


def test_image_mode_rejected_with_shards(native):
    r = subprocess.run([sys.executable, "-m", "psana_ray_amd.producer", "--exp", "synthetic", "--run", "1",
                        "--detector_name", "tiny_epix", "--panel_shards", "2", "--device", "cpu", "--local",
                        "--consumer_task", "peakfind"],
                       env=_env({"RANK": "0", "WORLD_SIZE": "2", "LOCAL_RANK": "0"}), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2 and "--panel_shards" in (r.stdout + r.stderr)


def _shard_stream(src_kw, shard, G, device, cm, n_events, rank):
    """One shard's producer pipeline (native engine on a GPU) into its own local queue; returns the
    leased items (the consumer side of a panel-sharded session, in one process)."""
    from psana_ray_amd.pipeline import ProducerPipeline
    from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint

    sh = PanelShardSource(SyntheticRun(**src_kw), shard, G)
    cal = Calibrator(sh.consts, device, Mode.calib, mask=sh.create_bad_pixel_mask(), common_mode=cm)
    ring = FrameRing(cal.out_shape, cal.out_dtype, device, 8, n_events)
    ep = QueueEndpoint(ring)
    pipe = ProducerPipeline(sh, cal, ep, rank=rank, chunk=4)
    assert pipe.engine is not None, "GPU shards must run through the native producer engine"
    assert pipe.run() == n_events
    items = []
    while True:
        try:
            it = ep.get(timeout=1.0)
        except EndOfStream:
            break
        if it is not None:
            items.append(it)
    return items, (ring, ep)


@pytest.mark.gpu
@pytest.mark.parametrize("det,G", [("tiny_epix", 2), ("epix10k2M", 4)])
def test_panel_shards_gpu_engine_assemble(native, cuda_device, det, G):
    """Shards staged from sub-spans of the pinned pool by the native engine, calibrated with
    common mode on the GPU, regrouped by the ShardAssembler (list-destination gather kernel):
    bitwise equal to the whole-frame GPU calibration."""
    n_events = 8
    kw = dict(exp="synthetic", run=7, detector_name=det, n_events=n_events, pool_frames=4, pinned=True,
              gen_device="cuda")
    cm = CommonModeParams.parse("default")
    full_src = SyntheticRun(**kw)
    full = Calibrator(full_src.consts, cuda_device, Mode.calib, mask=full_src.create_bad_pixel_mask(), common_mode=cm)
    ref = full(torch.from_numpy(full_src.pool.view(np.int16)).view(torch.uint16).to(cuda_device))
    keep, items = [], []
    for s in range(G):
        its, k = _shard_stream(kw, s, G, cuda_device, cm, n_events, rank=s)
        keep.append(k)
        assert [it.rank for it in its] == [s] * n_events and [it.gevt for it in its] == list(range(n_events))
        items += its
    random.Random(1).shuffle(items)
    asm = ShardAssembler(G, items[0].data.shape, cuda_device)
    frames = []
    for i in range(0, len(items), 7):
        frames += asm.add(items[i:i + 7])
    torch.cuda.synchronize()
    assert sorted(f.gevt for f in frames) == list(range(n_events)) and asm.pending == 0
    for f in frames:
        assert torch.equal(f.data, ref[f.gevt % 4]), f"event {f.gevt}"
