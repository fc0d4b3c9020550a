"""Experiment: H2D straight out of a registered file mapping (tmpfs / page cache) vs out of a
hipHostMalloc'd pinned buffer.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psana_ray_amd.ops import _ext  # noqa: E402
from psana_ray_amd.parallel.launch import bind_numa_to_device  # noqa: E402

C = _ext.load()
dev = torch.device("cuda:0")
numa = bind_numa_to_device(dev)
FB = 16 * 352 * 384 * 2
N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
CH = 32
path = "/dev/shm/psray_mmap_exp.bin"
a = np.memmap(path, dtype=np.uint16, mode="w+", shape=(N, FB // 2))
a[:] = (np.arange(FB // 2, dtype=np.uint32) % 16381).astype(np.uint16)[None]
a[:, 0] = np.arange(N, dtype=np.uint16)
a.flush()
del a
out = {"numa": numa, "frames": N}
try:
    t0 = time.perf_counter()
    mf = C.MappedFile(path, True)
    out["map_register_s"] = round(time.perf_counter() - t0, 3)
    out["register_s"] = round(mf.register_s, 3)
    dst = torch.empty((CH, FB // 2), dtype=torch.int16, device=dev)
    s = torch.cuda.Stream(device=dev)
    h = int(s.cuda_stream)

    def run(base, reps=2, per_frame=False):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            for c in range(0, N - CH + 1, CH):
                if per_frame:   # one copy per 4.3 MB frame (what scattered file payloads need)
                    for j in range(CH):
                        C.memcpy_h2d_async(int(dst.data_ptr()) + j * FB, base + (c + j) * FB, FB, h)
                else:
                    C.memcpy_h2d_async(int(dst.data_ptr()), base + c * FB, CH * FB, h)
        s.synchronize()
        return reps * (N // CH) * CH * FB / (time.perf_counter() - t) / 1e9

    run(mf.ptr, 1)
    out["mapped_GBps"] = round(run(mf.ptr), 2)
    out["mapped_per_frame_GBps"] = round(run(mf.ptr, per_frame=True), 2)
    # correctness: frame 37 copied from the mapping
    C.memcpy_h2d_async(int(dst.data_ptr()), mf.ptr + 37 * FB, FB, h)
    s.synchronize()
    out["mapped_ok"] = int(dst[0, 0].item()) == 37 and int(dst[0, 5].item()) == 5
    pin = C.PinnedBuffer(N * FB)
    np.frombuffer(pin, dtype=np.uint8)[:] = 1
    run(pin.ptr, 1)
    out["pinned_GBps"] = round(run(pin.ptr), 2)
    out["pinned_per_frame_GBps"] = round(run(pin.ptr, per_frame=True), 2)
    del mf
except Exception as e:  # noqa: BLE001
    out["error"] = repr(e)
finally:
    os.unlink(path)
print(json.dumps(out))
