"""Experiment: does the HIP runtime block the HOST on (a) large async pinned H2D copies or
(b) a copy stream waiting on an event of a busy compute stream?"""
import time
import torch
from psana_ray_amd.ops import _ext

C = _ext.load()
dev = torch.device("cuda:0")
frame = 16 * 352 * 384 * 2
chunk = 16 * frame
host = C.PinnedBuffer(8 * chunk)
dst = torch.empty(8 * chunk, dtype=torch.uint8, device=dev)
h2d = torch.cuda.Stream(device=dev)
comp = torch.cuda.Stream(device=dev)
torch.cuda.synchronize()

def issue(i):
    C.memcpy_h2d_async(int(dst.data_ptr()) + i * chunk, host.ptr + i * chunk, chunk, int(h2d.cuda_stream))

# (a) back-to-back copies
for _ in range(2):
    t = []
    t0 = time.perf_counter()
    for i in range(8):
        a = time.perf_counter(); issue(i); t.append(time.perf_counter() - a)
    issued = time.perf_counter() - t0
    h2d.synchronize()
    tot = time.perf_counter() - t0
print("a) per-call host us:", [round(x * 1e6) for x in t], "issue total ms", round(issued * 1e3, 2), "wall ms", round(tot * 1e3, 2),
      "GB/s", round(8 * chunk / tot / 1e9, 1))
# (b) copies waiting on events of a busy compute stream
evs = [torch.cuda.Event() for _ in range(8)]
for _ in range(2):
    with torch.cuda.stream(comp):
        for i in range(8):
            torch.cuda._sleep(2_000_000)     # ~1 ms busy kernel
            evs[i].record(comp)
    t = []
    t0 = time.perf_counter()
    for i in range(8):
        a = time.perf_counter(); h2d.wait_event(evs[i]); issue(i); t.append(time.perf_counter() - a)
    issued = time.perf_counter() - t0
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
print("b) per (wait+copy) host us:", [round(x * 1e6) for x in t], "issue total ms", round(issued * 1e3, 2), "wall ms",
      round(tot * 1e3, 2))
# (c) compute kernels concurrent with copies (no dependency)
for _ in range(2):
    with torch.cuda.stream(comp):
        for i in range(8):
            torch.cuda._sleep(2_000_000)
    t0 = time.perf_counter()
    for i in range(8):
        issue(i)
    h2d.synchronize()
    tot = time.perf_counter() - t0
    torch.cuda.synchronize()
print("c) copies beside busy kernels: wall ms", round(tot * 1e3, 2), "GB/s", round(8 * chunk / tot / 1e9, 1))
