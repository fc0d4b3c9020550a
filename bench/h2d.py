#!/usr/bin/env python3
"""Host->HBM staging bandwidth: pinned pool -> device, 1/2/4 concurrent streams (SDMA engines),
several chunk sizes.  Tells how close the producer's staging path is to PCIe Gen5 x16."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from psana_ray_amd.ops import _ext


def main():
    C = _ext.load()
    dev = torch.device("cuda:0")
    frame = 16 * 352 * 384 * 2
    nfr = 64
    host = C.PinnedBuffer(nfr * frame)
    import numpy as np
    np.frombuffer(host, dtype=np.uint8)[:] = 1
    dst = torch.empty(nfr * frame, dtype=torch.uint8, device=dev)
    res = []
    for chunk in (4, 16, 32):
        for nstreams in (1, 2, 4):
            streams = [torch.cuda.Stream(device=dev) for _ in range(nstreams)]
            def run(iters):
                for it in range(iters):
                    for c0 in range(0, nfr, chunk):
                        part = chunk * frame // nstreams
                        for k, s in enumerate(streams):
                            off = c0 * frame + k * part
                            C.memcpy_h2d_async(int(dst.data_ptr()) + off, host.ptr + off, part, int(s.cuda_stream))
                for s in streams:
                    s.synchronize()
            run(2)
            t0 = time.perf_counter()
            iters = 5
            run(iters)
            dt = time.perf_counter() - t0
            r = {"chunk_frames": chunk, "streams": nstreams, "GB_per_s": round(iters * nfr * frame / dt / 1e9, 2),
                 "epix_raw_frames_per_s": round(iters * nfr / dt, 1)}
            res.append(r)
            print(json.dumps(r), flush=True)
    # the producer engine's default staging path: copy_h2d_kernel with a few persistent workgroups
    s = torch.cuda.Stream(device=dev)
    for wgs in (16, 32, 64, 128):
        def runk(iters):
            for it in range(iters):
                for c0 in range(0, nfr, 32):
                    off = c0 * frame
                    assert C.copy_h2d_kernel(int(dst.data_ptr()) + off, host.ptr + off, 32 * frame, wgs,
                                             int(s.cuda_stream)), "copy kernel not applicable"
            s.synchronize()
        runk(2)
        t0 = time.perf_counter()
        iters = 5
        runk(iters)
        dt = time.perf_counter() - t0
        r = {"copy_kernel_workgroups": wgs, "chunk_frames": 32, "GB_per_s": round(iters * nfr * frame / dt / 1e9, 2),
             "epix_raw_frames_per_s": round(iters * nfr / dt, 1)}
        print(json.dumps(r), flush=True)
    assert torch.all(dst[:1 << 20] == 1).item(), "copy kernel wrote wrong bytes"


if __name__ == "__main__":
    main()
