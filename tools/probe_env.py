"""One-off environment probe run on the GPU box (H2D bandwidth, RCCL duplicate-GPU check)."""
import os, sys, time, json
import torch

def h2d_bw():
    dev = torch.device("cuda:0")
    out = {}
    for mb in (4, 35, 277):
        n = mb * (1 << 20)
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        h.fill_(1)
        d = torch.empty(n, dtype=torch.uint8, device=dev)
        s = torch.cuda.Stream()
        for _ in range(3):
            with torch.cuda.stream(s):
                d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        it = 20
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            for _ in range(it):
                d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out[f"h2d_{mb}MB_GBps"] = n * it / dt / 1e9
        # D2D
        d2 = torch.empty_like(d)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(it):
            d2.copy_(d)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out[f"d2d_{mb}MB_GBps(read+write)"] = 2 * n * it / dt / 1e9
    return out

def dup_gpu_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world)
        t = torch.ones(4, device="cuda:0") * (rank + 1)
        dist.all_reduce(t)
        torch.cuda.synchronize()
        buf = torch.zeros(1 << 20, device="cuda:0")
        if rank == 0:
            ops = [dist.P2POp(dist.isend, torch.full((1 << 20,), 7.0, device="cuda:0"), 1)]
        else:
            ops = [dist.P2POp(dist.irecv, buf, 0)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        torch.cuda.synchronize()
        q.put((rank, "ok", float(t[0]), float(buf[0])))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, "err", repr(e)[:500]))

if __name__ == "__main__":
    res = {"torch": torch.__version__, "hip": torch.version.hip,
           "device": torch.cuda.get_device_name(0), "n_gpus": torch.cuda.device_count()}
    p = torch.cuda.get_device_properties(0)
    res["cus"] = p.multi_processor_count
    res["mem_GB"] = p.total_memory / 1e9
    res["gcn"] = getattr(p, "gcnArchName", "?")
    res.update(h2d_bw())
    print(json.dumps(res), flush=True)
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=dup_gpu_worker, args=(r, 2, 29555, q)) for r in range(2)]
    for pr in procs: pr.start()
    outs = []
    for _ in range(2):
        try:
            outs.append(q.get(timeout=120))
        except Exception as e:
            outs.append(("timeout", repr(e)))
    for pr in procs:
        pr.join(timeout=10)
        if pr.is_alive(): pr.kill()
    res["dup_gpu_nccl"] = outs
    print(json.dumps(res), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/probe_env.json", "w") as f:
        json.dump(res, f, indent=1)
