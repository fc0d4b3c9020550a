"""Worker bodies for the multi-process (gloo, CPU) transport tests -- importable for spawn."""
import os
import time

import numpy as np
import torch


def transport_worker(rank, world, port, roles, n_events, policy, out_q, slow_rank=-1, mode="calib", xport="native",
                     shm_fail_rank=-1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["PSANA_RAY_XPORT"] = xport
    if shm_fail_rank >= 0:
        os.environ["PSANA_RAY_XPORT_TEST_FAIL_RANK"] = str(shm_fail_rank)
    os.environ["MASTER_PORT"] = str(port)
    try:
        from psana_ray_amd.models import Calibrator, Mode
        from psana_ray_amd.ops import reference
        from psana_ray_amd.parallel.comm import init_groups
        from psana_ray_amd.pipeline import ProducerPipeline
        from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint
        from psana_ray_amd.source import SyntheticRun

        comm = init_groups(rank, world, "cpu", master_addr="127.0.0.1", master_port=port, timeout_s=60)
        prods = [r for r in range(world) if "p" in roles[r]]
        cons = [r for r in range(world) if "c" in roles[r]]
        is_p, is_c = "p" in roles[rank], "c" in roles[rank]
        psize = len(prods)
        prank = prods.index(rank) if is_p else 0
        src = SyntheticRun("synthetic", 2, "tiny_epix", rank=prank, size=psize, n_events=n_events, pool_frames=3,
                           gen_device="cpu")
        cal = Calibrator(src.consts, "cpu", Mode(mode))
        ring = FrameRing(cal.out_shape, cal.out_dtype, "cpu", 4, 5 if is_c else 0 or 1)
        ep = QueueEndpoint(ring, rank, world, comm, producer_ranks=prods, consumer_ranks=cons, route=policy,
                           max_offer=8, is_producer=is_p, is_consumer=is_c)
        ep.start()
        import threading

        th = None
        if is_p:
            prod = ProducerPipeline(src, cal, ep, rank=prank, chunk=3)
            th = threading.Thread(target=prod.run)
            th.start()
        seen = []
        bad = 0
        refs = {}
        if is_c:
            while True:
                try:
                    it = ep.get(timeout=0.2)
                except EndOfStream:
                    break
                if it is None:
                    continue
                if rank == slow_rank:
                    time.sleep(0.02)
                key = (it.rank, it.idx)
                if mode == "calib":
                    if it.rank not in refs:
                        s2 = SyntheticRun("synthetic", 2, "tiny_epix", rank=it.rank, size=psize, pool_frames=3,
                                          gen_device="cpu")
                        refs[it.rank] = reference.calibrate_reference(torch.from_numpy(s2.pool.astype(np.int32)),
                                                                      s2.consts)
                    if not torch.equal(it.data, refs[it.rank][it.idx % 3]):
                        bad += 1
                assert it.gevt == it.rank + it.idx * psize
                seen.append(key)
                it.release()
        if th is not None:
            th.join(60)
        ep.join(60)
        st = ep.stats()
        st["xport_used"] = ep.xport
        out_q.put((rank, "ok", seen, bad, st))
        import torch.distributed as dist

        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback

        out_q.put((rank, "err", traceback.format_exc(), 0, {}))


def dying_consumer_worker(rank, world, port, out_q, xport="native"):
    """rank 1 (consumer) exits abruptly mid-stream; rank 0 (producer) must fail cleanly."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["PSANA_RAY_XPORT"] = xport
    os.environ["MASTER_PORT"] = str(port)
    from psana_ray_amd.models import Calibrator, Mode
    from psana_ray_amd.parallel.comm import init_groups
    from psana_ray_amd.pipeline import ProducerPipeline
    from psana_ray_amd.queue import FrameRing, QueueEndpoint, QueuePeerError

    comm = init_groups(rank, world, "cpu", master_addr="127.0.0.1", master_port=port, timeout_s=20)
    from psana_ray_amd.source import SyntheticRun

    src = SyntheticRun("synthetic", 2, "tiny_epix", rank=0, size=1, n_events=None, pool_frames=2, gen_device="cpu")
    cal = Calibrator(src.consts, "cpu", Mode.calib)
    is_p = rank == 0
    ring = FrameRing(cal.out_shape, cal.out_dtype, "cpu", 4, 4)
    ep = QueueEndpoint(ring, rank, world, comm, producer_ranks=[0], consumer_ranks=[1], max_offer=4,
                       is_producer=is_p, is_consumer=not is_p)
    ep.start()
    if rank == 1:
        n = 0
        while n < 5:
            it = ep.get(timeout=0.2)
            if it is not None:
                it.release()
                n += 1
        out_q.put((1, "exiting"))
        out_q.close()
        out_q.join_thread()   # flush before dying
        os._exit(0)   # fault injection: the consumer dies without any goodbye
    t0 = time.time()
    prod = ProducerPipeline(src, cal, ep, rank=0, chunk=2, acquire_timeout_s=0.1)
    try:
        prod.run()
        out_q.put((0, "no-error", time.time() - t0))
    except QueuePeerError as e:
        out_q.put((0, "peer-error", time.time() - t0))
    except Exception as e:
        out_q.put((0, f"other:{type(e).__name__}:{e}", time.time() - t0))
    out_q.close()
    out_q.join_thread()
    os._exit(0)
