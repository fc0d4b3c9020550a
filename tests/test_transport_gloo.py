"""Multi-process shared-queue protocol over gloo on the CPU (same code path as RCCL; only the
byte mover differs): exactly-once delivery, data integrity, EOS without barriers, load balance,
and failure detection when a peer dies."""
import multiprocessing as mp
import random

import pytest

from tests._mp_workers import dying_consumer_worker, transport_worker


XPORTS = ["native", "python"]


def _run(world, roles, n_events, policy, slow_rank=-1, mode="calib", timeout=120, xport="native", shm_fail_rank=-1,
         expect_xport=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    ps = [ctx.Process(target=transport_worker, args=(r, world, port, roles, n_events, policy, q, slow_rank, mode, xport,
                                                     shm_fail_rank))
          for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, status, seen, bad, st = q.get(timeout=timeout)
            assert status == "ok", seen
            assert st["xport_used"] == (expect_xport or xport)
            res[r] = (seen, bad, st)
    finally:
        for p in ps:
            p.join(20)
            if p.is_alive():
                p.kill()
    return res


@pytest.mark.parametrize("xport", XPORTS)
@pytest.mark.parametrize("policy", ["balanced", "spread", "local_first"])
def test_two_ranks_exactly_once(native, policy, xport):
    res = _run(2, ["pc", "pc"], 20, policy, xport=xport)
    allseen = [k for r in res for k in res[r][0]]
    assert sorted(allseen) == sorted([(0, i) for i in range(10)] + [(1, i) for i in range(10)])
    assert all(res[r][1] == 0 for r in res), "frame content corrupted in transit"
    for r in res:                                             # FIFO per producer within a shard
        for p in (0, 1):
            idxs = [i for (pr, i) in res[r][0] if pr == p]
            assert idxs == sorted(idxs)
    if policy == "spread":
        assert res[0][2]["bytes_sent"] > 0 and res[1][2]["bytes_sent"] > 0


@pytest.mark.parametrize("fail_rank", [0, 2])
def test_shm_failure_falls_back_to_python_everywhere(native, fail_rank):
    """The shared-memory segment cannot be created (rank 0) or attached (rank 2): every rank must
    agree on the python driver and the stream still completes exactly once."""
    res = _run(3, ["p", "pc", "c"], 12, "balanced", xport="native", shm_fail_rank=fail_rank, expect_xport="python")
    allseen = [k for r in res for k in res[r][0]]
    assert sorted(allseen) == sorted([(0, i) for i in range(6)] + [(1, i) for i in range(6)])


@pytest.mark.parametrize("xport", XPORTS)
def test_producer_only_and_consumer_only_ranks(native, xport):
    res = _run(3, ["p", "p", "c"], 15, "balanced", xport=xport)
    assert sorted(res[2][0]) == sorted([(0, i) for i in range(8)] + [(1, i) for i in range(7)])
    assert res[0][0] == [] and res[1][0] == []


@pytest.mark.parametrize("xport", XPORTS)
def test_competing_consumers_slow_one_gets_less(native, xport):
    res = _run(3, ["p", "c", "c"], 60, "balanced", slow_rank=2, xport=xport)
    n1, n2 = len(res[1][0]), len(res[2][0])
    assert n1 + n2 == 60
    assert n1 > n2, f"fast consumer got {n1}, slow got {n2}"


@pytest.mark.parametrize("xport", XPORTS)
def test_dead_consumer_makes_producer_fail_cleanly(native, xport):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    ps = [ctx.Process(target=dying_consumer_worker, args=(r, 2, port, q, xport)) for r in range(2)]
    for p in ps:
        p.start()
    msgs = {}
    try:
        for _ in range(2):
            m = q.get(timeout=120)
            msgs[m[0]] = m
    finally:
        for p in ps:
            p.join(20)
            if p.is_alive():
                p.kill()
    assert msgs[1][1] == "exiting"
    assert msgs[0][1] == "peer-error", msgs[0]


def test_init_groups_reuses_but_never_owns_a_callers_process_group():
    """Q-13 fixed: a caller's own default process group is reused (when it matches the queue world)
    and marked not-owned, so DataReader.close() leaves it alive; a mismatched one is refused."""
    import socket

    import torch.distributed as dist

    from psana_ray_amd.parallel.comm import init_groups

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    assert not dist.is_initialized()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        comm = init_groups(0, 1, "cpu")
        assert not comm.owns_default_group
        comm.close()
        assert dist.is_initialized()
        with pytest.raises(RuntimeError, match="does not match"):
            init_groups(1, 2, "cpu")
    finally:
        dist.destroy_process_group()
