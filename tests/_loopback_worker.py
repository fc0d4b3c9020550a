"""Loopback transport integrity check (run as a subprocess: it owns a process group).

world == 1 with a real Comm and ``loopback=True``: every frame takes the multi-GPU data path
(control all-gather -> plan -> grouped send/recv to self -> end_recv events), so on one GPU this
exercises the RCCL transport the 2/4/8-GPU runs use.  Prints ``LOOPBACK_OK <frames> <bytes>``."""
import os
import socket
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(device: str, n: int) -> int:
    from psana_ray_amd.parallel.comm import init_groups
    from psana_ray_amd.queue import EndOfStream, FrameRing, QueueEndpoint

    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    comm = init_groups(0, 1, dev, master_addr="127.0.0.1", master_port=port, timeout_s=60)
    ring = FrameRing((2, 24, 40), torch.float32, dev, 8, 6)
    ep = QueueEndpoint(ring, 0, 1, comm, max_offer=4, loopback=True)
    seen = {}
    k = 0
    while True:
        # produce while slots are free, then one transport round, then drain what arrived
        while k < n:
            s = ep.acquire(timeout=0)
            if s is None:
                break
            ep.slot_tensor(s).fill_(float(k) + 0.5)
            ep.commit(s, 0, k, 1000 + k, 9.5 + k)
            k += 1
        if k == n:
            ep.finish()
        ep.step()
        try:
            while True:
                it = ep.get(timeout=0)
                if it is None:
                    break
                with it:
                    v = it.data.float()
                    exp = float(it.idx) + 0.5
                    if not bool((v == exp).all()):
                        print(f"BAD frame idx={it.idx}: {v.flatten()[:4].tolist()} != {exp}")
                        return 1
                    if it.gevt != 1000 + it.idx or abs(it.photon_energy - (9.5 + it.idx)) > 1e-9:
                        print(f"BAD header {it.rank} {it.idx} {it.gevt} {it.photon_energy}")
                        return 1
                    seen[it.idx] = seen.get(it.idx, 0) + 1
        except EndOfStream:
            break
    if sorted(seen) != list(range(n)) or any(c != 1 for c in seen.values()):
        print(f"BAD coverage: {len(seen)} distinct of {n}")
        return 1
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    print(f"LOOPBACK_OK {n} {comm.bytes_sent} native={comm.rccl is not None} xport={ep.xport}")
    import torch.distributed as dist
    ep.close()
    comm.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 100))
