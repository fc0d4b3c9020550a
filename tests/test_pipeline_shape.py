"""Shared-GPU pipeline shape: ranks of one launch that share a GPU take the
shape measured for it (3 producer compute streams, 32-frame consumer batches) -- and the producer
CLI's pipeline, its co-consumer, psana-ray-consumer and bench.py all resolve it the same way
(`mpirun -n 4 psana-ray-producer` on a box with fewer GPUs, /root/reference/README.md:20)."""
import pytest
import torch

import bench
from psana_ray_amd import consumer as consumer_cli
from psana_ray_amd.config import CONSUMER_BATCH, PRODUCER_STREAMS, pipeline_shape
from psana_ray_amd.parallel.launch import detect, ranks_per_gpu
from psana_ray_amd.pipeline import PeakFinderConsumer, resolve_consumer_batch, resolve_producer_streams


@pytest.mark.parametrize("lws", [1, 2, 4])
@pytest.mark.parametrize("launcher", ["torchrun", "openmpi", "mpich"])
def test_cli_and_bench_resolve_the_same_shape(monkeypatch, lws, launcher):
    for k in ("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", "RANK", "WORLD_SIZE",
              "OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "PMI_RANK", "PMI_SIZE"):
        monkeypatch.delenv(k, raising=False)
    env = {"torchrun": {"RANK": "0", "WORLD_SIZE": str(lws), "LOCAL_WORLD_SIZE": str(lws)},
           "openmpi": {"OMPI_COMM_WORLD_RANK": "0", "OMPI_COMM_WORLD_SIZE": str(lws),
                       "OMPI_COMM_WORLD_LOCAL_SIZE": str(lws)},
           "mpich": {"PMI_RANK": "0", "PMI_SIZE": str(lws), "MPI_LOCALNRANKS": str(lws)}}[launcher]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)   # one GPU on the node
    assert detect().local_size == lws
    assert ranks_per_gpu() == lws
    shared = lws > 1
    want_streams = 3 if shared else PRODUCER_STREAMS["device"]
    want_batch = 32 if shared else CONSUMER_BATCH
    # the library
    assert pipeline_shape("device", lws) == {"producer_streams": want_streams, "consumer_batch": want_batch}
    assert resolve_producer_streams("device") == want_streams
    assert resolve_producer_streams("staged") == 1
    assert resolve_consumer_batch() == want_batch
    # psana-ray-consumer --task peakfind / train without --batch
    assert consumer_cli.resolve_batch(None) == want_batch
    # bench.py (device-resident and host-staged)
    for src, streams in (("device", want_streams), ("host", 1)):
        share, batch, cs = bench.resolve_shape(bench.parse(["--source", src]), gpu=True)
        assert (share, batch, cs) == (lws, want_batch, streams)
    # explicit flags win
    share, batch, cs = bench.resolve_shape(bench.parse(["--source", "device", "--batch", "8", "--compute-streams", "2"]),
                                           gpu=True)
    assert (batch, cs) == (8, 2)


def test_co_consumer_takes_the_resolved_batch(monkeypatch):
    """The producer CLI's co-located consumer is built without a batch: it gets the resolution."""
    from psana_ray_amd.queue import FrameRing, QueueEndpoint

    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    ring = FrameRing((1, 8, 8), torch.float32, torch.device("cpu"), 4, 4)
    ep = QueueEndpoint(ring)
    assert PeakFinderConsumer(ep, (1, 8, 8)).batch == 32
    assert PeakFinderConsumer(ep, (1, 8, 8), ranks_per_gpu=1).batch == CONSUMER_BATCH
