"""Shared defaults and configuration dataclasses.

One module owns every default so producer and consumer agree (fixes reference quirk Q-3: the
reference producer defaults ``queue_name='my'`` / ``ray_namespace='default'``
(psana_ray/producer.py:26-27) while its DataReader defaults ``queue_name='shared_queue'`` /
``ray_namespace='my'`` (psana_ray/data_reader.py:5), so the documented consumer cannot find the
documented producer's queue).  The producer CLI keeps the reference's exact flag defaults; the
consumer side now defaults to the SAME values.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Optional

# --- reference CLI defaults (psana_ray/producer.py:17-33) -------------------------------
DEFAULT_RAY_ADDRESS = "auto"          # :25
DEFAULT_RAY_NAMESPACE = "default"     # :26
DEFAULT_QUEUE_NAME = "my"             # :27
DEFAULT_QUEUE_SIZE = 100              # :28 (also shared_queue.py:6,33)
DEFAULT_NUM_CONSUMERS = 1             # :29
DEFAULT_LOG_LEVEL = "INFO"            # :31
LOG_LEVELS = ["DEBUG", "INFO", "WARNING", "ERROR", "CRITICAL"]  # :32

# --- reference retry / backoff constants -------------------------------------------------
BACKOFF_BASE_S = 0.1                  # producer.py:85
BACKOFF_MAX_S = 2.0                   # producer.py:86
BACKOFF_JITTER_S = 0.5                # producer.py:109
TRANSIENT_RETRY_SLEEP_S = 1.0         # producer.py:117
QUEUE_LOOKUP_RETRIES = 10             # producer.py:35
QUEUE_LOOKUP_DELAY_S = 1.0            # producer.py:35
CONSUMER_POLL_SLEEP_S = 1.0           # examples/psana_consumer.py:40

# --- consumer read-ahead (elastic fabric) ----------------------------------------------------
# A consumer holds at most this many frames noticed-but-not-taken plus grants outstanding: the
# bound on what a crashed consumer loses (the reference's get() pops ONE item,
# psana_ray/shared_queue.py:19-24).  One producer chunk (64 frames) keeps a copy in flight while the
# previous one is read; DataReader.batches(n) raises it to 2 x n.
DEFAULT_PREFETCH = 64
# Hardware-queue placement of the pipeline's own streams: "shared" = ordinary HIP streams,
# multiplexed onto the process's GPU_MAX_HW_QUEUES hardware queues (two streams on one queue run
# one after the other); "dedicated" = one hardware queue per stream (csrc/streams.h); "high" =
# high-priority streams.
STREAM_KINDS = {"shared": 0, "dedicated": 1, "high": 2}
# Producer: chunks alternate over this many compute streams.  Measured on MI355X (bench.py, 200
# steps, profiles/r3/streams*/): raw frames already in HBM -> 3 dedicated streams (140.9-143.6k
# fr/s vs 134.5-134.6k on one ordinary stream; image mode 110.4-115.5k vs 104.7-105.5k: one
# chunk's calibration fills the CUs its predecessor's tail leaves, and the peak finder no longer
# queues behind it); host-staged (PCIe-bound) -> one ordinary stream (13,064-13,069 vs
# 12,852-12,858 with 3: concurrent calibrations delay the staging copy kernel).
# Round 4 (profiles/r4/sweep3/, interleaved, 4 rounds): 4 streams with 64-frame consumer batches
# 151.2-153.9k vs 142.9-144.7k for 3 streams / 32 (4 streams alone 145.8-147.9k, batch 64 alone
# 144.8-147.6k); image mode 128.8-129.0k vs 124.6-125.1k (sweep4/).  5 streams 152.3-153.2k vs
# 151.1-154.1k for 4, 6 streams 146.8-148.4k (sweep6/).
PRODUCER_STREAMS = {"device": 4, "staged": 1}
PRODUCER_STREAM_KIND = {"device": "dedicated", "staged": "shared"}
# Ranks sharing ONE GPU (an N-rank launch on fewer GPUs, e.g. `mpirun -n 4` on a one-GPU box,
# README.md:20): every process's dedicated streams are hardware queues of that one GPU, so the
# pipeline takes the round-3 shape there -- 3 producer compute streams (raw frames in HBM) and
# 32-frame consumer batches.  2 ranks on one GPU, device-resident: 142.8k fr/s with it, 83.6k
# with the one-rank-per-GPU shape (4 streams, 64) (profiles/r4/n2final/).
SHARED_GPU_PRODUCER_STREAMS = {"device": 3, "staged": 1}
SHARED_GPU_CONSUMER_BATCH = 32


def pipeline_shape(where: str, ranks_per_gpu: int = 1) -> dict:
    """Producer compute streams and consumer batch for a producer whose raw frames are ``where``
    ("device": already in HBM; "staged": pinned host memory) on a GPU shared by ``ranks_per_gpu``
    ranks (parallel.launch.ranks_per_gpu).  The one resolution the producer / consumer CLIs,
    ProducerPipeline, PeakFinderConsumer and bench.py all use."""
    if where not in PRODUCER_STREAMS:
        raise ValueError(f"pipeline_shape: where must be one of {sorted(PRODUCER_STREAMS)}, not {where!r}")
    shared = int(ranks_per_gpu) > 1
    return {"producer_streams": (SHARED_GPU_PRODUCER_STREAMS if shared else PRODUCER_STREAMS)[where],
            "consumer_batch": SHARED_GPU_CONSUMER_BATCH if shared else CONSUMER_BATCH}


# Consumer: the peak finder's two alternating streams, each on its own hardware queue (ordinary
# streams landed both on ONE queue: rocprofv3 Queue_Id, profiles/r3/streams2/).  Round 5: ordinary
# streams are within the noise for one rank per GPU (+0.3-1.3 %, profiles/r5/sweep2/, sweep3/) but
# lose where ranks share a GPU or frames cross processes (2 ranks on one GPU: host-staged -2.5 %,
# cross windows -3.6 / -3.8 %, profiles/r5/n2ab/), so the queues stay dedicated.
CONSUMER_STREAM_KIND = "dedicated"
CONSUMER_STREAMS = 2
# Frames per peak-finder launch of the in-process consumer (bench.py --batch, the producer CLI's
# co-consumer): one full launch (kernels.MAX_FRAMES) -- half as many launch ramps and drains per
# frame as 32 (host-staged headline unchanged: 13.01-13.04k either way, PCIe-bound)
CONSUMER_BATCH = 64
# Queue fabric (csrc/fabric.h): how a producer moves frames into OTHER processes' GPU rings.
# "kernel": every frame of one fabric pass, to all its consumers, in ONE copy_runs_kernel launch on
# a stream with its own hardware queue: 512 workgroups when a consumer sits on the same GPU (HBM ->
# HBM), plus FABRIC_COPY_WORKGROUPS per distinct peer GPU written (one xGMI link each,
# QueueFabric::copy_grid_for); a link whose frames are not 16-B multiples copies by "runtime":
# hipMemcpyAsync per contiguous run on one ordinary stream per link (the round-3 path; A/B only).
# FABRIC_COPY_STREAM: hardware-queue placement of the kernel engine's copy stream (STREAM_KINDS).
# Env override: PSANA_RAY_AMD_FABRIC_COPY=kernel|runtime[:workgroups[:stream kind]].
FABRIC_COPY_ENGINES = {"kernel": 0, "runtime": 1}
FABRIC_COPY_ENGINE = "kernel"
FABRIC_COPY_WORKGROUPS = 32
FABRIC_COPY_STREAM = "dedicated"


def fabric_copy_setting(engine: Optional[str] = None, workgroups: Optional[int] = None,
                        stream: Optional[str] = None) -> tuple[str, int, str]:
    """(engine, workgroups, stream kind) for a new fabric: explicit arguments, else the environment,
    else the defaults above."""
    parts = (os.environ.get("PSANA_RAY_AMD_FABRIC_COPY", "").split(":") + ["", "", ""])[:3]
    eng = engine or parts[0] or FABRIC_COPY_ENGINE
    if eng not in FABRIC_COPY_ENGINES:
        raise ValueError(f"unknown fabric copy engine {eng!r} ({' | '.join(FABRIC_COPY_ENGINES)})")
    wgs = workgroups if workgroups else (int(parts[1]) if parts[1] else FABRIC_COPY_WORKGROUPS)
    kind = stream or parts[2] or FABRIC_COPY_STREAM
    if kind not in STREAM_KINDS:
        raise ValueError(f"unknown stream kind {kind!r} ({' | '.join(STREAM_KINDS)})")
    return eng, int(wgs), kind

# End-to-end frame checks of the fabric (csrc/verify.h): a producer attaches a content checksum to
# every FABRIC_VERIFY_EVERY-th frame (rank-local idx % N == 0) it sends to another process; the consumer re-sums
# it from its own ring before the caller reads it and counts matches / mismatches on the device.
# 1/64 of the routed frames = one extra 8.65-MB read per 64 frames on each side.  0 disables.
# Env override: PSANA_RAY_AMD_VERIFY_EVERY.
FABRIC_VERIFY_EVERY = 64


# Direct writes (csrc/fabric.h set_direct): while frames are routed to other processes (spread /
# remote_only), a GPU producer calibrates them straight into granted consumer slots instead of into
# its own slot plus a copy pass.  Env override: PSANA_RAY_AMD_FABRIC_DIRECT=0|1.
FABRIC_DIRECT = True


def fabric_direct() -> bool:
    v = os.environ.get("PSANA_RAY_AMD_FABRIC_DIRECT", "").strip()
    return FABRIC_DIRECT if not v else v not in ("0", "false", "off")


# Direct headroom (csrc/engine.h set_direct_headroom): producer slots kept for direct frames; frames
# in local slots (the copy path's backlog) stay within the rest of the budget (the one queue_size
# gives), and while grants are on offer a chunk that would pass it waits for grants (or for the
# backlog to drain; FABRIC_DIRECT_WAIT_S > 0 bounds the wait).  Producers that route to other
# processes add it to their slot budget (bench.py, psana-ray-producer), at most
# FABRIC_DIRECT_HEADROOM_BYTES of HBM.  Env overrides: PSANA_RAY_AMD_FABRIC_DIRECT_HEADROOM (slots;
# 0 = off: direct grants only when on offer at launch), PSANA_RAY_AMD_FABRIC_DIRECT_WAIT_S.
FABRIC_DIRECT_HEADROOM = 384
FABRIC_DIRECT_HEADROOM_BYTES = 8 << 30
FABRIC_DIRECT_WAIT_S = 0.0


def fabric_direct_headroom(frame_bytes: Optional[int] = None) -> int:
    if not fabric_direct():
        return 0
    v = os.environ.get("PSANA_RAY_AMD_FABRIC_DIRECT_HEADROOM", "").strip()
    n = max(0, int(v)) if v else FABRIC_DIRECT_HEADROOM
    if frame_bytes:
        n = min(n, FABRIC_DIRECT_HEADROOM_BYTES // max(1, int(frame_bytes)))
    return n


def fabric_direct_wait_s() -> float:
    v = os.environ.get("PSANA_RAY_AMD_FABRIC_DIRECT_WAIT_S", "").strip()
    return max(0.0, float(v)) if v else FABRIC_DIRECT_WAIT_S


def fabric_verify_every() -> int:
    v = os.environ.get("PSANA_RAY_AMD_VERIFY_EVERY", "")
    return max(0, int(v)) if v.strip() else FABRIC_VERIFY_EVERY


# --- rendezvous ---------------------------------------------------------------------------
DEFAULT_STORE_PORT = 6379             # the Ray head port of README.md:15, reused for the store
ENV_ADDRESS = "PSANA_RAY_ADDRESS"


def resolve_address(address: Optional[str]) -> tuple[str, int]:
    """Map the reference's ``--ray_address`` value to a rendezvous ``(host, port)``.

    ``"auto"`` (the reference default) means: ``$PSANA_RAY_ADDRESS`` if set, else
    ``127.0.0.1:6379``.  ``host``, ``host:port`` and ``ray://host:port`` are accepted.
    """
    if address is None or address == "auto":
        address = os.environ.get(ENV_ADDRESS, f"127.0.0.1:{DEFAULT_STORE_PORT}")
    if "://" in address:
        address = address.split("://", 1)[1]
    if ":" in address:
        host, port = address.rsplit(":", 1)
        return host or "127.0.0.1", int(port)
    return address, DEFAULT_STORE_PORT


@dataclass
class CommonModeParams:
    """psana "mode 7"-like common-mode parameters (K-03).

    flags: bit0 = rows by bank segment, bit1 = columns (within each ASIC).
    thr: only pixels with |ADU - pedestal| < thr estimate the median.
    maxcorr: corrections with |median| > maxcorr are skipped.
    npix_min: minimum number of participating pixels.
    """

    flags: int = 3
    thr: float = 30.0
    maxcorr: float = 50.0
    npix_min: int = 10
    bank_cols: Optional[int] = None   # None -> detector default (epix10ka: 48)

    @staticmethod
    def parse(text: Optional[str]) -> Optional["CommonModeParams"]:
        """``"off"``/``None`` -> None; ``"default"`` -> defaults; else ``flags,thr,maxcorr,npix_min[,bank]``."""
        if text is None or text.lower() in ("", "none", "off", "0"):
            return None
        if text.lower() in ("default", "on", "1"):
            return CommonModeParams()
        parts = [p.strip() for p in text.split(",")]
        cm = CommonModeParams(flags=int(parts[0]))
        if len(parts) > 1:
            cm.thr = float(parts[1])
        if len(parts) > 2:
            cm.maxcorr = float(parts[2]) if parts[2].lower() != "inf" else math.inf
        if len(parts) > 3:
            cm.npix_min = int(parts[3])
        if len(parts) > 4:
            cm.bank_cols = int(parts[4])
        return cm


# Common-mode kernel tables: carry each pixel's CM eligibility in the sign bit of its pedestal
# (CalibConstants.cm_signed_pedestals) instead of a separate bit-plane array, which saves one global
# load per 8-pixel group in the kernel's first phase.  Used when every pedestal is >= 0 (otherwise
# the bit-planes); False forces the bit-planes.
CM_SIGNED_PEDESTALS = True

# Common mode by detector family when the CLI says "auto" (the producer's default): psana's calib of
# an ePix10ka includes common mode (SURVEY E-03 / Appendix B), Jungfrau has none by default.
CM_AUTO_FAMILIES = ("epix10ka",)


def resolve_common_mode(text: Optional[str], spec) -> Optional["CommonModeParams"]:
    """``--common_mode`` value -> parameters for detector ``spec`` (models.detector.DetectorSpec):
    ``auto`` = the defaults for families whose psana calibration applies common mode, else off;
    anything else as :meth:`CommonModeParams.parse`.  The bank width comes from the detector."""
    if text is not None and text.lower() == "auto":
        cm = CommonModeParams() if spec.kind in CM_AUTO_FAMILIES else None
    else:
        cm = CommonModeParams.parse(text)
    if cm is not None and cm.bank_cols is None:
        cm.bank_cols = spec.bank_cols
    return cm


@dataclass
class PeakFinderParams:
    """K-07 consumer peak finder parameters."""

    thr_peak: float = 20.0   # keV-domain threshold on the calibrated pixel
    son_min: float = 5.0     # minimum signal-over-noise vs the background ring
    radius: int = 1          # local-maximum window radius (1 -> 3x3, 2 -> 5x5)
    max_peaks: int = 2048    # peak records kept per frame


@dataclass
class QueueConfig:
    """Everything that defines one shared queue instance."""

    queue_name: str = DEFAULT_QUEUE_NAME
    ray_namespace: str = DEFAULT_RAY_NAMESPACE
    address: str = DEFAULT_RAY_ADDRESS
    queue_size: int = DEFAULT_QUEUE_SIZE
    num_consumers: int = DEFAULT_NUM_CONSUMERS
    # physical HBM slots are capped by this fraction of free device memory (H-8: queue_size is
    # a LOGICAL bound, the reference never pre-allocates: shared_queue.py:7)
    hbm_fraction: float = 0.80
    producer_slots: int = 64          # calibrated frames a producer may hold un-routed
    route: str = "balanced"           # balanced | local_first | spread
    connect_timeout_s: float = 300.0
    extra: dict = field(default_factory=dict)
