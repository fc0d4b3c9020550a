"""Online training consumer: queue batches -> peak-finder labels -> PeakNetLite optimizer step.

The reference's consumers are meant to feed a "PyTorch Task" (architecture figure; PeakNet in
setup.py:11).  :class:`OnlinePeakNetTrainer` is that task for one consumer GPU: each
:class:`~psana_ray_amd.batching.FrameBatch` (one gather launch from the leased ring slots) is
labelled by the K-07 peak finder on the GPU, and one AdamW step of
:class:`~psana_ray_amd.models.peaknet.PeakNetLite` runs in bf16 autocast.  Everything stays on the
consumer's GPU; the queue keeps streaming while the step runs (slots were released after the
gather).  ``psana-ray-consumer --task train`` drives it from the command line.

Data parallel (``ddp=True``, ``psana-ray-consumer --task train --ddp`` under torchrun): several
consumer processes -- one per GPU, each draining its own queue shard -- train ONE model: the
gradients are all-reduced by DistributedDataParallel over RCCL (backend "nccl", xGMI between the
GPUs; gloo on the CPU).  Consumers see different numbers of batches (the queue balances by
speed), so the loop runs under :meth:`join` (DDP's uneven-input join: a rank that ran out shadows
the others' all-reduces until every rank is done).
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch
import torch.nn.functional as F

from .config import PeakFinderParams
from .models.peaknet import PeakNetLite, normalize_panels, peak_masks


class OnlinePeakNetTrainer:
    def __init__(self, frame_shape, device, width: int = 16, lr: float = 1e-3,
                 params: Optional[PeakFinderParams] = None, bf16: bool = True, pos_weight: float = 20.0,
                 miopen: bool = True, ddp: bool = False):
        if len(frame_shape) != 3:
            raise ValueError(f"PeakNetLite trains on (panels, H, W) frames, got {tuple(frame_shape)}")
        P, H, W = frame_shape
        if H % 4 or W % 4:
            raise ValueError("panel height / width must be divisible by 4 (two 2x pooling levels)")
        self.shape = tuple(int(x) for x in frame_shape)
        self.device = torch.device(device)
        # MIOpen: immediate-mode solver choice instead of compiling + benchmarking every candidate
        # kernel for each new convolution shape (minutes of JIT on a fresh node with an empty
        # kernel cache); an explicit MIOPEN_FIND_MODE from the environment wins
        os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
        # miopen=False: PyTorch's im2col + GEMM convolutions (no per-shape kernel JIT; slower steps)
        self.miopen = miopen
        self.params = params or PeakFinderParams()
        self.model = PeakNetLite(width).to(self.device).to(memory_format=torch.channels_last)
        self.net = self.model
        if ddp:
            import torch.distributed as dist
            from torch.nn.parallel import DistributedDataParallel

            if not dist.is_initialized():
                raise RuntimeError("OnlinePeakNetTrainer(ddp=True) needs an initialised torch.distributed group")
            # every rank starts from rank 0's weights (DDP broadcasts them at construction)
            self.net = DistributedDataParallel(
                self.model, device_ids=[self.device.index] if self.device.type == "cuda" else None,
                broadcast_buffers=False)
        self.opt = torch.optim.AdamW(self.model.parameters(), lr=lr)
        self._pf_scratch = None
        self.bf16 = bf16 and self.device.type == "cuda"
        self.pos_weight = torch.tensor([pos_weight], device=self.device)
        self.steps = 0
        self.frames = 0
        self.last_loss = float("nan")
        self.positives = 0

    def labels(self, frames: torch.Tensor):
        """[B, P, H, W] f32 -> (targets [B*P, 1, H, W], peaks found) from the K-07 peak finder."""
        B = frames.shape[0]
        mp = self.params.max_peaks
        if frames.device.type == "cuda":
            from .ops import kernels

            pk = torch.empty((B, mp, 8), dtype=torch.float32, device=frames.device)
            cnt = torch.empty(B, dtype=torch.int32, device=frames.device)
            sm = torch.empty((B, 2), dtype=torch.float32, device=frames.device)
            if self._pf_scratch is None:
                self._pf_scratch = torch.zeros(kernels.PF_SCRATCH_WORDS, dtype=torch.int32, device=frames.device)
            kernels.peakfind([frames[i] for i in range(B)], self.shape, self.params, pk, cnt, sm,
                             torch.cuda.current_stream(frames.device), scratch=self._pf_scratch)
        else:
            from .ops import reference

            lists, _ = reference.peakfind_reference(frames, self.params)
            pk = torch.zeros((B, mp, 8), dtype=torch.float32)
            cnt = torch.zeros(B, dtype=torch.int32)
            for i, p in enumerate(lists):
                k = min(p.shape[0], mp)
                pk[i, :k] = p[:k]
                cnt[i] = k
        return peak_masks(pk, cnt, self.shape), cnt

    def step(self, frames: torch.Tensor) -> float:
        """One optimizer step on a [B, P, H, W] float32 batch (on this trainer's device)."""
        frames = frames.to(self.device).reshape(-1, *self.shape)
        target, cnt = self.labels(frames)
        x = normalize_panels(frames).contiguous(memory_format=torch.channels_last)
        self.model.train()
        ctx = torch.autocast("cuda", dtype=torch.bfloat16) if self.bf16 else contextlib.nullcontext()
        with torch.backends.cudnn.flags(enabled=self.miopen), ctx:
            logits = self.net(x)
            loss = F.binary_cross_entropy_with_logits(logits.float(), target, pos_weight=self.pos_weight)
            self.opt.zero_grad(set_to_none=True)
            loss.backward()
        self.opt.step()
        self.steps += 1
        self.frames += frames.shape[0]
        self.last_loss = float(loss.detach())
        self.positives += int(cnt.sum())
        return self.last_loss

    def join(self):
        """Context for the training loop: DDP's uneven-input join when data parallel, else nothing."""
        return self.net.join() if self.net is not self.model else contextlib.nullcontext()

    @torch.no_grad()
    def param_checksum(self) -> float:
        """Sum of all parameters (float64): equal on every rank of a data-parallel run."""
        return float(sum(p.detach().double().sum() for p in self.model.parameters()))

    @torch.no_grad()
    def predict(self, frames: torch.Tensor) -> torch.Tensor:
        """Peak probabilities [B*P, 1, H, W] for a [B, P, H, W] batch (eval mode)."""
        self.model.eval()
        x = normalize_panels(frames.to(self.device).reshape(-1, *self.shape)).contiguous(
            memory_format=torch.channels_last)
        ctx = torch.autocast("cuda", dtype=torch.bfloat16) if self.bf16 else contextlib.nullcontext()
        with torch.backends.cudnn.flags(enabled=self.miopen), ctx:
            return torch.sigmoid(self.model(x).float())
