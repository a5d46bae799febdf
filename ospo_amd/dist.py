"""Data parallelism over RCCL (torch.distributed backend "nccl" == RCCL on ROCm).

One process per GPU; preference pairs are sharded across ranks (the
DistributedSampler role of PL's DDPStrategy, ospo/utils/train.py:26-28); the
only data-path collective is the sum of the flat fp32 LoRA-gradient buffer
(DDP's bucketed all-reduce), divided by world size.  Frozen weights are built
locally on every rank -- nothing but the LoRA init is broadcast.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def init(backend: Optional[str] = None):
    """Join the process group of a torchrun-style launch; returns (world, rank, device index).
    backend None: RCCL ("nccl") when a GPU is present, else gloo.  With gloo the ranks may share
    GPUs (device = LOCAL_RANK mod device count): the multi-rank rehearsal on a one-GPU box."""
    world, rank, local = env_world()
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "gloo" and torch.cuda.is_available():
        local = local % max(1, torch.cuda.device_count())
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
            if torch.cuda.is_available():
                torch.cuda.set_device(local)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return world, rank, local


class GradAllReduce:
    """Sum + average the flat fp32 gradient buffer in fixed-size buckets.

    Buckets are contiguous slices (whole layers of the LoRA layout), issued
    back-to-back as async collectives and waited together."""

    def __init__(self, world: int, bucket_elems: int = 16 * 1024 * 1024, group=None):
        self.world, self.bucket, self.group = world, bucket_elems, group

    def __call__(self, flat: torch.Tensor):
        if self.world <= 1:
            return flat
        works = []
        for i in range(0, flat.numel(), self.bucket):
            works.append(dist.all_reduce(flat[i:i + self.bucket], op=dist.ReduceOp.SUM, group=self.group,
                                         async_op=True))
        for w in works:
            w.wait()
        flat.mul_(1.0 / self.world)
        return flat

    # ---- overlapped form: buckets launched as the backward finishes layers
    def begin(self, flat: torch.Tensor):
        """Start a step: ``push`` contiguous ranges as they become final, then ``finish``."""
        self._flat, self._works, self._pend = flat, [], None

    def push(self, lo: int, hi: int):
        """Elements [lo, hi) of the flat buffer are final on the CURRENT stream.  Adjacent
        ranges are merged until a bucket is full, then all-reduced asynchronously (the
        collective waits for the current stream's work so far, not for the whole backward)."""
        if self.world <= 1:
            return
        if self._pend is None:
            self._pend = [lo, hi]
        elif hi == self._pend[0]:      # backward walks layers in reverse: ranges grow downwards
            self._pend[0] = lo
        elif lo == self._pend[1]:
            self._pend[1] = hi
        else:
            self._flush()
            self._pend = [lo, hi]
        if self._pend[1] - self._pend[0] >= self.bucket:
            self._flush()

    def _flush(self):
        if self._pend is not None:
            lo, hi = self._pend
            self._works.append(dist.all_reduce(self._flat[lo:hi], op=dist.ReduceOp.SUM, group=self.group,
                                               async_op=True))
            self._pend = None

    def finish(self):
        """Launch the last bucket, make the current stream wait for every collective, average."""
        if self.world <= 1:
            return self._flat
        self._flush()
        for w in self._works:
            w.wait()
        self._works = []
        self._flat.mul_(1.0 / self.world)
        return self._flat


def broadcast_(t: torch.Tensor, src: int = 0, group=None):
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(t, src, group=group)
    return t


def all_reduce_mean_(t: torch.Tensor, group=None):
    """sync_dist=True logging (train.py:91-93,435-443): one fused all-reduce of the scalars."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.mul_(1.0 / dist.get_world_size(group))
    return t


def barrier():
    if dist.is_initialized():
        dist.barrier()
