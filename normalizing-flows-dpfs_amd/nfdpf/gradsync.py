"""Data-parallel gradient reduction for batch-sharded training.

Every rank filters its own rows of the batch (global rows [rank*B, (rank+1)*B)) and
back-propagates its own shard's loss; the parameter gradients are then averaged over the
ranks with ONE all-reduce of a single flat fp32 bucket per step (RCCL over xGMI on the GPU
node; gloo on CPU).  The models are small (the coupling nets are ~1-5 k parameters, the frame
encoder/decoder a few hundred k), so one bucket is latency-optimal on xGMI's point-to-point
links -- splitting it would only add per-collective latency.  The reference trains on one
device (DPFs.py:304-383); the averaged gradient equals the gradient of the mean loss over the
whole batch when the shards are equal.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world_size(group=None) -> int:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


class GradBucket:
    """Flat buffer over a module's parameters; ``sync()`` averages their .grad over ranks."""

    def __init__(self, module: torch.nn.Module, group=None):
        self.params = [p for p in module.parameters() if p.requires_grad]
        self.group = group
        self._buf = None

    def sync(self) -> None:
        w = world_size(self.group)
        if w == 1 or not self.params:
            return
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        if self._buf is None or self._buf.numel() != n or self._buf.device != dev:
            self._buf = torch.empty(n, device=dev, dtype=torch.float32)
        buf = self._buf
        off = 0
        for p in self.params:  # a parameter with no gradient contributes zeros on this rank
            k = p.numel()
            if p.grad is None:
                buf[off:off + k].zero_()
            else:
                buf[off:off + k].copy_(p.grad.reshape(-1))
            off += k
        dist.all_reduce(buf, group=self.group)
        buf.mul_(1.0 / w)
        off = 0
        for p in self.params:
            k = p.numel()
            g = buf[off:off + k].view_as(p).to(p.dtype)
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.copy_(g)
            off += k


def global_mean(local_sum: torch.Tensor, local_count: int, group=None) -> torch.Tensor:
    """torch.mean over the whole (sharded) batch from this rank's sum and row count -- the
    batch-global ESS gate of DPFs.py:163-165 in the autograd loop."""
    if world_size(group) == 1:
        return local_sum / local_count
    t = torch.stack([local_sum.detach().double().reshape(()),
                     torch.tensor(float(local_count), dtype=torch.float64, device=local_sum.device)])
    dist.all_reduce(t, group=group)
    return (t[0] / t[1]).to(local_sum.dtype)
