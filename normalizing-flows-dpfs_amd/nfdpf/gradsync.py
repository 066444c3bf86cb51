"""Data-parallel gradient reduction for batch-sharded training.

Every rank filters its own rows of the batch (global rows [rank*B, (rank+1)*B)) and
back-propagates its own shard's loss; the parameter gradients are then averaged over the
ranks with ONE all-reduce of a single flat fp32 bucket per step (RCCL over xGMI on the GPU
node; gloo on CPU).  The models are small (the coupling nets are ~1-5 k parameters, the frame
encoder/decoder a few hundred k), so one bucket is latency-optimal on xGMI's point-to-point
links -- splitting it would only add per-collective latency.  The reference trains on one
device (DPFs.py:304-383).

What the average reproduces: for a loss that is a MEAN over batch rows (the auto-encoder MSE,
the pseudo-likelihood) the average of the per-shard gradients is the full-batch gradient
when the shards are equal.  The supervised loss is an RMSE, sqrt(mean(err^2)), whose per-shard
gradients do NOT average to the full-batch one; ``global_rmse`` therefore builds it from the
all-reduced sum of squared errors, with a gradient scaled so that the bucket's average is
exactly d RMSE_full / d theta.  Parameters no rank produced a gradient for keep ``.grad = None``
(as on one device), so the optimiser state matches the reference's.
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
        P = len(self.params)
        dev = self.params[0].device
        if self._buf is None or self._buf.numel() != n + P or self._buf.device != dev:
            self._buf = torch.empty(n + P, device=dev, dtype=torch.float32)
        buf = self._buf
        # the gradients (zeros where a parameter has none) in one cat, the presence flags in one
        # host->device copy: a few launches per step, not one per parameter
        grads = [p.grad.reshape(-1).to(torch.float32) if p.grad is not None
                 else torch.zeros(p.numel(), device=dev, dtype=torch.float32) for p in self.params]
        torch.cat(grads, out=buf[:n])
        flags = torch.tensor([0.0 if p.grad is None else 1.0 for p in self.params], dtype=torch.float32)
        buf[n:].copy_(flags)
        dist.all_reduce(buf, group=self.group)
        present = buf[n:].cpu()
        buf = buf[:n]
        buf.mul_(1.0 / w)
        off = 0
        for j, p in enumerate(self.params):
            k = p.numel()
            if float(present[j]) == 0.0:  # no rank touched it: leave it as one device would
                p.grad = None
            else:
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


def global_rmse(err2_sum: torch.Tensor, count: float, group=None) -> torch.Tensor:
    """sqrt(sum over ALL ranks of err2_sum / sum of count) -- the full-batch RMSE of a
    batch-sharded run (losses.py:18-31) -- with a gradient that GradBucket's average over the
    ranks turns into exactly d RMSE_full / d theta: the value is built from the all-reduced
    sum, the local term carries w times its gradient (the bucket divides by w)."""
    w = world_size(group)
    if w == 1:
        return torch.sqrt(err2_sum / count)
    t = torch.stack([err2_sum.detach().double().reshape(()),
                     torch.tensor(float(count), dtype=torch.float64, device=err2_sum.device)])
    dist.all_reduce(t, group=group)
    s_glob = t[0].to(err2_sum.dtype)
    s_eff = s_glob + w * (err2_sum - err2_sum.detach())
    return torch.sqrt(s_eff / t[1].to(err2_sum.dtype))


def sharded_supervised_loss(particle_list, particle_weight_list, true_state, mask, train, labeledRatio=1.0,
                            group=None):
    """losses.supervised_loss over the whole sharded batch (value and gradient of the
    single-device loss); returns (loss, this rank's predictions)."""
    prediction = torch.sum(particle_list * particle_weight_list[:, :, :, None], dim=2)
    err2 = (prediction - true_state[:, :, :2]) ** 2
    if not train:
        return global_rmse(err2.sum(), err2.numel(), group), prediction
    if labeledRatio > 0:
        return global_rmse((mask[:, :, None] * err2).sum(), err2.numel() * labeledRatio, group), prediction
    return 0
