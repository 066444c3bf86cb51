"""Differentiable resamplers (resamplers/resamplers.py of the reference) on libnfdpf.

* ``soft_resampler`` (resamplers.py:20-60): the HIP kernel reproduces the reference's
  indices bit for bit (same reduction orders, exact f64 prefix, lower-bound search) without
  the B x N x N comparison tensor; gradients (training) flow through the gathered weights
  p/q as in the reference, computed by nfdpf_soft_resample_backward.
* ``resampler_ot`` (resamplers.py:62-277): streamed Sinkhorn with the reference's
  batch-coupled stop rule; the transport matrix is never materialised.  As in the
  reference, the particles' gradient is T^T g with T treated as a constant (its own
  autograd.grad result is discarded, :241-245) -- nfdpf_ot_transport_backward.
"""
import torch
import torch.nn as nn

from nfdpf import ops as _ops
from nfdpf.gradsync import world_size

device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


class resampler(nn.Module):
    """Dispatch on ``param.resampler_type`` ('ot' | 'soft') (resamplers.py:6-17)."""

    def __init__(self, param):
        super().__init__()
        if param.resampler_type == "ot":
            self.kargs = {"eps": param.epsilon, "scaling": param.scaling, "threshold": param.threshold,
                          "max_iter": param.max_iter, "device": device}
            self.resampling = resampler_ot
        elif param.resampler_type == "soft":
            self.kargs = {"num_resampled": param.num_particles, "index": True, "alpha": param.alpha,
                          "device": device}
            self.resampling = soft_resampler

    def forward(self, particles, particle_probs):
        return self.resampling(particles, particle_probs, **self.kargs)


class _SoftResample(torch.autograd.Function):
    """soft_resampler with the HIP backward (nfdpf_soft_resample_backward): dL/dx by in-order
    run sums over the sorted indices, dL/dp through w = p / q and the output normalisation."""

    @staticmethod
    def forward(ctx, particles, particle_probs, alpha, offsets):
        xo, wo, idx = _ops.soft_resample(particles, particle_probs, alpha, offsets)
        ctx.save_for_backward(particle_probs, idx, wo)
        ctx.alpha, ctx.D, ctx.dtypes = alpha, particles.shape[-1], (particles.dtype, particle_probs.dtype)
        ctx.mark_non_differentiable(idx)
        return xo, wo, idx

    @staticmethod
    def backward(ctx, g_xo, g_wo, _g_idx):
        p, idx, wo = ctx.saved_tensors
        gx, gp = _ops.soft_resample_backward(p, idx, wo, g_xo, g_wo, ctx.alpha, ctx.D)
        return gx.to(ctx.dtypes[0]), gp.to(ctx.dtypes[1]), None, None


def soft_resampler(particles, particle_probs, alpha, num_resampled, index=True, device="cuda", offsets=None):
    """Soft resampling with q = alpha p + (1 - alpha)/N; the CPU-generator offset draw of
    the reference (:43) is kept (pass ``offsets`` to supply it)."""
    assert 0.0 < alpha <= 1.0
    B, N = particle_probs.shape
    if offsets is None:
        offsets = torch.FloatTensor(B).uniform_(0.0, 1.0 / num_resampled)
    if torch.is_grad_enabled() and (particles.requires_grad or particle_probs.requires_grad):
        xo, wo, idx = _SoftResample.apply(particles, particle_probs, alpha, offsets)
    else:
        xo, wo, idx = _ops.soft_resample(particles.detach(), particle_probs.detach(), alpha, offsets)
    return (xo, wo, idx) if index else (xo, wo)


# The process group the autograd loop's Sinkhorn stop is reduced over (None: the default
# group -- the group DPFs.DPF's ShardInfo.from_env shards the batch over, so both paths agree).
# A caller that shards a DPF over a subgroup must set this to that group as well.
SHARD_GROUP = None


def _ot_call(particles, weights, eps, scaling, threshold, max_iter, keep=None):
    """One Sinkhorn resampling with the reference's batch-coupled stop rule (the loop ends
    when ANY row converges, resamplers.py:126-129).  Batch-sharded (world > 1): each rank
    runs its rows with the local rule keeping every state's potentials, the ranks take the
    MIN of the stop iteration (the first row to converge anywhere) and each finishes at that
    state -- the unsharded loop's result, no iteration run twice (ops.ot_resample_sharded,
    as the no-grad engine)."""
    if world_size(SHARD_GROUP) > 1:
        return _ops.ot_resample_sharded(particles, weights, eps, scaling, threshold, max_iter,
                                        group=SHARD_GROUP, keep=keep)
    return _ops.ot_resample(particles, weights, eps, scaling, threshold, max_iter, keep=keep)


class _OtTransport(torch.autograd.Function):
    """x' = T x with the Sinkhorn plan T held constant in backward (resamplers.py:234-264):
    dL/dx = T^T g by nfdpf_ot_transport_backward from this call's own workspace; no gradient
    to the weights (the reference returns None for them)."""

    @staticmethod
    def forward(ctx, particles, weights, eps, scaling, threshold, max_iter):
        B, N, _ = particles.shape
        ws = _ops.ot_workspace(B, N, particles.device)
        xo, wo, idx, _ = _ot_call(particles, weights, eps, scaling, threshold, max_iter, keep=ws)
        ctx.ws, ctx.eps = ws, eps
        ctx.mark_non_differentiable(wo, idx)
        return xo, wo, idx

    @staticmethod
    def backward(ctx, g, _gw, _gi):
        gx = _ops.ot_transport_backward(ctx.ws, g, ctx.eps)
        return gx, None, None, None, None, None


def resampler_ot(particles, weights, eps=0.1, scaling=0.75, threshold=1e-3, max_iter=100, device="cuda",
                 flag=None):
    """OT resampling -> (x', uniform weights, identity flat index) (resamplers.py:62-70)."""
    if torch.is_grad_enabled() and particles.requires_grad:
        return _OtTransport.apply(particles, weights.detach(), eps, scaling, threshold, max_iter)
    xo, wo, idx, _ = _ot_call(particles.detach(), weights.detach(), eps, scaling, threshold, max_iter)
    return xo, wo, idx


def ot_resample_with_info(particles, weights, eps=0.1, scaling=0.75, threshold=1e-3, max_iter=100):
    """As resampler_ot, also returning the reference's Sinkhorn iteration count (:179)."""
    return _ops.ot_resample(particles, weights, eps, scaling, threshold, max_iter)
