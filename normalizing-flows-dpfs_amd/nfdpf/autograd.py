"""Autograd for the HIP flow / measurement ops (training).

The forward value always comes from the HIP kernel.  Backward: a runner with a HIP backward
(``runner.hip_backward``: the RealNVP(_cond) coupling stacks, MAF stacks, the cosine / CRNVP /
NN / gaussian / CGLOW measurements -- csrc/*_bwd.hip) returns the input and parameter gradients
from the kernel; where it declines (sizes or models its kernel does not cover), the runner's
math is re-run as PyTorch ops on the saved inputs and differentiated (activation-recompute
style).  ``NFDPF_HIP_BACKWARD=0`` sends every runner down the recompute path -- for comparison
only: a runner may bound the recompute (``recompute_limit(*inputs)`` -> the largest size it
finishes, with the input's size) and then refuses a larger one with NfdpfError instead of
stalling the device (CGLOW's recompute did not finish a 64 x 1 000-particle backward in 3 min).
"""
from __future__ import annotations

import os

import torch

HIP_BACKWARD = os.environ.get("NFDPF_HIP_BACKWARD", "1") != "0"


class _RecomputeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, runner, n_in, *tensors):
        ins = tensors[:n_in]
        ctx.runner = runner
        ctx.n_in = n_in
        ctx.save_for_backward(*tensors)
        with torch.no_grad():
            outs = runner.hip(*ins)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        saved = ctx.saved_tensors
        n_in = ctx.n_in
        ins, params = saved[:n_in], saved[n_in:]
        hb = getattr(ctx.runner, "hip_backward", None)
        if HIP_BACKWARD and hb is not None:
            got = hb(*ins, gouts)
            if got is not None:
                gin, gpar = got
                gin = [g if (t is not None and t.requires_grad) else None for g, t in zip(gin, ins)]
                gpar = [g if p.requires_grad else None for g, p in zip(gpar, params)]
                return (None, None) + tuple(gin) + tuple(gpar)
        lim = getattr(ctx.runner, "recompute_limit", None)
        if lim is not None:
            cap, size = lim(*ins)
            if size > cap:
                from ._lib import NfdpfError
                raise NfdpfError(f"{type(ctx.runner).__name__}: the PyTorch-recompute backward is bounded to {cap} "
                                 f"rows (got {size}); the HIP backward covers this size (NFDPF_HIP_BACKWARD=1)")
        with torch.enable_grad():
            leaves = [t.detach().requires_grad_(t.requires_grad) if t is not None and t.is_floating_point() else t
                      for t in ins]
            outs = ctx.runner.torch(*leaves)
            pairs = [(o, g) for o, g in zip(outs, gouts) if o is not None and g is not None and o.requires_grad]
            wrt = [t for t in list(leaves) + list(params) if t is not None and t.requires_grad]
            grads = torch.autograd.grad([o for o, _ in pairs], wrt, [g for _, g in pairs], allow_unused=True) \
                if pairs and wrt else [None] * len(wrt)
        it = iter(grads)
        res = []
        for t in list(leaves) + list(params):
            res.append(next(it) if t is not None and t.requires_grad else None)
        return (None, None) + tuple(res)


def needs_grad(*tensors) -> bool:
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors)


def apply(runner, inputs, params):
    """Run ``runner.hip(*inputs)``; when autograd is active, wire a recompute backward."""
    if needs_grad(*inputs, *params):
        return _RecomputeFn.apply(runner, len(inputs), *inputs, *params)
    with torch.no_grad():
        return tuple(runner.hip(*inputs))
