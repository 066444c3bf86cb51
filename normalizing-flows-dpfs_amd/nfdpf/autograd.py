"""HIP forward + recompute backward for the standalone flow / measurement ops.

Training (autograd) is §8(f1) "next" in SURVEY.md: the forward value always comes from the
HIP kernel; the backward re-runs the same math as PyTorch ops on the saved inputs and
differentiates that (activation-recompute style).  Dedicated HIP backward kernels replace
this in a later round.
"""
from __future__ import annotations

import torch


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
