"""Rational-quadratic splines of the neural spline flows (nf/utils.py of the reference, after
Durkan et al. 2019): ``searchsorted``, ``unconstrained_RQS``, ``RQS`` with the reference's
names, arguments, defaults and errors.

The spline itself is the HIP kernel ``nfdpf_rqs`` (csrc/rqs.hip): one element per lane with
its K bins in registers.  When autograd is recording, the backward differentiates a PyTorch
restatement of the same map on the saved inputs (``nfdpf.autograd``, the recompute path of
MAF and the NN / gaussian measurements).
"""
import numpy as np
import torch
import torch.nn.functional as F

from nfdpf import autograd as _ag
from nfdpf import ops as _ops

DEFAULT_MIN_BIN_WIDTH = 1e-3
DEFAULT_MIN_BIN_HEIGHT = 1e-3
DEFAULT_MIN_DERIVATIVE = 1e-3


def searchsorted(bin_locations, inputs, eps=1e-6):
    """Bin index of each input: #{k : input >= location_k} - 1, the last location lifted by
    ``eps`` IN PLACE (nf/utils.py:16-21 -- callers see the lifted tensor)."""
    bin_locations[..., -1] += eps
    return torch.sum(inputs[..., None] >= bin_locations, dim=-1) - 1


def _knots(u, lo, hi, min_bin):
    """Bin edges and lengths of one axis from unnormalised bin sizes (nf/utils.py:66-85)."""
    K = u.shape[-1]
    w = min_bin + (1 - min_bin * K) * torch.softmax(u, dim=-1)
    edges = F.pad(torch.cumsum(w, dim=-1), (1, 0), value=0.0)
    edges = (hi - lo) * edges + lo
    edges = torch.cat([torch.full_like(edges[..., :1], lo), edges[..., 1:-1], torch.full_like(edges[..., :1], hi)], -1)
    return edges, edges[..., 1:] - edges[..., :-1]


def _rqs_torch(inputs, uw, uh, ud, inverse, left, right, bottom, top, min_bin_width, min_bin_height,
               min_derivative):
    """The spline as PyTorch ops (for the backward): derivatives ``ud`` has K + 1 entries."""
    cw, wd = _knots(uw, left, right, min_bin_width)
    ch, ht = _knots(uh, bottom, top, min_bin_height)
    der = min_derivative + F.softplus(ud)
    loc = (ch if inverse else cw).detach().clone()
    idx = searchsorted(loc, inputs)[..., None].clamp(0, uw.shape[-1] - 1)
    pick = lambda t: t.gather(-1, idx)[..., 0]  # noqa: E731
    x0, w, y0, h = pick(cw), pick(wd), pick(ch), pick(ht)
    delta = h / w
    d0, d1 = pick(der), der[..., 1:].gather(-1, idx)[..., 0]
    s = d0 + d1 - 2 * delta
    if inverse:
        r = inputs - y0
        a = r * s + h * (delta - d0)
        b = h * d0 - r * s
        c = -delta * r
        theta = (2 * c) / (-b - torch.sqrt(b.pow(2) - 4 * a * c))
        out = theta * w + x0
    else:
        theta = (inputs - x0) / w
    tt = theta * (1 - theta)
    den = delta + s * tt
    num = delta.pow(2) * (d1 * theta.pow(2) + 2 * delta * tt + d0 * (1 - theta).pow(2))
    lad = torch.log(num) - 2 * torch.log(den)
    if inverse:
        return out, -lad
    return y0 + h * (delta * theta.pow(2) + d0 * tt) / den, lad


class _RqsRunner:
    """nfdpf.autograd runner: forward on the HIP kernel, backward through _rqs_torch."""

    def __init__(self, inverse, left, right, bottom, top, tails, mins):
        self.inverse, self.bounds, self.tails, self.mins = inverse, (left, right, bottom, top), tails, mins

    def hip(self, x, W, H, D):
        l, r, b, t = self.bounds
        return _ops.rqs(x, W, H, D, self.inverse, l, r, b, t, self.tails, *self.mins)

    def torch(self, x, W, H, D):
        l, r, b, t = self.bounds
        if D.shape[-1] == W.shape[-1] - 1:  # unconstrained: the constant boundary derivatives
            const = float(np.log(np.exp(1 - self.mins[2]) - 1))
            D = F.pad(D, (1, 1), value=const)
        inside = (x >= l) & (x <= r) if self.tails else torch.ones_like(x, dtype=torch.bool)
        xs = torch.where(inside, x, torch.zeros_like(x) + 0.5 * (l + r))
        y, ld = _rqs_torch(xs, W, H, D, self.inverse, l, r, b, t, *self.mins)
        return torch.where(inside, y, x), torch.where(inside, ld, torch.zeros_like(ld))


def unconstrained_RQS(inputs, unnormalized_widths, unnormalized_heights, unnormalized_derivatives, inverse=False,
                      tail_bound=1., min_bin_width=DEFAULT_MIN_BIN_WIDTH, min_bin_height=DEFAULT_MIN_BIN_HEIGHT,
                      min_derivative=DEFAULT_MIN_DERIVATIVE):
    """RQS on [-tail_bound, tail_bound]^2 with identity tails (nf/utils.py:23-53):
    unnormalized_derivatives holds the K - 1 inner knots' values; returns (outputs, logabsdet)."""
    B = float(tail_bound)
    run = _RqsRunner(bool(inverse), -B, B, -B, B, True, (min_bin_width, min_bin_height, min_derivative))
    return _ag.apply(run, (inputs, unnormalized_widths, unnormalized_heights, unnormalized_derivatives), ())


def RQS(inputs, unnormalized_widths, unnormalized_heights, unnormalized_derivatives, inverse=False, left=0.,
        right=1., bottom=0., top=1., min_bin_width=DEFAULT_MIN_BIN_WIDTH, min_bin_height=DEFAULT_MIN_BIN_HEIGHT,
        min_derivative=DEFAULT_MIN_DERIVATIVE):
    """The bounded spline (nf/utils.py:55-147): K + 1 unnormalised derivatives; the reference's
    domain and bin-size checks raise ValueError."""
    if torch.min(inputs) < left or torch.max(inputs) > right:
        raise ValueError("Input outside domain")
    num_bins = unnormalized_widths.shape[-1]
    if min_bin_width * num_bins > 1.0:
        raise ValueError('Minimal bin width too large for the number of bins')
    if min_bin_height * num_bins > 1.0:
        raise ValueError('Minimal bin height too large for the number of bins')
    run = _RqsRunner(bool(inverse), float(left), float(right), float(bottom), float(top), False,
                     (min_bin_width, min_bin_height, min_derivative))
    return _ag.apply(run, (inputs, unnormalized_widths, unnormalized_heights, unnormalized_derivatives), ())
