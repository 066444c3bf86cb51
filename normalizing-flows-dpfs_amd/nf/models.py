"""Flow stacks (nf/models.py of the reference): same classes / methods / returns.

A stack of RealNVP(_cond) or MAF flows runs as ONE HIP launch over all flows (the
reference loops over flows in Python, nf/models.py:16-18, 48-50).
"""
import torch
import torch.nn as nn

from nfdpf import autograd as _ag
from nf.flows import CouplingStack, MafStack, MAF

_MVN = torch.distributions.MultivariateNormal


def _isotropic(prior):
    """(mean, std) if ``prior`` is MultivariateNormal(m*1, s^2 I), else None."""
    if not isinstance(prior, _MVN):
        return None
    loc, cov = prior.loc, prior.covariance_matrix
    m, s2 = float(loc.reshape(-1)[0]), float(cov[0, 0])
    d = loc.shape[-1]
    eye = torch.eye(d, device=cov.device, dtype=cov.dtype)
    if torch.allclose(loc, torch.full_like(loc, m)) and torch.allclose(cov, eye * s2):
        return m, s2 ** 0.5
    return None


def _flow_kind(flows):
    kinds = {type(f).__name__ for f in flows}
    if kinds <= {"MAF"}:
        return "maf"
    if kinds <= {"RealNVP", "RealNVP_cond"}:
        return "coupling"
    raise TypeError(f"no HIP kernel for a stack of {sorted(kinds)}")


def _params(flows):
    return [p for f in flows for p in f.parameters()]


class NormalizingFlowModel(nn.Module):
    """Unconditional stack (nf/models.py:5-35): forward -> (z, None, log_det)."""

    def __init__(self, prior, flows, device="cuda"):
        super().__init__()
        self.prior = prior
        self.device = device
        self.flows = nn.ModuleList(flows).to(self.device)

    def _runner(self, inverse):
        fl = list(self.flows)
        if _flow_kind(fl) == "maf":
            return MafStack(self, fl, fl[0].dim, fl[0].hidden_dim, inverse)
        return CouplingStack(self, fl, fl[0].dim, 0, fl[0].hidden_dim, inverse)

    def forward(self, x):
        r = self._runner(False)
        args = (x,) if isinstance(r, MafStack) else (x, None)
        z, ld = _ag.apply(r, args, _params(self.flows))
        return z, None, ld

    def inverse(self, z):
        r = self._runner(True)
        args = (z,) if isinstance(r, MafStack) else (z, None)
        return _ag.apply(r, args, _params(self.flows))

    def sample(self, n_samples):
        z = self.prior.sample((n_samples,)).to(self.device)
        x, _ = self.inverse(z)
        return x


class NormalizingFlowModel_cond(nn.Module):
    """Conditional stack (nf/models.py:37-66): forward -> (z, prior.log_prob(z), log_det)."""

    def __init__(self, prior, flows, device="cuda"):
        super().__init__()
        self.prior = prior
        self.device = device
        self.flows = nn.ModuleList(flows).to(self.device)

    def forward(self, x, obser):
        fl = list(self.flows)
        iso = _isotropic(self.prior)
        r = CouplingStack(self, fl, fl[0].dim, fl[0].obser_dim, fl[0].hidden_dim, False, prior=iso)
        outs = _ag.apply(r, (x, obser), _params(fl))
        if iso is not None:
            z, ld, lp = outs
        else:
            z, ld = outs
            lp = self.prior.log_prob(z.float())
        return z, lp, ld

    def inverse(self, z, obser):
        fl = list(self.flows)
        r = CouplingStack(self, fl, fl[0].dim, fl[0].obser_dim, fl[0].hidden_dim, True)
        return _ag.apply(r, (z, obser), _params(fl))

    def sample(self, n_samples, obser):
        z = self.prior.sample((n_samples,)).to(self.device)
        x, _ = self.inverse(z, obser)
        return x
