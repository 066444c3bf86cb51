"""Flows of the hot path -- same classes, constructor arguments and state_dict keys as the
reference's nf/flows.py, forward/inverse run by libnfdpf (HIP, gfx950).

* ``RealNVP_cond`` (nf/flows.py:181-239): conditional affine coupling, the only flow the
  DPF instantiates (model/models.py:162);
* ``RealNVP`` (:117-179): unconditional coupling (the HIP kernel with obser_dim = 0);
* ``MAF`` (:241-284): masked autoregressive flow (BASELINE config 4 dynamic flow);
* ``FCNN`` (:101-114): the coupling nets' MLP.

Each ``forward``/``inverse`` call runs the whole flow in one kernel launch; a stack of
flows is run by ``nf.models`` in ONE launch over all flows.  Parameters are packed into a
cached fp32 blob (nfdpf.pack).  Tensors must live on the HIP device.
"""
import math

import torch
import torch.nn as nn
import torch.nn.init as init

from nfdpf import autograd as _ag
from nfdpf import ops as _ops
from nfdpf.pack import blob, blob_grad_to_params, flows_tensors

device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


class FCNN(nn.Module):
    """Linear(in,H) Tanh Linear(H,H) Tanh Linear(H,out) on ``x.float()`` (nf/flows.py:101-114)."""

    def __init__(self, in_dim, out_dim, hidden_dim):
        super().__init__()
        layers = [nn.Linear(in_dim, hidden_dim), nn.Tanh(), nn.Linear(hidden_dim, hidden_dim), nn.Tanh(),
                  nn.Linear(hidden_dim, out_dim)]
        self.network = nn.Sequential(*layers)

    def forward(self, x):
        return self.network(x.float())


def _coupling_nets(flow, in_dim, half, hidden_dim, base_network):
    for name in ("t1", "s1", "t2", "s2"):
        setattr(flow, name, base_network(in_dim, half, hidden_dim))


def _normal_init(flow, var):
    """zero_initialization (nf/flows.py:131-151 / 191-211): N(0, var^2) weights, zero biases."""
    for net in (flow.t1, flow.s1, flow.t2, flow.s2):
        for layer in net.network:
            if isinstance(layer, nn.Linear):
                nn.init.normal_(layer.weight, std=var)
                layer.bias.data.fill_(0)


# ------------------------------------------------------------------------------------------
# PyTorch restatement of the coupling math, used ONLY to differentiate in backward
# (nfdpf.autograd); the forward values come from the HIP kernel.
# ------------------------------------------------------------------------------------------
def torch_coupling(flow, x, obser, inverse):
    half = x.shape[1] // 2
    lo, up = x[:, :half], x[:, half:]
    cat = (lambda a: torch.cat([a, obser], dim=-1)) if obser is not None else (lambda a: a)
    if not inverse:
        s1_in = cat(lo)
        t1, s1 = flow.t1(s1_in), flow.s1(s1_in)
        up = t1 + up * torch.exp(s1)
        s2_in = cat(up)
        t2, s2 = flow.t2(s2_in), flow.s2(s2_in)
        lo = t2 + lo * torch.exp(s2)
        return torch.cat([lo, up], dim=1), s1.sum(1) + s2.sum(1)
    s2_in = cat(up)
    t2, s2 = flow.t2(s2_in), flow.s2(s2_in)
    lo = (lo - t2) * torch.exp(-s2)
    s1_in = cat(lo)
    t1, s1 = flow.t1(s1_in), flow.s1(s1_in)
    up = (up - t1) * torch.exp(-s1)
    return torch.cat([lo, up], dim=1), (-s1).sum(1) + (-s2).sum(1)


def torch_maf(flow, x, inverse):
    dim = x.shape[1]
    cols, ld = [], torch.zeros(x.shape[0], device=x.device)
    src = x.flip(dims=(1,)) if inverse else x
    for i in range(dim):
        if i == 0:
            mu, alpha = flow.initial_param[0], flow.initial_param[1]
        else:
            prev = torch.stack(cols, 1) if inverse else x[:, :i]
            out = flow.layers[i - 1](prev)
            mu, alpha = out[:, 0], out[:, 1]
        if inverse:
            cols.append(mu + torch.exp(alpha) * src[:, i])
            ld = ld + alpha
        else:
            cols.append((src[:, i] - mu) / torch.exp(alpha))
            ld = ld - alpha
    z = torch.stack(cols, 1)
    return (z, ld) if inverse else (z.flip(dims=(1,)), ld)


class CouplingStack:
    """Runner for a list of RealNVP(_cond) flows: one HIP launch for the whole stack."""

    def __init__(self, owner, flows, dim, obser_dim, hidden, inverse, prior=None):
        self.owner, self.flows, self.dim, self.obser_dim = owner, list(flows), dim, obser_dim
        self.hidden, self.inverse, self.prior = hidden, inverse, prior

    def hip(self, x, obser):
        b = blob(self.owner, "stack", self.flows, lambda: flows_tensors(self.flows), x.device)
        pm, ps = self.prior if self.prior is not None else (0.0, 1.0)
        out, ld, lp = _ops.cond_stack(b, len(self.flows), self.dim, self.obser_dim, self.hidden, x,
                                      obser, 1, self.inverse, pm, ps, want_prior=self.prior is not None)
        return (out, ld) if lp is None else (out, ld, lp)

    def hip_backward(self, x, obser, gouts):
        """d/d(x, obser, parameters) by nfdpf_cond_stack_backward (csrc/flows_bwd.hip); None when
        the kernel does not cover the case (autograd then differentiates ``torch``)."""
        rows = x.shape[0]
        if (self.dim not in (2, 4, 32) or self.hidden != 8 or not 1 <= len(self.flows) <= 4
                or (self.obser_dim and (obser is None or obser.dim() != 2 or obser.shape[0] != rows))):
            return None
        b = blob(self.owner, "stack", self.flows, lambda: flows_tensors(self.flows), x.device)
        g_out = gouts[0] if gouts[0] is not None else torch.zeros_like(x, dtype=torch.float32)
        g_ld = gouts[1] if gouts[1] is not None else torch.zeros(rows, device=x.device)
        g_lp = gouts[2] if len(gouts) > 2 else None
        pm, ps = self.prior if self.prior is not None else (0.0, 1.0)
        gx, gc, gb = _ops.cond_stack_backward(b, len(self.flows), self.dim, self.obser_dim, self.hidden,
                                              x.float(), obser.float() if self.obser_dim else None,
                                              self.inverse, g_out.float(), g_ld.float(),
                                              None if g_lp is None else g_lp.float(), pm, ps)
        # blob -> parameters: the packed blob is a fixed gather of the parameters (nfdpf.pack)
        params = _params(self.flows)
        gp = blob_grad_to_params(self.owner, "stack", params, lambda get: flows_tensors(self.flows, get), gb)
        gp = [g if p.requires_grad else None for g, p in zip(gp, params)]
        gobs = None if gc is None else gc.to(obser.dtype)
        return (gx.to(x.dtype), gobs), gp

    def torch(self, x, obser):
        ld = torch.zeros(x.shape[0], device=x.device)
        seq = self.flows[::-1] if self.inverse else self.flows
        for f in seq:
            x, l = torch_coupling(f, x, obser if self.obser_dim else None, self.inverse)
            ld = ld + l
        if self.prior is None:
            return x, ld
        pm, ps = self.prior
        d = x.shape[-1]
        z = (x - pm) / ps
        lp = -0.5 * (z * z).sum(-1) - d * math.log(ps) - 0.5 * d * math.log(2 * math.pi)
        return x, ld, lp


class MafStack:
    def __init__(self, owner, flows, dim, hidden, inverse):
        self.owner, self.flows, self.dim, self.hidden, self.inverse = owner, list(flows), dim, hidden, inverse

    def hip(self, x):
        b = blob(self.owner, "maf", self.flows, lambda: flows_tensors(self.flows), x.device)
        return _ops.maf_stack(b, len(self.flows), self.dim, self.hidden, x, self.inverse)

    def hip_backward(self, x, gouts):
        """d/d(x, parameters) by nfdpf_maf_stack_backward (csrc/maf_bwd.hip); None when the
        kernel does not cover the case (autograd then differentiates ``torch``)."""
        b = blob(self.owner, "maf", self.flows, lambda: flows_tensors(self.flows), x.device)
        got = _ops.maf_stack_backward(b, len(self.flows), self.dim, self.hidden, x.float(), self.inverse,
                                      None if gouts[0] is None else gouts[0].float(),
                                      None if gouts[1] is None else gouts[1].float())
        if got is None:
            return None
        gx, gb = got
        params = _params(self.flows)
        gp = blob_grad_to_params(self.owner, "maf", params, lambda get: flows_tensors(self.flows, get), gb)
        return (gx.to(x.dtype),), [g if p.requires_grad else None for g, p in zip(gp, params)]

    def torch(self, x):
        ld = torch.zeros(x.shape[0], device=x.device)
        for f in (self.flows[::-1] if self.inverse else self.flows):
            x, l = torch_maf(f, x, self.inverse)
            ld = ld + l
        return x, ld


def _params(mods):
    return [p for m in mods for p in m.parameters()]


class RealNVP(nn.Module):
    """Non-volume preserving flow (nf/flows.py:117-179) [Dinh et al. 2017]."""

    def __init__(self, dim, hidden_dim=8, base_network=FCNN):
        super().__init__()
        self.dim = dim
        self.hidden_dim = hidden_dim
        _coupling_nets(self, dim // 2, dim // 2, hidden_dim, base_network)

    def zero_initialization(self, var=0.1):
        _normal_init(self, var)

    def forward(self, x):
        r = CouplingStack(self, [self], self.dim, 0, self.hidden_dim, False)
        return _ag.apply(r, (x, None), _params([self]))

    def inverse(self, z):
        r = CouplingStack(self, [self], self.dim, 0, self.hidden_dim, True)
        return _ag.apply(r, (z, None), _params([self]))


class RealNVP_cond(nn.Module):
    """Conditional affine coupling (nf/flows.py:181-239): nets see [half, obser]."""

    def __init__(self, dim, hidden_dim=8, base_network=FCNN, obser_dim=None):
        super().__init__()
        self.dim = dim
        self.obser_dim = obser_dim
        self.hidden_dim = hidden_dim
        _coupling_nets(self, dim // 2 + obser_dim, dim // 2, hidden_dim, base_network)

    def zero_initialization(self, var=0.1):
        _normal_init(self, var)

    def forward(self, x, obser):
        r = CouplingStack(self, [self], self.dim, self.obser_dim, self.hidden_dim, False)
        return _ag.apply(r, (x, obser), _params([self]))

    def inverse(self, z, obser):
        r = CouplingStack(self, [self], self.dim, self.obser_dim, self.hidden_dim, True)
        return _ag.apply(r, (z, obser), _params([self]))


class MAF(nn.Module):
    """Masked autoregressive flow (nf/flows.py:241-284) [Papamakarios et al. 2018]."""

    def __init__(self, dim, hidden_dim=8, base_network=FCNN):
        super().__init__()
        self.dim = dim
        self.hidden_dim = hidden_dim
        self.layers = nn.ModuleList([base_network(i, 2, hidden_dim) for i in range(1, dim)])
        self.initial_param = nn.Parameter(torch.Tensor(2))
        self.reset_parameters()

    def reset_parameters(self):
        init.uniform_(self.initial_param, -math.sqrt(0.5), math.sqrt(0.5))

    def forward(self, x):
        return _ag.apply(MafStack(self, [self], self.dim, self.hidden_dim, False), (x,), _params([self]))

    def inverse(self, z):
        return _ag.apply(MafStack(self, [self], self.dim, self.hidden_dim, True), (z,), _params([self]))


# ------------------------------------------------------------------------------------------
# The reference's other flows (nf/flows.py:11-98, 287-458), not on the DPF path (SURVEY.md
# §8(f4)): same classes, constructor arguments, parameter names and returns.  The neural
# spline flows' rational-quadratic spline is the HIP kernel nfdpf_rqs (nf.utils); Planar,
# Radial, ActNorm and OneByOneConv are a few elementwise / (dim x dim) ops each and run as
# PyTorch ops on the tensors' device.
# ------------------------------------------------------------------------------------------
import numpy as np  # noqa: E402
import scipy as sp  # noqa: E402
import scipy.linalg  # noqa: E402,F401
import torch.nn.functional as F  # noqa: E402

from nf.utils import unconstrained_RQS  # noqa: E402

# supported non-linearities and their derivatives (nf/flows.py:11-18); evaluated on the
# input's own device
functional_derivatives = {
    torch.tanh: lambda x: 1 - torch.pow(torch.tanh(x), 2),
    F.leaky_relu: lambda x: (x > 0).to(x.dtype) + (x < 0).to(x.dtype) * -0.01,
    F.elu: lambda x: (x > 0).to(x.dtype) + (x < 0).to(x.dtype) * torch.exp(x),
}


class Planar(nn.Module):
    """Planar flow z = x + u h(w^T x + b) (nf/flows.py:22-64) [Rezende and Mohamed 2015]."""

    def __init__(self, dim, nonlinearity=torch.tanh):
        super().__init__()
        self.h = nonlinearity
        self.w = nn.Parameter(torch.Tensor(dim))
        self.u = nn.Parameter(torch.Tensor(dim))
        self.b = nn.Parameter(torch.Tensor(1))
        self.reset_parameters(dim)

    def reset_parameters(self, dim):
        bound = math.sqrt(1 / dim)
        for p in (self.w, self.u, self.b):
            init.uniform_(p, -bound, bound)

    def forward(self, x):
        if self.h in (F.elu, F.leaky_relu):
            u = self.u
        elif self.h == torch.tanh:
            # u constrained so that w^T u >= -1 (invertibility)
            wu = self.w @ self.u
            u = self.u + (torch.log(1 + torch.exp(wu)) - wu - 1) * self.w / torch.norm(self.w) ** 2
        else:
            raise NotImplementedError("Non-linearity is not supported.")
        lin = torch.unsqueeze(x @ self.w, 1) + self.b
        z = x + u * self.h(lin)
        phi = functional_derivatives[self.h](lin) * self.w
        return z, torch.log(torch.abs(1 + phi @ u) + 1e-4)

    def inverse(self, z):
        raise NotImplementedError("Planar flow has no algebraic inverse.")


class Radial(nn.Module):
    """Radial flow z = x + beta h(alpha, r) (x - x0) (nf/flows.py:67-98) [Rezende and Mohamed
    2015].  As in the reference, __init__ leaves the parameters uninitialised (reset_parameters
    is not called) and r is the norm over the whole input matrix."""

    def __init__(self, dim):
        super().__init__()
        self.x0 = nn.Parameter(torch.Tensor(dim))
        self.log_alpha = nn.Parameter(torch.Tensor(1))
        self.beta = nn.Parameter(torch.Tensor(1))

    def reset_parameters(self, dim):
        bound = math.sqrt(1 / dim)
        for p in (self.x0, self.log_alpha, self.beta):
            init.uniform_(p, -bound, bound)

    def forward(self, x):
        m, n = x.shape
        alpha = torch.exp(self.log_alpha)
        r = torch.norm(x - self.x0)
        h = 1 / (alpha + r)
        beta = -alpha + torch.log(1 + torch.exp(self.beta))
        z = x + beta * h * (x - self.x0)
        log_det = (n - 1) * torch.log(1 + beta * h) + torch.log(1 + beta * h - beta * r / (alpha + r) ** 2)
        return z, log_det


class ActNorm(nn.Module):
    """Per-dimension affine map with a scalar log-det (nf/flows.py:287-306) [Kingma and
    Dhariwal 2018]."""

    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.mu = nn.Parameter(torch.zeros(dim, dtype=torch.float))
        self.log_sigma = nn.Parameter(torch.zeros(dim, dtype=torch.float))

    def forward(self, x):
        return x * torch.exp(self.log_sigma) + self.mu, torch.sum(self.log_sigma)

    def inverse(self, z):
        return (z - self.mu) / torch.exp(self.log_sigma), -torch.sum(self.log_sigma)


class OneByOneConv(nn.Module):
    """Invertible 1x1 convolution, W = P L (U + diag S) from the LU of a random orthogonal
    matrix drawn with numpy's global generator (nf/flows.py:309-340) [Kingma and Dhariwal 2018].
    As in the reference, L, S and U are registered parameters only when ``device`` is the CPU
    (``nn.Parameter(...).to(device)`` returns a plain tensor on the GPU).  The inverse matrix is
    cached after the first ``inverse`` (the reference's ``if not self.W_inv`` raises on the
    second call for dim > 1; this build tests ``is None``)."""

    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        W, _ = sp.linalg.qr(np.random.randn(dim, dim))
        P, L, U = sp.linalg.lu(W)
        self.P = torch.tensor(P, dtype=torch.float).to(device)
        self.L = nn.Parameter(torch.tensor(L, dtype=torch.float)).to(device)
        self.S = nn.Parameter(torch.tensor(np.diag(U), dtype=torch.float)).to(device)
        self.U = nn.Parameter(torch.triu(torch.tensor(U, dtype=torch.float), diagonal=1)).to(device)
        self.W_inv = None

    def _w(self):
        eye = torch.diag(torch.ones(self.dim).to(device))
        L = torch.tril(self.L, diagonal=-1) + eye
        return self.P @ L @ (torch.triu(self.U, diagonal=1) + torch.diag(self.S))

    def forward(self, x):
        return x @ self._w(), torch.sum(torch.log(torch.abs(self.S)))

    def inverse(self, z):
        if self.W_inv is None:
            self.W_inv = torch.inverse(self._w())
        return z.float() @ self.W_inv, -torch.sum(torch.log(torch.abs(self.S)))


def _spline_params(out, K, B, dim):
    """(W, H, D) of a spline from a net output split K / K / K-1 along ``dim``: softmax'ed and
    scaled by 2B, softplus'ed -- the reference then hands these to unconstrained_RQS as its
    UNNORMALISED inputs (a second softmax inside; nf/flows.py:378-381)."""
    W, H, D = torch.split(out, K, dim=dim)
    W, H = 2 * B * torch.softmax(W, dim=dim), 2 * B * torch.softmax(H, dim=dim)
    return W, H, F.softplus(D)


class NSF_AR(nn.Module):
    """Neural spline flow, autoregressive (nf/flows.py:343-398) [Durkan et al. 2019]: dimension
    i's spline comes from FCNN(x[:, :i]) (the first from ``init_param``)."""

    def __init__(self, dim, K=5, B=3, hidden_dim=8, base_network=FCNN):
        super().__init__()
        self.dim = dim
        self.K = K
        self.B = B
        self.layers = nn.ModuleList()
        self.init_param = nn.Parameter(torch.Tensor(3 * K - 1))
        for i in range(1, dim):
            self.layers += [base_network(i, 3 * K - 1, hidden_dim)]
        self.reset_parameters()

    def reset_parameters(self):
        init.uniform_(self.init_param, -1 / 2, 1 / 2)

    def _params_of(self, i, x):
        if i == 0:
            out = self.init_param.expand(x.shape[0], 3 * self.K - 1)
        else:
            out = self.layers[i - 1](x[:, :i])
        return _spline_params(out, self.K, self.B, 1)

    def _run(self, v, inverse):
        out = torch.zeros_like(v).to(device)
        log_det = torch.zeros(out.shape[0]).to(device)
        src = out if inverse else v  # the inverse conditions on the dimensions already inverted
        for i in range(self.dim):
            W, H, D = self._params_of(i, src)
            out[:, i], ld = unconstrained_RQS(v[:, i], W, H, D, inverse=inverse, tail_bound=self.B)
            log_det += ld
        return out, log_det

    def forward(self, x):
        return self._run(x, False)

    def inverse(self, z):
        return self._run(z, True)


class NSF_CL(nn.Module):
    """Neural spline flow, coupling layer (nf/flows.py:401-458) [Durkan et al. 2019]."""

    def __init__(self, dim, K=5, B=3, hidden_dim=8, base_network=FCNN):
        super().__init__()
        self.dim = dim
        self.K = K
        self.B = B
        self.f1 = base_network(dim // 2, (3 * K - 1) * dim // 2, hidden_dim)
        self.f2 = base_network(dim // 2, (3 * K - 1) * dim // 2, hidden_dim)

    def _half(self, net, cond, v, inverse):
        out = net(cond).reshape(-1, self.dim // 2, 3 * self.K - 1)
        W, H, D = _spline_params(out, self.K, self.B, 2)
        y, ld = unconstrained_RQS(v, W, H, D, inverse=inverse, tail_bound=self.B)
        return y, torch.sum(ld, dim=1)

    def forward(self, x):
        log_det = torch.zeros(x.shape[0]).to(device)
        lower, upper = x[:, :self.dim // 2], x[:, self.dim // 2:]
        upper, ld = self._half(self.f1, lower, upper, False)
        log_det += ld
        lower, ld = self._half(self.f2, upper, lower, False)
        log_det += ld
        return torch.cat([lower, upper], dim=1), log_det

    def inverse(self, z):
        log_det = torch.zeros(z.shape[0]).to(device)
        lower, upper = z[:, :self.dim // 2], z[:, self.dim // 2:]
        lower, ld = self._half(self.f2, upper, lower, True)
        log_det += ld
        upper, ld = self._half(self.f1, lower, upper, True)
        log_det += ld
        return torch.cat([lower, upper], dim=1), log_det
