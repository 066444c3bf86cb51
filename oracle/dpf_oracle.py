"""CPU oracle for the NF-DPF particle-update hot path -- TEST INFRASTRUCTURE ONLY.

This module is a functional restatement, in PyTorch-CPU, of the reference's
per-timestep particle update (xiongjiechen/Normalizing-Flows-DPFs).  Every
function cites the reference file:line it restates.  It is used only by:

  * ``tests/``                     -- as the checker for the HIP path,
  * ``__graft_entry__.smoke()``    -- to check one small HIP invocation,
  * ``bench.py`` ``cpu_baseline``  -- the CPU leg timed beside the GPU.

The product path (``normalizing-flows-dpfs_amd/``) never imports this file.

It is "timing faithful": it keeps the reference's op structure (dense O(N^2)
marker matching in soft resampling, FP64 four-potential Sinkhorn with dense
cost matrices, per-step history concatenation), so timing it is a fair
stand-in for timing the reference on a box where the reference is absent.

Parity pinning: the restatement is checked against golden vectors produced by
running the reference itself in the build container
(``tests/golden/gen_golden.py`` -> ``tests/golden/*.npz``), see
``tests/test_oracle_golden.py``.

Parameters are plain ``dict[str, Tensor]`` keyed exactly like the reference's
``state_dict`` (e.g. ``flows.0.t1.network.2.weight``).
"""
from __future__ import annotations

import math
from typing import Callable, Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

Params = Dict[str, torch.Tensor]
NETS = ("t1", "s1", "t2", "s2")

# Working precision.  float32 = the reference's own arithmetic.  float64 (via ``precision``)
# evaluates the same algorithm in double: the GPU tests use |ref64 - ref32| as the
# reference's own rounding envelope where the computation is ill-conditioned (e.g. the
# cosine likelihood -log(1 - <a,b>) near alignment).
_DT = torch.float32


def _f(x: torch.Tensor) -> torch.Tensor:
    return x.to(_DT)


class precision:
    """``with precision(torch.float64): ...`` -- run the oracle in double."""

    def __init__(self, dt):
        self.dt = dt

    def __enter__(self):
        global _DT
        self.prev, self.prev_default = _DT, torch.get_default_dtype()
        _DT = self.dt
        torch.set_default_dtype(self.dt)

    def __exit__(self, *exc):
        global _DT
        _DT = self.prev
        torch.set_default_dtype(self.prev_default)


def cast_params(params: Params, dt) -> Params:
    return {k: (v.to(dt) if v.is_floating_point() else v) for k, v in params.items()}


def sub(params: Params, prefix: str) -> Params:
    """Slice a state-dict-like mapping down to ``prefix.*`` (prefix stripped)."""
    p = prefix + "."
    return {k[len(p):]: v for k, v in params.items() if k.startswith(p)}


# ----------------------------------------------------------------------------
# Flows -- nf/flows.py, nf/models.py
# ----------------------------------------------------------------------------
def fcnn(params: Params, x: torch.Tensor) -> torch.Tensor:
    """FCNN: Linear-Tanh-Linear-Tanh-Linear on ``x.float()`` (nf/flows.py:101-114)."""
    h = torch.tanh(F.linear(_f(x), params["network.0.weight"], params["network.0.bias"]))
    h = torch.tanh(F.linear(h, params["network.2.weight"], params["network.2.bias"]))
    return F.linear(h, params["network.4.weight"], params["network.4.bias"])


def realnvp_cond_forward(params: Params, x, obser):
    """One conditional affine coupling, forward (nf/flows.py:215-226)."""
    half = x.shape[1] // 2
    lo, up = x[:, :half], x[:, half:]
    lc = torch.cat([lo, obser], dim=-1)
    t1, s1 = fcnn(sub(params, "t1"), lc), fcnn(sub(params, "s1"), lc)
    up = t1 + up * torch.exp(s1)
    uc = torch.cat([up, obser], dim=-1)
    t2, s2 = fcnn(sub(params, "t2"), uc), fcnn(sub(params, "s2"), uc)
    lo = t2 + lo * torch.exp(s2)
    return torch.cat([lo, up], dim=1), s1.sum(dim=1) + s2.sum(dim=1)


def realnvp_cond_inverse(params: Params, z, obser):
    """One conditional affine coupling, inverse (nf/flows.py:228-239)."""
    half = z.shape[1] // 2
    lo, up = z[:, :half], z[:, half:]
    uc = torch.cat([up, obser], dim=-1)
    t2, s2 = fcnn(sub(params, "t2"), uc), fcnn(sub(params, "s2"), uc)
    lo = (lo - t2) * torch.exp(-s2)
    lc = torch.cat([lo, obser], dim=-1)
    t1, s1 = fcnn(sub(params, "t1"), lc), fcnn(sub(params, "s1"), lc)
    up = (up - t1) * torch.exp(-s1)
    return torch.cat([lo, up], dim=1), (-s1).sum(dim=1) + (-s2).sum(dim=1)


def realnvp_forward(params: Params, x):
    """Unconditional RealNVP coupling forward (nf/flows.py:155-166)."""
    half = x.shape[1] // 2
    lo, up = x[:, :half], x[:, half:]
    t1, s1 = fcnn(sub(params, "t1"), lo), fcnn(sub(params, "s1"), lo)
    up = t1 + up * torch.exp(s1)
    t2, s2 = fcnn(sub(params, "t2"), up), fcnn(sub(params, "s2"), up)
    lo = t2 + lo * torch.exp(s2)
    return torch.cat([lo, up], dim=1), s1.sum(dim=1) + s2.sum(dim=1)


def realnvp_inverse(params: Params, z):
    """Unconditional RealNVP coupling inverse (nf/flows.py:168-179)."""
    half = z.shape[1] // 2
    lo, up = z[:, :half], z[:, half:]
    t2, s2 = fcnn(sub(params, "t2"), up), fcnn(sub(params, "s2"), up)
    lo = (lo - t2) * torch.exp(-s2)
    t1, s1 = fcnn(sub(params, "t1"), lo), fcnn(sub(params, "s1"), lo)
    up = (up - t1) * torch.exp(-s1)
    return torch.cat([lo, up], dim=1), (-s1).sum(dim=1) + (-s2).sum(dim=1)


def maf_forward(params: Params, x):
    """MAF forward with the output flip (nf/flows.py:259-270).

    The reference builds ``log_det`` on the CPU; here everything is CPU anyway.
    """
    dim = x.shape[1]
    z = torch.zeros_like(x)
    log_det = torch.zeros(x.shape[0])
    for i in range(dim):
        if i == 0:
            mu, alpha = params["initial_param"][0], params["initial_param"][1]
        else:
            out = fcnn(sub(params, f"layers.{i - 1}"), x[:, :i])
            mu, alpha = out[:, 0], out[:, 1]
        z[:, i] = (x[:, i] - mu) / torch.exp(alpha)
        log_det = log_det - alpha
    return z.flip(dims=(1,)), log_det


def maf_inverse(params: Params, z):
    """MAF inverse, sequential over dims (nf/flows.py:272-284)."""
    dim = z.shape[1]
    x = torch.zeros_like(z)
    log_det = torch.zeros(z.shape[0])
    z = z.flip(dims=(1,))
    for i in range(dim):
        if i == 0:
            mu, alpha = params["initial_param"][0], params["initial_param"][1]
        else:
            out = fcnn(sub(params, f"layers.{i - 1}"), x[:, :i])
            mu, alpha = out[:, 0], out[:, 1]
        x[:, i] = mu + torch.exp(alpha) * z[:, i]
        log_det = log_det + alpha
    return x, log_det


def mvn_isotropic_logprob(z: torch.Tensor, mean: float, std: float) -> torch.Tensor:
    """Prior log-prob of ``build_conditional_nf`` (model/models.py:167-168): the same
    torch ``MultivariateNormal(mean*1, std^2 I)`` evaluated on ``z.float()`` (nf/models.py:51)."""
    d = z.shape[-1]
    mvn = torch.distributions.MultivariateNormal(torch.zeros(d) + mean, torch.eye(d) * std ** 2)
    return mvn.log_prob(_f(z))


def cond_stack_forward(params: Params, n_flows: int, x, obser, prior_mean=0.0, prior_std=1.0):
    """NormalizingFlowModel_cond.forward (nf/models.py:45-52) -> (z, prior_logprob, log_det)."""
    log_det = torch.zeros(x.shape[0])
    for i in range(n_flows):
        x, ld = realnvp_cond_forward(sub(params, f"flows.{i}"), x, obser)
        log_det = log_det + ld
    return x, mvn_isotropic_logprob(x, prior_mean, prior_std), log_det


def cond_stack_inverse(params: Params, n_flows: int, z, obser):
    """NormalizingFlowModel_cond.inverse (nf/models.py:54-61), flows in reverse."""
    log_det = torch.zeros(z.shape[0])
    for i in reversed(range(n_flows)):
        z, ld = realnvp_cond_inverse(sub(params, f"flows.{i}"), z, obser)
        log_det = log_det + ld
    return z, log_det


def stack_forward(params: Params, n_flows: int, x, kind="maf"):
    """NormalizingFlowModel.forward (nf/models.py:13-21) over MAF/RealNVP flows."""
    fwd = maf_forward if kind == "maf" else realnvp_forward
    log_det = torch.zeros(x.shape[0])
    for i in range(n_flows):
        x, ld = fwd(sub(params, f"flows.{i}"), x)
        log_det = log_det + ld
    return x, None, log_det


def stack_inverse(params: Params, n_flows: int, z, kind="maf"):
    """NormalizingFlowModel.inverse (nf/models.py:23-30)."""
    inv = maf_inverse if kind == "maf" else realnvp_inverse
    log_det = torch.zeros(z.shape[0])
    for i in reversed(range(n_flows)):
        z, ld = inv(sub(params, f"flows.{i}"), z)
        log_det = log_det + ld
    return z, log_det


# ----------------------------------------------------------------------------
# utils.py
# ----------------------------------------------------------------------------
def normal_density(noise: torch.Tensor, pos_noise: float, vel_noise: float) -> torch.Tensor:
    """compute_normal_density.forward (utils.py:22-37), same float32 op order."""
    log_c = -0.5 * torch.log(torch.tensor(2 * np.pi))
    sp, sv = torch.tensor(pos_noise), torch.tensor(vel_noise)
    npos, nvel = noise[:, :, :2], noise[:, :, 2:]
    d = noise.shape[-1]
    return (d * log_c - 2 * torch.log(sp) - torch.sum(npos ** 2 / (2 * sp ** 2), dim=-1)
            + -(d - 2) * torch.log(sv) - torch.sum(nvel ** 2 / (2 * sv ** 2), dim=-1))


def normalize_log_probs(logp: torch.Tensor) -> torch.Tensor:
    """Row max-shift, exp, divide by row sum (utils.py:39-44)."""
    e = (logp - logp.max(dim=1, keepdim=True)[0]).exp()
    return e / torch.sum(e, dim=1, keepdim=True)


def et_distance(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Cosine distance after L2 normalisation (utils.py:8-15)."""
    a = F.normalize(a, p=2, dim=-1, eps=1e-12)
    b = F.normalize(b, p=2, dim=-1, eps=1e-12)
    return 1.0 - torch.sum(a * b, dim=-1)


def particle_init(start_xy, width, n, state_dim=2, true_state=False, gen=None):
    """particle_initialization (utils.py:46-62), incl. the discarded randn draw."""
    B = start_xy.shape[0]
    if true_state:
        x = start_xy[:, None, :].repeat(1, n, 1) + torch.randn(B, n, state_dim, generator=gen)
    else:
        hi, lo = width / 2.0, -width / 2.0
        x = torch.tensor(hi - lo) * torch.rand(B, n, 2, generator=gen) + torch.tensor(lo)
        torch.randn(B, n, 2, generator=gen)  # drawn and discarded by the reference (:58)
    return x, torch.log(torch.ones([B, n]) / n)


# ----------------------------------------------------------------------------
# model/models.py -- dynamics, proposal, measurement
# ----------------------------------------------------------------------------
def motion(x, vel, pos_noise, noise=None, gen=None):
    """motion_update (model/models.py:191-204) -> (x + vel + eps, eps)."""
    B, N, _ = x.shape
    if noise is None:
        noise = torch.normal(mean=0.0, std=pos_noise, size=(B, N, 2), generator=gen)
    return x + vel[:, None, :].repeat((1, N, 1)) + noise, noise


def row_context(x: torch.Tensor) -> torch.Tensor:
    """[mean_n, std_n (unbiased)] per batch row, shape (B, 2D) (model/models.py:309-315)."""
    return torch.cat([x.mean(dim=1), x.std(dim=1)], dim=-1)


def dyn_flow(params: Params, n_flows, x, NF, forward=False, ctx=None, kind="RealNVP"):
    """nf_dynamic_model (model/models.py:305-332) -> (x', jac = -log_det).  kind "MAF": the
    context-free MAF stack (NormalizingFlowModel, nf/models.py:5-30) of --NF-dyn-flow MAF,
    which the reference builds (nf/flows.py:241-284) but does not wire into DPF."""
    B, N, D = x.shape
    if not NF:
        return x, torch.zeros(B, N)
    if kind == "MAF":
        flat = x.reshape(-1, D)
        if forward:
            y, _, ld = stack_forward(params, n_flows, flat, kind="maf")
        else:
            y, ld = stack_inverse(params, n_flows, flat, kind="maf")
        return y.reshape(B, N, D), (-ld).reshape(B, N)
    c = row_context(x) if ctx is None else ctx
    c = c[:, None, :].repeat(1, N, 1).reshape(B * N, -1)
    flat = x.reshape(-1, D)
    if forward:
        y, _, ld = cond_stack_forward(params, n_flows, flat, c)
    else:
        y, ld = cond_stack_inverse(params, n_flows, flat, c)
    return y.reshape(B, N, D), (-ld).reshape(B, N)


def nf_propose(params: Params, n_flows, x, enc):
    """normalising_flow_propose (model/models.py:334-356)."""
    B, N, D = x.shape
    c = torch.cat([enc, row_context(x)], dim=-1)[:, None, :].repeat(1, N, 1).reshape(B * N, -1)
    y, ld = cond_stack_inverse(params, n_flows, x.reshape(-1, D), c)
    return y.reshape(B, N, D), (-ld).reshape(B, N)


def particle_encode(params: Params, x):
    """build_particle_encoder MLP: Linear-ReLU-Linear-ReLU-Linear (model/models.py:130-150)."""
    h = F.relu(F.linear(_f(x), params["0.weight"], params["0.bias"]))
    h = F.relu(F.linear(h, params["2.weight"], params["2.bias"]))
    return F.linear(h, params["4.weight"], params["4.bias"])


def meas_cos(pe_params: Params, enc, x):
    """measurement_model_cosine_distance (model/models.py:206-219)."""
    es = particle_encode(pe_params, x)
    eo = enc[:, None, :].repeat(1, x.shape[1], 1)
    return (1 / (1e-7 + et_distance(eo, es))).log()


def meas_nn(pe_params: Params, lik_params: Params, enc, x):
    """measurement_model_NN (model/models.py:221-235) with build_likelihood (:119-128)."""
    es = particle_encode(pe_params, x)
    eo = enc[:, None, :].repeat(1, x.shape[1], 1)
    h = torch.cat([eo, es], dim=-1)
    h = F.relu(F.linear(h, lik_params["0.weight"], lik_params["0.bias"]))
    h = F.relu(F.linear(h, lik_params["2.weight"], lik_params["2.bias"]))
    h = torch.sigmoid(F.linear(h, lik_params["4.weight"], lik_params["4.bias"]))
    return h[..., 0].log()


def meas_gaussian(pe_params: Params, enc, x):
    """measurement_model_Gaussian with N(1, 100 I) (DPFs.py:84-86, model/models.py:237-254)."""
    es = particle_encode(pe_params, x)
    eo = enc[:, None, :].repeat(1, x.shape[1], 1)
    H = enc.shape[-1]
    mvn = torch.distributions.MultivariateNormal(torch.ones(H), 100 * torch.eye(H))
    lik = mvn.log_prob(eo - es)
    return lik - lik.max(dim=-1, keepdim=True)[0]


def meas_crnvp(pe_params: Params, cnf_params: Params, n_flows, enc, x, prior_std=2.5):
    """measurement_model_cnf (model/models.py:256-278): flow input = obs encoding."""
    B, N, _ = x.shape
    H = enc.shape[-1]
    es = particle_encode(pe_params, x).reshape(-1, H)
    eo = enc[:, None, :].repeat(1, N, 1).reshape(-1, H)
    _, lp, ld = cond_stack_forward(cnf_params, n_flows, eo, es, 0.0, prior_std)
    lik = (lp + ld).reshape(B, N)
    return lik - lik.max(dim=-1, keepdim=True)[0]


def proposal_likelihood(dyn_p, cond_p, n_flows, meas: Callable, x_dyn, x_phys, enc, noise, jac,
                        NF, NF_cond, pos_noise, vel_noise, dyn_kind="RealNVP"):
    """proposal_likelihood (model/models.py:358-379) -> (x_prop, lik, prior, propose)."""
    dens = lambda e: normal_density(e, pos_noise, vel_noise)
    if NF_cond:
        x_prop, jac_prop = nf_propose(cond_p, n_flows, x_dyn, enc.detach())
        if NF:
            ctx = row_context(x_phys)
            back, jac_back = dyn_flow(dyn_p, n_flows, x_prop, True, forward=True, ctx=ctx, kind=dyn_kind)
            prior = dens(back - (x_phys - noise)) - jac_back
        else:
            prior = dens(x_prop - (x_phys - noise))
        propose = dens(noise) + jac + jac_prop
    else:
        x_prop = x_dyn
        prior = dens(noise) + jac
        propose = dens(noise) + jac
    return x_prop, meas(enc, x_prop), prior, propose


# ----------------------------------------------------------------------------
# Conditional GLOW measurement -- nf/cglow/*.py (K steps, L = 1)
# ----------------------------------------------------------------------------
def _split(t, how):
    C = t.shape[1]
    return (t[:, :C // 2], t[:, C // 2:]) if how == "split" else (t[:, 0::2], t[:, 1::2])


def _cond_net(p: Params, x, B):
    """x_Con (3 resize convs + ReLU) then x_Linear (3 linears) -- modules.py:84-101,145-162."""
    h = x
    for i in (0, 2, 4):  # Conv2dResize halving H and W: stride 2 (modules.py:47-61)
        h = F.relu(F.conv2d(h, p[f"x_Con.{i}.weight"], p[f"x_Con.{i}.bias"], stride=2))
    h = h.reshape(B, -1)
    h = F.relu(F.linear(h, p["x_Linear.0.weight"], p["x_Linear.0.bias"]))
    h = F.relu(F.linear(h, p["x_Linear.2.weight"], p["x_Linear.2.bias"]))
    return torch.tanh(F.linear(h, p["x_Linear.4.weight"], p["x_Linear.4.bias"]))


def cglow_step(p: Params, x, y, logdet):
    """CondGlowStep forward: actnorm -> invconv -> affine (CGlowModel.py:24-37)."""
    B = x.shape[0]
    # CondActNorm (modules.py:104-132)
    a = _cond_net(sub(p, "actnorm"), x, B).reshape(B, -1, 1, 1)
    logs, bias = _split(a, "split")
    hw = y.shape[2] * y.shape[3]
    y = (y + bias) * torch.exp(logs)
    logdet = logdet + hw * torch.sum(logs, dim=(1, 2, 3))
    # Cond1x1Conv (modules.py:165-211)
    C = y.shape[1]
    w = _cond_net(sub(p, "invconv"), x, B).reshape(B, C, C)
    logdet = logdet + torch.slogdet(w)[1] * hw
    Bc, _, H, W = y.shape
    y = F.conv2d(y.reshape(1, B * C, H, W), w.reshape(B * C, C, 1, 1), groups=B).reshape(B, C, H, W)
    # CondAffineCoupling (modules.py:282-303)
    q = sub(p, "affine")
    z1, z2 = _split(y, "split")
    h = F.relu(F.conv2d(x, q["resize_x.0.weight"], q["resize_x.0.bias"], padding=1))
    h = F.relu(F.conv2d(h, q["resize_x.2.weight"], q["resize_x.2.bias"],
                        stride=(x.shape[2] // z1.shape[2], x.shape[3] // z1.shape[3])))
    h = F.relu(F.conv2d(h, q["resize_x.4.weight"], q["resize_x.4.bias"], padding=1))
    h = torch.cat((h, z1), dim=1)
    h = F.conv2d(h, q["f.0.weight"], None, padding=1)
    h = F.relu((h + q["f.0.actnorm.bias"]) * torch.exp(q["f.0.actnorm.logs"]))
    h = F.conv2d(h, q["f.2.weight"], None)
    h = F.relu((h + q["f.2.actnorm.bias"]) * torch.exp(q["f.2.actnorm.logs"]))
    h = F.conv2d(h, q["f.4.weight"], q["f.4.bias"], padding=1)
    h = torch.tanh((h + q["f.4.newbias"]) * torch.exp(q["f.4.logs"] * 3.0))
    shift, scale = _split(h, "cross")
    scale = torch.sigmoid(scale + 2.0)
    z2 = (z2 + shift) * scale
    logdet = torch.sum(torch.log(scale), dim=(1, 2, 3)) + logdet
    return torch.cat((z1, z2), dim=1), logdet


def squeeze2d(t, f=2):
    """SqueezeLayer.squeeze2d (modules.py:321-331)."""
    B, C, H, W = t.shape
    t = t.reshape(B, C, H // f, f, W // f, f).permute(0, 1, 3, 5, 2, 4)
    return t.reshape(B, C * f * f, H // f, W // f)


def cglow_nll(p: Params, K: int, x, y, n_bins=256.0):
    """CondGlowModel.forward, reverse=False (CGlowModel.py:167-176), L = 1, learn_top=False."""
    dims = y.shape[1] * y.shape[2] * y.shape[3]
    logdet = torch.zeros_like(y[:, 0, 0, 0]) + float(-np.log(n_bins) * dims)
    y = squeeze2d(y)
    for k in range(K):
        y, logdet = cglow_step(sub(p, f"flow.layers.{k + 1}"), x, y, logdet)
    # GaussianDiag.logp with mean = logs = 0 (modules.py:381-387)
    logp = torch.sum(-0.5 * (y ** 2.0 + float(np.log(2 * np.pi))), dim=(1, 2, 3))
    obj = logdet + logp
    return y, -obj / float(np.log(2.0) * dims)


def meas_cglow(pe_params: Params, glow_params: Params, K: int, enc, x):
    """measurement_model_cglow (model/models.py:280-303)."""
    B, N, D = x.shape
    es = particle_encode(pe_params, x.reshape(-1, D)).reshape(B * N, 3, 8, 8)
    eo = enc[:, None, :].repeat(1, N, 1).reshape(B * N, 3, 8, 8)
    _, nll = cglow_nll(glow_params, K, es, eo)
    lik = -nll.reshape(B, N)
    return lik - lik.max(dim=-1, keepdim=True)[0]


# ----------------------------------------------------------------------------
# resamplers/resamplers.py
# ----------------------------------------------------------------------------
def soft_resample(x, p, alpha, offsets=None, gen=None):
    """soft_resampler (resamplers.py:20-60), dense O(N^2) marker matching as in the reference.

    ``offsets`` (B,) replaces the CPU-generator draw ``FloatTensor(B).uniform_(0, 1/N)`` (:43)
    when given.  Returns (x', w', flat index).
    """
    assert 0.0 < alpha <= 1.0
    B, N = p.shape
    uni = torch.ones((B, N)) / N
    if alpha < 1.0:
        q = torch.stack((p * alpha, uni * (1.0 - alpha)), dim=-1).sum(dim=-1)
        q = q / q.sum(dim=-1, keepdim=True)
        w = p / q
    else:
        q, w = p, uni
    base = torch.linspace(0.0, (N - 1.0) / N, N)
    if offsets is None:
        offsets = torch.empty(B).uniform_(0.0, 1.0 / N, generator=gen)
    markers = offsets[:, None] + base[None, :]
    cum = torch.cumsum(q, axis=1)
    cum[:, -1] = 1.0
    cnt = (markers[:, :, None] > cum[:, None, :]).sum(axis=2).int()
    idx = cnt + N * torch.arange(B)[:, None].repeat((1, N))
    xr = x.reshape(B * N, -1)[idx, :]
    wr = w.reshape(B * N)[idx]
    wr = wr / wr.sum(dim=-1, keepdim=True)
    return xr, wr, idx


def _softmin(eps, C, f):
    """softmin (resamplers.py:94-110): -eps * LSE_j(f_j - C_ij / eps)."""
    b, n = C.shape[0], C.shape[1]
    return -eps.reshape(-1, 1) * torch.logsumexp(f.reshape(b, 1, n) - C / eps.reshape(-1, 1, 1), dim=2)


# Number of Sinkhorn potentials iterated.  4 = the reference's op structure (timing-faithful,
# the CPU baseline).  2 = a_y and b_x only: a_x and b_y never reach the output or the stop
# test (resamplers.py:139-147 vs :149-156, 175-178), so the result is bit-identical and the
# call half the cost -- the large-size parity tests set this.
OT_POTENTIALS = 4


def ot_resample(x, w, eps=0.1, scaling=0.75, threshold=1e-3, max_iter=100, return_info=False):
    """resampler_ot / OT_resampling (resamplers.py:62-70, 211-277), FP64, 4 potentials
    (``OT_POTENTIALS``).

    Returns (x', w', flat index) and, with ``return_info``, a dict with the Sinkhorn
    iteration count (``total_iter + 2`` as the reference returns, :179) and the
    final potentials (a_y, b_x after the post-loop softmin, :175-176).
    """
    live4 = OT_POTENTIALS == 4
    logw = w.log()
    B, N, D = x.shape
    eps_t = torch.tensor(eps, dtype=torch.float)
    log_n = torch.log(torch.tensor(N, dtype=torch.float))
    uni_log = -log_n * torch.ones_like(logw)
    xc = x - x.mean(dim=1, keepdim=True)
    sd = x.std(dim=1, unbiased=False).max(dim=-1)[0]
    diam = torch.where(sd == 0.0, 1.0, sd.double())                  # diameter (:72-76) -> FP64
    xs = xc / (diam.reshape(-1, 1, 1) * torch.sqrt(torch.tensor(D)))
    C = torch.cdist(xs, xs, p=2.0) ** 2 / 2.0                        # cost (:79-84)
    # max_min (:87-91), incl. the reference's use of x.max(...).min for the min term
    mm = torch.maximum(xs.max(dim=1)[0].max(dim=1)[0], xs.max(dim=1)[0].max(dim=1)[0]) - \
        torch.minimum(xs.max(dim=1)[0].min(dim=1)[0], xs.min(dim=1)[0].min(dim=1)[0])
    eps0 = mm ** 2
    sf = scaling ** 2
    a_y, b_x = _softmin(eps0, C, logw), _softmin(eps0, C, uni_log)
    if live4:
        a_x, b_y = _softmin(eps0, C, logw), _softmin(eps0, C, uni_log)
    cont = torch.ones(B, dtype=torch.bool)
    run_eps = eps0
    it = 0
    while it < max_iter - 1 and bool(torch.all(cont)):                 # sinkhorn_loop (:113-179)
        re = run_eps.reshape(-1, 1)
        at_y = _softmin(run_eps, C, logw + b_x / re)
        bt_x = _softmin(run_eps, C, uni_log + a_y / re)
        if live4:
            at_x = _softmin(run_eps, C, logw + a_x / re)
            bt_y = _softmin(run_eps, C, uni_log + b_y / re)
            a_x, b_y = (a_x + at_x) / 2, (b_y + bt_y) / 2
        ny, nx = (a_y + at_y) / 2, (b_x + bt_x) / 2
        local = torch.logical_or((ny - a_y).abs().max(dim=1)[0] > threshold,
                                 (nx - b_x).abs().max(dim=1)[0] > threshold)
        a_y, b_x = ny, nx
        new_eps = torch.maximum(run_eps * sf, eps_t)
        cont = torch.logical_or(new_eps < run_eps, local)
        run_eps = new_eps
        it += 1
    e = eps_t.reshape(-1, 1)
    f = _softmin(eps_t.reshape(1).expand(B), C, logw + b_x / e)
    g = _softmin(eps_t.reshape(1).expand(B), C, uni_log + a_y / e)
    # transport_from_potentials (:194-210)
    tmp = (f[:, :, None] + g[:, None, :] - C) / eps_t
    tmp = tmp - torch.logsumexp(tmp, dim=1, keepdim=True) + log_n
    T = torch.exp(tmp + logw[:, None, :])
    xr = torch.matmul(_f(T), _f(x))                           # apply_transport_matrix (:254-264)
    wr = torch.ones_like(w) / _f(torch.tensor(N))
    idx = (torch.arange(N) + N * torch.arange(B)[:, None].repeat((1, N))).long()
    if return_info:
        return xr, wr, idx, {"iters": it + 2, "a_y": f, "b_x": g, "T": T}
    return xr, wr, idx


# ----------------------------------------------------------------------------
# DPFs.py -- the filtering loop, and losses.py RMSE
# ----------------------------------------------------------------------------
class HostRNG:
    """The reference's CPU-generator draw sequence (DPFs.py:105,151,166,172).

    Draws: init rand/randn (utils.py:54-58); per step [offsets(B) if resampling]
    then normal(B,N,2).  ``gen=None`` uses torch's global CPU generator.
    """

    def __init__(self, gen: Optional[torch.Generator] = None):
        self.gen = gen

    def offsets(self, B, N):
        return torch.empty(B).uniform_(0.0, 1.0 / N, generator=self.gen)

    def noise(self, B, N, std):
        return torch.normal(mean=0.0, std=std, size=(B, N, 2), generator=self.gen)


def filter_step(cfg: dict, params: Params, meas: Callable, x, p, vel, enc_t, rng: HostRNG,
                force_resample=False):
    """One iteration of the T loop of DPF.filtering_pos (DPFs.py:160-214).

    ``x``/``p`` are the particles / probabilities after the previous step, ``vel`` the
    velocity used by this step's motion.  Returns a dict of this step's history entries.
    """
    N = cfg["N"]
    B = x.shape[0]
    nfl = cfg.get("n_flows", 2)
    dyn_p, cond_p = sub(params, "nf_dyn"), sub(params, "cond_model")
    idx = (torch.arange(N) + N * torch.arange(B)[:, None].repeat((1, N))).long()
    ess = torch.mean(1 / torch.sum(p ** 2, dim=-1))
    fired = bool(force_resample or ess < 0.5 * N)
    if fired:
        if cfg["resampler"] == "soft":
            xr, pr, idx = soft_resample(x, p, cfg["alpha"], rng.offsets(B, N))
        else:
            xr, pr, idx = ot_resample(x, p, cfg["eps"], cfg["scaling"], cfg["threshold"], cfg["max_iter"])
        lr = pr.log()
    else:
        xr, lr = x, p.log()
    x_phys, noise = motion(xr, vel, cfg["pos_noise"], rng.noise(B, N, cfg["pos_noise"]))
    dk = cfg.get("dyn_flow", "RealNVP")
    x_dyn, jac = dyn_flow(dyn_p, nfl, x_phys, cfg["NF_dyn"], kind=dk)
    xp, lik, prior, prop = proposal_likelihood(dyn_p, cond_p, nfl, meas, x_dyn, x_phys, _f(enc_t),
                                               noise, jac, cfg["NF_dyn"], cfg["NF_cond"],
                                               cfg["pos_noise"], cfg["vel_noise"], dyn_kind=dk)
    lw = lr + lik + prior - prop
    return dict(x=xp, p=normalize_log_probs(lw) + 1e-12, noise=noise, lik=lik, idx=idx, jac=jac,
                prior=prior, lw_mean=lw.mean(), fired=fired, logw=lw)


def make_measurement(cfg: dict, params: Params) -> Callable:
    """Measurement-model dispatch of DPF.build_model (DPFs.py:74-89)."""
    nfl = cfg.get("n_flows", 2)
    pe_p = sub(params, "particle_encoder")
    m = cfg["measurement"]
    if m == "cos":
        return lambda e, x: meas_cos(pe_p, e, x)
    if m == "CRNVP":
        return lambda e, x: meas_crnvp(pe_p, sub(params, "cnf_measurement"), nfl, e, x)
    if m == "NN":
        return lambda e, x: meas_nn(pe_p, sub(params, "likelihood_est"), e, x)
    if m == "gaussian":
        return lambda e, x: meas_gaussian(pe_p, e, x)
    if m == "CGLOW":
        return lambda e, x: meas_cglow(pe_p, sub(params, "cglow_measurement"), cfg.get("cglow_K", 1), e, x)
    raise ValueError(m)


def filtering(cfg: dict, params: Params, enc: torch.Tensor, start_state, vel_input,
              rng: Optional[HostRNG] = None, force_resample=False, init=None):
    """DPF.filtering_pos (DPFs.py:144-216) with precomputed frame encodings ``enc`` (B,T,H).

    ``cfg`` keys: N, NF_dyn, NF_cond, measurement, resampler ('soft'|'ot'), alpha, eps, scaling,
    threshold, max_iter, pos_noise, vel_noise, width, n_flows, init_with_true_state, cglow_K.
    History is concatenated step by step as the reference does (:207-214).
    Returns the reference's 9-tuple.
    """
    rng = rng or HostRNG()
    N, T = cfg["N"], enc.shape[1]
    meas = make_measurement(cfg, params)
    if init is None:
        x, logw0 = particle_init(start_state[:, :2], cfg["width"], N, 2,
                                 cfg.get("init_with_true_state", False), rng.gen)
    else:
        x, logw0 = init
    p = normalize_log_probs(logw0)
    obs_lik = 0.0
    vel = start_state[:, 2:]
    keys = ("x", "p", "noise", "lik", "idx", "jac", "prior")
    hist = {}
    for t in range(T):
        r = filter_step(cfg, params, meas, x, p, vel, enc[:, t], rng, force_resample)
        vel = vel_input[:, t, :]
        x, p = r["x"], r["p"]
        obs_lik += r["lw_mean"]
        for k in keys:
            v = r[k][:, None]
            hist[k] = v if t == 0 else torch.cat([hist[k], v], dim=1)
    nf = cfg["NF_dyn"]
    return (hist["x"], hist["p"], hist["noise"], hist["lik"], logw0, hist["idx"],
            hist["jac"] if nf else None, hist["prior"] if nf else None, obs_lik)


def rmse(particles, probs, state):
    """supervised_loss, eval branch (losses.py:18-31) -> (rmse, prediction)."""
    pred = torch.sum(particles * probs[:, :, :, None], dim=2)
    return torch.sqrt(torch.mean((pred - state[:, :, :2]) ** 2)), pred
