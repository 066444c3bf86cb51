"""Model assembly (model/models.py of the reference): builders, dynamics, proposal and
measurement models with the reference's names, signatures and state_dict keys.

Hot-path pieces run on libnfdpf: the flow stacks (via nf.models), the measurement models
(``nfdpf_measurement``) and -- inside ``DPF.filtering_pos`` -- everything fused into one
kernel per step (nfdpf.engine).  The frame encoder / decoder CNNs are per-image work
(B x T frames, not B x N x T particles) and stay on PyTorch/MIOpen.
"""
import math

import torch
from torch import nn

from nf.flows import FCNN, RealNVP, RealNVP_cond, MAF  # noqa: F401  (reference re-exports nf.flows)
from nf.models import NormalizingFlowModel, NormalizingFlowModel_cond
from nfdpf import autograd as _ag
from nfdpf import ops as _ops
from nfdpf._lib import NfdpfError
from nfdpf.pack import blob, blob_grad_to_params, encoder_tensors, flows_tensors, paired_mlp_tensors
from utils import et_distance

device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")

_CHANNELS = (3, 16, 32, 64, 128, 256)


def _conv_stack(out_features):
    """5 x [Conv(4, s2, p1, no bias) ReLU BN] + Linear(256*4*4, out) (model/models.py:10-60)."""
    layers = []
    for cin, cout in zip(_CHANNELS[:-1], _CHANNELS[1:]):
        layers += [nn.Conv2d(cin, cout, kernel_size=4, stride=2, padding=1, bias=False), nn.ReLU(True),
                   nn.BatchNorm2d(cout)]
    layers += [nn.Flatten(), nn.Linear(256 * 4 * 4, out_features)]
    return nn.Sequential(*layers)


def _deconv_stack(in_features):
    """Linear + Unflatten + 5 x ConvTranspose (model/models.py:62-117), sigmoid output."""
    layers = [nn.Linear(in_features, 256 * 4 * 4), nn.Unflatten(-1, (256, 4, 4))]
    rev = _CHANNELS[::-1]
    for k, (cin, cout) in enumerate(zip(rev[:-1], rev[1:])):
        layers.append(nn.ConvTranspose2d(cin, cout, kernel_size=4, padding=1, stride=2, bias=False))
        if cout != 3:
            layers.append(nn.ReLU(True))
        layers.append(nn.BatchNorm2d(cout))
    layers.append(nn.Sigmoid())
    return nn.Sequential(*layers)


def build_encoder(hidden_size):
    return _conv_stack(hidden_size)


def build_encoder_cglow(hidden_size):
    return _conv_stack(192)


def build_decoder(hidden_size):
    return _deconv_stack(hidden_size)


def build_decoder_cglow(hidden_size):
    return _deconv_stack(192)


def _mlp(sizes, act, last_act=None):
    layers = []
    for i, (a, b) in enumerate(zip(sizes[:-1], sizes[1:])):
        layers.append(nn.Linear(a, b))
        if i < len(sizes) - 2:
            layers.append(act())
    if last_act is not None:
        layers.append(last_act())
    return nn.Sequential(*layers)


def build_likelihood(hidden_size, state_dim):
    """likelihood_est: Linear(2H,64) ReLU Linear(64,64) ReLU Linear(64,1) Sigmoid (:119-128)."""
    return _mlp([2 * hidden_size, 64, 64, 1], lambda: nn.ReLU(True), nn.Sigmoid)


def build_particle_encoder(hidden_size, state_dim):
    """Linear(D,16) ReLU Linear(16,32) ReLU Linear(32,H) (:130-139)."""
    return _mlp([state_dim, 16, 32, hidden_size], nn.ReLU)


def build_particle_encoder_cglow(hidden_size, state_dim):
    return _mlp([state_dim, 16, 32, 192], nn.ReLU)


def build_transition_model(state_dim):
    return _mlp([state_dim, 64, 64, state_dim], nn.ReLU)


def build_conditional_nf(n_sequence, hidden_size, state_dim, init_var=0.01, prior_mean=0.0, prior_std=1.0):
    """Stack of RealNVP_cond(dim=state_dim, obser_dim=hidden_size) with N(0, init_var^2)
    weights and an isotropic MVN prior (model/models.py:161-172)."""
    flows = [RealNVP_cond(dim=state_dim, obser_dim=hidden_size) for _ in range(n_sequence)]
    for f in flows:
        f.zero_initialization(var=init_var)
    prior = torch.distributions.MultivariateNormal(torch.zeros(state_dim).to(device) + prior_mean,
                                                   torch.eye(state_dim).to(device) * prior_std ** 2)
    return NormalizingFlowModel_cond(prior, flows, device=device)


def build_maf_dyn(n_sequence, state_dim, hidden_dim=8):
    """MAF dynamic flow stack for --NF-dyn-flow MAF (BASELINE config 4; not wired in the
    reference)."""
    flows = [MAF(dim=state_dim, hidden_dim=hidden_dim) for _ in range(n_sequence)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(state_dim).to(device), torch.eye(state_dim).to(device))
    return NormalizingFlowModel(prior, flows, device=device)


def build_conditional_glow(args):
    from nf.cglow.CGlowModel import CondGlowModel
    return CondGlowModel(args)


def build_dyn_nf(n_sequence, hidden_size, state_dim, init_var=0.01):
    flows = [RealNVP(dim=state_dim) for _ in range(n_sequence)]
    for f in flows:
        f.zero_initialization(var=init_var)
    prior = torch.distributions.MultivariateNormal(torch.zeros(state_dim).to(device), torch.eye(state_dim).to(device))
    return NormalizingFlowModel(prior, flows, device=device)


def motion_update(particles, vel, pos_noise=20.0):
    """x + vel + N(0, pos_noise^2) noise drawn on the CPU generator (model/models.py:191-204)."""
    B, N, _ = particles.shape
    noise = torch.normal(mean=0., std=pos_noise, size=(B, N, 2)).to(particles.device)
    return particles + vel[:, None, :].repeat((1, N, 1)) + noise, noise


# ------------------------------------------------------------------------------------------
# measurement models: forward(encodings (B,H), particles (B,N,2)) -> log-likelihood (B,N)
# ------------------------------------------------------------------------------------------
class _MeasRunner:
    def __init__(self, model, kind):
        self.model, self.kind = model, kind

    def hip(self, enc, x):
        m = self.model
        pe = blob(m, "pe", m.particle_encoder, lambda: encoder_tensors(m.particle_encoder), x.device)
        meas, nfl, pstd = None, 0, 2.5
        if self.kind == "CRNVP":
            meas = blob(m, "meas", m.CNF.flows, lambda: flows_tensors(m.CNF.flows), x.device)
            nfl = len(m.CNF.flows)
            pstd = math.sqrt(float(m.CNF.prior.covariance_matrix[0, 0]))
        elif self.kind == "NN":
            meas = blob(m, "meas", m.likelihood_estimator, lambda: paired_mlp_tensors(m.likelihood_estimator), x.device)
        return (_ops.measurement(self.kind, pe, meas, nfl, enc, x, pstd),)

    def hip_backward(self, enc, x, gouts):
        """d/d(enc, x, encoder and model parameters) on the HIP kernels: cosine by
        nfdpf_cos_measurement_backward (csrc/measure_bwd.hip), gaussian / CRNVP / NN through the
        particle encoder's kernels and the model's own backward; None where a model falls outside
        the kernels (autograd then differentiates ``torch``)."""
        m = self.model
        if self.kind not in ("cos", "CRNVP", "gaussian", "NN") or enc.dim() != 2 or enc.shape[-1] != 32 or x.dim() != 3 \
                or x.shape[-1] != 2:
            return None
        pe = blob(m, "pe", m.particle_encoder, lambda: encoder_tensors(m.particle_encoder), x.device)
        g = gouts[0] if gouts[0] is not None else torch.zeros(x.shape[:2], device=x.device)
        g = g.float()
        pe_params = list(m.particle_encoder.parameters())
        if self.kind == "cos":
            g_enc, gx, gp = _ops.cos_measurement_backward(pe, enc.float(), x.float(), g)
            extra = []
        elif self.kind == "gaussian":
            out = self._gaussian_backward(pe, enc.float(), x.float(), g)
            if out is None:
                return None
            g_enc, gx, gp = out
            extra = []
        elif self.kind == "NN":
            g_enc, gx, gp, extra = self._nn_backward(pe, enc.float(), x.float(), g)
        else:
            out = self._crnvp_backward(pe, enc.float(), x.float(), g)
            if out is None:
                return None
            g_enc, gx, gp, extra = out
        res, off = [], 0
        for p in pe_params:  # the encoder's W1 b1 W2 b2 W3 b3, nn.Linear layout
            res.append(gp[off:off + p.numel()].view_as(p).to(p.dtype) if p.requires_grad else None)
            off += p.numel()
        res += extra  # CRNVP: the flow's parameters (m.parameters() lists the encoder first)
        return (g_enc.to(enc.dtype), gx.to(x.dtype)), res

    def _gaussian_backward(self, pe, enc, x, g):
        """measurement_model_Gaussian (model/models.py:237-254): lik = log N(o - e; mu, s^2 I) minus
        the row max.  The max routes -sum_n g to the row's argmax; dlik/de = (o - e - mu) / s^2
        (elementwise on the (B, N, 32) encodings); the particle encoder forward and backward are
        the HIP kernels (nfdpf_particle_encoder modes 0 / 1)."""
        dist = self.model.gaussian_distribution
        cov = dist.covariance_matrix
        var = float(cov[0, 0])
        if not torch.equal(cov, torch.eye(cov.shape[0], device=cov.device, dtype=cov.dtype) * var):
            return None  # a non-isotropic covariance: differentiate the PyTorch restatement
        B, N, _ = x.shape
        es = _ops.particle_encoder_forward(pe, x).view(B, N, 32)
        d = enc[:, None, :] - es - dist.loc.to(es.dtype)
        u = -0.5 * (d * d).sum(-1)  # the log-density up to a constant: only its argmax is used
        am = u.argmax(-1)
        g_u = g.clone()
        g_u[torch.arange(B, device=g.device), am] -= g.sum(-1)
        r = g_u[..., None] * d / var        # = dL/de (lik rises as e approaches o - mu)
        gx, gp = _ops.particle_encoder_backward(pe, x, r.reshape(B * N, 32).contiguous())
        return -r.sum(1), gx, gp

    def _nn_backward(self, pe, enc, x, g):
        """measurement_model_NN (model/models.py:221-235): the head's backward
        (nfdpf_nn_measurement_backward, csrc/nn_bwd.hip) gives d/d the particle encodings, the
        frame encoding and likelihood_est's parameters; the encoder backward (HIP) takes g_e on
        to x and the encoder's parameters."""
        m = self.model
        B, N, _ = x.shape
        mb = blob(m, "meas", m.likelihood_estimator, lambda: paired_mlp_tensors(m.likelihood_estimator), x.device)
        es = _ops.particle_encoder_forward(pe, x)
        g_es, g_enc, g_mp = _ops.nn_measurement_backward(mb, enc, es, g)
        gx, gp = _ops.particle_encoder_backward(pe, x, g_es)
        extra, off = [], 0
        for p in m.likelihood_estimator.parameters():
            extra.append(g_mp[off:off + p.numel()].view_as(p).to(p.dtype) if p.requires_grad else None)
            off += p.numel()
        return g_enc, gx, gp, extra

    def _crnvp_backward(self, pe, enc, x, g):
        """measurement_model_cnf (model/models.py:256-278): lik = u - max_n u with u = log N(z) +
        log-det of the CNF stack on the frame encoding conditioned on the particle encoding.
        The max routes -sum_n g to the row's argmax; then the stack backward (HIP) gives d/d the
        condition (-> encoder backward, HIP) and d/d the repeated frame encoding (summed per row)."""
        from nf.models import _isotropic
        m = self.model
        fl = list(m.CNF.flows)
        iso = _isotropic(m.CNF.prior)
        if iso is None or fl[0].dim != 32 or fl[0].hidden_dim != 8 or not 1 <= len(fl) <= 4:
            return None
        pm, ps = iso
        B, N, _ = x.shape
        cb = blob(m, "meas", m.CNF.flows, lambda: flows_tensors(m.CNF.flows), x.device)
        es = _ops.particle_encoder_forward(pe, x)
        eo = enc[:, None, :].expand(B, N, 32).reshape(B * N, 32).contiguous()
        _, ld, lp = _ops.cond_stack(cb, len(fl), 32, 32, 8, eo, es, 1, False, pm, ps, want_prior=True)
        am = (lp + ld).view(B, N).argmax(-1)
        g_u = g.clone()
        g_u[torch.arange(B, device=g.device), am] -= g.sum(-1)
        g_u = g_u.reshape(-1)
        g_eo, g_es, g_cb = _ops.cond_stack_backward(cb, len(fl), 32, 32, 8, eo, es, False, torch.zeros_like(eo),
                                                    g_u, g_u, pm, ps)
        gx, gp = _ops.particle_encoder_backward(pe, x, g_es)
        cnf_params = [p for f in fl for p in f.parameters()]
        gf = blob_grad_to_params(m, "meas", cnf_params, lambda get: flows_tensors(fl, get), g_cb)
        gf = [gi if p.requires_grad else None for gi, p in zip(gf, cnf_params)]
        return g_eo.view(B, N, 32).sum(1), gx, gp, gf

    def torch(self, enc, x):
        return (self.model.torch_forward(enc, x),)


def _meas_apply(model, kind, enc, x):
    return _ag.apply(_MeasRunner(model, kind), (enc, x), list(model.parameters()))[0]


def _obs_rep(encodings, n):
    return encodings[:, None, :].repeat(1, n, 1)


class measurement_model_cosine_distance(nn.Module):
    """log(1/(1e-7 + cos-distance(enc_obs, enc_particle))) (model/models.py:206-219)."""

    def __init__(self, particle_encoder):
        super().__init__()
        self.particle_encoder = particle_encoder

    def forward(self, encodings, update_particles):
        return _meas_apply(self, "cos", encodings, update_particles)

    def torch_forward(self, encodings, particles):
        es = self.particle_encoder(particles.float())
        return (1 / (1e-7 + et_distance(_obs_rep(encodings, particles.shape[1]), es))).log()


class measurement_model_NN(nn.Module):
    """sigmoid-MLP on [enc_obs, enc_particle] (model/models.py:221-235)."""

    def __init__(self, particle_encoder, likelihood_estimator):
        super().__init__()
        self.particle_encoder = particle_encoder
        self.likelihood_estimator = likelihood_estimator

    def forward(self, encodings, update_particles):
        return _meas_apply(self, "NN", encodings, update_particles)

    def torch_forward(self, encodings, particles):
        es = self.particle_encoder(particles.float())
        h = torch.cat([_obs_rep(encodings, particles.shape[1]), es], dim=-1)
        return self.likelihood_estimator(h)[..., 0].log()


class measurement_model_Gaussian(nn.Module):
    """N(1, 100 I) log-density of enc_obs - enc_particle, minus the row max (:237-254)."""

    def __init__(self, particle_encoder, gaussian_distribution):
        super().__init__()
        self.particle_encoder = particle_encoder
        self.gaussian_distribution = gaussian_distribution

    def forward(self, encodings, update_particles):
        return _meas_apply(self, "gaussian", encodings, update_particles)

    def torch_forward(self, encodings, particles):
        es = self.particle_encoder(particles.float())
        lik = self.gaussian_distribution.log_prob(_obs_rep(encodings, particles.shape[1]) - es)
        return lik - lik.max(dim=-1, keepdim=True)[0]


class measurement_model_cnf(nn.Module):
    """Conditional-RealNVP likelihood of the frame encoding given the particle encoding,
    minus the row max (model/models.py:256-278)."""

    def __init__(self, particle_encoder, CNF):
        super().__init__()
        self.particle_encoder = particle_encoder
        self.CNF = CNF

    def forward(self, encodings, update_particles):
        return _meas_apply(self, "CRNVP", encodings, update_particles)

    def torch_forward(self, encodings, particles):
        from nf.flows import CouplingStack
        from nf.models import _isotropic
        B, N = particles.shape[:2]
        H = encodings.shape[-1]
        es = self.particle_encoder(particles.float()).reshape(-1, H)
        eo = _obs_rep(encodings, N).reshape(-1, H)
        fl = list(self.CNF.flows)
        _, ld, lp = CouplingStack(self.CNF, fl, H, H, fl[0].hidden_dim, False,
                                  prior=_isotropic(self.CNF.prior)).torch(eo, es)
        lik = (lp + ld).reshape(B, N)
        return lik - lik.max(dim=-1, keepdim=True)[0]


class _CglowRunner:
    """measurement_model_cglow's raw likelihood -nll: the fused HIP kernel forward (particle
    encoder + CGLOW, csrc/cglow.hip) and the HIP backward (nfdpf_cglow_measurement_backward,
    csrc/cglow_bwd.hip); ``torch`` is the PyTorch restatement (the particle encoder, then
    CondGlowModel.torch_forward) that NFDPF_HIP_BACKWARD=0 differentiates instead, bounded to
    RECOMPUTE_ROWS particles (nfdpf.autograd: 4 000 took 3.96 ms there, 64 000 did not finish in
    3 minutes on the GPU box)."""

    RECOMPUTE_ROWS = 16384

    def __init__(self, model):
        self.model = model

    def recompute_limit(self, enc, x):
        return self.RECOMPUTE_ROWS, x.numel() // x.shape[-1]

    def hip(self, enc, x):
        from nfdpf.pack import cglow_tensors
        m = self.model
        pe = blob(m, "pe", m.particle_encoder, lambda: encoder_tensors(m.particle_encoder), x.device)
        glow = blob(m, "glow", m.CGLOW, lambda: cglow_tensors(m.CGLOW), x.device)
        return (_ops.cglow_measurement(pe, glow, enc.float(), x.float()),)

    def torch(self, enc, x):
        return (self.model.torch_forward_raw(enc, x),)

    def hip_backward(self, enc, x, gouts):
        """d/d(enc, x, encoder and CGLOW parameters) on nfdpf_cglow_measurement_backward
        (csrc/cglow_bwd.hip); None (recompute) outside the kernel's configuration."""
        from nfdpf.pack import blob_param_grads, cglow_tensors
        m = self.model
        if enc.dim() != 2 or enc.shape[-1] != 192 or x.dim() != 3 or x.shape[-1] != 2 \
                or not m.CGLOW.kernel_supported():
            return None
        pe = blob(m, "pe", m.particle_encoder, lambda: encoder_tensors(m.particle_encoder), x.device)
        glow = blob(m, "glow", m.CGLOW, lambda: cglow_tensors(m.CGLOW), x.device)
        g = gouts[0] if gouts[0] is not None else torch.zeros(x.shape[:2], device=x.device)
        g_enc, gx, g_glow, g_pe = _ops.cglow_measurement_backward(pe, glow, enc.float(), x.float(), g.float())
        pe_params, gl_params = list(m.particle_encoder.parameters()), list(m.CGLOW.parameters())
        res = blob_param_grads(m, "pe_grad", pe_params, lambda get: encoder_tensors(m.particle_encoder, get), g_pe)
        res += blob_param_grads(m, "glow_grad", gl_params, lambda get: cglow_tensors(m.CGLOW, get), g_glow)
        return (g_enc.to(enc.dtype), gx.to(x.dtype)), res


class measurement_model_cglow(nn.Module):
    """Conditional-GLOW likelihood (model/models.py:280-303)."""

    def __init__(self, particle_encoder, CGLOW):
        super().__init__()
        self.particle_encoder = particle_encoder
        self.CGLOW = CGLOW

    def forward(self, encodings, update_particles):
        """One HIP kernel (csrc/cglow.hip: particle encoder, conditioning nets, actnorm, 1x1 conv
        with its 12x12 log-determinant, affine coupling, Gaussian log-prob), then the row-max
        shift.  Under autograd the particle encoder and every CGLOW parameter get their
        gradients through the recompute backward of _CglowRunner."""
        if not self.CGLOW.kernel_supported():
            raise NfdpfError("measurement_model_cglow: the HIP kernel is built for the reference's default CGLOW "
                             "(K = 1, L = 1, 3x8x8, learn_top off, 256 bins)")
        lik = _ag.apply(_CglowRunner(self), (encodings, update_particles), list(self.parameters()))[0]
        return lik - lik.max(dim=-1, keepdim=True)[0]

    def torch_forward_raw(self, encodings, particles):
        """-nll before the row-max shift (model/models.py:285-300), PyTorch."""
        B, N, D = particles.shape
        es = self.particle_encoder(particles.reshape(-1, D).float()).reshape(B * N, 3, 8, 8)
        eo = encodings[:, None, :].repeat(1, N, 1).reshape(B * N, 3, 8, 8)
        _, nll = self.CGLOW.torch_forward(es, eo)
        return -nll.reshape(B, N)


# ------------------------------------------------------------------------------------------
# dynamics / proposal (model/models.py:305-379)
# ------------------------------------------------------------------------------------------
def _row_context(x, mean=None, std=None):
    n = x.shape[1]
    m = x.mean(dim=1, keepdim=True) if mean is None else mean
    s = x.std(dim=1, keepdim=True) if std is None else std
    return torch.cat([m.detach().clone().repeat([1, n, 1]).reshape(-1, x.shape[-1]),
                      s.detach().clone().repeat([1, n, 1]).reshape(-1, x.shape[-1])], dim=-1)


def nf_dynamic_model(dynamical_nf, dynamic_particles, jac_shape, NF=False, forward=False, mean=None, std=None):
    """Dynamic flow with per-row [mean, std] context; returns (x', jac = -log_det) (:305-332)."""
    if not NF:
        return dynamic_particles, torch.zeros(jac_shape).to(dynamic_particles.device)
    B, N, D = dynamic_particles.shape
    ctx = _row_context(dynamic_particles, mean, std)
    flat = dynamic_particles.reshape(-1, D)
    if isinstance(dynamical_nf, NormalizingFlowModel):  # MAF dynamic flow: no context
        if forward:
            out, _, ld = dynamical_nf.forward(flat)
        else:
            out, ld = dynamical_nf.inverse(flat)
    elif forward:
        out, _, ld = dynamical_nf.forward(flat, ctx)
    else:
        out, ld = dynamical_nf.inverse(flat, ctx)
    return out.reshape(B, N, D), (-ld).reshape(B, N)


def normalising_flow_propose(cond_model, particles_pred, obs, flow=RealNVP_cond, n_sequence=2, hidden_dimension=8,
                             obser_dim=None):
    """Proposal flow conditioned on [frame encoding, mean, std] (:334-356)."""
    B, N, D = particles_pred.shape
    ctx = _row_context(particles_pred)
    cond = torch.cat([obs[:, None, :].repeat([1, N, 1]).reshape(B * N, -1), ctx], dim=-1)
    out, ld = cond_model.inverse(particles_pred.reshape(-1, D), cond)
    return out.reshape(B, N, D), (-ld).reshape(B, N)


def proposal_likelihood(cond_model, dynamical_nf, measurement_model, particles_dynamic, particles_physical,
                        encodings, noise, jac_dynamic, NF, NF_cond, prototype_density):
    """(proposal particles, lik, prior, proposal log-density) (:358-379)."""
    enc = encodings.detach().clone()
    if NF_cond:
        prop, jac_prop = normalising_flow_propose(cond_model, particles_dynamic, enc)
        if NF:
            back, jac_back = nf_dynamic_model(dynamical_nf, prop, jac_dynamic.shape, NF=NF, forward=True,
                                              mean=particles_physical.mean(dim=1, keepdim=True),
                                              std=particles_physical.std(dim=1, keepdim=True))
            prior = prototype_density(back - (particles_physical - noise)) - jac_back
        else:
            prior = prototype_density(prop - (particles_physical - noise))
        propose = prototype_density(noise) + jac_dynamic + jac_prop
    else:
        prop = particles_dynamic
        prior = prototype_density(noise) + jac_dynamic
        propose = prototype_density(noise) + jac_dynamic
    return prop, measurement_model(encodings, prop), prior, propose
