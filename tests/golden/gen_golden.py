"""Generate golden vectors by RUNNING THE REFERENCE (build container only).

    python tests/golden/gen_golden.py            # writes tests/golden/*.npz

The reference lives read-only at /root/reference and never travels: only the
inputs/outputs it produced are committed, as small .npz fixtures.  Two modules
the reference imports but never uses on this path (``cv2`` in DPFs.py:13,
``torch.utils.tensorboard`` in DPFs.py:10, used only by ``train_val``) are not
installed here, so empty placeholder modules are put in ``sys.modules`` before
import; nothing else is altered.

Fixtures:
  G1 flows.npz        RealNVP_cond forward/inverse, (D,O) in {(2,4),(2,36),(2,196),(32,32)},
                      init std 0.01 (reference init) and 0.3
  G2 stacks.npz       NormalizingFlowModel_cond fwd/inv (n=2) incl. prior log-prob;
                      NormalizingFlowModel of MAF flows (D=2, D=4)
  G3 soft.npz         soft_resampler: inputs, CPU-generator offsets, indices, weights
  G4 ot.npz           OT resampler (FP64 Sinkhorn): x', iteration count, potentials
  G5 meas.npz         cos / CRNVP / NN / gaussian / CGLOW measurement outputs
  G6 e2e_*.npz        DPF.filtering_pos end to end (encoder = identity on precomputed
                      encodings), with the CPU-generator draws recorded
  G7                  RMSE (losses.supervised_loss) stored inside each e2e file
  G8 fwd_*.npz        DPF.forward(inputs, train=False) end to end -- 128x128 frames, the
                      frame encoder / decoder swapped for tests/_tiny.py in the reference's
                      DPF (its CNNs are 1.6 M parameters), global CPU generator seeded
  G9 state_dict_keys.json  DPF(args).state_dict() key -> shape for every measurement model
  G11 cglow_flow.npz  CondGlowModel.forward(x, y) -> (z, nll)
  G14 autoencoder.npz frame encoder / decoder CNNs + autoencoder_loss (seeded init checksums,
                      features, reconstruction sample, loss; train and eval mode)
  G13 dataset.npz     the disk generator's trajectories (start state, states, q)
  G12 flows_extra.npz the flows off the DPF path (Planar, Radial, ActNorm, OneByOneConv,
                      NSF_AR, NSF_CL -- forward / inverse, spline-flow gradients) and the
                      rational-quadratic spline (unconstrained_RQS, RQS)
  G10 grads.npz       the reference's AUTOGRAD gradients (training): flow stacks
                      (forward and inverse), MAF, soft and OT resamplers, all five measurement
                      models, each for a random linear functional of its outputs; and one
                      DPF.forward(train=True) + total_loss.backward() (tiny frame encoder /
                      decoder) with every parameter's gradient
"""
import argparse
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    for name in ("cv2", "torch.utils.tensorboard"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["torch.utils.tensorboard"].SummaryWriter = object
    import torch  # noqa
    import DPFs  # noqa
    return sys.modules


def sd_np(module, prefix=""):
    return {prefix + k: v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


def perturb(module, std, gen):
    import torch
    with torch.no_grad():
        for p in module.parameters():
            p.copy_(torch.randn(p.shape, generator=gen) * std)


def gen_flows(mods):
    import torch
    from nf.flows import RealNVP_cond
    out = {}
    g = torch.Generator().manual_seed(11)
    for D, O in ((2, 4), (2, 36), (2, 196), (32, 32)):
        for tag, std in (("init", 0.01), ("wide", 0.3)):
            torch.manual_seed(100 + D + O)
            f = RealNVP_cond(dim=D, obser_dim=O)
            f.zero_initialization(var=0.01)
            if tag == "wide":
                perturb(f, std, g)
            M = 96
            x = torch.randn(M, D, generator=g) * 5
            c = torch.randn(M, O, generator=g)
            with torch.no_grad():
                z, ldf = f.forward(x, c)
                xi, ldi = f.inverse(x, c)
            k = f"D{D}_O{O}_{tag}"
            for kk, v in sd_np(f).items():
                out[f"{k}/w/{kk}"] = v
            out[f"{k}/x"], out[f"{k}/c"] = x.numpy(), c.numpy()
            out[f"{k}/z"], out[f"{k}/ld_fwd"] = z.numpy(), ldf.numpy()
            out[f"{k}/xinv"], out[f"{k}/ld_inv"] = xi.numpy(), ldi.numpy()
    np.savez_compressed(os.path.join(OUT, "flows.npz"), **out)


def gen_stacks(mods):
    import torch
    from model.models import build_conditional_nf
    from nf.flows import MAF
    from nf.models import NormalizingFlowModel
    from torch.distributions import MultivariateNormal
    out = {}
    g = torch.Generator().manual_seed(12)
    for D, O, pstd in ((2, 4, 1.0), (2, 36, 1.0), (32, 32, 2.5)):
        torch.manual_seed(200 + D + O)
        m = build_conditional_nf(2, O, D, init_var=0.01, prior_std=pstd)
        perturb(m.flows, 0.2, g)
        M = 80
        x = torch.randn(M, D, generator=g) * 3
        c = torch.randn(M, O, generator=g)
        with torch.no_grad():
            z, lp, ldf = m.forward(x, c)
            xi, ldi = m.inverse(x, c)
        k = f"cond_D{D}_O{O}"
        for kk, v in sd_np(m.flows, "flows.").items():
            out[f"{k}/w/{kk}"] = v
        out[f"{k}/prior_std"] = np.float32(pstd)
        for name, v in (("x", x), ("c", c), ("z", z), ("lp", lp), ("ld_fwd", ldf), ("xinv", xi), ("ld_inv", ldi)):
            out[f"{k}/{name}"] = v.numpy()
    for D in (2, 4):
        torch.manual_seed(300 + D)
        flows = [MAF(dim=D) for _ in range(2)]
        perturb(torch.nn.ModuleList(flows), 0.3, g)
        m = NormalizingFlowModel(MultivariateNormal(torch.zeros(D), torch.eye(D)), flows, device="cpu")
        M = 80
        x = torch.randn(M, D, generator=g) * 2
        with torch.no_grad():
            z, _, ldf = m.forward(x)
            xi, ldi = m.inverse(x)
        k = f"maf_D{D}"
        for kk, v in sd_np(m.flows, "flows.").items():
            out[f"{k}/w/{kk}"] = v
        for name, v in (("x", x), ("z", z), ("ld_fwd", ldf), ("xinv", xi), ("ld_inv", ldi)):
            out[f"{k}/{name}"] = v.numpy()
    np.savez_compressed(os.path.join(OUT, "stacks.npz"), **out)


def _probs(kind, B, N, g):
    import torch
    from utils import normalize_log_probs
    if kind == "rand":
        lw = torch.randn(B, N, generator=g) * 3
    elif kind == "peaky":
        lw = torch.randn(B, N, generator=g) * 30
    elif kind == "uniform":
        lw = torch.zeros(B, N)
    else:  # one dominant particle per row
        lw = torch.full((B, N), -80.0)
        lw[torch.arange(B), torch.randint(0, N, (B,), generator=g)] = 0.0
    return normalize_log_probs(lw) + 1e-12


def gen_soft(mods):
    import torch
    from resamplers.resamplers import soft_resampler
    out = {}
    g = torch.Generator().manual_seed(13)
    cases = [(16, 100, "rand", 0.5), (32, 1000, "rand", 0.5), (2, 10000, "rand", 0.5), (8, 1000, "peaky", 0.5),
             (4, 256, "uniform", 0.5), (4, 300, "onehot", 0.5), (3, 1, "rand", 0.5), (5, 7, "rand", 0.5),
             (5, 33, "rand", 0.5), (4, 500, "rand", 0.3), (4, 500, "rand", 1.0)]
    for i, (B, N, kind, alpha) in enumerate(cases):
        x = torch.randn(B, N, 2, generator=g) * 40
        p = _probs(kind, B, N, g)
        seed = 1000 + i
        torch.manual_seed(seed)
        xr, wr, idx = soft_resampler(x, p, alpha, N, index=True, device="cpu")
        torch.manual_seed(seed)
        off = torch.FloatTensor(B).uniform_(0.0, 1.0 / N)
        k = f"c{i}"
        out[f"{k}/alpha"] = np.float32(alpha)
        out[f"{k}/x"], out[f"{k}/p"], out[f"{k}/offsets"] = x.numpy(), p.numpy(), off.numpy()
        out[f"{k}/idx"] = idx.numpy().astype(np.int32)
        out[f"{k}/w"] = wr.numpy()
        assert torch.equal(xr, x.reshape(B * N, 2)[idx])
    out["n_cases"] = np.int32(len(cases))
    np.savez_compressed(os.path.join(OUT, "soft.npz"), **out)


def gen_ot(mods):
    import torch
    import resamplers.resamplers as R
    out = {}
    g = torch.Generator().manual_seed(14)
    cases = [(4, 128, "rand"), (8, 200, "rand"), (3, 64, "peaky")]
    for i, (B, N, kind) in enumerate(cases):
        x = torch.randn(B, N, 2, generator=g) * 30 + torch.randn(B, 1, 2, generator=g) * 10
        p = _probs(kind, B, N, g)
        with torch.no_grad():
            xr, wr, idx = R.resampler_ot(x, p, eps=0.1, scaling=0.75, threshold=1e-3, max_iter=100, device="cpu")
            # the same intermediate path as transport_function (resamplers.py:211-227) for iters / potentials
            logw = p.log()
            eps = torch.tensor(0.1, dtype=torch.float)
            log_n = torch.log(torch.tensor(N, dtype=torch.float))
            uni = -log_n * torch.ones_like(logw)
            xc = x - x.mean(dim=1, keepdim=True)
            scale = R.diameter(x, x).reshape([-1, 1, 1]) * torch.sqrt(torch.tensor(2))
            xs = xc / scale
            a_y, b_x, _, _, iters = R.sinkhorn_potentials(logw, xs, uni, xs, eps, 0.75, 1e-3, 100, device="cpu")
        k = f"c{i}"
        out[f"{k}/x"], out[f"{k}/p"] = x.numpy(), p.numpy()
        out[f"{k}/xr"], out[f"{k}/wr"] = xr.numpy(), wr.numpy()
        out[f"{k}/iters"] = np.int32(iters)
        out[f"{k}/a_y"], out[f"{k}/b_x"] = a_y.numpy(), b_x.numpy()
    out["n_cases"] = np.int32(len(cases))
    np.savez_compressed(os.path.join(OUT, "ot.npz"), **out)


def make_args(**kw):
    import arguments
    saved = sys.argv
    sys.argv = ["gen"]
    try:
        a = arguments.parse_args()
    finally:
        sys.argv = saved
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def gen_meas(mods):
    import torch
    from DPFs import DPF
    out = {}
    g = torch.Generator().manual_seed(15)
    B, N = 3, 50
    for meas, H in (("cos", 32), ("CRNVP", 32), ("NN", 32), ("gaussian", 32), ("CGLOW", 192)):
        torch.manual_seed(400)
        a = make_args(measurement=meas, hiddensize=H, num_particles=N, batchsize=B)
        dpf = DPF(a)
        perturb(dpf.particle_encoder, 0.3, g)
        if meas == "CRNVP":
            perturb(dpf.cnf_measurement.flows, 0.1, g)
        if meas == "CGLOW":
            perturb(dpf.cglow_measurement, 0.1, g)
        if meas == "NN":
            perturb(dpf.likelihood_est, 0.2, g)
        enc = torch.randn(B, 192 if meas == "CGLOW" else H, generator=g)
        x = torch.randn(B, N, 2, generator=g) * 30
        with torch.no_grad():
            lik = dpf.measurement_model(enc, x)
        k = meas
        for kk, v in sd_np(dpf).items():
            if kk.split(".")[0] in ("particle_encoder", "cnf_measurement", "cglow_measurement", "likelihood_est"):
                out[f"{k}/w/{kk}"] = v
        out[f"{k}/enc"], out[f"{k}/x"], out[f"{k}/lik"] = enc.numpy(), x.numpy(), lik.numpy()
    np.savez_compressed(os.path.join(OUT, "meas.npz"), **out)


E2E = {
    # name: (flag overrides, B, N, T, H, particle-encoder std, flow std, encodings)
    # "aligned" encodings = particle_encoder(true position) + 30 % noise, as a trained encoder
    # would give; it makes the ESS gate fire on some steps and not on others.
    "c1": (dict(NF_dyn=False, NF_cond=False, measurement="cos", resampler_type="soft"), 4, 64, 6, 32, 0.5, 0.05, "aligned"),
    "c2": (dict(NF_dyn=True, NF_cond=True, measurement="cos", resampler_type="soft"), 4, 64, 6, 32, 0.5, 0.05, "aligned"),
    "c2w": (dict(NF_dyn=True, NF_cond=True, measurement="cos", resampler_type="soft"), 4, 64, 5, 32, 0.5, 0.3, "aligned"),
    "c3": (dict(NF_dyn=False, NF_cond=False, measurement="CRNVP", resampler_type="ot"), 3, 48, 4, 32, 0.5, 0.05, "random"),
    "c3n": (dict(NF_dyn=True, NF_cond=True, measurement="CRNVP", resampler_type="ot"), 3, 48, 4, 32, 0.5, 0.3, "random"),
    "c5": (dict(NF_dyn=True, NF_cond=True, measurement="CGLOW", resampler_type="soft", hiddensize=192), 3, 40, 4, 192, 1.0, 0.05, "random"),
    # C4: MAF dynamic flow (nf/flows.py:241-284) behind a context-dropping adapter -- the
    # reference builds MAF but never wires it into DPF -- with OT resampling
    "c4": (dict(NF_dyn=True, NF_cond=True, measurement="cos", resampler_type="ot", NF_dyn_flow="MAF"), 3, 48, 4, 32, 0.5, 0.3, "aligned"),
}


def maf_adapter(n_flows=2, dim=2, hidden=8):
    """The reference's MAF stack (nf/flows.py MAF in nf/models.py NormalizingFlowModel) with
    nf_dynamic_model's (x, context) call signature; the context is ignored."""
    import torch
    from nf.flows import MAF
    from nf.models import NormalizingFlowModel

    class Adapter(torch.nn.Module):
        def __init__(self):
            super().__init__()
            prior = torch.distributions.MultivariateNormal(torch.zeros(dim), torch.eye(dim))
            self.m = NormalizingFlowModel(prior, [MAF(dim=dim, hidden_dim=hidden) for _ in range(n_flows)],
                                          device="cpu")
            self.flows = self.m.flows

        def forward(self, x, context=None):
            return self.m.forward(x)

        def inverse(self, z, context=None):
            return self.m.inverse(z)

    return Adapter()


def gen_e2e(mods, name):
    import torch
    from DPFs import DPF
    from losses import supervised_loss
    flags, B, N, T, H, pe_std, fl_std, enc_mode = E2E[name]
    g = torch.Generator().manual_seed(16)
    torch.manual_seed(500)
    dyn_kind = flags.get("NF_dyn_flow", "RealNVP")
    flags = {k: v for k, v in flags.items() if k != "NF_dyn_flow"}
    a = make_args(num_particles=N, batchsize=B, sequence_length=T, **flags)
    dpf = DPF(a)
    if dyn_kind == "MAF":
        dpf.nf_dyn = maf_adapter()
        dpf.nf_dyn.eval()
    dpf.eval()
    # sharpen the likelihood so ESS-gated resampling fires within a few steps
    perturb(dpf.particle_encoder, pe_std, g)
    for m in (dpf.nf_dyn.flows, dpf.cond_model.flows):
        perturb(m, fl_std, g)
    if flags["measurement"] == "CRNVP":
        perturb(dpf.cnf_measurement.flows, 0.1, g)
    if flags["measurement"] == "CGLOW":
        perturb(dpf.cglow_measurement, 0.1, g)
    dpf.encoder = torch.nn.Identity()
    Henc = 192 if flags["measurement"] == "CGLOW" else H
    start = torch.cat([torch.rand(B, 2, generator=g) * 100 - 50, torch.randn(B, 2, generator=g) * 3], -1)
    vel = torch.randn(B, T, 2, generator=g) * 3
    pos = start[:, None, :2] + torch.cumsum(vel, 1)
    if enc_mode == "aligned":
        with torch.no_grad():
            enc = dpf.particle_encoder(pos)
        enc = enc + 0.3 * enc.abs().mean() * torch.randn(enc.shape, generator=g)
    else:
        enc = torch.randn(B, T, Henc, generator=g)
    state = torch.cat([pos + torch.randn(B, T, 2, generator=g) * 2, vel], -1)
    seed = 600
    torch.manual_seed(seed)
    with torch.no_grad():
        res = dpf.filtering_pos(enc, start, vel)
    (xl, pl, nl, ll, lw0, il, jl, prl, obs) = res
    # replay the global CPU generator to record the draws (order: SURVEY §8c)
    torch.manual_seed(seed)
    init_x = torch.rand(B, N, 2) * 128.0 - 64.0
    torch.randn(B, N, 2)
    from utils import normalize_log_probs
    p = normalize_log_probs(lw0)
    offsets, fired = [], []
    for t in range(T):
        ess = torch.mean(1 / torch.sum(p ** 2, dim=-1))
        f = bool(ess < 0.5 * N)
        fired.append(f)
        offsets.append(torch.FloatTensor(B).uniform_(0.0, 1.0 / N) if (f and flags["resampler_type"] == "soft")
                       else torch.zeros(B))
        noise = torch.normal(mean=0.0, std=a.pos_noise, size=(B, N, 2))
        assert torch.equal(noise, nl[:, t]), "draw replay diverged"
        p = pl[:, t]
    loss, pred = supervised_loss(xl, pl, state, 1.0, False)
    out = {"B": np.int32(B), "N": np.int32(N), "T": np.int32(T), "H": np.int32(Henc)}
    for k, v in flags.items():
        out[f"flag/{k}"] = np.array(v)
    if dyn_kind != "RealNVP":
        out["flag/NF_dyn_flow"] = np.array(dyn_kind)
    for k, v in sd_np(dpf).items():
        k = k.replace("nf_dyn.m.", "nf_dyn.")  # the adapter's stack -> DPF's nf_dyn key names
        if k.split(".")[0] in ("nf_dyn", "cond_model", "particle_encoder", "cnf_measurement", "cglow_measurement"):
            out[f"w/{k}"] = v
    out.update(enc=enc.numpy(), start=start.numpy(), vel=vel.numpy(), state=state.numpy(),
               init_x=init_x.numpy(), offsets=torch.stack(offsets, 1).numpy(), fired=np.array(fired),
               x=xl.numpy(), p=pl.numpy(), noise=nl.numpy(), lik=ll.numpy(), logw0=lw0.numpy(),
               idx=il.numpy().astype(np.int32), obs_lik=np.float32(obs), rmse=np.float32(loss), pred=pred.numpy())
    if jl is not None:
        out.update(jac=jl.numpy(), prior=prl.numpy())
    np.savez_compressed(os.path.join(OUT, f"e2e_{name}.npz"), **out)
    print(name, "resample fired at steps", [t for t, f in enumerate(fired) if f])


FWD = {
    # name: (flag overrides, B, N, T)
    "fwd_c2_sdpf": (dict(NF_dyn=True, NF_cond=True, measurement="cos", resampler_type="soft", trainType="SDPF",
                         block_length=2), 3, 64, 4),
    "fwd_c1_sdpf": (dict(NF_dyn=False, NF_cond=False, measurement="cos", resampler_type="soft", trainType="SDPF",
                         block_length=2), 3, 64, 4),
    "fwd_c3": (dict(NF_dyn=False, NF_cond=False, measurement="CRNVP", resampler_type="ot", trainType="DPF"), 2, 48,
               3),
}


def gen_forward(mods, name):
    """DPF.forward(inputs, train=False) (DPFs.py:96-142) of the reference, all 13 outputs."""
    import torch
    sys.path.insert(0, os.path.dirname(OUT))
    from _tiny import TinyDecoder, TinyEncoder
    from DPFs import DPF
    flags, B, N, T = FWD[name]
    g = torch.Generator().manual_seed(21)
    torch.manual_seed(700)
    a = make_args(num_particles=N, batchsize=B, sequence_length=T, **flags)
    dpf = DPF(a)
    dpf.encoder, dpf.decoder = TinyEncoder(a.hiddensize), TinyDecoder(a.hiddensize)
    perturb(dpf.encoder, 0.3, g)
    perturb(dpf.decoder, 0.3, g)
    perturb(dpf.particle_encoder, 0.5, g)
    for m in (dpf.nf_dyn.flows, dpf.cond_model.flows):
        perturb(m, 0.05, g)
    if flags["measurement"] == "CRNVP":
        perturb(dpf.cnf_measurement.flows, 0.1, g)
    dpf.eval()
    start = torch.cat([torch.rand(B, 2, generator=g) * 100 - 50, torch.randn(B, 2, generator=g) * 3], -1)
    vel = torch.randn(B, T, 2, generator=g) * 3
    pos = start[:, None, :2] + torch.cumsum(vel, 1)
    state = torch.cat([pos + torch.randn(B, T, 2, generator=g) * 2, vel], -1)
    # frames: 16x16 random blocks of 8x8 pixels (stored small; fwd_frames() expands them)
    img = torch.randint(0, 256, (B, T, 16, 16, 3), generator=g, dtype=torch.uint8)
    start_img = torch.randint(0, 256, (B, 16, 16, 3), generator=g, dtype=torch.uint8)
    up = lambda t: t.float().div(255).repeat_interleave(8, -3).repeat_interleave(8, -2)  # noqa: E731
    inputs = (up(start_img), start, up(img), state, torch.zeros(B, T), torch.ones(B, T))
    seed = 800
    torch.manual_seed(seed)
    with torch.no_grad():
        out = dpf.forward(inputs, train=False)
    (total, sup, pseud, ae, pred, pl, pwl, st, ss, image, ll, nl, obs) = out
    res = {"B": np.int32(B), "N": np.int32(N), "T": np.int32(T), "seed": np.int32(seed), "H": np.int32(a.hiddensize)}
    for k, v in flags.items():
        res[f"flag/{k}"] = np.array(v)
    for k, v in sd_np(dpf).items():
        if k.split(".")[0] in ("encoder", "decoder", "nf_dyn", "cond_model", "particle_encoder", "cnf_measurement"):
            res[f"w/{k}"] = v
    res.update(start=start.numpy(), state=state.numpy(), img=img.numpy(), start_img=start_img.numpy(),
               total=np.float32(total), sup=np.float32(sup), ae=np.float32(ae), pred=pred.numpy(), x=pl.numpy(),
               p=pwl.numpy(), lik=ll.numpy(), noise=nl.numpy(), obs_lik=np.float32(obs))
    if pseud is not None:
        res["pseud"] = np.float32(pseud)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **res)
    print(name, "total", float(total), "sup", float(sup))


def gen_keys(mods):
    """state_dict key -> shape of the reference's DPF for every measurement model (checkpoint
    compatibility of the drop-in, SURVEY.md §5 checkpoint row)."""
    import json
    import torch
    from DPFs import DPF
    out = {}
    for meas, H in (("cos", 32), ("CRNVP", 32), ("NN", 32), ("gaussian", 32), ("CGLOW", 192)):
        torch.manual_seed(0)
        dpf = DPF(make_args(measurement=meas, hiddensize=H, NF_dyn=True, NF_cond=meas != "CGLOW"))
        out[meas] = {k: list(v.shape) for k, v in dpf.state_dict().items()}
    with open(os.path.join(OUT, "state_dict_keys.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)


def _grad_pack(out, key, named):
    for k, v in named:
        out[f"{key}/g/{k}"] = (v.grad if v.grad is not None else torch_zeros_like(v)).detach().numpy().copy()


def torch_zeros_like(v):
    import torch
    return torch.zeros_like(v)


def gen_grads(mods):
    """Reference autograd gradients of L = sum(out * g_out) for random g_out."""
    import torch
    import resamplers.resamplers as R
    from DPFs import DPF
    from model.models import build_conditional_nf
    from nf.flows import MAF
    from nf.models import NormalizingFlowModel
    from torch.distributions import MultivariateNormal
    out = {}
    g = torch.Generator().manual_seed(31)
    # -- conditional RealNVP stacks (nf/models.py:37-66), forward and inverse
    for D, O, pstd in ((2, 4, 1.0), (2, 36, 1.0), (32, 32, 2.5)):
        for inv in (False, True):
            torch.manual_seed(900 + D + O)
            m = build_conditional_nf(2, O, D, init_var=0.01, prior_std=pstd)
            perturb(m.flows, 0.2, g)
            M = 64
            x = (torch.randn(M, D, generator=g) * 3).requires_grad_(True)
            c = torch.randn(M, O, generator=g).requires_grad_(True)
            gz, gl, gp = torch.randn(M, D, generator=g), torch.randn(M, generator=g), torch.randn(M, generator=g)
            if inv:
                z, ld = m.inverse(x, c)
                loss = (z * gz).sum() + (ld * gl).sum()
            else:
                z, lp, ld = m.forward(x, c)
                loss = (z * gz).sum() + (ld * gl).sum() + (lp * gp).sum()
            loss.backward()
            k = f"cond_D{D}_O{O}_{'inv' if inv else 'fwd'}"
            for kk, v in sd_np(m.flows, "flows.").items():
                out[f"{k}/w/{kk}"] = v
            out[f"{k}/prior_std"] = np.float32(pstd)
            for name, v in (("x", x), ("c", c), ("gz", gz), ("gl", gl), ("gp", gp)):
                out[f"{k}/{name}"] = v.detach().numpy()
            out[f"{k}/dx"], out[f"{k}/dc"] = x.grad.numpy(), c.grad.numpy()
            _grad_pack(out, k, [("flows." + n, q) for n, q in m.flows.named_parameters()])
    # -- MAF stack (nf/flows.py:241-284), D = 2: forward only -- the reference's MAF.inverse
    # writes x in place while reading it (:279-283), so its autograd raises ("modified by an
    # inplace operation"); there is no reference gradient to pin for the inverse
    for inv in (False,):
        torch.manual_seed(950)
        flows = [MAF(dim=2) for _ in range(2)]
        perturb(torch.nn.ModuleList(flows), 0.3, g)
        m = NormalizingFlowModel(MultivariateNormal(torch.zeros(2), torch.eye(2)), flows, device="cpu")
        x = (torch.randn(64, 2, generator=g) * 2).requires_grad_(True)
        gz, gl = torch.randn(64, 2, generator=g), torch.randn(64, generator=g)
        z, ld = m.inverse(x) if inv else m.forward(x)[::2]
        ((z * gz).sum() + (ld * gl).sum()).backward()
        k = f"maf_{'inv' if inv else 'fwd'}"
        for kk, v in sd_np(m.flows, "flows.").items():
            out[f"{k}/w/{kk}"] = v
        for name, v in (("x", x), ("gz", gz), ("gl", gl)):
            out[f"{k}/{name}"] = v.detach().numpy()
        out[f"{k}/dx"] = x.grad.numpy()
        _grad_pack(out, k, [("flows." + n, q) for n, q in m.flows.named_parameters()])
    # -- soft resampler (resamplers.py:20-60): d/dx through the gather, d/dp through p / q
    B, N = 4, 200
    x = (torch.randn(B, N, 2, generator=g) * 30).requires_grad_(True)
    lw = torch.randn(B, N, generator=g) * 2
    p = (torch.softmax(lw, -1) + 1e-12).requires_grad_(True)
    gx, gw = torch.randn(B, N, 2, generator=g), torch.randn(B, N, generator=g)
    torch.manual_seed(77)
    xo, wo, idx = R.soft_resampler(x, p, 0.5, N, index=True, device="cpu")
    torch.manual_seed(77)
    off = torch.FloatTensor(B).uniform_(0.0, 1.0 / N)
    ((xo * gx).sum() + (wo * gw).sum()).backward()
    out.update({"soft/x": x.detach().numpy(), "soft/p": p.detach().numpy(), "soft/offsets": off.numpy(),
                "soft/gx": gx.numpy(), "soft/gw": gw.numpy(), "soft/dx": x.grad.numpy(), "soft/dp": p.grad.numpy(),
                "soft/idx": idx.numpy().astype(np.int32)})
    # -- OT resampler (resamplers.py:234-264): T held constant, no gradient to the weights
    B, N = 3, 96
    x = (torch.randn(B, N, 2, generator=g) * 30).requires_grad_(True)
    p = torch.softmax(torch.randn(B, N, generator=g) * 2, -1) + 1e-12
    gx = torch.randn(B, N, 2, generator=g)
    xo, wo, idx = R.resampler_ot(x, p, eps=0.1, scaling=0.75, threshold=1e-3, max_iter=100, device="cpu")
    (xo * gx).sum().backward()
    out.update({"ot/x": x.detach().numpy(), "ot/p": p.numpy(), "ot/gx": gx.numpy(), "ot/dx": x.grad.numpy()})
    # -- measurement models (model/models.py:206-303): d/d(encodings, particles, parameters)
    for meas, H in (("cos", 32), ("CRNVP", 32), ("NN", 32), ("gaussian", 32), ("CGLOW", 192)):
        torch.manual_seed(960)
        dpf = DPF(make_args(measurement=meas, hiddensize=H, num_particles=40, batchsize=3))
        perturb(dpf.particle_encoder, 0.3, g)
        if meas == "CRNVP":
            perturb(dpf.cnf_measurement.flows, 0.1, g)
        if meas == "CGLOW":
            perturb(dpf.cglow_measurement, 0.1, g)
        if meas == "NN":
            perturb(dpf.likelihood_est, 0.2, g)
        mm = dpf.measurement_model
        enc = torch.randn(3, 192 if meas == "CGLOW" else H, generator=g).requires_grad_(True)
        x = (torch.randn(3, 40, 2, generator=g) * 30).requires_grad_(True)
        gl = torch.randn(3, 40, generator=g)
        (mm(enc, x) * gl).sum().backward()
        k = f"meas_{meas}"
        for kk, v in sd_np(dpf).items():
            if kk.split(".")[0] in ("particle_encoder", "cnf_measurement", "cglow_measurement", "likelihood_est"):
                out[f"{k}/w/{kk}"] = v
        out.update({f"{k}/enc": enc.detach().numpy(), f"{k}/x": x.detach().numpy(), f"{k}/gl": gl.numpy(),
                    f"{k}/denc": enc.grad.numpy(), f"{k}/dx": x.grad.numpy()})
        _grad_pack(out, k, [n_q for n_q in mm.named_parameters()])
    np.savez_compressed(os.path.join(OUT, "grads.npz"), **out)


def gen_train_step(mods, name="train_c2"):
    """One training forward + backward of the reference (DPFs.py:318-331): DPF.forward(inputs,
    train=True) -> total_loss.backward(), every parameter's gradient recorded."""
    import torch
    sys.path.insert(0, os.path.dirname(OUT))
    from _tiny import TinyDecoder, TinyEncoder
    from DPFs import DPF
    flags = dict(NF_dyn=True, NF_cond=True, measurement="cos", resampler_type="soft", trainType="SDPF",
                 block_length=2)
    B, N, T = 3, 48, 4
    g = torch.Generator().manual_seed(41)
    torch.manual_seed(710)
    a = make_args(num_particles=N, batchsize=B, sequence_length=T, **flags)
    dpf = DPF(a)
    dpf.encoder, dpf.decoder = TinyEncoder(a.hiddensize), TinyDecoder(a.hiddensize)
    perturb(dpf.encoder, 0.3, g)
    perturb(dpf.decoder, 0.3, g)
    perturb(dpf.particle_encoder, 0.5, g)
    for m in (dpf.nf_dyn.flows, dpf.cond_model.flows):
        perturb(m, 0.05, g)
    dpf.train()
    start = torch.cat([torch.rand(B, 2, generator=g) * 100 - 50, torch.randn(B, 2, generator=g) * 3], -1)
    vel = torch.randn(B, T, 2, generator=g) * 3
    pos = start[:, None, :2] + torch.cumsum(vel, 1)
    state = torch.cat([pos + torch.randn(B, T, 2, generator=g) * 2, vel], -1)
    img = torch.randint(0, 256, (B, T, 16, 16, 3), generator=g, dtype=torch.uint8)
    start_img = torch.randint(0, 256, (B, 16, 16, 3), generator=g, dtype=torch.uint8)
    up = lambda t: t.float().div(255).repeat_interleave(8, -3).repeat_interleave(8, -2)  # noqa: E731
    inputs = (up(start_img), start, up(img), state, torch.zeros(B, T), torch.ones(B, T))
    seed = 810
    np.random.seed(seed)
    torch.manual_seed(seed)
    outp = dpf.forward(inputs, train=True)
    dpf.zero_grad()
    outp[0].backward()
    res = {"B": np.int32(B), "N": np.int32(N), "T": np.int32(T), "seed": np.int32(seed), "H": np.int32(a.hiddensize)}
    for k, v in flags.items():
        res[f"flag/{k}"] = np.array(v)
    for k, v in sd_np(dpf).items():
        if k.split(".")[0] in ("encoder", "decoder", "nf_dyn", "cond_model", "particle_encoder"):
            res[f"w/{k}"] = v
    res.update(start=start.numpy(), state=state.numpy(), img=img.numpy(), start_img=start_img.numpy(),
               total=np.float32(outp[0].detach()), sup=np.float32(outp[1].detach()),
               pseud=np.float32(outp[2].detach()), ae=np.float32(outp[3].detach()),
               x=outp[5].detach().numpy(), p=outp[6].detach().numpy())
    for n, q in dpf.named_parameters():
        if q.grad is not None:
            res[f"g/{n}"] = q.grad.numpy().copy()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **res)
    print(name, "total", float(outp[0]), "grads", sum(1 for k in res if k.startswith("g/")))


def gen_cglow_flow(mods):
    """CondGlowModel.forward(x, y) (nf/cglow/CGlowModel.py:167-176) -> (z, nll), reference
    defaults (K = 1, L = 1).  (Its reverse, :178-184, raises in the reference: Cond1x1Conv
    .view()s the non-contiguous inverse weight, modules.py:195 -- nothing to record.)"""
    import torch
    from nf.cglow.CGlowModel import CondGlowModel
    g = torch.Generator().manual_seed(51)
    torch.manual_seed(52)
    m = CondGlowModel(make_args())
    perturb(m, 0.1, g)
    with torch.no_grad():
        m.new_mean.zero_()
        m.new_logs.zero_()
    M = 40
    x = torch.randn(M, 3, 8, 8, generator=g)
    y = torch.randn(M, 3, 8, 8, generator=g)
    with torch.no_grad():
        z, nll = m(x, y)
    out = {f"w/{k}": v for k, v in sd_np(m).items()}
    out.update(x=x.numpy(), y=y.numpy(), z=z.numpy(), nll=nll.numpy())
    np.savez_compressed(os.path.join(OUT, "cglow_flow.npz"), **out)


def gen_flows_extra(mods):
    """The flows the DPF never instantiates (nf/flows.py:22-98, 287-458) and
    the rational-quadratic spline (nf/utils.py:23-147): forward / inverse outputs, and for the
    spline flows the autograd gradients of a random linear functional of (z, log_det)."""
    import torch
    import torch.nn.functional as F
    from nf import flows as fl
    from nf.utils import RQS, unconstrained_RQS
    out = {}
    g = torch.Generator().manual_seed(61)
    # splines: K bins, inputs partly outside the tail bound
    for K, B in ((5, 3.0), (8, 2.0)):
        M = 300
        x = (torch.rand(M, generator=g) * 2 - 1) * (B * 1.3)
        W, H, D = (torch.randn(M, K, generator=g) * 1.5, torch.randn(M, K, generator=g) * 1.5,
                   torch.randn(M, K - 1, generator=g))
        y, ld = unconstrained_RQS(x, W.clone(), H.clone(), D.clone(), inverse=False, tail_bound=B)
        xi, ldi = unconstrained_RQS(y, W.clone(), H.clone(), D.clone(), inverse=True, tail_bound=B)
        k = f"urqs_K{K}/"
        out.update({k + "x": x.numpy(), k + "W": W.numpy(), k + "H": H.numpy(), k + "D": D.numpy(),
                    k + "B": np.float32(B), k + "y": y.numpy(), k + "ld": ld.numpy(), k + "xi": xi.numpy(),
                    k + "ldi": ldi.numpy()})
        xb = torch.rand(M, generator=g) * 0.98 + 0.01
        Df = torch.randn(M, K + 1, generator=g)
        yb, ldb = RQS(xb, W.clone(), H.clone(), Df.clone())
        xbi, ldbi = RQS(yb, W.clone(), H.clone(), Df.clone(), inverse=True)
        k = f"rqs_K{K}/"
        out.update({k + "x": xb.numpy(), k + "D": Df.numpy(), k + "y": yb.numpy(), k + "ld": ldb.numpy(),
                    k + "xi": xbi.numpy(), k + "ldi": ldbi.numpy()})
    # neural spline flows (forward, inverse of the forward output, gradients)
    for name, ctor, D in (("nsf_ar_D2", lambda: fl.NSF_AR(2), 2), ("nsf_ar_D4", lambda: fl.NSF_AR(4), 4),
                          ("nsf_cl_D4", lambda: fl.NSF_CL(4), 4), ("nsf_cl_D6", lambda: fl.NSF_CL(6, K=6, B=2), 6)):
        torch.manual_seed(70 + D)
        m = ctor()
        M = 64
        x = torch.randn(M, D, generator=g) * 1.5
        z, ld = m(x)
        xi, ldi = m.inverse(z.detach())
        k = name + "/"
        out.update({k + "w/" + n: v for n, v in sd_np(m).items()})
        out.update({k + "x": x.numpy(), k + "z": z.detach().numpy(), k + "ld": ld.detach().numpy(),
                    k + "xi": xi.detach().numpy(), k + "ldi": ldi.detach().numpy()})
        xg = x.clone().requires_grad_(True)
        z, ld = m(xg)
        cz, cl = torch.randn(M, D, generator=g), torch.randn(M, generator=g)
        ((z * cz).sum() + (ld * cl).sum()).backward()
        out.update({k + "cz": cz.numpy(), k + "cl": cl.numpy(), k + "gx": xg.grad.numpy()})
        for n, p_ in m.named_parameters():
            out[k + "g/" + n] = p_.grad.numpy().copy()
    # planar (three non-linearities), radial, actnorm, 1x1 convolution
    for nl, tag in ((torch.tanh, "tanh"), (F.leaky_relu, "leaky_relu"), (F.elu, "elu")):
        torch.manual_seed(80)
        m = fl.Planar(3, nonlinearity=nl)
        x = torch.randn(50, 3, generator=g) * 2
        with torch.no_grad():
            z, ld = m(x)
        k = f"planar_{tag}/"
        out.update({k + "w/" + n: v for n, v in sd_np(m).items()})
        out.update({k + "x": x.numpy(), k + "z": z.numpy(), k + "ld": ld.numpy()})
    torch.manual_seed(81)
    m = fl.Radial(3)
    m.reset_parameters(3)
    x = torch.randn(50, 3, generator=g)
    with torch.no_grad():
        z, ld = m(x)
    out.update({"radial/w/" + n: v for n, v in sd_np(m).items()})
    out.update({"radial/x": x.numpy(), "radial/z": z.numpy(), "radial/ld": ld.numpy()})
    m = fl.ActNorm(3)
    perturb(m, 0.5, g)
    x = torch.randn(50, 3, generator=g)
    with torch.no_grad():
        z, ld = m(x)
        xi, ldi = m.inverse(z)
    out.update({"actnorm/w/" + n: v for n, v in sd_np(m).items()})
    out.update({"actnorm/x": x.numpy(), "actnorm/z": z.numpy(), "actnorm/ld": np.float32(ld),
                "actnorm/xi": xi.numpy(), "actnorm/ldi": np.float32(ldi)})
    np.random.seed(82)
    m = fl.OneByOneConv(3)
    x = torch.randn(50, 3, generator=g)
    with torch.no_grad():
        z, ld = m(x)
        xi, ldi = m.inverse(z)
    out.update({"conv1x1/P": m.P.numpy(), "conv1x1/L": m.L.detach().numpy(), "conv1x1/S": m.S.detach().numpy(),
                "conv1x1/U": m.U.detach().numpy(), "conv1x1/x": x.numpy(), "conv1x1/z": z.numpy(),
                "conv1x1/ld": np.float32(ld), "conv1x1/xi": xi.numpy(), "conv1x1/ldi": np.float32(ldi)})
    np.savez_compressed(os.path.join(OUT, "flows_extra.npz"), **out)


def gen_autoencoder(mods):
    """The frame encoder / decoder CNNs and autoencoder_loss (model/models.py:10-117,
    losses.py:5-16).  The networks are 1.6 M parameters: instead of storing
    them, each is built right after torch.manual_seed(s) -- the same layers in the same order
    draw the same default init -- and the fixture holds a checksum of every parameter, the
    input frames' seed, the features, a fixed subsample of the reconstruction and the loss,
    in train (batch statistics) and eval mode."""
    import torch
    from model.models import build_decoder, build_decoder_cglow, build_encoder, build_encoder_cglow
    from losses import autoencoder_loss
    out = {}
    for tag, benc, bdec, H in (("h32", build_encoder, build_decoder, 32),
                               ("cglow", build_encoder_cglow, build_decoder_cglow, 192)):
        torch.manual_seed(301)
        enc = benc(H)
        torch.manual_seed(302)
        dec = bdec(H)
        for name, m in (("enc", enc), ("dec", dec)):
            for k, v in m.state_dict().items():
                out[f"{tag}/{name}/sum/{k}"] = np.float64(v.double().sum())
                out[f"{tag}/{name}/abs/{k}"] = np.float64(v.double().abs().sum())
        g = torch.Generator().manual_seed(303)
        img = torch.rand(2, 2, 3, 128, 128, generator=g)
        idx = torch.randint(0, 4 * 3 * 128 * 128, (512,), generator=g)
        out[f"{tag}/idx"] = idx.numpy()
        for mode in ("train", "eval"):
            enc.train(mode == "train")
            dec.train(mode == "train")
            with torch.no_grad():
                x = img.reshape(4, 3, 128, 128)
                f = enc(x)
                r = dec(f)
                loss = autoencoder_loss(img, mode == "train", enc, dec)
            out[f"{tag}/{mode}/feature"] = f.numpy()
            out[f"{tag}/{mode}/recon_sample"] = r.reshape(-1)[idx].numpy()
            out[f"{tag}/{mode}/recon_mean"] = r.mean(dim=(0, 2, 3)).numpy()
            out[f"{tag}/{mode}/loss"] = np.float32(loss)
    np.savez_compressed(os.path.join(OUT, "autoencoder.npz"), **out)


def gen_dataset(mods):
    """The disk generator's trajectories (data/disk/create_dataset.py:120-216): start state,
    states and q of a few sequences drawn from numpy's global generator.  The reference draws
    its frames with cv2.circle; cv2 is not installed, so for THIS fixture its placeholder
    module gets a no-op ``circle`` -- circle draws no random numbers, so the recorded
    trajectories are the reference's own; its frames / visibility are not recorded."""
    import importlib.util
    sys.modules["cv2"].circle = lambda *a, **k: None
    spec = importlib.util.spec_from_file_location("ref_create_dataset", os.path.join(REF, "data/disk/create_dataset.py"))
    cd = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cd)
    import tempfile
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        param = types.SimpleNamespace(width=128, out_dir=tmp, name="fixture", num_examples=4, sequence_length=6,
                                      file_size=500)
        ex = cd.ToyExample(param)
        for case, (nd, pn, seed) in enumerate(((0, 2.0, 91), (3, 2.0, 92), (25, 5.0, 93))):
            np.random.seed(seed)
            for n in range(2):
                v = ex._get_data(nd, pn)
                for k in ("start_state", "state", "q"):
                    out[f"c{case}/s{n}/{k}"] = np.asarray(v[k])
            out[f"c{case}/cfg"] = np.array([nd, pn, seed], dtype=np.float64)
            out[f"c{case}/next_uniform"] = np.float64(np.random.uniform())  # the RNG state after
    np.savez_compressed(os.path.join(OUT, "dataset.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    mods = import_reference()
    jobs = {"flows": gen_flows, "stacks": gen_stacks, "soft": gen_soft, "ot": gen_ot, "meas": gen_meas}
    for k, fn in jobs.items():
        if not args.only or args.only == k:
            fn(mods)
            print("wrote", k)
    for name in E2E:
        if not args.only or args.only == name:
            gen_e2e(mods, name)
    for name in FWD:
        if not args.only or args.only == name:
            gen_forward(mods, name)
    if not args.only or args.only == "keys":
        gen_keys(mods)
    if not args.only or args.only == "cglow_flow":
        gen_cglow_flow(mods)
    if not args.only or args.only == "flows_extra":
        gen_flows_extra(mods)
    if not args.only or args.only == "dataset":
        gen_dataset(mods)
    if not args.only or args.only == "autoencoder":
        gen_autoencoder(mods)
    if not args.only or args.only == "grads":
        gen_grads(mods)
    if not args.only or args.only == "train_c2":
        gen_train_step(mods)


if __name__ == "__main__":
    main()
