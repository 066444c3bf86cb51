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


if __name__ == "__main__":
    main()
