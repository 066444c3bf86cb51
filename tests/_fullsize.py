"""Workloads at the BASELINE sizes for the host-RNG parity tests (tests/test_gpu_parity_full.py).

Each case builds the DPF's modules with this package's builders, perturbs them from a seeded
generator (the reference init, N(0, 0.01^2) coupling weights, makes every flow the identity to
~1e-2 and the likelihood flat -- nothing to test), draws a synthetic disk trajectory with
"aligned" frame encodings (the particle encoder applied to the true position plus noise, as a
trained encoder would give) so that the ESS gate fires on some steps, and runs the CPU oracle
(oracle/dpf_oracle.py, pinned to the reference by tests/golden) with the reference's
CPU-generator draw order, recording the draws on a tape the HIP engine then replays.
"""
import time

import numpy as np
import torch

from oracle import dpf_oracle as O

# name: (flags, B, N, T, particle-encoder std, flow std, measurement-net std, force_resample)
CASES = {
    # BASELINE configs[1]: CNF-DPF (--NF-dyn --NF-cond, RealNVP), cos, soft, N=1000, B=64, T=50
    # (coupling weights ~ N(0, 0.01^2), the reference's own init; the gate fires in 17 of 50 steps)
    "c2_full": (dict(NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft"), 64, 1000, 50, 0.5, 0.01, 0.0,
                False),
    # BASELINE configs[2]: DPF-CM (--measurement CRNVP), OT, N=1000, B=64 -- T cut to 10 steps (every
    # fired step is one FP64 Sinkhorn of the oracle at B=64: ~10 s on 16 host cores; each is run
    # once and recorded, see build)
    "c3_full": (dict(NF_dyn=False, NF_cond=False, measurement="CRNVP", resampler="ot"), 64, 1000, 10, 0.5, 0.05, 0.1,
                False),
    # BASELINE configs[3] shape: MAF dynamic flow, NF proposal, cos, OT at N=4000, resampling every
    # step, 8 rows (the batch-coupled stop rule over 8 rows; a C4 rank holds 32)
    "c4_n4000": (dict(NF_dyn=True, NF_cond=True, measurement="cos", resampler="ot", dyn_flow="MAF"), 8, 4000, 3, 0.5,
                 0.05, 0.0, True),
    # BASELINE configs[4] shape: CNF-DPF + CGLOW measurement (--hiddensize 192), soft resampling at
    # N=10000 every step (40 tiles per row in the front launch), 8 rows = 80 000 particles: the
    # CGLOW kernel's persistent grid (768 workgroups x 16 particles) takes ~7 tiles per workgroup
    "c5_n10000": (dict(NF_dyn=True, NF_cond=True, measurement="CGLOW", resampler="soft"), 8, 10000, 3, 0.5, 0.05,
                  0.1, True),
}


def cfg_dict(flags, N):
    return dict(N=N, NF_dyn=flags["NF_dyn"], NF_cond=flags["NF_cond"], measurement=flags["measurement"],
                resampler=flags["resampler"], alpha=0.5, eps=0.1, scaling=0.75, threshold=1e-3, max_iter=100,
                pos_noise=20.0, vel_noise=20.0, width=128, n_flows=2, cglow_K=1,
                dyn_flow=flags.get("dyn_flow", "RealNVP"))


def hidden(flags):
    """--hiddensize: 192 for CGLOW (the reference crashes with 32), else 32."""
    return 192 if flags["measurement"] == "CGLOW" else 32


class Holder(torch.nn.Module):
    """The DPF attribute names the engine reads (nf_dyn, cond_model, particle_encoder, ...)."""

    def __init__(self, flags):
        super().__init__()
        from model.models import (build_conditional_nf, build_maf_dyn, build_particle_encoder,
                                  build_particle_encoder_cglow)
        H = hidden(flags)
        self.nf_dyn = build_maf_dyn(2, 2) if flags.get("dyn_flow") == "MAF" else build_conditional_nf(2, 4, 2)
        self.cond_model = build_conditional_nf(2, 4 + H, 2)
        if flags["measurement"] == "CGLOW":
            from arguments import parse_args
            from nf.cglow.CGlowModel import CondGlowModel
            self.particle_encoder = build_particle_encoder_cglow(H, 2)
            self.cglow_measurement = CondGlowModel(parse_args(["--hiddensize", str(H)]))
        else:
            self.particle_encoder = build_particle_encoder(H, 2)
        if flags["measurement"] == "CRNVP":
            self.cnf_measurement = build_conditional_nf(2, H, H, prior_std=2.5)


def _perturb(module, std, g):
    with torch.no_grad():
        for p in module.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * std)


class RecordingRNG(O.HostRNG):
    """The reference's CPU-generator draws (seeded generator), recorded per step."""

    def __init__(self, seed):
        super().__init__(torch.Generator().manual_seed(seed))
        self.noise_tape, self.off_tape = [], []

    def offsets(self, B, N):
        v = super().offsets(B, N)
        self.off_tape.append((len(self.noise_tape), v.clone()))  # belongs to the step drawing noise next
        return v

    def noise(self, B, N, std):
        v = super().noise(B, N, std)
        self.noise_tape.append(v.clone())
        return v


class Tape:
    """Replays a RecordingRNG's draws to nfdpf.engine.FilterEngine (host-RNG mode)."""

    def __init__(self, rec: RecordingRNG):
        self.noise_tape = rec.noise_tape
        self.off = dict(rec.off_tape)
        self.t = 0

    def offsets(self, B, N):
        return self.off[self.t].clone()

    def noise(self, B, N, std):
        v = self.noise_tape[self.t].clone()
        self.t += 1
        return v


def workload(name, seed=0, B=None, N=None, T=None):
    """The case's modules, trajectory and aligned frame encodings (no oracle run); B / N / T
    override the case's sizes.  -> dict(flags, models (CPU), enc, start, vel, state, force, g)."""
    flags, B0, N0, T0, pe_std, fl_std, m_std, force = CASES[name]
    B, N, T = B or B0, N or N0, T or T0
    g = torch.Generator().manual_seed(1000 + seed)
    torch.manual_seed(2000 + seed)
    models = Holder(flags)
    _perturb(models.particle_encoder, pe_std, g)
    _perturb(models.nf_dyn.flows, fl_std, g)
    _perturb(models.cond_model.flows, fl_std, g)
    if flags["measurement"] == "CRNVP":
        _perturb(models.cnf_measurement.flows, m_std, g)
    if flags["measurement"] == "CGLOW":
        _perturb(models.cglow_measurement, m_std, g)
    start = torch.cat([torch.rand(B, 2, generator=g) * 100 - 50, torch.randn(B, 2, generator=g) * 3], -1)
    vel = torch.randn(B, T, 2, generator=g) * 3
    pos = start[:, None, :2] + torch.cumsum(vel, 1)
    with torch.no_grad():
        enc = models.particle_encoder(pos)
    enc = enc + 0.3 * enc.abs().mean() * torch.randn(enc.shape, generator=g)
    state = torch.cat([pos + torch.randn(B, T, 2, generator=g) * 2, vel], -1)
    return dict(flags=flags, models=models, enc=enc, start=start, vel=vel, state=state, force=force, g=g,
                B=B, N=N, T=T)


def build(name, seed=0):
    """-> dict(cfg, flags, models (CPU), params (oracle dict), enc, start, vel, state, force,
    ref (oracle 9-tuple), fired, tape (RecordingRNG), oracle_s)."""
    flags, B, N, T, pe_std, fl_std, m_std, force = CASES[name]
    wl = workload(name, seed)
    models, enc, start, vel, state, g = wl["models"], wl["enc"], wl["start"], wl["vel"], wl["state"], wl["g"]
    params = {k: v.detach().float().cpu().clone() for k, v in models.state_dict().items()}
    cfg = cfg_dict(flags, N)
    init_x = torch.rand(B, N, 2, generator=g) * 128.0 - 64.0
    logw0 = torch.log(torch.ones(B, N) / N)
    rec = RecordingRNG(3000 + seed)
    saved, step, ot = O.OT_POTENTIALS, O.filter_step, O.ot_resample
    O.OT_POTENTIALS = 2  # bit-identical outputs, half the FP64 work (oracle/dpf_oracle.py)
    fired = []
    ot_calls = {}  # step -> the oracle's Sinkhorn call (input, output, iterations, x' in fp64)

    def step_rec(*a, **k):
        r = step(*a, **k)
        fired.append(bool(r["fired"]))
        print(f"  [{name}] oracle step {len(fired) - 1}: fired {fired[-1]} ({time.perf_counter() - t0:.1f} s)",
              flush=True)  # progress: a long oracle run must not look hung
        return r

    def ot_rec(x, w, *a, **k):
        # each FP64 Sinkhorn of the oracle runs once: the direct OT test and the float64
        # envelope reuse it (x' = T x with the oracle's own fp64 transport matrix, in fp64)
        xr, wr, idx, info = ot(x, w, *a, return_info=True, **k)
        ot_calls[len(fired)] = dict(x=x.clone(), w=w.clone(), xr=xr.clone(), iters=int(info["iters"]),
                                    xr64=torch.matmul(info["T"].double(), x.double()))
        return xr, wr, idx

    O.filter_step, O.ot_resample = step_rec, ot_rec
    t0 = time.perf_counter()
    try:
        with torch.no_grad():
            ref = O.filtering(cfg, params, enc, start, vel, rng=rec, force_resample=force, init=(init_x, logw0))
        dt = time.perf_counter() - t0
    finally:
        O.OT_POTENTIALS, O.filter_step, O.ot_resample = saved, step, ot
    return dict(cfg=cfg, flags=flags, models=models, params=params, enc=enc, start=start, vel=vel, state=state,
                force=force, init=(init_x, logw0), ref=ref, fired=fired, rec=rec, oracle_s=dt, B=B, N=N, T=T,
                ot_calls=ot_calls)


def frac_within(ours, ref, rtol, atol):
    """Fraction of elements with |ours - ref| <= rtol |ref| + atol, and the worst offenders."""
    a = np.asarray(ours, dtype=np.float64)
    b = np.asarray(ref, dtype=np.float64)
    d = np.abs(a - b)
    ok = d <= rtol * np.abs(b) + atol
    worst = np.argsort((d - rtol * np.abs(b)).ravel())[-3:][::-1]
    return float(ok.mean()), [(np.unravel_index(i, a.shape), float(a.ravel()[i]), float(b.ravel()[i])) for i in worst]
