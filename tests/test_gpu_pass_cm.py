"""The C3-shaped one-launch pass (nfdpf_filter_pass_tiled -> tiled_pass_cm_kernel: no dynamic flow,
no conditional proposal, the conditional-RealNVP measurement, the speculative ESS gate) against
the step-by-step launches and against the CPU oracle replaying the pass's own device draws.
GPU box only.  (The C2-shaped pass: test_gpu_pass.py.)"""
import os

import numpy as np
import pytest
import torch

from _util import assert_close, e2e_cfg, load, weights
from oracle import dpf_oracle as O
from test_gpu_parity import _Models, _check_envelope
from test_gpu_pass import _Replay, _fractions, _inputs

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from nfdpf import _lib
    _lib.load()
    assert torch.cuda.is_available()


# the no-flow pass's measurements: C3 (CRNVP + OT), C1 (cosine + soft), and the gaussian one
MEAS = {"CRNVP": ("CRNVP", "ot", "c3"), "cos": ("cos", "soft", "c1"), "gaussian": ("gaussian", "soft", "c1")}


def _models(fixture, meas="CRNVP"):
    """bench: DPF(args) of BASELINE's C3 (or C1; bench.py CONFIGS) at its init weights, seed 2,
    with the measurement ``meas``; else the e2e fixture's weights (tests/golden, the reference's
    own C3 model)."""
    if fixture == "bench":
        import bench
        from DPFs import DPF
        m, r, cfgname = MEAS[meas]
        flags, B, N, T, _, _ = bench.CONFIGS[cfgname]
        torch.manual_seed(2)
        return DPF(bench.make_args(flags, B, N, T, {"measurement": m, "resampler_type": r})).to(DEV).eval()
    fx = load(fixture)
    return _Models(weights(fx), e2e_cfg(fx))


def _cfg(N, meas="CRNVP"):
    c = e2e_cfg(load("e2e_c3.npz"))  # the C3 flags: NF_dyn / NF_cond off, CRNVP, OT
    c["N"] = N
    c["measurement"], c["resampler"] = MEAS[meas][:2]
    return c


def _engine(models, N, seed, spec=True, meas="CRNVP"):
    from nfdpf.engine import FilterConfig, FilterEngine
    m, r, _ = MEAS[meas]
    cfg = FilterConfig(N=N, NF_dyn=False, NF_cond=False, measurement=m, resampler=r, seed=seed,
                       kernel="tiled", speculate_gate=spec)
    return FilterEngine(cfg, models)


CASES = [(4, 1000, 10, "bench", "CRNVP"), (3, 257, 6, "bench", "CRNVP"), (2, 1024, 8, "bench", "CRNVP"),
         (5, 100, 5, "bench", "CRNVP"), (4, 1000, 8, "e2e_c3.npz", "CRNVP"), (64, 1000, 50, "bench", "CRNVP"),
         # C1 (BASELINE configs[0]: 16 x 100 x 24, cosine, soft) and a larger cosine row; gaussian
         (16, 100, 24, "bench", "cos"), (4, 1000, 10, "bench", "cos"), (4, 257, 8, "bench", "gaussian")]


@pytest.mark.parametrize("B,N,T,fixture,meas", CASES)
def test_cm_pass_matches_step_launches(B, N, T, fixture, meas, monkeypatch):
    """One launch == T x the step launches of the same speculative pass: noise, indices and
    particles bit-equal (the bootstrap proposal is the same two adds); likelihoods, weights,
    predictions and the obs-likelihood to rounding (the per-tile partials merge over 4 particle
    groups in the pass, over the block in the step launch).  Ragged rows (257: a last tile of
    one particle; 100: empty groups), the maximum N, the C3 shape 64 x 1000 x 50."""
    models = _models(fixture, meas)
    enc, start, vel = _inputs(B, T, seed=B * 1000 + N)
    eng = _engine(models, N, 41, meas=meas)
    a = eng.run(enc, start, vel)
    torch.cuda.synchronize()
    assert eng.pass_launches == 1, "the one-launch C3 pass did not run"
    monkeypatch.setenv("NFDPF_PASS", "0")
    if not eng.last_pass:
        # the fixture's sharp likelihood fires a gate: the verification caught it and the result
        # is the step-by-step rerun (OT where the gates fire), bit for bit the step launches
        eng_b = _engine(models, N, 41, spec=False, meas=meas)
        b = eng_b.run(enc, start, vel)
        torch.cuda.synchronize()
        for f in ("particles", "probs", "noise", "lik", "index", "pred", "obs_likelihood"):
            assert torch.equal(getattr(a, f), getattr(b, f)), f
        return
    eng_b = _engine(models, N, 41, meas=meas)
    b = eng_b.run(enc, start, vel)
    torch.cuda.synchronize()
    assert not eng_b.last_pass
    assert torch.equal(a.noise, b.noise)
    assert torch.equal(a.index, b.index)
    ident = torch.arange(N, device=DEV) + N * torch.arange(B, device=DEV)[:, None]
    assert torch.equal(a.index, ident[:, None, :].expand(B, T, N)), "a verified pass resamples nothing"
    assert torch.equal(a.particles, b.particles)
    assert_close(a.lik.cpu(), b.lik.cpu(), 1e-5, 1e-4, "likelihood")
    assert_close(a.probs.cpu(), b.probs.cpu(), 1e-4, 1e-9, "weights")
    assert_close(a.pred.cpu(), b.pred.cpu(), 1e-5, 1e-3, "prediction")
    assert abs(float(a.obs_likelihood) - float(b.obs_likelihood)) <= 1e-5 * abs(float(b.obs_likelihood)) + 1e-4


# (the e2e_c3 fixture's sharp likelihood fires a gate on every input tried: its rerun is compared
# with the step launches above and in test_cm_pass_gate_fired_reruns)
ORACLE_CASES = [(4, 1000, 10, "bench", "CRNVP"), (3, 257, 6, "bench", "CRNVP"), (2, 1024, 8, "bench", "CRNVP"),
                (64, 1000, 50, "bench", "CRNVP"), (16, 100, 24, "bench", "cos"), (4, 1000, 10, "bench", "cos"),
                (4, 257, 1, "bench", "gaussian")]  # (its gate fires from step 1 at init weights)


@pytest.mark.parametrize("B,N,T,fixture,meas", ORACLE_CASES)
def test_cm_pass_vs_oracle(B, N, T, fixture, meas):
    """The C3 pass against the oracle (float32 and float64) on the same initial particles and
    motion noise, free-running over T steps with every gate off (checked: the verified pass, and
    every step's ESS above 0.6 N so that no rounding can tip one): particles, weights and the
    shifted likelihood inside the float32 oracle's own error envelope (test_gpu_parity.
    _check_envelope: 4x max / 2.5x mean of its error against float64), the obs-likelihood too.
    The first of a fixed list of input seeds whose gates stay off by that margin is used."""
    from nfdpf import ops
    c = _cfg(N, meas)
    models = _models(fixture, meas)
    w = {k: v.detach().cpu() for k, v in models.state_dict().items()}
    quiet = False
    for k in range(12 if fixture != "bench" else 3):
        enc, start, vel = _inputs(B, T, seed=7 * N + B + 1000 * k)
        x0, logw0 = ops.particle_init(start[:, :2], B, N, 128.0, False, 5, 0, DEV)
        eng = _engine(models, N, 5, meas=meas)
        res = eng.run(enc, start, vel, init=(x0, logw0))
        torch.cuda.synchronize()
        ess = (1.0 / (res.probs[:, :-1].double() ** 2).sum(-1)).mean(0)
        quiet = eng.last_pass and eng.pass_launches == 1
        if quiet and (T == 1 or float(ess.min()) > 0.6 * N):
            break
    assert quiet and (T == 1 or float(ess.min()) > 0.6 * N), "no input seed kept the gate off by a margin"
    outs = {}
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    for dt in (torch.float32, torch.float64):
        with O.precision(dt):
            wd = O.cast_params(w, dt)
            r = O.filtering(c, wd, enc.cpu().to(dt), start.cpu().to(dt), vel.cpu().to(dt), rng=_Replay(res.noise),
                            init=(x0.cpu().to(dt), logw0.cpu().to(dt)))
        outs[dt] = [a.double().numpy() if torch.is_tensor(a) else a for a in r]
    r32, r64 = outs[torch.float32], outs[torch.float64]
    np.testing.assert_array_equal(res.index.cpu().numpy(), r32[5])  # no resampling in the oracle either
    print(f"\nno-flow pass ({meas}) vs oracle, B={B} N={N} T={T} ({fixture}):")
    for i, what, rtol, atol in ((0, "particles", 1e-5, 1e-4), (1, "weights", 1e-5, 1e-9), (3, "likelihood", 1e-5, 2e-5)):
        ours = getattr(res, ("particles", "probs", None, "lik")[i]).cpu()
        _check_envelope(ours, r32[i], r64[i], rtol, atol, what)
        _fractions(what, ours, r32[i], r64[i], 1e-5, 0.0)
    obs64 = float(r64[8])
    assert abs(float(res.obs_likelihood) - obs64) <= 4 * abs(float(r32[8]) - obs64) + 1e-5 * abs(obs64) + 1e-4


def test_cm_pass_gate_fired_reruns(monkeypatch):
    """The e2e_c3 fixture (the reference's own C3 model, inputs and sizes) fires the ESS gate: the
    speculative C3 pass's verification catches it and the engine reruns the pass step by step
    (the FP64-faithful OT resampler where the gates fire) -- bit for bit the step launches run
    directly, the fired steps' indices included."""
    from _util import t
    fx = load("e2e_c3.npz")
    models = _Models(weights(fx), e2e_cfg(fx))
    enc, start, vel = t(fx["enc"]).to(DEV), t(fx["start"]).to(DEV), t(fx["vel"]).to(DEV)
    N = int(fx["N"])
    eng = _engine(models, N, 9)
    a = eng.run(enc, start, vel)
    torch.cuda.synchronize()
    assert eng.pass_launches == 1 and not eng.last_pass, "the fired speculation was not rerun step by step"
    assert eng.last_ot_calls > 0, "the gate never fired"
    monkeypatch.setenv("NFDPF_PASS", "0")
    eng_b = _engine(models, N, 9, spec=False)
    b = eng_b.run(enc, start, vel)
    torch.cuda.synchronize()
    assert eng_b.last_ot_calls == eng.last_ot_calls
    for f in ("particles", "probs", "noise", "lik", "index", "pred"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    assert torch.equal(a.obs_likelihood, b.obs_likelihood)
