"""The whole filtering pass as ONE persistent launch (nfdpf_filter_pass_tiled, csrc/filter_pass.hpp)
against (a) the step-by-step tiled launches on the same device-RNG draws and (b) the oracle
(the reference's algorithm, float32 and float64) replaying those draws.  GPU box only.

Three modes: speculative (every ESS gate, DPFs.py:163-165, taken as off and verified after the
pass; a fired gate reruns the pass), forced (the row resampled at the top of every step) and
gated (the batch-global gate decided inside the launch at every step -- the default on one GPU).
Against the step launches the pass differs in the order of the row's x_phys sums and in the
coupling nets' rounding (the tanh algebra is folded into the pass layout's weights), so (a) is
a rounding-level comparison; (b) is the reference-parity check: every history within the
reference's own float32 envelope, the gate decisions and resampling indices exact.
"""
import os

import numpy as np
import pytest
import torch

from _util import assert_close, e2e_cfg, load, t, weights
from oracle import dpf_oracle as O
from test_gpu_parity import _Models, _check_envelope

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from nfdpf import _lib
    _lib.load()
    assert torch.cuda.is_available()


def _inputs(B, T, seed, scale=10.0):
    g = torch.Generator().manual_seed(seed)
    enc = torch.randn(B, T, 32, generator=g).to(DEV)
    start = (torch.randn(B, 4, generator=g) * scale).to(DEV)
    vel = (torch.randn(B, T, 2, generator=g) * 3).to(DEV)
    return enc, start, vel


def _models(fixture):
    """The fixture's flows (e2e_c2: std 0.05, e2e_c2w: std 0.3) with a default-initialised
    particle encoder: the fixtures' encoder is sharpened so that the ESS gate fires (what the
    gate tests need); a pass whose gate fires is rerun step by step, and the comparison here is
    of the one-launch pass itself."""
    from model.models import build_particle_encoder
    if fixture == "bench":  # the bench's model: DPF(args) at its init weights, seed 2 (bench.py)
        import bench
        from DPFs import DPF
        flags, B, N, T, _, _ = bench.CONFIGS["c2"]
        torch.manual_seed(2)
        return DPF(bench.make_args(flags, B, N, T, {})).to(DEV).eval()
    fx = load(fixture)
    m = _Models(weights(fx), e2e_cfg(fx))
    torch.manual_seed(12)
    m.particle_encoder = build_particle_encoder(32, 2).to(DEV)
    return m


def _run(models, N, enc, start, vel, spec, seed=41, env=None, monkeypatch=None):
    from nfdpf.engine import FilterConfig, FilterEngine
    if monkeypatch is not None:
        monkeypatch.setenv("NFDPF_PASS", env or "1")
    cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=seed,
                       kernel="tiled", speculate_gate=spec)
    eng = FilterEngine(cfg, models)
    res = eng.run(enc, start, vel)
    torch.cuda.synchronize()
    return eng, res


CASES = [(6, 1000, 8, "e2e_c2.npz"), (6, 1000, 8, "e2e_c2w.npz"), (5, 777, 6, "e2e_c2.npz"),
         (5, 777, 6, "e2e_c2w.npz"), (3, 100, 5, "e2e_c2.npz"), (4, 257, 7, "e2e_c2.npz"),
         (4, 257, 7, "e2e_c2w.npz"), (2, 1024, 4, "e2e_c2.npz"), (64, 1000, 50, "bench"),
         (64, 1000, 50, "e2e_c2w.npz"),
         # more rows than the device holds at once (MI355X: 256 CUs, 64 rows of 4 tiles): the
         # speculative pass runs them in resident chunks of rows, one launch each
         (96, 1000, 6, "bench"), (80, 777, 5, "e2e_c2.npz")]


@pytest.mark.parametrize("B,N,T,fixture", CASES)
def test_pass_matches_step_launches(B, N, T, fixture, monkeypatch):
    """One launch == T x (front + proposal launches): noise and indices bit-equal; histories to
    rounding.  Ragged rows (777, 257: a last tile of 9 / 1 particles), one tile with empty wave
    groups (N = 100), the maximum N (1024), the C2 shape (64 x 1000 x 50, the bench's model).  The wide flows
    (e2e_c2w, std 0.3) degenerate the weights within a step or two, so the ESS gate fires: the
    verification must catch it and the step-by-step rerun is returned (bit-equal); with the
    e2e_c2 flows the gate stays off and the one-launch pass itself is compared."""
    models = _models(fixture)
    enc, start, vel = _inputs(B, T, seed=B * 1000 + N)
    eng, a = _run(models, N, enc, start, vel, spec=True)
    assert eng.pass_launches >= 1, "the one-launch pass did not run"
    if fixture == "e2e_c2w.npz" and not eng.last_gates.eq(0).all():
        # a gate fired: the verification caught it and the rerun -- the gated one-launch pass --
        # is the result, bit for bit the gated pass run directly
        assert eng.pass_launches == 2 and eng.last_gate_pass
        eng_g, g = _run(models, N, enc, start, vel, spec=False)
        assert eng_g.last_gate_pass and eng_g.pass_launches == 1
        for f in ("particles", "probs", "noise", "lik", "index", "jac", "prior", "pred", "obs_likelihood"):
            assert torch.equal(getattr(a, f), getattr(g, f)), f
        return
    _, b = _run(models, N, enc, start, vel, spec=False, env="0", monkeypatch=monkeypatch)  # the step launches
    assert eng.last_pass, f"a gate fired on the {fixture} flows"
    assert torch.equal(a.noise, b.noise)
    assert torch.equal(a.index, b.index)
    ident = torch.arange(N, device=DEV) + N * torch.arange(B, device=DEV)[:, None]
    assert torch.equal(a.index, ident[:, None, :].expand(B, T, N)), "a verified pass resamples nothing"
    assert_close(a.particles.cpu(), b.particles.cpu(), 1e-5, 1e-4, "particles")
    assert_close(a.probs.cpu(), b.probs.cpu(), 1e-4, 1e-9, "weights")
    assert_close(a.lik.cpu(), b.lik.cpu(), 1e-4, 1e-5, "likelihood")
    assert_close(a.jac.cpu(), b.jac.cpu(), 1e-5, 1e-5, "jac")
    assert_close(a.prior.cpu(), b.prior.cpu(), 1e-5, 1e-4, "prior")
    assert_close(a.pred.cpu(), b.pred.cpu(), 1e-5, 1e-3, "prediction")
    assert abs(float(a.obs_likelihood) - float(b.obs_likelihood)) <= 1e-5 * abs(float(b.obs_likelihood)) + 1e-4


class _Replay:
    """The device draws of our own pass replayed into the oracle (HostRNG's interface)."""

    def __init__(self, noise):
        self.noise_t = noise.detach().cpu()
        self.k = 0
        self.gen = None

    def offsets(self, B, N):
        raise AssertionError("the oracle resampled: the gate fired")

    def noise(self, B, N, std):
        v = self.noise_t[:, self.k].clone()
        self.k += 1
        return v


def _fractions(what, ours, r32, r64, rtol, atol):
    """north_star's 1e-5 bar: the fraction of elements within rtol |ref64| + atol of the float64
    oracle, ours next to the reference's own float32 run (printed for the round's record)."""
    ours, r32, r64 = (np.asarray(a, dtype=np.float64) for a in (ours, r32, r64))
    bar = rtol * np.abs(r64) + atol
    f_ours, f_ref = float(np.mean(np.abs(ours - r64) <= bar)), float(np.mean(np.abs(r32 - r64) <= bar))
    print(f"  {what}: within {rtol:g} rel + {atol:g}: ours {100 * f_ours:.3f} %, reference float32 "
          f"{100 * f_ref:.3f} %; max err ours {np.abs(ours - r64).max():.3e} vs float32 {np.abs(r32 - r64).max():.3e}")


PASS_ORACLE_CASES = [(4, 1000, 10, "bench"), (3, 257, 6, "bench"), (2, 1024, 8, "bench"), (4, 1000, 6, "e2e_c2.npz"),
                     (3, 257, 6, "e2e_c2.npz"), (2, 1024, 8, "e2e_c2.npz"),
                     # the BASELINE C2 shape itself, the bench's model (DPF(args) at its init weights)
                     (64, 1000, 50, "bench")]


@pytest.mark.parametrize("B,N,T,fixture", PASS_ORACLE_CASES)
def test_pass_vs_oracle(B, N, T, fixture):
    """The pass against the oracle run on the same initial particles and motion noise: ours vs
    the oracle in float64 within 4x (max) / 2.5x (mean) of the oracle float32's own error
    (test_gpu_parity._check_envelope, the one-step tests' bar), free-running over T steps (no
    resampling: nothing discrete can diverge).  Includes the headline shape, 64 x 1000 x 50.
    The e2e_c2 flows (std 0.05) degenerate the weights on some draws and the gate then fires
    (compared elsewhere): the first of a fixed list of input seeds whose gates all stay off by a
    margin (every step's ESS above 0.6 N, so that the oracle's own rounding cannot tip one) is
    used -- deterministic, and never a skip."""
    from nfdpf import ops
    c = e2e_cfg(load("e2e_c2.npz"))  # the C2 flags
    c["N"] = N
    models = _models(fixture)
    w = {k: v.detach().cpu() for k, v in models.state_dict().items()}
    from nfdpf.engine import FilterConfig, FilterEngine
    cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=5,
                       kernel="tiled", speculate_gate=True)
    for k in range(12 if fixture != "bench" else 1):
        enc, start, vel = _inputs(B, T, seed=7 * N + B + 1000 * k)
        x0, logw0 = ops.particle_init(start[:, :2], B, N, 128.0, False, 5, 0, DEV)
        eng = FilterEngine(cfg, models)
        res = eng.run(enc, start, vel, init=(x0, logw0))
        torch.cuda.synchronize()
        ess = (1.0 / (res.probs[:, :-1].double() ** 2).sum(-1)).mean(0)  # the gates of steps 1 .. T-1
        quiet = eng.last_pass and not eng.last_gate_pass and eng.pass_launches == 1  # the speculative pass verified
        if quiet and (T == 1 or float(ess.min()) > 0.6 * N):
            break
    assert quiet and (T == 1 or float(ess.min()) > 0.6 * N), \
        "no input seed kept the gate off by a margin (a fired gate reruns the pass gated)"
    outs = {}
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    for dt in (torch.float32, torch.float64):
        with O.precision(dt):
            wd = O.cast_params(w, dt)
            r = O.filtering(c, wd, enc.cpu().to(dt), start.cpu().to(dt), vel.cpu().to(dt), rng=_Replay(res.noise),
                            init=(x0.cpu().to(dt), logw0.cpu().to(dt)))
        outs[dt] = [a.double().numpy() if torch.is_tensor(a) else a for a in r]
    r32, r64 = outs[torch.float32], outs[torch.float64]
    np.testing.assert_array_equal(res.index.cpu().numpy(), r32[5])
    print(f"\npass vs oracle, B={B} N={N} T={T} ({fixture}):")
    for i, what, rtol, atol in ((0, "particles", 1e-5, 1e-4), (1, "weights", 1e-5, 1e-9), (3, "likelihood", 1e-5, 2e-5),
                                (6, "jac", 1e-5, 1e-6), (7, "prior", 1e-5, 1e-5)):
        ours = getattr(res, ("particles", "probs", None, "lik", None, None, "jac", "prior")[i]).cpu()
        _check_envelope(ours, r32[i], r64[i], rtol, atol, what)
        _fractions(what, ours, r32[i], r64[i], 1e-5, 0.0 if what != "jac" else 1e-6)
    obs64 = float(r64[8])
    assert abs(float(res.obs_likelihood) - obs64) <= 4 * abs(float(r32[8]) - obs64) + 1e-5 * abs(obs64) + 1e-4


def test_pass_gate_fired_reruns(monkeypatch):
    """Encodings aligned with the true state: the ESS gate fires.  The speculative pass's
    verification catches it and reruns -- as the gated one-launch pass, which decides every gate
    inside the launch: the result is that pass run directly, bit for bit (histories, decisions,
    obs-likelihood).  (The gated pass against the reference at every step, decisions and indices
    exact: test_gated_pass_every_step_vs_oracle.)"""
    fx = load("e2e_c2.npz")
    models = _Models(weights(fx), e2e_cfg(fx))
    enc, start, vel = t(fx["enc"]).to(DEV), t(fx["start"]).to(DEV), t(fx["vel"]).to(DEV)
    N = int(fx["N"])
    eng_a, a = _run(models, N, enc, start, vel, spec=True)
    assert eng_a.pass_launches == 2 and eng_a.last_gate_pass, "the fired speculation was not rerun as the gated pass"
    ga = eng_a.last_gates.clone()
    eng_b, b = _run(models, N, enc, start, vel, spec=False)
    assert eng_b.pass_launches == 1 and eng_b.last_gate_pass
    for f in ("particles", "probs", "noise", "lik", "index", "jac", "prior", "pred"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    assert torch.equal(a.obs_likelihood, b.obs_likelihood)
    assert torch.equal(ga, eng_b.last_gates)
    B, T = enc.shape[0], enc.shape[1]
    ident = torch.arange(N, device=DEV) + N * torch.arange(B, device=DEV)[:, None]
    fired_rows = (a.index != ident[:, None, :]).any(-1).any(0).int()
    assert int(fired_rows.sum()) > 0, "the gate never fired"
    # a fired step resamples (almost surely moves some index), a quiet one leaves the identity
    assert torch.equal(fired_rows, ga.int()), (fired_rows.tolist(), ga.tolist())


def test_pass_deterministic_and_graph_replay():
    """Two passes give identical bits; a hipGraph-captured pass (the bench's mode: run(finish=
    False) captured, finish_pending after each replay) replays to the same result."""
    models = _models("bench")
    B, N, T = 8, 1000, 12
    enc, start, vel = _inputs(B, T, seed=99)
    eng, a = _run(models, N, enc, start, vel, spec=True)
    assert eng.last_pass
    _, b = _run(models, N, enc, start, vel, spec=True)
    for f in ("particles", "probs", "lik", "jac", "prior", "pred"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cap = eng.run(enc, start, vel, finish=False, speculate=True)
    for _ in range(3):
        g.replay()
        assert eng.finish_pending()
        torch.cuda.synchronize()
        for f in ("particles", "probs", "lik", "pred"):
            assert torch.equal(getattr(cap, f), getattr(a, f)), f
        assert torch.equal(cap.obs_likelihood, a.obs_likelihood)


@pytest.mark.parametrize("T,B,N", [(37, 5, 300), (50, 64, 1000), (1, 3, 1024)])
def test_pass_verify_matches_gate_batch(T, B, N):
    """ops.pass_verify (one launch: gates + fired count + the hand-off fault counter) == the
    batch gate kernel on the same partials, with a mix of fired and quiet steps."""
    from nfdpf import ops
    tiles = (N + 255) // 256
    g = torch.Generator().manual_seed(T * 7 + B)
    odd = (torch.arange(T)[:, None, None] % 2 == 1).double()
    m = torch.randn(T, B, tiles, generator=g, dtype=torch.float64) * odd
    # even steps nearly uniform weights (ESS ~ N: quiet), odd steps peaked (fired)
    spread = 0.01 + 30.0 * odd
    e = torch.rand(T, B, tiles, generator=g, dtype=torch.float64) * 250 + 1
    sq = e * e / 256 * (1 + spread)
    parts = torch.stack([m, e, sq, torch.zeros_like(m)], -1).to(DEV)
    ref = ops.ess_gate_tiled_batch(parts, N, 0, False)
    lw = (torch.randn(B, T, generator=g) * 50).to(DEV)
    gates, flags, obs = ops.pass_verify(parts, lw, N)
    torch.cuda.synchronize()
    assert torch.equal(gates, ref)
    assert flags.tolist() == [int(ref.sum()), 0]
    obs_ref = float((lw.double().sum(0) / (B * N)).sum())
    assert abs(float(obs) - obs_ref) <= 1e-6 * abs(obs_ref) + 1e-6
    if T > 1:
        assert 0 < int(ref.sum()) < T, "the case should mix fired and quiet steps"


@pytest.mark.parametrize("world", [2, 3])
def test_row_terms_gates_match_gate_batch(world):
    """The sharded verification's two halves (each rank: nfdpf_ess_row_terms of its rows; after
    the gather: nfdpf_ess_gate_terms over B_global rows) == the batch gate kernel on the gathered
    partials, bit for bit, with fired and quiet steps; the fault word rides at the end."""
    from nfdpf import ops
    T, B, N = 12, 8, 1000
    tiles = (N + 255) // 256
    g = torch.Generator().manual_seed(world)
    odd = (torch.arange(T)[:, None, None] % 2 == 1).double()
    m = torch.randn(T, world * B, tiles, generator=g, dtype=torch.float64) * odd
    e = torch.rand(T, world * B, tiles, generator=g, dtype=torch.float64) * 250 + 1
    sq = e * e / 256 * (1 + 0.01 + 30.0 * odd)
    parts = torch.stack([m, e, sq, torch.zeros_like(m)], -1).to(DEV)
    ref = ops.ess_gate_tiled_batch(parts, N, 0, False)
    per_rank = [ops.ess_row_terms(parts[:, r * B:(r + 1) * B], N) for r in range(world)]
    assert all(int(t[T * B:].view(torch.int32)) == 0 for t in per_rank)  # no hand-off fault
    terms = torch.stack([t[:T * B].view(T, B) for t in per_rank], 1).reshape(T, world * B)
    gates = ops.ess_gate_terms(terms, N)
    torch.cuda.synchronize()
    assert torch.equal(gates, ref), (gates.tolist(), ref.tolist())
    assert 0 < int(ref.sum()) < T


def test_pass_disabled_by_env(monkeypatch):
    """NFDPF_PASS=0 keeps the step-by-step launches (the library reads it per call)."""
    fx = load("e2e_c2.npz")
    models = _Models(weights(fx), e2e_cfg(fx))
    enc, start, vel = _inputs(2, 3, seed=3)
    monkeypatch.setenv("NFDPF_PASS", "0")
    eng, _ = _run(models, 300, enc, start, vel, spec=True)
    assert not eng.last_pass


def test_pass_shape_fallback_is_reported(monkeypatch):
    """A C2-shaped run beyond the pass's shape limits (here N > 1024 particles per row) runs the
    step launches and says so: one RuntimeWarning per engine and ``pass_fallback_reason``;
    NFDPF_PASS=0 (chosen, not a limit) stays quiet.  A speculative pass of more rows than the
    device holds at once is NOT such a limit: its rows run in resident chunks."""
    fx = load("e2e_c2.npz")
    models = _Models(weights(fx), e2e_cfg(fx))
    enc, start, vel = _inputs(2, 2, seed=5)
    with pytest.warns(RuntimeWarning, match="one-launch pass does not cover"):
        eng, _ = _run(models, 1100, enc, start, vel, spec=True)
    assert not eng.last_pass and eng.pass_launches == 0
    assert "1024" in eng.pass_fallback_reason
    import warnings
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    B = cus // 4 + 1  # N = 1000: 4 tiles per row, one row more than resident at once
    enc, start, vel = _inputs(B, 2, seed=5)
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        eng2, _ = _run(models, 1000, enc, start, vel, spec=True)
        assert eng2.pass_launches >= 1 and eng2.pass_fallback_reason is None
        assert not eng2._gate_resident  # (the gated pass needs every row resident: not here)
        monkeypatch.setenv("NFDPF_PASS", "0")
        eng3, _ = _run(models, 1000, enc[:2], start[:2], vel[:2], spec=True)
    assert not eng3.last_pass


def _philox_offsets(seed, T, B, N, row_base=0):
    """The device RNG's soft-resampling offsets (csrc/common.hpp rng_draw(seed, kTagOffset = 1,
    t, row, 0) -> u01 / N), restated on the host: offsets [T, B] float32."""
    M = 0xFFFFFFFF

    def philox(c, k0, k1):
        x, y, z, w = c
        for _ in range(10):
            p0, p1 = x * 0xD2511F53, z * 0xCD9E8D57
            x, y, z, w = ((p1 >> 32) ^ y ^ k0) & M, p1 & M, ((p0 >> 32) ^ w ^ k1) & M, p0 & M
            k0, k1 = (k0 + 0x9E3779B9) & M, (k1 + 0xBB67AE85) & M
        return x
    out = np.zeros((T, B), dtype=np.float32)
    for t in range(T):
        for b in range(B):
            row = row_base + b
            u = philox((0, row & M, ((row >> 32) ^ (t << 8)) & M, 1), seed & M, (seed >> 32) & M)
            out[t, b] = np.float32((u >> 8) * np.float32(2.0 ** -24)) * np.float32(np.float32(1.0) / np.float32(N))
    return out


@pytest.mark.parametrize("B,N,T", [(6, 1000, 8), (4, 257, 6), (3, 100, 5), (64, 1000, 50)])
def test_forced_pass_resampling_bit_exact(B, N, T):
    """--force-resample: the pass resamples every row every step inside the launch.  Every
    step's indices equal the ORACLE's soft resampler (resamplers.py:20-60 restated, pinned to the
    reference's golden vectors) on the pass's own previous slot and the device offsets, bit for
    bit; the resampled log-weights likewise feed the same step; the whole pass against the
    step-by-step launches: index agreement and predictions as test_gpu_parity's tiled == fused."""
    models = _models("e2e_c2.npz")
    enc, start, vel = _inputs(B, T, seed=B * 31 + N)
    from nfdpf.engine import FilterConfig, FilterEngine
    out = {}
    for env in ("1", "0"):
        import os
        os.environ["NFDPF_PASS"] = env
        try:
            cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=77,
                               kernel="tiled", force_resample=True)
            eng = FilterEngine(cfg, models)
            out[env] = eng.run(enc, start, vel)
            torch.cuda.synchronize()
            assert eng.last_pass == (env == "1")
        finally:
            os.environ.pop("NFDPF_PASS", None)
    a, b = out["1"], out["0"]
    off = _philox_offsets(77, T, B, N)
    x, p, idx = a.particles.cpu(), a.probs.cpu(), a.index.cpu()
    for t in range(1, T):
        _, _, ref_idx = O.soft_resample(x[:, t - 1].contiguous(), p[:, t - 1].contiguous(), 0.5,
                                        torch.from_numpy(off[t]))
        assert torch.equal(idx[:, t], ref_idx.long()), f"step {t}: indices differ from the oracle's"
    assert torch.equal(a.noise, b.noise)
    # step 0 resamples the initial state: identical inputs, identical indices; later a marker within
    # rounding of a CDF step flips an index and the row then follows other particles (resampling
    # every step compounds it: ~70 % agreement after 50 forced steps) -- the per-step oracle
    # check above is the parity claim
    assert torch.equal(a.index[:, 0], b.index[:, 0])
    agree = (a.index == b.index).float().mean().item()
    print(f"forced pass vs step launches: indices agree {100 * agree:.2f} %")
    assert torch.allclose(a.particles[:, :1], b.particles[:, :1], rtol=1e-4, atol=1e-2)
    assert torch.allclose(a.pred[:, :1], b.pred[:, :1], rtol=1e-4, atol=1e-2)
    assert torch.isfinite(a.probs).all()
    s = a.probs.sum(-1)
    assert torch.allclose(s, torch.ones_like(s) + N * 1e-12, atol=1e-5)


class _StepDraws:
    """One step's device draws replayed into the oracle: the soft-resampling offsets and the
    motion noise (the HostRNG interface of oracle.filter_step)."""

    def __init__(self, off, noise):
        self.off, self.nz = off, noise

    def offsets(self, B, N):
        return self.off.clone()

    def noise(self, B, N, std):
        return self.nz.clone()


def _soft_indices32(soft32):
    """The float64 oracle's soft resampler with the reference's own (float32) indices: the
    marker search is the one discrete step, and float64 arithmetic can move a marker across a
    CDF step -- the envelope then measures the continuous arithmetic around the same indices
    (test_gpu_parity._oracle64_one_step does the same)."""
    def soft64(x, p, alpha, offsets=None, gen=None):
        with O.precision(torch.float32):
            _, _, idx = soft32(x.float(), p.float(), alpha, offsets.float())
        B, N = p.shape
        q = alpha * p + (1 - alpha) / N
        q = q / q.sum(-1, keepdim=True)
        w = (p / q).reshape(B * N)[idx]
        return x.reshape(B * N, -1)[idx], w / w.sum(-1, keepdim=True), idx
    return soft64


# (80 rows of N = 1000: more than the device holds at once -- resident chunks, the last first)
@pytest.mark.parametrize("B,N,T", [(6, 1000, 8), (4, 257, 6), (3, 100, 5), (64, 1000, 50), (80, 1000, 6)])
def test_forced_pass_every_step_vs_oracle(B, N, T, monkeypatch):
    """--force-resample inside the one-launch pass, every step against the oracle's step
    (oracle.filter_step = DPFs.py:160-192 with resamplers.py:20-60) started from the PASS's own
    slot t-1 (particles, normalised weights) with the pass's device offsets and motion noise:
    the indices bit for bit against the float32 oracle, and the resampled weights' consequence --
    the normalised weights p -- with the particles, likelihood, jac and prior of every slot within
    the reference's own float32 envelope against the float64 oracle (_check_envelope).  Teacher
    forcing from our own state: a marker within rounding of a CDF step cannot make the two runs
    follow different particles, so every step of a 64 x 1000 x 50 forced pass is pinned."""
    from nfdpf import ops
    from nfdpf.engine import FilterConfig, FilterEngine
    models = _models("e2e_c2.npz")
    w = {k: v.detach().cpu() for k, v in models.state_dict().items()}
    c = e2e_cfg(load("e2e_c2.npz"))
    c["N"] = N
    enc, start, vel = _inputs(B, T, seed=B * 31 + N)
    x0, logw0 = ops.particle_init(start[:, :2], B, N, 128.0, False, 77, 0, DEV)
    p0, _ = ops.normalize_log_probs(logw0)
    cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=77,
                       kernel="tiled", force_resample=True)
    eng = FilterEngine(cfg, models)
    res = eng.run(enc, start, vel, init=(x0, logw0))
    torch.cuda.synchronize()
    assert eng.last_pass, "the forced pass did not run as one launch"
    off = torch.from_numpy(_philox_offsets(77, T, B, N))
    xs, ps, nz = res.particles.cpu(), res.probs.cpu(), res.noise.cpu()
    x0c, p0c, encc, startc, velc = x0.cpu(), p0.cpu(), enc.cpu(), start.cpu(), vel.cpu()
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    keys = ("x", "p", "lik", "jac", "prior")
    outs = {}
    soft32 = O.soft_resample
    for dt in (torch.float32, torch.float64):
        if dt == torch.float64:
            monkeypatch.setattr(O, "soft_resample", _soft_indices32(soft32))
        acc = {k: [] for k in keys + ("idx",)}
        with O.precision(dt):
            wd = O.cast_params(w, dt)
            meas = O.make_measurement(c, wd)
            for t_ in range(T):
                xp = (x0c if t_ == 0 else xs[:, t_ - 1]).to(dt)
                pp = (p0c if t_ == 0 else ps[:, t_ - 1]).to(dt)
                v = (startc[:, 2:] if t_ == 0 else velc[:, t_ - 1]).to(dt)
                r = O.filter_step(c, wd, meas, xp, pp, v, encc[:, t_].to(dt), _StepDraws(off[t_], nz[:, t_].to(dt)),
                                  force_resample=True)
                for k in keys + ("idx",):
                    acc[k].append(r[k])
        outs[dt] = {k: torch.stack(v, 1).double().numpy() for k, v in acc.items()}
    r32, r64 = outs[torch.float32], outs[torch.float64]
    np.testing.assert_array_equal(res.index.cpu().numpy(), r32["idx"].astype(np.int64))
    print(f"\nforced pass vs oracle step by step, B={B} N={N} T={T}:")
    for k, ours, rtol, atol in (("x", xs, 1e-5, 1e-4), ("p", ps, 1e-5, 1e-9), ("lik", res.lik.cpu(), 1e-5, 2e-5),
                                ("jac", res.jac.cpu(), 1e-5, 1e-6), ("prior", res.prior.cpu(), 1e-5, 1e-5)):
        _check_envelope(ours, r32[k], r64[k], rtol, atol, k)
        _fractions(k, ours, r32[k], r64[k], 1e-5, 0.0 if k != "jac" else 1e-6)


@pytest.mark.parametrize("N,true_state", [(1000, False), (1000, True), (900, False), (1024, True), (65, False),
                                          (1, False)])
def test_filter_init_equals_three_launches(N, true_state):
    """nfdpf_filter_init (one launch) == nfdpf_particle_init + nfdpf_normalize_log_probs +
    nfdpf_filter_tiled_init bit for bit: particles, log-weights, p0, 1 / sum p0^2 and the t = 0
    gate partials, on ragged N (a last tile of fewer waves) and both init modes."""
    from nfdpf import ops
    B = 5
    start = (torch.randn(B, 4) * 30).to(DEV)
    T = 7
    vel_in = (torch.randn(B, T + 2, 2) * 3).to(DEV)
    x, lw, p, ie, vel = ops.filter_init(start, B, N, 128.0, true_state, 11, 3, DEV,
                                        ess := torch.full((B, ops.tiled_tiles(N), 4), float("nan"), device=DEV,
                                                          dtype=torch.float64), vel_input=vel_in, T=T)
    x3, lw3 = ops.particle_init(start[:, :2], B, N, 128.0, true_state, 11, 3, DEV)
    p3, ie3 = ops.normalize_log_probs(lw3)
    ess3 = ops.tiled_init(p3, torch.empty_like(ess))
    torch.cuda.synchronize()
    vel3 = torch.cat([start[:, None, 2:4], vel_in[:, :T - 1]], 1).transpose(0, 1).contiguous()
    for a, b in ((x, x3), (lw, lw3), (p, p3), (ie, ie3), (ess, ess3), (vel, vel3)):
        assert torch.equal(a.cpu(), b.cpu())


@pytest.mark.parametrize("N", [8, 100, 257, 1000, 1024])
def test_cascade_row_sum_1k_equals_generic(N):
    """The forced pass's load-ahead cascade sum (cascade_row_sum_1k) == the generic device
    cascade sum == ATen's CPU order restated (oracle/cascade.py), bit for bit, on rows of mixed
    magnitudes (the resampler's q and gathered weights)."""
    from nfdpf import _lib
    from oracle.cascade import torch_cpu_row_sum
    g = torch.Generator().manual_seed(N)
    B = 33
    x = torch.rand(B, N, generator=g) * torch.exp(torch.randn(B, N, generator=g) * 3)
    x[0] = 1.0 / N
    xd = x.to(DEV).contiguous()
    out = [torch.empty(B, device=DEV) for _ in range(2)]
    for v in range(2):
        _lib.check(_lib.lib().nfdpf_cascade_row_sum(xd.data_ptr(), B, N, v, out[v].data_ptr(),
                                                    torch.cuda.current_stream().cuda_stream), "cascade_row_sum")
    torch.cuda.synchronize()
    ref = np.array([torch_cpu_row_sum(r) for r in x.numpy()], dtype=np.float32)
    np.testing.assert_array_equal(out[0].cpu().numpy(), ref)
    np.testing.assert_array_equal(out[1].cpu().numpy(), ref)
    assert torch.equal(x.sum(-1), torch.from_numpy(ref))  # the restatement is torch's own order here


@pytest.mark.parametrize("force", [False, True])
def test_pass_timeout_falls_back(force, monkeypatch):
    """A one-launch pass whose row hand-off waits time out (NFDPF_PASS_WAIT_US=1: a 1 us bound,
    standing in for a grid that is not all resident) drains, counts its faults, warns, turns the
    pass off for the engine and reruns the step launches: the returned result is the step
    launches' own, bit for bit, and the next run does not try the pass again."""
    models = _models("e2e_c2.npz")
    B, N, T = 4, 1000, 6
    enc, start, vel = _inputs(B, T, seed=5)
    from nfdpf.engine import FilterConfig, FilterEngine
    cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=9, kernel="tiled",
                       speculate_gate=None if force else True, force_resample=force)
    monkeypatch.setenv("NFDPF_PASS_WAIT_US", "1")
    eng = FilterEngine(cfg, models)
    with pytest.warns(RuntimeWarning, match="timed out"):
        a = eng.run(enc, start, vel)
    torch.cuda.synchronize()
    monkeypatch.delenv("NFDPF_PASS_WAIT_US")
    assert eng.pass_disabled and eng.pass_launches == 1 and not eng.last_pass
    eng.run(enc, start, vel)
    assert eng.pass_launches == 1, "the pass ran again after a fault"
    monkeypatch.setenv("NFDPF_PASS", "0")
    b = FilterEngine(cfg, models).run(enc, start, vel)
    torch.cuda.synchronize()
    for f in ("particles", "probs", "noise", "lik", "index", "jac", "prior", "pred"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    from nfdpf import _lib
    assert _lib.lib().nfdpf_split_fault(1, torch.cuda.current_stream().cuda_stream) == 0


@pytest.mark.parametrize("B,N,T", [(64, 1000, 50), (6, 777, 12), (3, 100, 8)])
def test_gated_pass_every_step_vs_oracle(B, N, T, monkeypatch):
    """The gated one-launch pass (the ESS gate decided INSIDE the launch at every step,
    DPFs.py:163-170) on the c2_full workload -- the C2 flags and size with frame encodings aligned
    with the true state, so the gate fires on a mix of steps -- against the oracle's step
    (oracle.filter_step, DPFs.py:160-192) started from the PASS's own slot t-1 with its device
    offsets and motion noise: every step's gate decision equals the reference's
    torch.mean(1 / sum p^2) < 0.5 N on the same weights, the indices are bit-exact, and the
    particles, weights, likelihood, jac and prior of every slot lie within the reference's own
    float32 envelope against the float64 oracle.  Both fired and quiet steps must occur."""
    import _fullsize as F
    from nfdpf import ops
    from nfdpf.engine import FilterConfig, FilterEngine
    wl = F.workload("c2_full", B=B, N=N, T=T)
    models = wl["models"].to(DEV)
    w = {k: v.detach().cpu() for k, v in models.state_dict().items()}
    c = F.cfg_dict(wl["flags"], N)
    enc, start, vel = wl["enc"].to(DEV), wl["start"].to(DEV), wl["vel"].to(DEV)
    x0, logw0 = ops.particle_init(start[:, :2], B, N, 128.0, False, 4242, 0, DEV)
    p0, _ = ops.normalize_log_probs(logw0)
    cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=4242, kernel="tiled",
                       speculate_gate=False)  # the gated pass from the first pass on
    eng = FilterEngine(cfg, models)
    res = eng.run(enc, start, vel, init=(x0, logw0))
    torch.cuda.synchronize()
    assert eng.last_pass and eng.last_gate_pass, "the gated one-launch pass did not run"
    gates = eng.last_gates.cpu()
    off = torch.from_numpy(_philox_offsets(4242, T, B, N))
    xs, ps, nz = res.particles.cpu(), res.probs.cpu(), res.noise.cpu()
    x0c, p0c, encc, startc, velc = x0.cpu(), p0.cpu(), enc.cpu(), start.cpu(), vel.cpu()
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    keys = ("x", "p", "lik", "jac", "prior", "idx", "lw_mean")
    outs, fired = {}, {}
    soft32 = O.soft_resample
    for dt in (torch.float32, torch.float64):
        if dt == torch.float64:
            monkeypatch.setattr(O, "soft_resample", _soft_indices32(soft32))
        acc = {k: [] for k in keys}
        fired[dt] = []
        with O.precision(dt):
            wd = O.cast_params(w, dt)
            meas = O.make_measurement(c, wd)
            for t_ in range(T):
                xp = (x0c if t_ == 0 else xs[:, t_ - 1]).to(dt)
                pp = (p0c if t_ == 0 else ps[:, t_ - 1]).to(dt)
                v = (startc[:, 2:] if t_ == 0 else velc[:, t_ - 1]).to(dt)
                # float64: the reference's own (float32) decision, as its indices
                r = O.filter_step(c, wd, meas, xp, pp, v, encc[:, t_].to(dt), _StepDraws(off[t_], nz[:, t_].to(dt)),
                                  force_resample=bool(gates[t_]) if dt == torch.float64 else False)
                fired[dt].append(bool(r["fired"]))
                for k in keys:
                    acc[k].append(r[k] if k != "lw_mean" else r[k].reshape(1))
        outs[dt] = {k: torch.stack(v, 1 if k != "lw_mean" else 0).double().numpy() for k, v in acc.items()}
    dec = [bool(g) for g in gates.tolist()]
    assert dec == fired[torch.float32], f"gate decisions differ from the reference's: {dec} vs {fired[torch.float32]}"
    n_fired = sum(dec)
    print(f"\ngated pass vs oracle step by step, B={B} N={N} T={T}: the gate fired in {n_fired} of {T} steps")
    assert 0 < n_fired < T, "the case should mix fired and quiet steps"
    r32, r64 = outs[torch.float32], outs[torch.float64]
    np.testing.assert_array_equal(res.index.cpu().numpy(), r32["idx"].astype(np.int64))
    for k, ours, rtol, atol in (("x", xs, 1e-5, 1e-4), ("p", ps, 1e-5, 1e-9), ("lik", res.lik.cpu(), 1e-5, 2e-5),
                                ("jac", res.jac.cpu(), 1e-5, 1e-6), ("prior", res.prior.cpu(), 1e-5, 1e-5)):
        _check_envelope(ours, r32[k], r64[k], rtol, atol, k)
        _fractions(k, ours, r32[k], r64[k], 1e-5, 0.0 if k != "jac" else 1e-6)
    obs32, obs64 = r32["lw_mean"].sum(), r64["lw_mean"].sum()
    assert abs(float(res.obs_likelihood) - obs64) <= 4 * abs(obs32 - obs64) + 1e-5 * abs(obs64) + 1e-4


def test_gated_pass_quiet_equals_speculative():
    """On a workload whose gate never fires (the bench's model at its init weights, N(0,1)
    encodings) the gated pass takes the speculative pass's path at every step: identical bits,
    obs-likelihood included, and no decision fired."""
    models = _models("bench")
    B, N, T = 16, 1000, 20
    enc, start, vel = _inputs(B, T, seed=77)
    eng_s, s_ = _run(models, N, enc, start, vel, spec=True)
    eng_g, g_ = _run(models, N, enc, start, vel, spec=False)  # (no speculation: the gated pass)
    assert eng_s.last_pass and not eng_s.last_gate_pass and eng_s.pass_launches == 1
    assert eng_g.last_pass and eng_g.last_gate_pass
    assert int(eng_g.last_gates.sum()) == 0
    for f in ("particles", "probs", "noise", "lik", "index", "jac", "prior", "pred", "obs_likelihood"):
        assert torch.equal(getattr(s_, f), getattr(g_, f)), f


def test_gated_pass_decisions_match_gate_kernel():
    """The in-launch decisions (from registers, after each step's row exchange) equal the batch
    gate kernel (nfdpf_ess_gate_tiled_batch) on the same pass's own per-step partials -- the two
    evaluate one arithmetic."""
    from nfdpf import ops
    import _fullsize as F
    B, N, T = 8, 1000, 16
    wl = F.workload("c2_full", B=B, N=N, T=T)
    models = wl["models"].to(DEV)
    from nfdpf.engine import FilterConfig, FilterEngine
    cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=99, kernel="tiled",
                       speculate_gate=False)
    eng = FilterEngine(cfg, models)
    captured = {}
    orig = ops.filter_init

    def keep(*a, **k):  # the engine's [T + 1, B, tiles, 4] partials: slot 0 is the initial one
        captured["base"] = a[8] if len(a) > 8 else k["ess_out"]
        return orig(*a, **k)
    ops.filter_init = keep
    try:
        eng.run(wl["enc"].to(DEV), wl["start"].to(DEV), wl["vel"].to(DEV))
    finally:
        ops.filter_init = orig
    torch.cuda.synchronize()
    assert eng.last_gate_pass
    tiles = ops.tiled_tiles(N)
    base = captured["base"]
    hist = torch.as_strided(base, (T, B, tiles, 4), base.stride() if base.dim() == 4 else
                            (B * tiles * 4, tiles * 4, 4, 1))
    ref = ops.ess_gate_tiled_batch(hist.contiguous(), N, 0, False)
    assert torch.equal(ref.cpu(), eng.last_gates.cpu()), (ref.tolist(), eng.last_gates.tolist())
    assert 0 < int(ref.sum()) < T


def test_auto_mode_switches_between_speculative_and_gated():
    """Auto mode on one GPU: a quiet workload keeps the speculative pass (verified, no gate fired);
    when a speculative pass misses, the rerun is the gated pass and the engine stays gated while
    gates keep firing; after two gated passes without a fired gate it speculates again."""
    import _fullsize as F
    from nfdpf.engine import FilterConfig, FilterEngine
    B, N, T = 8, 1000, 12
    wl = F.workload("c2_full", B=B, N=N, T=T)
    models = wl["models"].to(DEV)
    cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=5, kernel="tiled")
    eng = FilterEngine(cfg, models)
    fire = (wl["enc"].to(DEV), wl["start"].to(DEV), wl["vel"].to(DEV))
    g = torch.Generator().manual_seed(1)
    quiet = (torch.randn(B, T, 32, generator=g).to(DEV) * 0.0, wl["start"].to(DEV), wl["vel"].to(DEV))
    eng.run(*fire)
    assert eng.pass_launches == 2 and eng.last_gate_pass and int(eng.last_gates.sum()) > 0  # missed, rerun gated
    eng.run(*fire)
    assert eng.pass_launches == 3 and eng.last_gate_pass  # stays gated while gates fire
    for k in range(2):
        eng.run(*quiet)
        assert eng.last_gate_pass and int(eng.last_gates.sum()) == 0
    eng.run(*quiet)
    assert eng.last_pass and not eng.last_gate_pass, "two quiet gated passes: speculation again"


def _c2_full(B, N, T, **kw):
    import _fullsize as F
    from nfdpf.engine import FilterConfig, FilterEngine
    wl = F.workload("c2_full", B=B, N=N, T=T)
    models = wl["models"].to(DEV)
    cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=5, kernel="tiled", **kw)
    return FilterEngine(cfg, models), (wl["enc"].to(DEV), wl["start"].to(DEV), wl["vel"].to(DEV))


PLAN_FIELDS = ("particles", "probs", "noise", "lik", "index", "jac", "prior", "pred", "obs_likelihood")


@pytest.mark.parametrize("B,N,T", [(8, 1000, 16), (64, 1000, 50), (5, 777, 9)])
def test_plan_pass_equals_gated(B, N, T, monkeypatch):
    """The pass following a gate plan (d.pass_plan: no batch-wide exchange inside the launch) given
    the gated pass's own decisions == the gated pass, bit for bit (histories, decisions, obs); its
    epilogue verifies the plan against the pass's own partials: no rerun.  The gated pass's motion
    noise is the step launches' (Philox keyed on step, row, particle) at every step -- also at the
    steps whose speculated attempt it dropped and redid after the gate fired."""
    eng_g, inp = _c2_full(B, N, T, speculate_gate=False)
    g = eng_g.run(*inp)
    assert eng_g.last_gate_pass
    gates = eng_g.last_gates.cpu().numpy()
    monkeypatch.setenv("NFDPF_PASS", "0")
    eng_s, _ = _c2_full(B, N, T, speculate_gate=False)
    s = eng_s.run(*inp)
    monkeypatch.delenv("NFDPF_PASS")
    assert not eng_s.last_pass
    assert torch.equal(s.noise, g.noise), "the gated pass's motion noise differs from the step launches'"
    if T >= 16:
        assert 0 < gates.sum() < T, "the case should mix fired and quiet steps"
    eng_p, _ = _c2_full(B, N, T)
    p = eng_p.run(*inp, plan=gates)
    assert eng_p.last_plan_pass and eng_p.pass_launches == 1 and eng_p.last_verify == "ok" and eng_p.plan_misses == 0
    assert np.array_equal(eng_p.last_gates.cpu().numpy(), gates)
    for f in PLAN_FIELDS:
        assert torch.equal(getattr(p, f), getattr(g, f)), f


@pytest.mark.parametrize("flip", ["drop", "add"])
def test_plan_pass_wrong_plan_reruns(flip):
    """A plan that differs from the actual gates (a fired gate dropped, or a quiet step resampled):
    the verification catches it, the pass reruns exactly (the gated pass) and the engine's plan
    becomes that pass's gates; the result is the gated pass's, bit for bit."""
    B, N, T = 8, 1000, 16
    eng_g, inp = _c2_full(B, N, T, speculate_gate=False)
    g = eng_g.run(*inp)
    gates = eng_g.last_gates.cpu().numpy()
    wrong = gates.copy()
    k = int(np.flatnonzero(gates)[-1]) if flip == "drop" else int(np.flatnonzero(gates == 0)[-1])
    wrong[k] ^= 1
    eng, _ = _c2_full(B, N, T, pass_plan=True)
    r = eng.run(*inp, plan=wrong)
    assert eng.plan_misses == 1 and eng.pass_launches == 2 and eng.last_gate_pass and not eng.last_plan_pass
    assert np.array_equal(eng._plan, gates)
    for f in PLAN_FIELDS:
        assert torch.equal(getattr(r, f), getattr(g, f)), f


def test_auto_plan_mode_one_gpu():
    """cfg.pass_plan = True on one GPU: the first pass speculates and misses, the gated rerun's
    decisions become the plan, and the next passes follow it (verified, no rerun) -- the gated
    pass's result each time; a hipGraph-captured plan pass (run(finish=False), finish_pending
    after the replay) too."""
    B, N, T = 8, 1000, 16
    eng, inp = _c2_full(B, N, T, pass_plan=True)
    g = eng.run(*inp)
    assert eng.pass_launches == 2 and eng.last_gate_pass and eng._plan is not None and eng._plan.any()
    assert eng.plans()
    for _ in range(2):
        p = eng.run(*inp)
        assert eng.last_plan_pass and eng.last_verify == "ok" and eng.plan_misses == 0
        for f in PLAN_FIELDS:
            assert torch.equal(getattr(p, f), getattr(g, f)), f
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        cap = eng.run(*inp, finish=False)
    pend = eng.take_pending()
    assert eng.last_plan_pass
    for _ in range(2):
        eng.arm_flags(pend)
        graph.replay()
        assert eng.finish_pending(pend), eng.last_verify
        for f in PLAN_FIELDS:
            assert torch.equal(getattr(cap, f), getattr(g, f)), f


def test_plan_pass_rows_beyond_resident():
    """More rows than the device holds at once (the gated pass does not apply): auto mode's
    speculative pass misses, the exact rerun (step launches, the batch gate per step) records its
    gates as the plan, and the next pass follows it in resident chunks of rows -- verified (its
    gates are the step launches') and, row for row, bit-equal to a resident plan pass of the first
    rows given the same plan (rows depend on the batch only through the gates)."""
    from nfdpf import _lib as L
    N, T = 1000, 12
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    B = min(256, 2 * (cus // 4) + 8)  # (4 workgroups a row at N = 1000: more rows than CUs / 4)
    eng, inp = _c2_full(B, N, T)
    eng.run(*inp)
    assert eng.last_pass_ok and not eng._gate_resident, "the gated pass should not fit this many rows"
    assert eng._plan is not None and eng._plan.any(), "the exact rerun recorded no firing plan"
    plan = eng._plan.copy()
    p = eng.run(*inp)
    assert eng.last_plan_pass and eng.last_verify == "ok" and eng.plan_misses == 0
    assert np.array_equal(eng.last_gates.cpu().numpy(), plan)
    b = min(8, B)
    eng_s, _ = _c2_full(b, N, T)
    sub = eng_s.run(*(x[:b] for x in inp), plan=plan, finish=False)
    eng_s.take_pending()
    torch.cuda.synchronize()
    for f in PLAN_FIELDS[:-1]:
        assert torch.equal(getattr(sub, f), getattr(p, f)[:b]), f
    assert L.lib().nfdpf_split_fault(1, torch.cuda.current_stream().cuda_stream) == 0
