"""HIP filter vs the CPU oracle at the BASELINE sizes, host-RNG mode (the reference's own
CPU-generator draws replayed from a tape).  GPU box only.

Cases (tests/_fullsize.py): C2 at full size (B=64, N=1000, T=50; soft resampling fires in 17 of
the 50 steps), C3 at B=64, N=1000, T=10 (CRNVP + OT), a C4-shaped OT case (MAF dynamic flow,
N=4000, B=8, OT every step) and a C5-shaped case (CGLOW measurement, N=10000, B=8, soft resampling
every step: 40 tiles per row in the front launch, ~7 tiles per workgroup of the CGLOW kernel's
persistent grid).  test_cglow_measurement_fullsize runs the CGLOW kernel alone at 64 x 10000
particles (52 tiles per workgroup) and on a ragged size.

``NFDPF_PARITY_TABLE=<file>`` appends the printed 1e-5 fraction tables to that file
(profiles/r03_parity_fractions.txt is such a record).

* Teacher-forced: every step starts from the oracle's own state after the previous step, so
  each step is compared on identical inputs.  Exact: gate decisions, resampling indices,
  motion noise.  The north-star bar (BASELINE.json: "within 1e-5 rel on flow log-dets and
  particle weights") is measured elementwise as |ours - ref| <= 1e-5 |ref| + atol against the
  oracle's float32 run (the reference's arithmetic), atol 1e-6 for the log-dets (jac, prior)
  and 1e-9 for the weights (pure relative error is meaningless on near-zero
  log-dets); the fraction that meets it is printed and asserted, the elements that miss are
  listed.  C2 also runs the envelope check against the float64 oracle (test_gpu_parity.py).
* Free-running: the whole sequence from the same initial particles and draws.  Gate decisions
  must be identical at every step.  Indices are exact up to the first step where a marker
  lands within rounding of a CDF step (weights agree to ~1e-7 relative, markers are 1/N
  apart): from there on the row follows other particles and the trajectories legitimately
  part, so the test reports the agreeing fraction and the first divergence and asserts the
  prediction / RMSE stay within the filter's own noise.
"""
import os

import numpy as np
import pytest
import torch

import _fullsize as F
from oracle import dpf_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
_CACHE = {}


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from nfdpf import _lib
    _lib.load()
    assert torch.cuda.is_available()
    torch.set_num_threads(16)


def _case(name):
    if name not in _CACHE:
        w = F.build(name)
        print(f"\n{name}: oracle {w['oracle_s']:.1f} s, gate fired at steps "
              f"{[i for i, f in enumerate(w['fired']) if f]}")
        _CACHE[name] = w
    return _CACHE[name]


def _engine(w):
    from nfdpf.engine import FilterConfig, FilterEngine
    c, fl = w["cfg"], w["flags"]
    cfg = FilterConfig(N=c["N"], NF_dyn=c["NF_dyn"], NF_cond=c["NF_cond"], measurement=c["measurement"],
                       resampler=c["resampler"], rng_mode="host", kernel="tiled", dyn_flow=c["dyn_flow"],
                       force_resample=w["force"])
    return FilterEngine(cfg, w["models"].to(DEV))


def _run(w, teacher):
    eng = _engine(w)
    ref = w["ref"]
    kw = dict(host=F.Tape(w["rec"]), init=w["init"])
    if teacher:
        kw["teacher"] = {"x": ref[0], "p": ref[1]}
    return eng.run(w["enc"].to(DEV), w["start"].to(DEV), w["vel"].to(DEV), **kw)


def _table(line):
    """Print a line of the parity record and append it to $NFDPF_PARITY_TABLE when set."""
    print(line)
    path = os.environ.get("NFDPF_PARITY_TABLE")
    if path:
        with open(path, "a") as f:
            f.write(line.rstrip("\n").lstrip("\n") + "\n")


def _report(what, ours, ref, rtol, atol):
    frac, worst = F.frac_within(ours, ref, rtol, atol)
    _table(f"  {what:10s} within {rtol:g} rel + {atol:g}: {100 * frac:.4f} %   worst {worst[0]}")
    return frac


def _oracle64_teacher(w):
    """Step t of the oracle in float64 from the float32 oracle's step t-1 state (resampling
    indices from the float32 run): |ref64 - ref32| is the reference's own rounding envelope."""
    ref = w["ref"]
    cfg, T = w["cfg"], w["T"]
    idx32 = ref[5]
    out = {k: [] for k in ("x", "p", "lik", "jac", "prior")}
    soft32 = O.soft_resample
    t_box = [0]

    def soft64(x, p, alpha, offsets=None, gen=None):
        B, N = p.shape
        idx = idx32[:, t_box[0]]
        q = alpha * p + (1 - alpha) / N
        q = q / q.sum(-1, keepdim=True)
        wv = (p / q).reshape(B * N)[idx]
        return x.reshape(B * N, -1)[idx], wv / wv.sum(-1, keepdim=True), idx

    ot64 = O.ot_resample

    def ot_recorded(x, p, *a, **k):
        # the oracle's Sinkhorn of this step from the float32 run (the same input values; FP64
        # throughout, x' = T x in fp64): not re-solved (~10 s per call at B=64)
        c = w["ot_calls"].get(t_box[0])
        if c is None:
            return ot64(x, p, *a, **k)
        B, N = p.shape
        idx = (torch.arange(N) + N * torch.arange(B)[:, None]).long()
        return c["xr64"].clone(), torch.ones_like(p) / N, idx

    O.soft_resample, O.ot_resample = soft64, ot_recorded
    tape = F.Tape(w["rec"])
    try:
        with O.precision(torch.float64), torch.no_grad():
            params = O.cast_params(w["params"], torch.float64)
            meas = O.make_measurement(cfg, params)
            x, p = w["init"][0].double(), O.normalize_log_probs(w["init"][1].double())
            vel = w["start"].double()[:, 2:]
            for s in range(T):
                t_box[0] = s
                r = O.filter_step(cfg, params, meas, x, p, vel, w["enc"].double()[:, s], tape, w["force"])
                for k in out:
                    out[k].append(r[k])
                x, p = ref[0][:, s].double(), ref[1][:, s].double()
                vel = w["vel"].double()[:, s]
    finally:
        O.soft_resample, O.ot_resample = soft32, ot64
    return {k: torch.stack(v, 1).numpy() for k, v in out.items()}


# (quantity, history index in the 9-tuple, key of the float64 run, atol)
QUANTITIES = (("weights", 1, "p", 1e-9), ("particles", 0, "x", 1e-4), ("likelihood", 3, "lik", 2e-5),
              ("jac", 6, "jac", 1e-6), ("prior", 7, "prior", 1e-5))


def _r64(name, w):
    if "r64" not in w:
        w["r64"] = _oracle64_teacher(w)
    return w["r64"]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", list(F.CASES))
def test_fullsize_teacher_forced(name):
    from test_gpu_parity import _check_envelope
    w = _case(name)
    ref = w["ref"]
    res = _run(w, teacher=True)
    torch.cuda.synchronize()
    assert res.fired == w["fired"]
    np.testing.assert_array_equal(res.index.cpu().numpy(), ref[5].numpy())
    np.testing.assert_array_equal(res.noise.cpu().numpy(), ref[2].numpy())
    ot = w["cfg"]["resampler"] == "ot"
    r64 = _r64(name, w)
    _table(f"\n{name} teacher-forced (B={w['B']}, N={w['N']}, T={w['T']}, measurement {w['cfg']['measurement']}, "
           f"{w['cfg']['resampler']}, gate fired in {sum(w['fired'])}/{w['T']} steps): elements within 1e-5 rel + atol")
    ours_all = {"weights": res.probs, "particles": res.particles, "likelihood": res.lik, "jac": res.jac,
                "prior": res.prior}
    cglow = w["cfg"]["measurement"] == "CGLOW"
    if cglow:
        # The CGLOW likelihood is steep in the particle position (|d lik / d x| up to ~2e3 at
        # C5, scripts/archive/diag_c5.py), so a particle's own fp32 rounding (checked under "particles")
        # moves it by ~1e-2 in any float32 evaluation.  The measurement is therefore asserted on
        # IDENTICAL particles: our CGLOW kernel on the reference's own teacher-forced proposals
        # against the float64 measurement there, next to the reference's float32 likelihood
        # (the same positions); the whole step's own-particle comparison is printed below.
        lik64_ours = _cglow_lik64_at(w, res.particles.cpu())
        lik64_ref = _cglow_lik64_at(w, ref[0])
        k_lik = _cglow_kernel_lik_at(w, ref[0])
        e_k, e_r = np.abs(k_lik - lik64_ref), np.abs(ref[3].numpy() - lik64_ref)
        _table(f"  likelihood, kernel alone on the reference's particles vs float64: max err {e_k.max():.3e} "
               f"(reference float32 {e_r.max():.3e}, ratio {e_k.max() / max(e_r.max(), 1e-30):.2f}), mean "
               f"{e_k.mean():.3e} (reference {e_r.mean():.3e})")
        # The kernel alone, on the reference's own particles: mean <= 2.5x and the 99.9th
        # percentile <= 4x the reference float32's, and every element within 4x the reference's
        # case maximum PLUS its own float32 floor: 4 sigma_i, sigma_i = the likelihood's
        # first-order response to rounding the 12x12 1x1-conv matrix W_i to float32 (iid errors
        # of half an ulp of max|W_i|: sigma = hw / (ln2 dims) 2^-24 max|W_i| ||W_i^-1||_F).  The
        # round-4 outlier (b 6, step 2, n 8339; 4.6-6x the reference's max) is such an element:
        # W has cond 5.9e6, our W is within 1.2 ulp of the float64 W (rms error 9.2e-9, the
        # reference float32's 8.5e-9) and our LU's log|det| within 7e-3 of float64 slogdet of OUR
        # W, yet log|det W| moves 0.18 -- random W errors of that rms move it 0.044 median, 0.155
        # at p99 (scripts/archive/r05_cglow_w.py).  No layer is worse than the
        # reference's float32; the element is the tail of the conditioning amplification.
        qk, qr = np.quantile(e_k, 0.999), np.quantile(e_r, 0.999)
        sig = _cglow_w_sigma(w, ref[0])
        bar = 4 * e_r.max() + 2e-5 + 4 * sig
        n_floor = int((4 * sig > 4 * e_r.max() + 2e-5).sum())
        worst = np.unravel_index(np.argmax(e_k - bar), e_k.shape)
        _table(f"  likelihood, kernel alone: 99.9th percentile err {qk:.3e} (reference {qr:.3e}, ratio "
               f"{qk / max(qr, 1e-30):.2f}); max ratio {e_k.max() / max(e_r.max(), 1e-30):.2f}; elements whose "
               f"float32 W floor exceeds 4x the reference max: {n_floor}; tightest element {tuple(map(int, worst))} "
               f"err {e_k[worst]:.3e} bar {bar[worst]:.3e} (sigma {sig[worst]:.3e})")
        ill = sig > 1e-4  # the ill-conditioned W: error in units of the element's float32 floor
        if ill.any():
            _table(f"  likelihood at the {int(ill.sum())} elements with sigma > 1e-4: max err / sigma ours "
                   f"{(e_k[ill] / sig[ill]).max():.2f}, reference float32 {(e_r[ill] / sig[ill]).max():.2f}")
        assert qk <= 4 * qr + 2e-5, (qk, qr)
        assert e_k.mean() <= 2.5 * e_r.mean() + 2e-5, (e_k.mean(), e_r.mean())
        assert (e_k <= bar).all(), (tuple(map(int, worst)), e_k[worst], bar[worst], sig[worst], e_r.max())
    fails = []
    for what, i, k, atol in QUANTITIES:
        if ref[i] is None:
            continue
        o = ours_all[what].cpu()
        if cglow and what == "likelihood":
            f_ours, worst = F.frac_within(o, lik64_ours, 1e-5, atol)
            f_ref, _ = F.frac_within(ref[i], lik64_ref, 1e-5, atol)
            e_o, e_r = np.abs(o.numpy() - lik64_ours), np.abs(ref[i].numpy() - lik64_ref)
            _table(f"  {what:10s} (atol {atol:g}) vs float64 at each run's own particles: ours {100 * f_ours:8.4f} %, "
                   f"reference float32 {100 * f_ref:8.4f} %; max err ours {e_o.max():.3e} ref {e_r.max():.3e}, "
                   f"mean ours {e_o.mean():.3e} ref {e_r.mean():.3e}")
            if f_ours < f_ref - 2e-3:
                fails.append((what, f_ours, f_ref, worst))
            # at each run's own particles the case maximum is one element where the likelihood
            # is steepest, a draw of ~ulp x slope for ours and the reference alike (measured 4.6x
            # in round 3): a diagnostic only -- the kernel is asserted on identical particles above
            _table(f"  likelihood at own particles: max ratio {e_o.max() / max(e_r.max(), 1e-30):.2f}, "
                   f"mean ratio {e_o.mean() / max(e_r.mean(), 1e-30):.2f} (diagnostic)")
            assert e_o.mean() <= 2.5 * e_r.mean() + atol, (e_o.mean(), e_r.mean())
            continue
        f32, _ = F.frac_within(o, ref[i], 1e-5, atol)
        f_ours, worst = F.frac_within(o, r64[k], 1e-5, atol)
        f_ref, _ = F.frac_within(ref[i], r64[k], 1e-5, atol)
        _table(f"  {what:10s} (atol {atol:g}): ours vs float32 oracle {100 * f32:8.4f} %  |  vs float64: ours "
               f"{100 * f_ours:8.4f} %, reference float32 {100 * f_ref:8.4f} %   worst {worst[0]}")
        # the north-star bar (1e-5 rel on log-dets and weights) met on at least as many
        # elements as the reference's own float32 run meets it ...
        if f_ours < f_ref - 2e-3:
            fails.append((what, f_ours, f_ref, worst))
        # ... and inside the reference's own rounding envelope: case max / mean, and (without
        # OT) every element against its row's.  With OT the Sinkhorn's pair work runs in fp32
        # against the reference's fp64 loop (x' within ~2e-5 relative, test_fullsize_ot_direct),
        # an error the reference's float32 run does not have, so rows where the reference's
        # own error happens to be tiny carry no per-row bound there.
        if ot and what == "particles":
            # x' of an OT step carries the fp32 pair work of our Sinkhorn (the reference
            # iterates in fp64): bounded, as in test_fullsize_ot_direct, relative to the scale
            # of the row's cloud rather than by the reference's float32 envelope
            o64, r = o.numpy().astype(np.float64), r64[k]
            scale = np.maximum(np.abs(r).max(axis=(2, 3), keepdims=True), 1.0)
            rel = (np.abs(o64 - r) / scale).max()
            _table(f"  particles: max error / row scale {rel:.2e} (bound 5e-5)")
            assert rel <= 5e-5, rel
            continue
        _check_envelope(o, ref[i], r64[k], 1e-5, atol, what, k_row=np.inf if ot else 16.0)
    dump = os.environ.get("NFDPF_PARITY_DUMP")
    if dump:  # diagnostics: per-(row, step) miss counts and the rows where ours misses most
        out = {}
        for what, i, k, atol in QUANTITIES:
            if ref[i] is None:
                continue
            o = ours_all[what].cpu().numpy().astype(np.float64)
            rr = ref[i].numpy().astype(np.float64)
            miss_o = np.abs(o - r64[k]) > 1e-5 * np.abs(r64[k]) + atol
            miss_r = np.abs(rr - r64[k]) > 1e-5 * np.abs(r64[k]) + atol
            ax = tuple(range(2, o.ndim))
            out[f"miss_ours_{what}"], out[f"miss_ref_{what}"] = miss_o.sum(ax), miss_r.sum(ax)
        d = out["miss_ours_weights"] - out["miss_ref_weights"]
        sel = np.argsort(d.ravel())[-4:]
        bt = np.stack(np.unravel_index(sel, d.shape), -1)
        out["sel"] = bt
        for what, i, k, atol in QUANTITIES:
            if ref[i] is None:
                continue
            o = ours_all[what].cpu().numpy()
            out[f"ours_{what}"] = np.stack([o[b, t] for b, t in bt])
            out[f"ref_{what}"] = np.stack([ref[i].numpy()[b, t] for b, t in bt])
            out[f"r64_{what}"] = np.stack([r64[k][b, t] for b, t in bt])
        np.savez_compressed(os.path.join(dump, f"{name}_teacher.npz"), **out)
    assert not fails, fails


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["c3_full", "c4_n4000"])
def test_fullsize_ot_direct(name):
    """The Sinkhorn resampler alone on every OT step's own input (the oracle's state after the
    previous step), at B=64 x N=1000 (C3) and B=8 x N=4000 (C4 shape: the batch-coupled stop
    rule over 8 rows): the iteration count of the reference's stop rule exactly, x' against the
    oracle's FP64 loop (its transport matrix applied in fp64, recorded when the case was built)."""
    from nfdpf import ops
    w = _case(name)
    assert w["ot_calls"], "no OT step in the case"
    for t, c in sorted(w["ot_calls"].items()):
        x, p = c["x"].float().contiguous(), c["w"].float().contiguous()
        xo, wo, idx, it = ops.ot_resample(x.to(DEV), p.to(DEV))
        xr = c["xr64"]
        e = (xo.cpu().double() - xr).abs()
        rel = float((e / xr.abs().clamp_min(1.0)).max())
        _table(f"{name} OT step {t} (B={x.shape[0]}, N={x.shape[1]}): iterations {int(it.item())} (reference "
               f"{c['iters']}), max |x'| {float(xr.abs().max()):.1f}, max abs err {float(e.max()):.2e}, rel {rel:.2e}")
        assert int(it.item()) == c["iters"]
        assert rel <= 5e-5
        assert torch.all(wo.cpu() == 1.0 / w["N"])
        ident = torch.arange(x.shape[1]) + x.shape[1] * torch.arange(x.shape[0])[:, None]
        assert torch.equal(idx.cpu(), ident)


@pytest.mark.timeout(120)
def test_ot_stop_at_c4_share():
    """One Sinkhorn call at a C4 rank's share, 32 rows x N = 4000 (BASELINE configs[3]: B = 256
    over 8 GPUs): the reference's stop rule ends the loop when ANY row of the batch has converged
    (resamplers.py:126-129), so it is pinned at the batch the ranks actually run -- iteration
    count exact, x' against the oracle's FP64 transport (tests/golden/ot_c4_share.npz, written by
    tests/golden/gen_ot_share.py; the input is regenerated from its seed)."""
    import sys
    from nfdpf import ops
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from gen_ot_share import ot_share_input
    fx = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ot_c4_share.npz"))
    x, w = ot_share_input(int(fx["seed"]))
    xo, wo, idx, it = ops.ot_resample(torch.from_numpy(x).to(DEV), torch.from_numpy(w).to(DEV))
    xr = torch.from_numpy(fx["xr"]).double()
    e = (xo.cpu().double() - xr).abs()
    rel = float((e / xr.abs().clamp_min(1.0)).max())
    _table(f"C4 share OT (B={x.shape[0]}, N={x.shape[1]}): iterations {int(it.item())} (oracle {int(fx['iters'])}), "
           f"max |x'| {float(xr.abs().max()):.1f}, max abs err {float(e.max()):.2e}, rel {rel:.2e}")
    assert int(it.item()) == int(fx["iters"])
    assert rel <= 5e-5
    assert torch.all(wo.cpu() == 1.0 / x.shape[1])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", list(F.CASES))
def test_fullsize_free_running(name):
    w = _case(name)
    ref = w["ref"]
    res = _run(w, teacher=False)
    torch.cuda.synchronize()
    assert res.fired == w["fired"], [i for i, (a, b) in enumerate(zip(res.fired, w["fired"])) if a != b]
    idx, idr = res.index.cpu(), ref[5]
    same = (idx == idr)
    per_step = same.float().mean(dim=(0, 2))
    bad = [t for t in range(w["T"]) if per_step[t] < 1.0]
    first = bad[0] if bad else None
    rows_exact = int(same.all(-1).all(-1).sum())
    _table(f"\n{name} free-running: indices equal {100 * float(same.float().mean()):.4f} %, "
           f"rows exact over the whole pass {rows_exact}/{w['B']}, first step with a differing index {first}")
    # every step before the first divergence is identical in its indices
    if first is not None:
        assert first >= 1
    rm, pred = O.rmse(res.particles.cpu(), res.probs.cpu(), w["state"])
    rr, predr = O.rmse(ref[0], ref[1], w["state"])
    _table(f"  RMSE ours {float(rm):.4f} oracle {float(rr):.4f}")
    assert abs(float(rm) - float(rr)) <= 0.03 * float(rr) + 0.05
    if first is None:
        _report("weights", res.probs.cpu(), ref[1], 1e-5, 1e-9)


def _cglow_lik64_at(w, x):
    """The float64 CGLOW likelihood (row-max shifted, model/models.py:280-303) of a case's
    frame encodings at the particles x (B, T, N, 2), step by step."""
    out = [_cglow_oracle(w["params"], w["enc"][:, t], x[:, t].float(), torch.float64) for t in range(x.shape[1])]
    return np.stack(out, 1)


def _cglow_w_sigma(w, x, rows=8):
    """Per element (B, T, N): the std of the likelihood's first-order response to rounding the
    1x1-conv matrix W (O.cglow_step's invconv, float64) to float32 with iid errors of half an ulp
    of max|W|: d lik / d log|det W| = hw / (ln2 dims) and d log|det W| = tr(W^-1 dW), whose std
    for iid dW of std s is s ||W^-1||_F.  One flow step (K = 1, as the cases)."""
    p = O.cast_params(w["params"], torch.float64)
    pe = O.sub(p, "particle_encoder")
    inv = O.sub(O.sub(O.sub(p, "cglow_measurement"), "flow.layers.1"), "invconv")
    assert not any(k.startswith("cglow_measurement.flow.layers.2.") for k in p)
    hw, dims = 16.0, 192.0
    out = []
    with O.precision(torch.float64), torch.no_grad():
        for t in range(x.shape[1]):
            per = []
            for b in range(0, x.shape[0], rows):
                xb = x[b:b + rows, t].double()
                Bc, N = xb.shape[:2]
                es = O.particle_encode(pe, xb.reshape(-1, 2)).reshape(Bc * N, 3, 8, 8)
                W = O._cond_net(inv, es, Bc * N).reshape(-1, 12, 12)
                s = torch.linalg.inv(W).pow(2).sum((1, 2)).sqrt() * W.abs().amax((1, 2)) * 2.0 ** -24
                per.append((s * hw / (np.log(2.0) * dims)).reshape(Bc, N))
            out.append(torch.cat(per).numpy())
    return np.stack(out, 1)


def _cglow_kernel_lik_at(w, x):
    """Our CGLOW kernel (nfdpf_cglow_measurement, the row-max shift of model/models.py:301-302
    applied after it, as the filter's phase 2) on the particles x (B, T, N, 2), step by step."""
    from nfdpf import ops
    from nfdpf.pack import cglow_tensors, encoder_tensors
    m = w["models"]
    pe = torch.cat([a.detach().reshape(-1) for a in encoder_tensors(m.particle_encoder)]).float().to(DEV)
    glow = torch.cat([a.detach().reshape(-1) for a in cglow_tensors(m.cglow_measurement)]).float().to(DEV)
    out = []
    for t in range(x.shape[1]):
        raw = ops.cglow_measurement(pe, glow, w["enc"][:, t].float().contiguous().to(DEV),
                                    x[:, t].float().contiguous().to(DEV))
        out.append((raw - raw.max(dim=-1, keepdim=True)[0]).cpu().numpy().astype(np.float64))
    return np.stack(out, 1)


def _cglow_oracle(w, enc, x, dt, rows=8):
    """O.meas_cglow in ``dt`` over row chunks (the row-max shift is per row: chunking is exact)."""
    with O.precision(dt), torch.no_grad():
        p = O.cast_params(w, dt)
        pe, gl = O.sub(p, "particle_encoder"), O.sub(p, "cglow_measurement")
        out = [O.meas_cglow(pe, gl, 1, enc[b:b + rows].to(dt), x[b:b + rows].to(dt))
               for b in range(0, x.shape[0], rows)]
    return torch.cat(out).numpy().astype(np.float64)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("B,N", [(64, 10000), (3, 9999)])
def test_cglow_measurement_fullsize(B, N):
    """measurement_model_cglow (model/models.py:280-303, nf/cglow/CGlowModel.py:123-176) at the
    C5 per-GPU size, 64 rows x N=10000 = 640 000 particles: the kernel's persistent grid
    (csrc/cglow.hip, 3 workgroups per CU x 16 particles) runs ~52 tiles per workgroup, so the
    cross-tile state (per-launch constants, LDS reuse under wave fences, the y prefetch) is
    exercised; (3, 9999) is ragged (29 997 particles, a partial last tile of 13).  Weights: the
    reference's CGLOW fixture (tests/golden/meas.npz).  Bar: the golden test's envelope against
    the oracle in float64 -- max error <= 4x and mean <= 2.5x the oracle's own float32 error
    (the reference's arithmetic) -- and the fraction within 1e-5 rel + 5e-5 of float64 at least
    the reference float32 evaluation's."""
    from nfdpf import ops
    from nfdpf.pack import cglow_tensors
    from _util import group, load, weights
    from test_gpu_parity import _enc_blob, _glow_module
    fx = group(load("meas.npz"), "CGLOW")
    w = weights(fx)
    pe = _enc_blob(w)
    glow = torch.cat([a.detach().reshape(-1) for a in cglow_tensors(_glow_module(w))]).to(DEV)
    g = torch.Generator().manual_seed(55)
    enc = torch.randn(B, 192, generator=g)
    x = torch.rand(B, N, 2, generator=g) * 128.0 - 64.0
    raw = ops.cglow_measurement(pe, glow, enc.to(DEV), x.to(DEV))
    lik = (raw - raw.max(dim=-1, keepdim=True)[0]).cpu().numpy().astype(np.float64)
    assert np.isfinite(lik).all()
    ref32 = _cglow_oracle(w, enc, x, torch.float32)
    ref64 = _cglow_oracle(w, enc, x, torch.float64)
    e_ours, e_ref = np.abs(lik - ref64), np.abs(ref32 - ref64)
    f_ours, _ = F.frac_within(lik, ref64, 1e-5, 5e-5)
    f_ref, _ = F.frac_within(ref32, ref64, 1e-5, 5e-5)
    _table(f"\nCGLOW measurement B={B} N={N} ({B * N} particles): max |ours - f64| {e_ours.max():.3e} mean "
           f"{e_ours.mean():.3e}; reference f32 max {e_ref.max():.3e} mean {e_ref.mean():.3e}; within 1e-5 rel + "
           f"5e-5 of f64: ours {100 * f_ours:.4f} %, reference f32 {100 * f_ref:.4f} %")
    assert e_ours.max() <= 4 * e_ref.max() + 1e-5
    assert e_ours.mean() <= 2.5 * e_ref.mean() + 1e-6
    # the likelihood is steep in x for some particles (|d lik / d x| ~ 2e3 measured, scripts/
    # diag_c5.py): there the float32 rounding of the particle encoding alone moves it by ~1e-2,
    # in the reference's own float32 run as much as in ours (max 9.7e-2 vs f64 at 64 x 10000), so
    # no elementwise bar holds for either; the north-star bar is met on at least as many
    # elements as the reference's own float32 evaluation meets it
    assert f_ours >= f_ref - 2e-4, (f_ours, f_ref)
