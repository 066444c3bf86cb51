"""The CPU oracle (oracle/dpf_oracle.py) against golden vectors produced by the reference.

These pin the oracle before it is trusted as the checker for the HIP path.
"""
import numpy as np
import pytest
import torch

from _util import assert_close, e2e_cfg, group, load, t, TapeRNG, weights
from oracle import dpf_oracle as O

FLOW_CASES = [f"D{D}_O{O_}_{tag}" for D, O_ in ((2, 4), (2, 36), (2, 196), (32, 32)) for tag in ("init", "wide")]


@pytest.mark.parametrize("case", FLOW_CASES)
def test_realnvp_cond(case):
    fx = group(load("flows.npz"), case)
    w = weights(fx)
    z, ld = O.realnvp_cond_forward(w, t(fx["x"]), t(fx["c"]))
    assert_close(z, fx["z"], 1e-6, 1e-6, "z")
    assert_close(ld, fx["ld_fwd"], 1e-6, 1e-6, "logdet fwd")
    xi, ldi = O.realnvp_cond_inverse(w, t(fx["x"]), t(fx["c"]))
    assert_close(xi, fx["xinv"], 1e-6, 1e-6, "x inv")
    assert_close(ldi, fx["ld_inv"], 1e-6, 1e-6, "logdet inv")


@pytest.mark.parametrize("case", ["cond_D2_O4", "cond_D2_O36", "cond_D32_O32"])
def test_cond_stack(case):
    fx = group(load("stacks.npz"), case)
    w = weights(fx)
    z, lp, ld = O.cond_stack_forward(w, 2, t(fx["x"]), t(fx["c"]), 0.0, float(fx["prior_std"]))
    assert_close(z, fx["z"], 1e-6, 1e-6, "z")
    assert_close(lp, fx["lp"], 1e-5, 1e-5, "prior log-prob")
    assert_close(ld, fx["ld_fwd"], 1e-6, 1e-6, "logdet")
    xi, ldi = O.cond_stack_inverse(w, 2, t(fx["x"]), t(fx["c"]))
    assert_close(xi, fx["xinv"], 1e-6, 1e-6, "x inv")
    assert_close(ldi, fx["ld_inv"], 1e-6, 1e-6, "logdet inv")


@pytest.mark.parametrize("D", [2, 4])
def test_maf_stack(D):
    fx = group(load("stacks.npz"), f"maf_D{D}")
    w = weights(fx)
    z, _, ld = O.stack_forward(w, 2, t(fx["x"]), "maf")
    assert_close(z, fx["z"], 1e-6, 1e-6, "z")
    assert_close(ld, fx["ld_fwd"], 1e-6, 1e-6, "logdet")
    xi, ldi = O.stack_inverse(w, 2, t(fx["x"]), "maf")
    assert_close(xi, fx["xinv"], 1e-6, 1e-6, "x inv")
    assert_close(ldi, fx["ld_inv"], 1e-6, 1e-6, "logdet inv")


def test_soft_resampler_bit_exact():
    fx = load("soft.npz")
    for i in range(int(fx["n_cases"])):
        c = group(fx, f"c{i}")
        xr, wr, idx = O.soft_resample(t(c["x"]), t(c["p"]), float(c["alpha"]), t(c["offsets"]))
        np.testing.assert_array_equal(idx.numpy(), c["idx"], err_msg=f"case {i}")
        np.testing.assert_array_equal(wr.numpy(), c["w"], err_msg=f"case {i}")


def test_ot_resampler():
    fx = load("ot.npz")
    for i in range(int(fx["n_cases"])):
        c = group(fx, f"c{i}")
        xr, wr, idx, info = O.ot_resample(t(c["x"]), t(c["p"]), return_info=True)
        assert info["iters"] == int(c["iters"])
        assert_close(xr, c["xr"], 1e-6, 1e-4, f"OT x' case {i}")
        assert_close(info["a_y"], c["a_y"], 1e-9, 1e-12, "a_y")
        np.testing.assert_array_equal(wr.numpy(), c["wr"])


@pytest.mark.parametrize("meas", ["cos", "CRNVP", "NN", "gaussian", "CGLOW"])
def test_measurements(meas):
    fx = group(load("meas.npz"), meas)
    w = weights(fx)
    enc, x = t(fx["enc"]), t(fx["x"])
    pe = O.sub(w, "particle_encoder")
    if meas == "cos":
        lik = O.meas_cos(pe, enc, x)
    elif meas == "CRNVP":
        lik = O.meas_crnvp(pe, O.sub(w, "cnf_measurement"), 2, enc, x)
    elif meas == "NN":
        lik = O.meas_nn(pe, O.sub(w, "likelihood_est"), enc, x)
    elif meas == "gaussian":
        lik = O.meas_gaussian(pe, enc, x)
    else:
        lik = O.meas_cglow(pe, O.sub(w, "cglow_measurement"), 1, enc, x)
    assert_close(lik, fx["lik"], 1e-5, 1e-5, meas)


@pytest.mark.parametrize("name", ["c1", "c2", "c2w", "c3", "c3n", "c4", "c5"])
def test_filtering_e2e(name):
    fx = load(f"e2e_{name}.npz")
    cfg = e2e_cfg(fx)
    w = weights(fx)
    init = (t(fx["init_x"]), t(fx["logw0"]))
    out = O.filtering(cfg, w, t(fx["enc"]), t(fx["start"]), t(fx["vel"]), rng=TapeRNG(fx), init=init)
    x, p, noise, lik, lw0, idx, jac, prior, obs = out
    np.testing.assert_array_equal(idx.numpy(), fx["idx"])
    assert_close(x, fx["x"], 1e-5, 1e-4, "particles")
    assert_close(p, fx["p"], 1e-5, 1e-9, "probs")
    assert_close(lik, fx["lik"], 1e-5, 1e-5, "lik")
    if jac is not None:
        assert_close(jac, fx["jac"], 1e-5, 1e-5, "jac")
        assert_close(prior, fx["prior"], 1e-5, 1e-5, "prior")
    assert abs(float(obs) - float(fx["obs_lik"])) <= 1e-5 * abs(float(fx["obs_lik"])) + 1e-4
    rm, _ = O.rmse(x, p, t(fx["state"]))
    assert abs(float(rm) - float(fx["rmse"])) <= 1e-5 * float(fx["rmse"])


@pytest.mark.parametrize("name", ["c1", "c2", "c2w", "c3", "c3n", "c4", "c5"])
def test_filter_step_teacher_forced(name):
    """Each step from the reference's own previous-step state: tight tolerances."""
    fx = load(f"e2e_{name}.npz")
    cfg = e2e_cfg(fx)
    w = weights(fx)
    meas = O.make_measurement(cfg, w)
    rng = TapeRNG(fx)
    T = int(fx["T"])
    x, p = t(fx["init_x"]), O.normalize_log_probs(t(fx["logw0"]))
    vel = t(fx["start"])[:, 2:]
    for s in range(T):
        r = O.filter_step(cfg, w, meas, x, p, vel, t(fx["enc"])[:, s], rng)
        assert r["fired"] == bool(fx["fired"][s])
        np.testing.assert_array_equal(r["idx"].numpy(), fx["idx"][:, s])
        assert_close(r["x"], fx["x"][:, s], 1e-5, 1e-4, f"particles step {s}")
        assert_close(r["p"], fx["p"][:, s], 1e-5, 1e-9, f"probs step {s}")
        assert_close(r["lik"], fx["lik"][:, s], 1e-5, 1e-5, f"lik step {s}")
        if cfg["NF_dyn"]:
            assert_close(r["jac"], fx["jac"][:, s], 1e-5, 1e-5, f"jac step {s}")
            assert_close(r["prior"], fx["prior"][:, s], 1e-5, 1e-5, f"prior step {s}")
        x, p = t(fx["x"][:, s]), t(fx["p"][:, s])
        vel = t(fx["vel"])[:, s]
