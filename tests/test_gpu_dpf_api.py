"""The drop-in boundary exercised through the public class: DPF(args) with --rng-mode host
(the reference's CPU-generator draws) against outputs of the reference's own DPF.  GPU box only.

* ``DPF.filtering_pos`` (DPFs.py:144-216) on the e2e fixtures (frame encoder = identity on the
  fixture's encodings, global generator seeded as the fixture generator seeded it);
* ``DPF.forward(inputs, train=False)`` (DPFs.py:96-142) -- 128x128 frames, the 13-tuple with
  the supervised / auto-encoder / pseudo-likelihood losses -- and ``DPF.testing`` (:419-451),
  on the fwd_* fixtures (frame encoder / decoder swapped for tests/_tiny.py on both sides);
* a batch shard with row_base > 0 returns indices flat into its own B * N, as the reference
  and the pseudo-likelihood losses expect;
* ``particle_initialization`` in device-RNG mode (nfdpf_particle_init, utils.py:46-62).

Tolerances as test_gpu_parity.test_filtering_free_running: indices and noise exact, particles
1e-4 rel + 1e-3, weights 1e-4 rel + 1e-7 (whole-sequence runs: rounding compounds over steps).
"""
import os

import numpy as np
import pytest
import torch

from _util import assert_close, load, t, weights

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from nfdpf import _lib
    _lib.load()
    assert torch.cuda.is_available()


def _flag(fx, k, default=None):
    key = f"flag/{k}"
    return fx[key].item() if key in fx else default


def _dpf(fx, extra=None):
    from arguments import parse_args
    from DPFs import DPF
    a = parse_args([])
    a.num_particles, a.batchsize, a.sequence_length = int(fx["N"]), int(fx["B"]), int(fx["T"])
    for k in ("NF_dyn", "NF_cond", "measurement", "resampler_type", "hiddensize", "trainType", "block_length",
              "NF_dyn_flow"):
        v = _flag(fx, k)
        if v is not None:
            setattr(a, k, v)
    a.rng_mode = "host"
    for k, v in (extra or {}).items():
        setattr(a, k, v)
    torch.manual_seed(0)
    return DPF(a)


def _load(dpf, fx):
    sd = dpf.state_dict()
    w = weights(fx)
    missing = [k for k in w if k not in sd]
    assert not missing, missing[:5]
    sd.update(w)
    dpf.load_state_dict(sd)


# whole sequences (c2w, the 0.3-std flows, is a teacher-forced case only: its wide flows
# amplify rounding past a whole-run tolerance, as in test_gpu_parity.test_filtering_free_running)
E2E = ["c1", "c2", "c3", "c4", "c5"]


@pytest.mark.parametrize("name", E2E)
def test_dpf_filtering_pos_host_rng(name):
    """DPF(args).filtering_pos with --rng-mode host draws the reference's own CPU-generator
    sequence (init, per-step offsets and noise) and returns the reference's 9-tuple."""
    fx = load(f"e2e_{name}.npz")
    extra = {"hiddensize": 192} if _flag(fx, "measurement") == "CGLOW" else {}
    dpf = _dpf(fx, extra)
    dpf.encoder = torch.nn.Identity()
    _load(dpf, fx)
    dpf.to(DEV).eval()
    torch.manual_seed(600)  # the fixture generator's seed right before filtering_pos
    with torch.no_grad():
        out = dpf.filtering_pos(t(fx["enc"]).to(DEV), t(fx["start"]).to(DEV), t(fx["vel"]).to(DEV))
    xl, pl, nl, ll, lw0, il, jl, prl, obs = out
    np.testing.assert_array_equal(nl.cpu().numpy(), fx["noise"])
    np.testing.assert_array_equal(il.cpu().numpy(), fx["idx"].astype(np.int64))
    # log(1/N) (utils.py:60): the device log may differ from the CPU's by an ulp
    np.testing.assert_allclose(lw0.cpu().numpy(), fx["logw0"], rtol=2.5e-7, atol=0)
    assert_close(xl.cpu(), fx["x"], 1e-4, 1e-3, "particles")
    assert_close(pl.cpu(), fx["p"], 1e-4, 1e-7, "weights")
    assert_close(ll.cpu(), fx["lik"], 1e-4, 1e-3, "likelihood")
    if "jac" in fx:
        assert_close(jl.cpu(), fx["jac"], 1e-4, 1e-5, "jac")
        assert_close(prl.cpu(), fx["prior"], 1e-4, 1e-3, "prior")
    else:
        assert jl is None and prl is None
    assert abs(float(obs) - float(fx["obs_lik"])) <= 1e-4 * abs(float(fx["obs_lik"])) + 1e-3


def _fwd_setup(name):
    from _tiny import TinyDecoder, TinyEncoder
    fx = load(f"{name}.npz")
    dpf = _dpf(fx)
    H = int(fx["H"])
    dpf.encoder, dpf.decoder = TinyEncoder(H), TinyDecoder(H)
    _load(dpf, fx)
    dpf.to(DEV).eval()
    up = lambda a: t(a).float().div(255).repeat_interleave(8, -3).repeat_interleave(8, -2)  # noqa: E731
    B, T = int(fx["B"]), int(fx["T"])
    inputs = (up(fx["start_img"]), t(fx["start"]), up(fx["img"]), t(fx["state"]), torch.zeros(B, T),
              torch.ones(B, T))
    return fx, dpf, inputs


FWD = ["fwd_c2_sdpf", "fwd_c1_sdpf", "fwd_c3"]


@pytest.mark.parametrize("name", FWD)
def test_dpf_forward_eval(name):
    """DPF.forward(inputs, train=False): the reference's 13-tuple (losses, predictions,
    histories) from the same frames, weights and generator state."""
    fx, dpf, inputs = _fwd_setup(name)
    torch.manual_seed(int(fx["seed"]))
    with torch.no_grad():
        out = dpf.forward(inputs, train=False)
    (total, sup, pseud, ae, pred, pl, pwl, st, ss, image, ll, nl, obs) = out
    np.testing.assert_array_equal(nl.cpu().numpy(), fx["noise"])
    assert_close(pl.cpu(), fx["x"], 1e-4, 1e-3, "particles")
    assert_close(pwl.cpu(), fx["p"], 1e-4, 1e-7, "weights")
    assert_close(ll.cpu(), fx["lik"], 1e-4, 1e-3, "likelihood")
    assert_close(pred.cpu(), fx["pred"], 1e-4, 1e-3, "predictions")
    for v, k in ((sup, "sup"), (ae, "ae"), (total, "total"), (obs, "obs_lik")):
        assert abs(float(v) - float(fx[k])) <= 1e-4 * abs(float(fx[k])) + 1e-4, (k, float(v), float(fx[k]))
    if "pseud" in fx:
        assert abs(float(pseud) - float(fx["pseud"])) <= 1e-4 * abs(float(fx["pseud"])) + 1e-3
    else:
        assert pseud is None
    assert tuple(image.shape) == (int(fx["B"]), int(fx["T"]), 3, 128, 128)


def test_dpf_testing_writes_reference_outputs(tmp_path, monkeypatch):
    """DPF.testing (DPFs.py:419-451): the test-set RMSE file and result dump."""
    fx, dpf, inputs = _fwd_setup("fwd_c2_sdpf")
    monkeypatch.chdir(tmp_path)
    torch.manual_seed(int(fx["seed"]))
    dpf.testing([inputs], "run")
    loss = np.load(tmp_path / "logs" / "run" / "data" / "test_loss_epoch.npy")
    assert loss.shape == (1,)
    assert abs(float(loss[0]) - float(fx["sup"])) <= 1e-4 * float(fx["sup"])
    res = np.load(tmp_path / "logs" / "run" / "data" / "test_result.npz")
    for k in ("particle_list", "particle_weight_list", "likelihood_list", "state", "pred", "images", "noise"):
        assert k in res.files, k
    assert_close(res["pred"], fx["pred"], 1e-4, 1e-3, "dumped predictions")


def test_dpf_shard_returns_local_indices(monkeypatch):
    """A batch shard (row_base > 0) keeps global indices on the engine's FilterResult but
    returns them flat into its own B * N in the reference tuple, so the SDPF pseudo-likelihood
    loss (losses.py:33-69) indexes its own rows."""
    import DPFs
    from losses import pseudolikelihood_loss_nf
    from nfdpf.engine import ShardInfo
    fx = load("e2e_c2.npz")
    dpf = _dpf(fx, {"force_resample": True, "rng_mode": "device"})
    dpf.encoder = torch.nn.Identity()
    _load(dpf, fx)
    dpf.to(DEV).eval()
    B, N = int(fx["B"]), int(fx["N"])
    # rows [B, 2B) of a larger batch, run without a process group (B_global = B: the gate is
    # this shard's own; the device RNG is keyed on the global rows)
    monkeypatch.setattr(DPFs.ShardInfo, "from_env", staticmethod(lambda b, group=None: ShardInfo(1, 0, b, b, None)))
    torch.manual_seed(600)
    with torch.no_grad():
        out = dpf.filtering_pos(t(fx["enc"]).to(DEV), t(fx["start"]).to(DEV), t(fx["vel"]).to(DEV))
    idx = out[5]
    rows = torch.arange(B, device=DEV)[:, None, None] * N
    assert bool(((idx >= rows) & (idx < rows + N)).all())
    assert bool((dpf.last_filter_result.index - idx == B * N).all())
    for k in (0, 1, 2, 3, 6, 7):
        assert bool(torch.isfinite(out[k]).all()), (k, out[k])
    loss = pseudolikelihood_loss_nf(out[1], out[2], out[3], idx, out[6], out[7], 2)
    assert torch.isfinite(loss), loss


def test_particle_init_kernel():
    """particle_initialization (utils.py:46-62) in device-RNG mode: positions uniform on
    [-width/2, width/2)^2, log-weights log(1/N); the init_with_true_state branch draws
    start + N(0, 1); draws keyed on the global row (shard-invariant) and repeatable."""
    from nfdpf import ops
    B, N, W = 6, 20000, 128.0
    start = (torch.randn(B, 2, generator=torch.Generator().manual_seed(1)) * 30).to(DEV)
    x, lw = ops.particle_init(start, B, N, W, False, 5, 0, DEV)
    xc = x.cpu()
    assert float(xc.min()) >= -64.0 and float(xc.max()) < 64.0
    assert abs(float(xc.mean())) < 0.5 and abs(float(xc.std()) - 128.0 / 12 ** 0.5) < 0.3
    hist = torch.histc(xc.flatten(), bins=16, min=-64, max=64)
    assert float((hist / hist.mean() - 1).abs().max()) < 0.05  # flat
    ref_lw = float(torch.log(torch.ones(1) / N))  # torch.log(ones / N) (utils.py:60), fp32
    np.testing.assert_allclose(lw.cpu().numpy(), np.full((B, N), ref_lw, np.float32), rtol=2e-7, atol=0)
    x2, _ = ops.particle_init(start, B, N, W, False, 5, 0, DEV)
    assert torch.equal(x, x2)
    xs, _ = ops.particle_init(start[3:], B - 3, N, W, False, 5, 3, DEV)  # rows [3, 6) of a shard at row 3
    assert torch.equal(xs, x[3:])
    xt, lwt = ops.particle_init(start, B, N, W, True, 5, 0, DEV)
    d = (xt - start[:, None, :]).cpu()
    assert abs(float(d.mean())) < 0.03 and abs(float(d.std()) - 1.0) < 0.02
    assert torch.equal(lwt, lw)
    x3, _ = ops.particle_init(start, B, N, W, False, 6, 0, DEV)
    assert not torch.equal(x3, x)


def test_cond_glow_model_forward_kernel():
    """CondGlowModel.forward(x, y) (nf/cglow/CGlowModel.py:167-176) on the HIP kernel
    (nfdpf_cglow_flow) -> the reference's (z, nll); and the reverse of that z (PyTorch, off the
    DPF path) recovers y (the reference's own reverse raises, modules.py:195)."""
    from arguments import parse_args
    from nf.cglow.CGlowModel import CondGlowModel
    fx = load("cglow_flow.npz")
    m = CondGlowModel(parse_args([]))
    sd = m.state_dict()
    sd.update(weights(fx))
    m.load_state_dict(sd)
    m.to(DEV)
    x, y = t(fx["x"]).to(DEV), t(fx["y"]).to(DEV)
    with torch.no_grad():
        z, nll = m(x, y)
    assert tuple(z.shape) == (x.shape[0], 12, 4, 4)
    assert_close(z.cpu(), fx["z"], 1e-5, 2e-5, "z")
    assert_close(nll.cpu(), fx["nll"], 1e-5, 2e-6, "nll")
    with torch.no_grad():
        yr, _ = m(x, z, reverse=True)
    assert_close(yr.cpu(), fx["y"], 1e-4, 1e-4, "reverse(forward(y))")
    # under autograd the kernel value carries the PyTorch recompute's backward
    xg = x.clone().requires_grad_(True)
    z2, nll2 = m(xg, y)
    assert torch.equal(z2.detach(), z) and torch.equal(nll2.detach(), nll)
    nll2.sum().backward()
    assert xg.grad is not None and torch.isfinite(xg.grad).all()
