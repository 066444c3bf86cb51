"""Training parity pinned to the REFERENCE's autograd: the gradients of this
package's modules -- HIP forward, HIP backward where one exists (coupling stacks, soft and OT
resamplers, cosine and CRNVP measurements), the recompute backward elsewhere (MAF, NN,
gaussian, CGLOW) -- against the gradients the reference itself computed
(tests/golden/grads.npz and train_c2.npz, written by tests/golden/gen_golden.py).  GPU box only.

Bar: every gradient tensor elementwise within rtol |ref| + atol * max|ref| (rtol 1e-3, atol
2e-4: fp32 backward chains through exp / tanh / log differ from the reference's Sleef / MKL
arithmetic at ~1e-6 relative per op and compound through the nets).  The whole training step
(DPF.forward(train=True) -> total_loss.backward(), 106 parameter tensors) is held to 2e-3
of each tensor's scale.
"""
import numpy as np
import pytest
import torch

from _util import group, load, t, weights

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
G = {}


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from nfdpf import _lib
    _lib.load()
    assert torch.cuda.is_available()
    G.update(load("grads.npz"))


def _close(ours, ref, what, rtol=1e-3, atol=2e-4):
    o = ours.detach().double().cpu().numpy() if torch.is_tensor(ours) else np.asarray(ours, np.float64)
    r = np.asarray(ref, np.float64)
    assert o.shape == r.shape, (what, o.shape, r.shape)
    scale = float(np.abs(r).max()) if r.size else 0.0
    err = np.abs(o - r) - (rtol * np.abs(r) + atol * scale)
    assert float(err.max()) <= 0 if err.size else True, \
        f"{what}: worst excess {float(err.max()):.3e} (scale {scale:.3e}, max |d| {float(np.abs(o - r).max()):.3e})"


def _load_into(module, w, prefix):
    sd = module.state_dict()
    upd = {k[len(prefix):]: v for k, v in w.items() if k.startswith(prefix)}
    assert upd and all(k in sd for k in upd), list(upd)[:3]
    sd.update(upd)
    module.load_state_dict(sd)


def _param_grads(fx, named, what):
    for n, p in named:
        key = f"g/{n}"
        assert key in fx, (what, key)
        ref = fx[key]
        if p.grad is None:
            assert not np.any(ref), (what, n)
            continue
        _close(p.grad, ref, f"{what} d/d{n}")


@pytest.mark.parametrize("case", ["cond_D2_O4", "cond_D2_O36", "cond_D32_O32"])
@pytest.mark.parametrize("direction", ["fwd", "inv"])
def test_cond_stack_grads_vs_reference(case, direction):
    """NormalizingFlowModel_cond forward / inverse (nf/models.py:37-66): d/dx, d/dcond and every
    coupling-net parameter, HIP backward (nfdpf_cond_stack_backward)."""
    from model.models import build_conditional_nf
    fx = group(G, f"{case}_{direction}")
    D, O_ = int(case.split("_")[1][1:]), int(case.split("_")[2][1:])
    m = build_conditional_nf(2, O_, D, init_var=0.01, prior_std=float(fx["prior_std"]))
    _load_into(m.flows, weights(fx), "flows.")
    m.flows.to(DEV)
    x = t(fx["x"]).to(DEV).requires_grad_(True)
    c = t(fx["c"]).to(DEV).requires_grad_(True)
    gz, gl, gp = (t(fx[k]).to(DEV) for k in ("gz", "gl", "gp"))
    if direction == "inv":
        z, ld = m.inverse(x, c)
        loss = (z * gz).sum() + (ld * gl).sum()
    else:
        z, lp, ld = m.forward(x, c)
        loss = (z * gz).sum() + (ld * gl).sum() + (lp * gp).sum()
    loss.backward()
    _close(x.grad, fx["dx"], "d/dx")
    _close(c.grad, fx["dc"], "d/dcond")
    _param_grads(fx, [("flows." + n, p) for n, p in m.flows.named_parameters()], case)


def test_maf_grads_vs_reference():
    """MAF stack forward (nf/flows.py:259-271): d/dx and every parameter.  (The reference's
    MAF.inverse writes its output in place while reading it, so its autograd raises: no
    reference gradient exists for the inverse.)"""
    from model.models import build_maf_dyn
    fx = group(G, "maf_fwd")
    m = build_maf_dyn(2, 2)
    _load_into(m.flows, weights(fx), "flows.")
    m.flows.to(DEV)
    x = t(fx["x"]).to(DEV).requires_grad_(True)
    z, _, ld = m.forward(x)
    ((z * t(fx["gz"]).to(DEV)).sum() + (ld * t(fx["gl"]).to(DEV)).sum()).backward()
    _close(x.grad, fx["dx"], "d/dx")
    _param_grads(fx, [("flows." + n, p) for n, p in m.flows.named_parameters()], "MAF")


def test_soft_resampler_grads_vs_reference():
    """soft_resampler (resamplers.py:20-60): indices bit-exact, d/dx through the gather, d/dp
    through w = p / q and the renormalisation (nfdpf_soft_resample_backward)."""
    from resamplers.resamplers import soft_resampler
    fx = group(G, "soft")
    x = t(fx["x"]).to(DEV).requires_grad_(True)
    p = t(fx["p"]).to(DEV).requires_grad_(True)
    N = x.shape[1]
    xo, wo, idx = soft_resampler(x, p, 0.5, N, index=True, offsets=t(fx["offsets"]))
    np.testing.assert_array_equal(idx.cpu().numpy(), fx["idx"].astype(np.int64))
    ((xo * t(fx["gx"]).to(DEV)).sum() + (wo * t(fx["gw"]).to(DEV)).sum()).backward()
    _close(x.grad, fx["dx"], "d/dx")
    _close(p.grad, fx["dp"], "d/dp")


def test_ot_resampler_grads_vs_reference():
    """resampler_ot (resamplers.py:234-264): dL/dx = T^T g with the plan held constant, as the
    reference's transport Function returns (nfdpf_ot_transport_backward); the fp32 Sinkhorn
    pair work vs the reference's fp64 gives the plan ~1e-5 relative -- atol 1e-3 of scale."""
    from resamplers.resamplers import resampler_ot
    fx = group(G, "ot")
    x = t(fx["x"]).to(DEV).requires_grad_(True)
    xo, wo, idx = resampler_ot(x, t(fx["p"]).to(DEV))
    (xo * t(fx["gx"]).to(DEV)).sum().backward()
    _close(x.grad, fx["dx"], "d/dx", rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("meas", ["cos", "CRNVP", "NN", "gaussian", "CGLOW"])
def test_measurement_grads_vs_reference(meas):
    """The measurement models (model/models.py:206-303): d/d(frame encoding, particles) and every
    parameter (particle encoder, CNF / likelihood_est / CGLOW)."""
    from arguments import parse_args
    from DPFs import DPF
    fx = group(G, f"meas_{meas}")
    a = parse_args([])
    a.measurement, a.hiddensize, a.num_particles, a.batchsize = meas, 192 if meas == "CGLOW" else 32, 40, 3
    torch.manual_seed(0)
    dpf = DPF(a)
    sd = dpf.state_dict()
    sd.update(weights(fx))
    dpf.load_state_dict(sd)
    dpf.to(DEV)
    mm = dpf.measurement_model
    enc = t(fx["enc"]).to(DEV).requires_grad_(True)
    x = t(fx["x"]).to(DEV).requires_grad_(True)
    (mm(enc, x) * t(fx["gl"]).to(DEV)).sum().backward()
    _close(enc.grad, fx["denc"], f"{meas} d/denc")
    _close(x.grad, fx["dx"], f"{meas} d/dx")
    _param_grads(fx, list(mm.named_parameters()), meas)


def test_training_step_grads_vs_reference():
    """One e2e_train iteration of the reference (DPFs.py:318-331): DPF.forward(inputs,
    train=True) with the SDPF losses, then total_loss.backward() -- the losses and all 106
    parameter gradients (frame encoder / decoder swapped for tests/_tiny.py on both sides)."""
    from _tiny import TinyDecoder, TinyEncoder
    from arguments import parse_args
    from DPFs import DPF
    fx = load("train_c2.npz")
    a = parse_args([])
    a.num_particles, a.batchsize, a.sequence_length = int(fx["N"]), int(fx["B"]), int(fx["T"])
    for k in ("NF_dyn", "NF_cond", "measurement", "resampler_type", "trainType", "block_length"):
        setattr(a, k, fx[f"flag/{k}"].item())
    torch.manual_seed(0)
    dpf = DPF(a)
    dpf.encoder, dpf.decoder = TinyEncoder(a.hiddensize), TinyDecoder(a.hiddensize)
    sd = dpf.state_dict()
    sd.update(weights(fx))
    dpf.load_state_dict(sd)
    dpf.to(DEV).train()
    up = lambda v: t(v).float().div(255).repeat_interleave(8, -3).repeat_interleave(8, -2)  # noqa: E731
    B, T = int(fx["B"]), int(fx["T"])
    inputs = (up(fx["start_img"]), t(fx["start"]), up(fx["img"]), t(fx["state"]), torch.zeros(B, T),
              torch.ones(B, T))
    np.random.seed(int(fx["seed"]))
    torch.manual_seed(int(fx["seed"]))
    out = dpf.forward(inputs, train=True)
    dpf.zero_grad()
    out[0].backward()
    _close(out[5], fx["x"], "particles", 1e-4, 1e-5)
    _close(out[6], fx["p"], "weights", 1e-4, 1e-5)
    for v, k in ((out[0], "total"), (out[1], "sup"), (out[2], "pseud"), (out[3], "ae")):
        assert abs(float(v) - float(fx[k])) <= 1e-4 * abs(float(fx[k])) + 1e-4, (k, float(v), float(fx[k]))
    n = 0
    for name, p in dpf.named_parameters():
        key = f"g/{name}"
        if key not in fx:
            assert p.grad is None or not bool(p.grad.any()), name
            continue
        assert p.grad is not None, name
        _close(p.grad, fx[key], f"d total / d {name}", rtol=2e-3, atol=2e-3)
        n += 1
    assert n == sum(1 for k in fx if k.startswith("g/"))
