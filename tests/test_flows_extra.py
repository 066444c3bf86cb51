"""The reference's flows off the DPF path against fixtures written by the
reference itself (tests/golden/gen_golden.py gen_flows_extra -> flows_extra.npz).

CPU: Planar / Radial / ActNorm / OneByOneConv (PyTorch ops on the tensors' device), the
PyTorch restatement of the rational-quadratic spline that the spline flows' backward
differentiates (nf.utils._rqs_torch), state_dict keys.  GPU (marked): the HIP spline kernel
(nfdpf_rqs) through unconstrained_RQS / RQS, NSF_AR and NSF_CL forward / inverse and their
gradients.  Tolerances: 1e-5 relative + 1e-5 absolute on outputs and log-dets (the kernel's
softmax / exp / log differ from ATen's at the ulp level), gradients 1e-4 + 1e-5.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from _util import assert_close, group, load, t

FX = "flows_extra.npz"


def _fx(prefix):
    return group(load(FX), prefix)


def _load(m, fx):
    sd = {k[len("w/"):]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("w/")}
    assert set(sd) == set(m.state_dict()), (sorted(sd), sorted(m.state_dict()))
    m.load_state_dict(sd)
    return m


@pytest.mark.parametrize("tag,nl", [("tanh", torch.tanh), ("leaky_relu", F.leaky_relu), ("elu", F.elu)])
def test_planar(tag, nl):
    from nf.flows import Planar
    fx = _fx(f"planar_{tag}")
    m = _load(Planar(3, nonlinearity=nl), fx)
    with torch.no_grad():
        z, ld = m(t(fx["x"]))
    assert_close(z, fx["z"], 1e-5, 1e-6, "planar z")
    assert_close(ld, fx["ld"], 1e-5, 1e-6, "planar log-det")
    with pytest.raises(NotImplementedError):
        m.inverse(t(fx["z"]))


def test_radial():
    from nf.flows import Radial
    fx = _fx("radial")
    m = _load(Radial(3), fx)
    with torch.no_grad():
        z, ld = m(t(fx["x"]))
    assert_close(z, fx["z"], 1e-5, 1e-6, "radial z")
    assert_close(ld, fx["ld"], 1e-5, 1e-6, "radial log-det")


def test_actnorm():
    from nf.flows import ActNorm
    fx = _fx("actnorm")
    m = _load(ActNorm(3), fx)
    with torch.no_grad():
        z, ld = m(t(fx["x"]))
        xi, ldi = m.inverse(z)
    assert_close(z, fx["z"], 1e-6, 1e-6, "actnorm z")
    assert_close(xi, fx["xi"], 1e-6, 1e-6, "actnorm inverse")
    assert abs(float(ld) - float(fx["ld"])) <= 1e-6 and abs(float(ldi) - float(fx["ldi"])) <= 1e-6


def test_one_by_one_conv():
    from nf import flows
    fx = _fx("conv1x1")
    np.random.seed(82)  # the reference drew its QR / LU from numpy's global generator
    m = flows.OneByOneConv(3)
    np.testing.assert_allclose(m.P.cpu().numpy(), fx["P"], atol=0)
    np.testing.assert_allclose(m.L.detach().cpu().numpy(), fx["L"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(m.S.detach().cpu().numpy(), fx["S"], rtol=1e-6, atol=1e-7)
    with torch.no_grad():
        z, ld = m(t(fx["x"]).to(flows.device))
        xi, ldi = m.inverse(z)
        xi2, _ = m.inverse(z)  # the cached inverse
    assert_close(z.cpu(), fx["z"], 1e-5, 1e-6, "1x1 z")
    assert_close(xi.cpu(), fx["xi"], 1e-5, 1e-5, "1x1 inverse")
    assert torch.equal(xi, xi2)
    assert abs(float(ld) - float(fx["ld"])) <= 1e-5 and abs(float(ldi) - float(fx["ldi"])) <= 1e-5


@pytest.mark.parametrize("K", [5, 8])
def test_rqs_torch_restatement(K):
    """The spline math the backward differentiates, on the CPU, vs the reference's outputs."""
    from nf.utils import _RqsRunner
    fx = _fx(f"urqs_K{K}")
    B = float(fx["B"])
    x, W, H, D = (t(fx[k]) for k in ("x", "W", "H", "D"))
    fwd = _RqsRunner(False, -B, B, -B, B, True, (1e-3, 1e-3, 1e-3))
    y, ld = fwd.torch(x, W, H, D)
    assert_close(y, fx["y"], 1e-5, 1e-5, "y")
    assert_close(ld, fx["ld"], 1e-5, 1e-5, "log-det")
    inv = _RqsRunner(True, -B, B, -B, B, True, (1e-3, 1e-3, 1e-3))
    xi, ldi = inv.torch(t(fx["y"]), W, H, D)
    assert_close(xi, fx["xi"], 1e-5, 1e-5, "x inverse")
    # (ATen's CPU kernels vectorise differently on different hosts: ulp-level log-det noise)
    assert_close(ldi, fx["ldi"], 1e-5, 3e-5, "log-det inverse")
    fb = _fx(f"rqs_K{K}")
    bnd = _RqsRunner(False, 0.0, 1.0, 0.0, 1.0, False, (1e-3, 1e-3, 1e-3))
    yb, ldb = bnd.torch(t(fb["x"]), W, H, t(fb["D"]))
    assert_close(yb, fb["y"], 1e-5, 1e-6, "bounded y")
    assert_close(ldb, fb["ld"], 1e-5, 1e-5, "bounded log-det")


def test_rqs_domain_errors():
    from nf.utils import RQS
    x = torch.tensor([0.5, 1.5])
    W = torch.zeros(2, 4)
    with pytest.raises(ValueError, match="Input outside domain"):
        RQS(x, W, W, torch.zeros(2, 5))
    with pytest.raises(ValueError, match="Minimal bin width"):
        RQS(torch.tensor([0.5]), torch.zeros(1, 4), torch.zeros(1, 4), torch.zeros(1, 5), min_bin_width=0.3)


@pytest.mark.parametrize("name", ["nsf_ar_D2", "nsf_ar_D4", "nsf_cl_D4", "nsf_cl_D6"])
def test_nsf_state_dict_keys(name):
    from nf.flows import NSF_AR, NSF_CL
    fx = _fx(name)
    D = int(name[-1])
    m = NSF_AR(D) if "ar" in name else (NSF_CL(4) if D == 4 else NSF_CL(6, K=6, B=2))
    _load(m, fx)


# ---------------------------------------------------------------------- GPU (HIP spline) --
DEV = torch.device("cuda:0")


@pytest.mark.gpu
@pytest.mark.parametrize("K", [5, 8])
def test_rqs_kernel_golden(K):
    from nfdpf import _lib
    from nf.utils import RQS, unconstrained_RQS
    _lib.load()
    fx = _fx(f"urqs_K{K}")
    B = float(fx["B"])
    x, W, H, D = (t(fx[k]).to(DEV) for k in ("x", "W", "H", "D"))
    y, ld = unconstrained_RQS(x, W, H, D, inverse=False, tail_bound=B)
    assert_close(y.cpu(), fx["y"], 1e-5, 1e-5, "y")
    # log-det of a near-flat bin (e^ld ~ 1e-3) carries the ulp-level exp / log differences
    # from ATen's (Sleef) relative to a tiny derivative: 3e-5 absolute
    assert_close(ld.cpu(), fx["ld"], 1e-5, 3e-5, "log-det")
    out = torch.abs(t(fx["x"])) > B
    assert torch.equal(y.cpu()[out], t(fx["x"])[out]) and torch.all(ld.cpu()[out] == 0)
    xi, ldi = unconstrained_RQS(t(fx["y"]).to(DEV), W, H, D, inverse=True, tail_bound=B)
    # the inverse is ill-conditioned where the spline is flat (dy/dx = e^ld small): a knot that
    # differs from ATen's by an ulp (the kernel's exp / softmax are not Sleef's) moves x by
    # ~ulp / (dy/dx).  Bound per element: the forward bar 1e-5 (1 + |x|) carried through
    # 1 / (dy/dx), plus the reference's own round-trip error (its conditioning).
    amp = 1.0 + np.exp(-fx["ld"].astype(np.float64))
    env = 2 * np.abs(fx["xi"] - fx["x"]) + 1e-5 * (1 + np.abs(fx["xi"])) * amp
    err = np.abs(xi.cpu().numpy() - fx["xi"])
    assert np.all(err <= env), f"x inverse: worst excess {(err - env).max():.3e}"
    steep = fx["ld"] > np.log(0.1)  # where dy/dx >= 0.1 the plain bar holds
    assert np.all((err <= 1e-5 * np.abs(fx["xi"]) + 1e-5)[steep & (np.abs(fx["x"]) <= B)])
    # the inverse log-det moves with the knots through the spline's curvature as well: x10
    env = 2 * np.abs(fx["ldi"] + fx["ld"]) + 1e-4 * (1 + np.abs(fx["ldi"])) * amp
    assert np.all(np.abs(ldi.cpu().numpy() - fx["ldi"]) <= env), "log-det inverse"
    fb = _fx(f"rqs_K{K}")
    yb, ldb = RQS(t(fb["x"]).to(DEV), W, H, t(fb["D"]).to(DEV))
    assert_close(yb.cpu(), fb["y"], 1e-5, 1e-6, "bounded y")
    assert_close(ldb.cpu(), fb["ld"], 1e-5, 3e-5, "bounded log-det")
    xbi, ldbi = RQS(t(fb["y"]).to(DEV), W, H, t(fb["D"]).to(DEV), inverse=True)
    ampb = 1.0 + np.exp(-fb["ld"].astype(np.float64))
    env = 2 * np.abs(fb["xi"] - fb["x"]) + 1e-5 * (1 + np.abs(fb["xi"])) * ampb
    assert np.all(np.abs(xbi.cpu().numpy() - fb["xi"]) <= env), "bounded inverse"
    env = 2 * np.abs(fb["ldi"] + fb["ld"]) + 1e-4 * (1 + np.abs(fb["ldi"])) * ampb
    assert np.all(np.abs(ldbi.cpu().numpy() - fb["ldi"]) <= env), "bounded inverse log-det"


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["nsf_ar_D2", "nsf_ar_D4", "nsf_cl_D4", "nsf_cl_D6"])
def test_nsf_golden(name):
    from nfdpf import _lib
    from nf.flows import NSF_AR, NSF_CL
    _lib.load()
    fx = _fx(name)
    D = int(name[-1])
    m = NSF_AR(D) if "ar" in name else (NSF_CL(4) if D == 4 else NSF_CL(6, K=6, B=2))
    m = _load(m, fx).to(DEV)
    with torch.no_grad():
        z, ld = m(t(fx["x"]).to(DEV))
        xi, ldi = m.inverse(t(fx["z"]).to(DEV))
    assert_close(z.cpu(), fx["z"], 1e-5, 1e-5, "z")
    assert_close(ld.cpu(), fx["ld"], 1e-5, 1e-5, "log-det")
    assert_close(xi.cpu(), fx["xi"], 1e-5, 1e-5, "x inverse")
    assert_close(ldi.cpu(), fx["ldi"], 1e-5, 1e-5, "log-det inverse")
    # gradients of the reference's random functional (HIP forward, recompute backward)
    xg = t(fx["x"]).to(DEV).requires_grad_(True)
    z, ld = m(xg)
    ((z * t(fx["cz"]).to(DEV)).sum() + (ld * t(fx["cl"]).to(DEV)).sum()).backward()
    assert_close(xg.grad.cpu(), fx["gx"], 1e-4, 1e-5, "d/dx")
    for n, p in m.named_parameters():
        assert_close(p.grad.cpu(), fx[f"g/{n}"], 1e-4, 1e-5, f"d/d{n}")
