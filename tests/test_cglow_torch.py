"""CPU: the PyTorch restatement of CondGlowModel (nf/cglow: the layers' forwards, used as the
recompute backward of the CGLOW kernel and for reverse sampling) against the reference's own
CondGlowModel.forward output (tests/golden/cglow_flow.npz) and the measurement golden vector."""
import torch

from _util import assert_close, group, load, t, weights


def _model(fx):
    from arguments import parse_args
    from nf.cglow.CGlowModel import CondGlowModel
    m = CondGlowModel(parse_args([]))
    sd = m.state_dict()
    sd.update(weights(fx))
    m.load_state_dict(sd)
    return m


def test_cglow_torch_forward_matches_reference():
    fx = load("cglow_flow.npz")
    m = _model(fx)
    with torch.no_grad():
        z, nll = m.torch_forward(t(fx["x"]), t(fx["y"]))
        yr, _ = m(t(fx["x"]), z, reverse=True)
    assert_close(z, fx["z"], 1e-6, 1e-6, "z")
    assert_close(nll, fx["nll"], 1e-6, 1e-6, "nll")
    assert_close(yr, fx["y"], 1e-4, 1e-4, "reverse round trip")


def test_cglow_measurement_torch_matches_reference():
    from model.models import build_particle_encoder_cglow, measurement_model_cglow
    fx = group(load("meas.npz"), "CGLOW")
    w = weights(fx)
    glow = _model({f"w/{k[len('cglow_measurement.'):]}": v.numpy() for k, v in w.items()
                   if k.startswith("cglow_measurement.")})
    pe = build_particle_encoder_cglow(192, 2)
    pe.load_state_dict({k[len("particle_encoder."):]: v for k, v in w.items() if k.startswith("particle_encoder.")})
    mm = measurement_model_cglow(pe, glow)
    with torch.no_grad():
        raw = mm.torch_forward_raw(t(fx["enc"]), t(fx["x"]))
    assert_close(raw - raw.max(-1, keepdim=True)[0], fx["lik"], 1e-6, 1e-6, "CGLOW likelihood")
