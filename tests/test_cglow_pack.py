"""CPU: the blob-layout gradient of the CGLOW backward maps back to the modules' parameters
(nfdpf.pack.blob_param_grads over cglow_tensors / encoder_tensors with a getter): packing a
per-parameter tensor set with the same layout functions and scattering it back returns the
same tensors, and parameters the blob does not pack (CondGlowModel's new_mean / new_logs with
learn_top off) get None, as under autograd."""
import torch


def _roundtrip(owner, params, build, name):
    from nfdpf.pack import blob_param_grads
    g = torch.Generator().manual_seed(len(params))
    fake = {id(p): torch.randn(p.shape, generator=g) for p in params}
    blob = torch.cat([t.reshape(-1) for t in build(lambda p: fake[id(p)])])
    got = blob_param_grads(owner, name, params, build, blob)
    return fake, got


def test_cglow_blob_grads_roundtrip():
    from arguments import parse_args
    from nf.cglow.CGlowModel import CondGlowModel
    from nfdpf.pack import cglow_tensors
    m = CondGlowModel(parse_args([]))
    params = list(m.parameters())
    fake, got = _roundtrip(m, params, lambda get: cglow_tensors(m, get), "glow_grad")
    names = [n for n, _ in m.named_parameters()]
    for n, p, gp in zip(names, params, got):
        if n in ("new_mean", "new_logs"):
            assert gp is None, n
        else:
            assert gp is not None and torch.equal(gp, fake[id(p)]), n


def test_encoder_blob_grads_roundtrip():
    from model.models import build_particle_encoder_cglow
    from nfdpf.pack import encoder_tensors
    pe = build_particle_encoder_cglow(192, 2)
    params = list(pe.parameters())
    fake, got = _roundtrip(pe, params, lambda get: encoder_tensors(pe, get), "pe_grad")
    for p, gp in zip(params, got):
        assert torch.equal(gp, fake[id(p)])


def test_cglow_blob_size_matches_kernel_layout():
    """The packed blob is the kernel's layout size (csrc/cglow.hpp kStep = 7 980 floats)."""
    from arguments import parse_args
    from nf.cglow.CGlowModel import CondGlowModel
    from nfdpf.pack import cglow_tensors
    m = CondGlowModel(parse_args([]))
    assert sum(t.numel() for t in cglow_tensors(m)) == 7980
