"""HIP backward of the MAF stack (csrc/maf_bwd.hip, nfdpf_maf_stack_backward) against the
reference's autograd gradients (tests/golden/grads.npz, written by the reference) and against
the PyTorch-recompute path on larger random inputs.  GPU box only."""
import numpy as np
import pytest
import torch

from _util import group, load, t

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from nfdpf import _lib
    _lib.load()


def _maf(D, n=2, seed=0, scale=0.3):
    from model.models import build_maf_dyn
    torch.manual_seed(seed)
    m = build_maf_dyn(n, D)
    with torch.no_grad():
        for p in m.parameters():
            p.mul_(1.0).add_(torch.randn_like(p) * scale)
    return m.to(DEV)


def _grads(m, x, inverse, cz, cl, hip):
    from nfdpf import autograd as ag
    old = ag.HIP_BACKWARD
    ag.HIP_BACKWARD = hip
    try:
        m.zero_grad(set_to_none=True)
        xg = x.clone().requires_grad_(True)
        if inverse:
            z, ld = m.inverse(xg)
        else:
            z, _, ld = m(xg)
        ((z * cz).sum() + (ld * cl).sum()).backward()
        return xg.grad.clone(), [p.grad.clone() for p in m.parameters()]
    finally:
        ag.HIP_BACKWARD = old


@pytest.mark.parametrize("D", [2, 4])
@pytest.mark.parametrize("inverse", [False, True])
def test_maf_hip_backward_matches_recompute(D, inverse):
    m = _maf(D, seed=D)
    g = torch.Generator().manual_seed(7)
    rows = 1000  # ragged: 15 full waves + 40 rows
    x = (torch.randn(rows, D, generator=g) * 2).to(DEV)
    cz = torch.randn(rows, D, generator=g).to(DEV)
    cl = torch.randn(rows, generator=g).to(DEV)
    gx_h, gp_h = _grads(m, x, inverse, cz, cl, True)
    gx_r, gp_r = _grads(m, x, inverse, cz, cl, False)
    torch.testing.assert_close(gx_h, gx_r, rtol=2e-4, atol=1e-5)
    for a, b in zip(gp_h, gp_r):
        scale = float(b.abs().max()) + 1e-6
        assert float((a - b).abs().max()) <= 5e-4 * scale + 1e-5, (float((a - b).abs().max()), scale)


def test_maf_hip_backward_is_taken():
    """The MAF runner's backward is the kernel (the reference-fixture gradients are checked by
    test_gpu_grad_golden.py::test_maf_grads_vs_reference, which now runs through it)."""
    from nf.flows import MafStack
    m = _maf(2)
    x = torch.randn(100, 2, device=DEV)
    r = MafStack(m, list(m.flows), 2, 8, False)
    got = r.hip_backward(x, (torch.ones_like(x), torch.ones(100, device=DEV)))
    assert got is not None
    (gx,), gp = got
    assert gx.shape == x.shape and len(gp) == len(list(m.flows.parameters()))
