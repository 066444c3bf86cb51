"""Block pseudo-likelihood on the HIP kernels (csrc/pseudo_lik.hip) vs the PyTorch restatement
of compute_block_density_nf (losses.py:37-68) in float64, forward and gradients, on
filter-shaped histories (sorted soft-resampling ancestor maps, identity steps, the
out-of-range edge that points at the next row's first particle).  GPU box only.  (End to end,
the reference's own SDPF loss value is pinned by test_gpu_dpf_api.py's fwd_*_sdpf fixtures.)"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from nfdpf import _lib
    _lib.load()


def _hist(B, T, N, seed, edge=False):
    g = torch.Generator().manual_seed(seed)
    w = torch.softmax(torch.randn(B, T, N, generator=g), -1)
    lik = torch.randn(B, T, N, generator=g)
    prior = torch.randn(B, T, N, generator=g) * 3
    idx = torch.empty(B, T, N, dtype=torch.int64)
    for b in range(B):
        for t in range(T):
            if t % 3 == 0:  # a step without resampling (or OT): identity
                src = torch.arange(N)
            else:           # soft resampling: sorted sources of the row
                src = torch.sort(torch.randint(0, N, (N,), generator=g)).values
            idx[b, t] = src + N * b
    if edge and B > 1:
        idx[0, 4, -1] = N  # the reference's marker-above-1 edge: row 0 points at row 1's first
    return w, lik, prior, idx


@pytest.mark.parametrize("B,T,N,L,edge", [(3, 25, 50, 10, False), (4, 30, 257, 10, True), (2, 12, 1000, 4, False),
                                          (1, 9, 7, 10, False)])
def test_pseudo_lik_forward_backward(B, T, N, L, edge):
    from losses import _block_density_nf_torch, compute_block_density_nf
    w, lik, prior, idx = _hist(B, T, N, 11 + N, edge)
    if T // L == 0:  # no complete block: the restatement path (the reference divides by 0 there)
        return
    ref = [x.double().requires_grad_(True) for x in (w, lik, prior)]
    Qr = _block_density_nf_torch(ref[0], ref[1], idx, ref[2], L)
    gQ = torch.randn(B, dtype=torch.float64, generator=torch.Generator().manual_seed(N))
    Qr.backward(gQ)
    dev = [x.to(DEV).requires_grad_(True) for x in (w, lik, prior)]
    Q = compute_block_density_nf(dev[0], None, dev[1], idx.to(DEV), None, dev[2], L)
    torch.testing.assert_close(Q.double().cpu(), Qr.detach(), rtol=2e-6, atol=1e-5)
    Q.backward(gQ.float().to(DEV))
    for name, a, r in zip(("w", "lik", "prior"), dev, ref):
        _close_scaled(a.grad, r.grad, name)


def _close_scaled(ours, ref, name):
    """Within 1e-5 relative + 2e-6 of the tensor's largest |gradient|: eta is an fp32 running sum
    over up to T steps of prior + likelihood (losses.py:65), so where it cancels towards zero its
    rounding (~1e-6 of the summands) is all that is left of dw = gQ eta."""
    o = ours.double().cpu()
    d = (o - ref).abs()
    tol = 1e-5 * ref.abs() + 2e-6 * float(ref.abs().max())
    assert bool((d <= tol).all()), f"{name}: max |d| {float(d.max()):.3g}, worst excess {float((d - tol).max()):.3g}"


def test_pseudo_lik_non_monotone_falls_back():
    from losses import _block_density_nf_torch, compute_block_density_nf
    w, lik, prior, idx = _hist(2, 10, 30, 3)
    idx[1, 5] = idx[1, 5].flip(0)  # not a filter's map: the backward takes the PyTorch path
    ref = [x.double().requires_grad_(True) for x in (w, lik, prior)]
    _block_density_nf_torch(ref[0], ref[1], idx, ref[2], 10).sum().backward()
    dev = [x.to(DEV).requires_grad_(True) for x in (w, lik, prior)]
    compute_block_density_nf(dev[0], None, dev[1], idx.to(DEV), None, dev[2], 10).sum().backward()
    for name, a, r in zip(("w", "lik", "prior"), dev, ref):
        _close_scaled(a.grad, r.grad, name)
