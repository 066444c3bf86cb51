"""HIP backward of the coupling-flow stacks (csrc/flows_bwd.hip, nfdpf_cond_stack_backward)
against PyTorch autograd of the same math in float64 (and float32 to size the tolerance).
GPU box only.

The reference's training path differentiates NormalizingFlowModel_cond.forward / .inverse
(nf/models.py:45-61) over RealNVP_cond (nf/flows.py:215-239) with autograd; the module API
here routes that backward through the HIP kernel (nfdpf.autograd).

Tolerance: per tensor, |d| <= 4 * |err32| + 1e-6 * max|ref|, elementwise, where err32 is the
float32 autograd's own error against float64 on the same inputs, plus a global cap
|d| <= 2e-4 |ref| + 2e-5 max|ref| -- the parameter gradients are sums over every row, so
their accumulation order (per-64-row partials, then per-workgroup) differs from ATen's.
"""
import copy
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _ref_stack(flows, x, c, inverse, prior, dtype):
    """RealNVP_cond stack (nf/flows.py:215-239, nf/models.py:45-61) in plain torch ops."""
    def net(m, a):
        l0, l2, l4 = [l for l in m.network if isinstance(l, torch.nn.Linear)]
        h = torch.tanh(F.linear(a, l0.weight.to(dtype), l0.bias.to(dtype)))
        h = torch.tanh(F.linear(h, l2.weight.to(dtype), l2.bias.to(dtype)))
        return F.linear(h, l4.weight.to(dtype), l4.bias.to(dtype))

    cat = (lambda a: torch.cat([a, c], -1)) if c is not None else (lambda a: a)
    ld = torch.zeros(x.shape[0], dtype=dtype, device=x.device)
    for f in (flows[::-1] if inverse else flows):
        half = x.shape[1] // 2
        lo, up = x[:, :half], x[:, half:]
        if not inverse:
            t1, s1 = net(f.t1, cat(lo)), net(f.s1, cat(lo))
            up = t1 + up * torch.exp(s1)
            t2, s2 = net(f.t2, cat(up)), net(f.s2, cat(up))
            lo = t2 + lo * torch.exp(s2)
            ld = ld + s1.sum(1) + s2.sum(1)
        else:
            t2, s2 = net(f.t2, cat(up)), net(f.s2, cat(up))
            lo = (lo - t2) * torch.exp(-s2)
            t1, s1 = net(f.t1, cat(lo)), net(f.s1, cat(lo))
            up = (up - t1) * torch.exp(-s1)
            ld = ld - s1.sum(1) - s2.sum(1)
        x = torch.cat([lo, up], 1)
    if prior is None or inverse:
        return x, ld, None
    pm, ps = prior
    d = x.shape[1]
    z = (x - pm) / ps
    lp = -0.5 * (z * z).sum(-1) - d * math.log(ps) - 0.5 * d * math.log(2 * math.pi)
    return x, ld, lp


def _build(D, O, n_flows, std, seed):
    from nf.flows import RealNVP_cond, RealNVP
    torch.manual_seed(seed)
    flows = []
    for _ in range(n_flows):
        f = RealNVP_cond(D, 8, obser_dim=O) if O else RealNVP(D, 8)
        f.zero_initialization(std)
        # non-zero biases, so every bias gradient path is exercised
        with torch.no_grad():
            for p in f.parameters():
                if p.dim() == 1:
                    p.normal_(0, std)
        flows.append(f)
    return flows


def _grads(loss, tensors):
    return torch.autograd.grad(loss, tensors, allow_unused=True)


def _check(ours, r32, r64, what, rel_cap=2e-4, abs_cap=2e-5):
    ours, r32, r64 = ours.double().cpu(), r32.double().cpu(), r64.double().cpu()
    scale = float(r64.abs().max()) + 1e-30
    d = (ours - r64).abs()
    e32 = (r32 - r64).abs()
    env = 4 * e32 + 1e-6 * scale
    cap = rel_cap * r64.abs() + abs_cap * scale
    bad = (d > torch.maximum(env, cap))
    assert not bool(bad.any()), (
        f"{what}: {int(bad.sum())}/{d.numel()} outside; max |d| {float(d.max()):.3g} "
        f"(fp32 err max {float(e32.max()):.3g}, scale {scale:.3g})")


def _check_tensor(ours, r32, r64, what, rmax=1e-4, rmean=5e-5):
    """Tensor-level envelope for cancellation-heavy gradients: max and mean |ours - f64| within
    4x the float32 autograd's own error (elementwise placement of fp32 rounding is arbitrary
    there), or within 1e-4 / 2e-5 of the tensor's scale: the kernels' tanh (1 - 2/(1 + e^2x),
    csrc/flows.hpp) has an ABSOLUTE error ~6e-8, which is a 1e-5..1e-4 relative error on the
    ~1e-3 activations of the reference init (std 0.01) that dW3 = sum g (x) h2 then sums."""
    ours, r32, r64 = ours.double().cpu(), r32.double().cpu(), r64.double().cpu()
    scale = float(r64.abs().max()) + 1e-30
    d, e32 = (ours - r64).abs(), (r32 - r64).abs()
    assert float(d.max()) <= max(4 * float(e32.max()), rmax * scale) + 1e-6 * scale, \
        f"{what}: max |d| {float(d.max()):.3g} vs fp32 {float(e32.max()):.3g} (scale {scale:.3g})"
    assert float(d.mean()) <= max(4 * float(e32.mean()), rmean * scale) + 1e-7 * scale, \
        f"{what}: mean |d| {float(d.mean()):.3g} vs fp32 {float(e32.mean()):.3g} (scale {scale:.3g})"


CASES = [  # (D, O, n_flows, std, rows)
    (2, 4, 2, 0.01, 5000),     # nf_dyn, reference init (nf/flows.py:191-211)
    (2, 4, 2, 0.3, 4097),
    (2, 36, 2, 0.3, 3001),     # NF proposal context (model/models.py:334-356)
    (2, 196, 2, 0.1, 777),     # CGLOW-size context
    (32, 32, 2, 0.3, 1000),    # CRNVP measurement flow
    (4, 0, 2, 0.3, 2048),      # unconditional RealNVP
    (2, 36, 1, 0.3, 1),        # one row, one flow
    (2, 4, 4, 0.3, 65),        # four flows, ragged last wave
]


@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("D,O,n_flows,std,rows", CASES)
def test_cond_stack_backward_vs_autograd(D, O, n_flows, std, rows, inverse, monkeypatch):
    from nf.models import NormalizingFlowModel, NormalizingFlowModel_cond
    from nfdpf import ops
    calls = []
    real = ops.cond_stack_backward
    monkeypatch.setattr(ops, "cond_stack_backward", lambda *a, **k: calls.append(1) or real(*a, **k))
    flows = _build(D, O, n_flows, std, seed=D * 1000 + O * 10 + n_flows)
    ref_flows = copy.deepcopy(flows)
    g = torch.Generator().manual_seed(rows)
    x = (torch.randn(rows, D, generator=g) * 3).to(DEV).requires_grad_(True)
    c = torch.randn(rows, O, generator=g).to(DEV).requires_grad_(True) if O else None
    w_out = torch.randn(rows, D, generator=g)
    w_ld = torch.randn(rows, generator=g)
    w_lp = torch.randn(rows, generator=g)
    prior = (0.0, 2.5)
    if O:
        prior_d = torch.distributions.MultivariateNormal(torch.zeros(D, device=DEV), 6.25 * torch.eye(D, device=DEV))
        model = NormalizingFlowModel_cond(prior_d, flows, device=DEV)
    else:
        model = NormalizingFlowModel(None, flows, device=DEV)

    if inverse:
        out, ld = model.inverse(x, c) if O else model.inverse(x)
        lp = None
    elif O:
        out, lp, ld = model.forward(x, c)
    else:
        out, _, ld = model.forward(x)
        lp = None
    loss = (out * w_out.to(DEV)).sum() + (ld * w_ld.to(DEV)).sum()
    if lp is not None:
        loss = loss + (lp * w_lp.to(DEV)).sum()
    params = [p for f in flows for p in f.parameters()]
    ins = [x] + ([c] if O else [])
    ours = _grads(loss, ins + params)
    assert len(calls) == 1, "the backward did not run through nfdpf_cond_stack_backward"

    refs = []
    for dt in (torch.float32, torch.float64):
        rf = copy.deepcopy(ref_flows)
        for p in rf:
            p.to(dtype=dt)
        xr = x.detach().cpu().to(dt).requires_grad_(True)
        cr = c.detach().cpu().to(dt).requires_grad_(True) if O else None
        o_, l_, p_ = _ref_stack(rf, xr, cr, inverse, prior if O else None, dt)
        lr = (o_ * w_out.to(dt)).sum() + (l_ * w_ld.to(dt)).sum()
        if p_ is not None:
            lr = lr + (p_ * w_lp.to(dt)).sum()
        rp = [p for f in rf for p in f.parameters()]
        refs.append(_grads(lr, [xr] + ([cr] if O else []) + rp))
    names = ["x"] + (["cond"] if O else []) + [f"param{i}" for i in range(len(params))]
    for name, a, r32, r64 in zip(names, ours, refs[0], refs[1]):
        assert a is not None, name
        _check(a, r32, r64, f"{name} (D={D} O={O} flows={n_flows} inv={inverse})")


def test_cond_stack_backward_deterministic():
    """Fixed-order partial sums: two backward calls give identical bits."""
    from nfdpf import ops
    from nfdpf.pack import flows_tensors
    flows = _build(2, 36, 2, 0.3, 7)
    b = torch.cat([t.detach().reshape(-1) for t in flows_tensors(flows)]).to(DEV)
    x = torch.randn(10000, 2, device=DEV)
    c = torch.randn(10000, 36, device=DEV)
    go, gl = torch.randn(10000, 2, device=DEV), torch.randn(10000, device=DEV)
    a = ops.cond_stack_backward(b, 2, 2, 36, 8, x, c, True, go, gl)
    bb = ops.cond_stack_backward(b, 2, 2, 36, 8, x, c, True, go, gl)
    for u, v in zip(a, bb):
        assert torch.equal(u, v)


def test_cond_stack_backward_zero_rows():
    from nfdpf import ops
    from nfdpf.pack import flows_tensors
    flows = _build(2, 4, 2, 0.3, 3)
    b = torch.cat([t.detach().reshape(-1) for t in flows_tensors(flows)]).to(DEV)
    x = torch.zeros(0, 2, device=DEV)
    c = torch.zeros(0, 4, device=DEV)
    gx, gc, gb = ops.cond_stack_backward(b, 2, 2, 4, 8, x, c, False, torch.zeros(0, 2, device=DEV),
                                         torch.zeros(0, device=DEV))
    assert gx.shape == (0, 2) and gc.shape == (0, 4) and bool((gb == 0).all())


@pytest.mark.parametrize("meas", ["cos", "CRNVP"])
def test_training_step_hip_backward_matches_recompute(meas):
    """One training pass of the reference loop (DPFs.py:144-216 under autograd, as e2e_train
    runs it): parameter gradients with the HIP flow backward == with the PyTorch-recompute
    backward (same HIP forward, so only the backward differs)."""
    import sys
    import os
    import torch.nn as nn
    from nfdpf import autograd as ag
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import make_args, synthetic_disk
    from DPFs import DPF
    B, N, T = 4, 200, 4
    flags = dict(NF_dyn=True, NF_cond=True, measurement=meas, resampler_type="soft", force_resample=True)
    torch.manual_seed(5)
    a = make_args(flags, B, N, T, {})
    dpf = DPF(a).to(DEV)
    dpf.encoder = nn.Identity()
    start, state, vel_in, enc = (x.to(DEV) for x in synthetic_disk(B, T, 3, a.hiddensize))
    grads = {}
    for mode in (True, False):
        ag.HIP_BACKWARD = mode
        try:
            dpf.zero_grad(set_to_none=True)
            torch.manual_seed(11)
            out = dpf.filtering_pos(enc, start, vel_in)
            xs, ps = out[0], out[1]
            pred = (xs * ps[..., None]).sum(2)
            loss = ((pred - state[:, :, :2]) ** 2).mean() + 0.01 * out[-1]
            loss.backward()
        finally:
            ag.HIP_BACKWARD = True
        grads[mode] = {n: p.grad.detach().clone() for n, p in dpf.named_parameters() if p.grad is not None}
    flow_keys = [k for k in grads[False] if k.startswith(("nf_dyn.", "cond_model."))]
    assert flow_keys and set(grads[True]) == set(grads[False])
    for k in grads[False]:
        a_, b_ = grads[True][k].double(), grads[False][k].double()
        scale = float(b_.abs().max()) + 1e-30
        d = float((a_ - b_).abs().max())
        assert d <= 2e-3 * scale + 1e-7, f"{k}: max |d| {d:.3g} vs scale {scale:.3g}"


@pytest.mark.parametrize("B,N,kind", [(4, 128, "random"), (3, 1000, "peaked"), (2, 257, "zero_w")])
def test_ot_transport_backward_vs_oracle(B, N, kind):
    """dL/dx through resampler_ot under autograd == T^T g with the oracle's float64 transport
    matrix (the reference treats T as a constant in backward, resamplers.py:234-245)."""
    from oracle import dpf_oracle as O
    from resamplers.resamplers import resampler_ot
    g = torch.Generator().manual_seed(N)
    x = torch.randn(B, N, 2, generator=g) * 20
    logits = torch.randn(B, N, generator=g) * (4.0 if kind == "peaked" else 1.0)
    w = torch.softmax(logits, -1)
    if kind == "zero_w":
        w[:, ::7] = 0.0
        w = w / w.sum(-1, keepdim=True)
    gout = torch.randn(B, N, 2, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    xo, wo, idx = resampler_ot(xd, w.to(DEV))
    (xo * gout.to(DEV)).sum().backward()
    _, _, _, info = O.ot_resample(x.double(), w.double(), return_info=True)
    ref = torch.einsum("bij,bic->bjc", info["T"].double(), gout.double())
    d = (xd.grad.double().cpu() - ref).abs()
    scale = float(ref.abs().max())
    tol = 1e-4 * ref.abs() + 5e-5 * scale
    assert bool((d <= tol).all()), f"max |d| {float(d.max()):.3g} (scale {scale:.3g})"
    if kind == "zero_w":
        assert bool((xd.grad[:, ::7].abs() == 0).all())


def _soft_ref(x, p, idx, alpha):
    """resamplers.py:28-56 in float64 with the given indices (and this library's edge rule:
    an index past the row reads the next row's first particle with weight 0; past the batch,
    the row's own last particle)."""
    B, N = p.shape
    M = B * N
    if alpha < 1.0:
        q = p * alpha + (1.0 - alpha) / N
        q = q / q.sum(-1, keepdim=True)
        w = p / q
    else:
        w = torch.ones_like(p) / N
    tg = idx.clamp(max=M - 1)
    xo = x.reshape(M, -1)[tg]
    same = (tg // N) == torch.arange(B)[:, None]
    a = torch.where(same, w.reshape(M)[tg], torch.zeros_like(p))
    return xo, a / a.sum(-1, keepdim=True)


def _soft_check(ours, ref, what):
    ours, ref = ours.double().cpu(), ref.double().cpu()
    scale = float(ref.abs().max()) + 1e-30
    d = (ours - ref).abs()
    ok = d <= 1e-4 * ref.abs() + 2e-5 * scale
    assert bool(ok.all()), f"{what}: max |d| {float(d.max()):.3g} (scale {scale:.3g})"


@pytest.mark.parametrize("B,N,alpha,kind", [(4, 100, 0.5, "random"), (3, 1000, 0.5, "peaked"), (2, 7, 1.0, "random"),
                                            (5, 333, 0.3, "random"), (3, 1, 0.5, "random")])
def test_soft_resampler_backward_vs_autograd(B, N, alpha, kind):
    """dL/d(x, p) through resampler.soft_resampler under autograd (HIP backward) == float64
    autograd of the reference's formulas (resamplers.py:28-56) on the kernel's indices."""
    from resamplers.resamplers import soft_resampler
    g = torch.Generator().manual_seed(B * N)
    x = torch.randn(B, N, 2, generator=g) * 10
    logits = torch.randn(B, N, generator=g) * (6.0 if kind == "peaked" else 1.0)
    p = torch.softmax(logits, -1)
    gx_out, gw_out = torch.randn(B, N, 2, generator=g), torch.randn(B, N, generator=g)
    xd, pd = x.to(DEV).requires_grad_(True), p.to(DEV).requires_grad_(True)
    xo, wo, idx = soft_resampler(xd, pd, alpha, N)
    ((xo * gx_out.to(DEV)).sum() + (wo * gw_out.to(DEV)).sum()).backward()
    xr, pr = x.double().requires_grad_(True), p.double().requires_grad_(True)
    xo_r, wo_r = _soft_ref(xr, pr, idx.cpu(), alpha)
    ((xo_r * gx_out.double()).sum() + (wo_r * gw_out.double()).sum()).backward()
    _soft_check(xo.detach(), xo_r.detach(), "x'")
    _soft_check(wo.detach(), wo_r.detach(), "w'")
    _soft_check(xd.grad, xr.grad, "dL/dx")
    if pr.grad is None:  # hard resampling (alpha = 1): w = 1/N, no path to p
        assert pd.grad is None or bool((pd.grad == 0).all())
    else:
        _soft_check(pd.grad, pr.grad, "dL/dp")


def test_soft_resample_backward_edges():
    """Hand-made sorted indices with long runs, unreferenced sources and the out-of-range
    edge (into the next row, and past the last row)."""
    from nfdpf import ops
    B, N = 3, 6
    idx = torch.tensor([[0, 0, 0, 0, 3, 6],        # row 0: a run of 4, a skip, the edge into row 1
                        [6, 6, 9, 10, 11, 11],
                        [12, 12, 12, 12, 12, 18]])  # row 2: past the batch -> own particle 5
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, N, 2, generator=g)
    p = torch.softmax(torch.randn(B, N, generator=g), -1)
    gx_out, gw_out = torch.randn(B, N, 2, generator=g), torch.randn(B, N, generator=g)
    xr, pr = x.double().requires_grad_(True), p.double().requires_grad_(True)
    xo_r, wo_r = _soft_ref(xr, pr, idx, 0.5)
    ((xo_r * gx_out.double()).sum() + (wo_r * gw_out.double()).sum()).backward()
    gx, gp = ops.soft_resample_backward(p.to(DEV), idx.to(DEV), wo_r.detach().float().to(DEV), gx_out.to(DEV),
                                        gw_out.to(DEV), 0.5, 2)
    _soft_check(gx, xr.grad, "dL/dx")
    _soft_check(gp, pr.grad, "dL/dp")


@pytest.mark.parametrize("B,N,scale", [(4, 1000, 1.0), (3, 77, 20.0), (2, 1, 1.0)])
def test_cos_measurement_backward_vs_autograd(B, N, scale, monkeypatch):
    """measurement_model_cosine_distance under autograd (HIP backward) == float64 autograd of
    model/models.py:206-219 + et_distance utils.py:8-15 (d/d encodings, particles, encoder)."""
    import torch.nn as nn
    from model.models import measurement_model_cosine_distance
    from nfdpf import ops
    calls = []
    real = ops.cos_measurement_backward
    monkeypatch.setattr(ops, "cos_measurement_backward", lambda *a, **k: calls.append(1) or real(*a, **k))
    torch.manual_seed(B * 100 + N)
    pe = nn.Sequential(nn.Linear(2, 16), nn.ReLU(), nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 32))
    ref_pe = copy.deepcopy(pe).double()
    m = measurement_model_cosine_distance(pe.to(DEV))
    g = torch.Generator().manual_seed(N)
    enc = torch.randn(B, 32, generator=g)
    x = torch.randn(B, N, 2, generator=g) * scale
    gl = torch.randn(B, N, generator=g)
    encd, xd = enc.to(DEV).requires_grad_(True), x.to(DEV).requires_grad_(True)
    lik = m(encd, xd)
    (lik * gl.to(DEV)).sum().backward()
    assert len(calls) == 1, "the backward did not run through nfdpf_cos_measurement_backward"
    er, xr = enc.double().requires_grad_(True), x.double().requires_grad_(True)
    es = ref_pe(xr)
    eo = er[:, None, :].repeat(1, N, 1)
    cosd = 1.0 - (torch.nn.functional.normalize(eo, p=2, dim=-1, eps=1e-12) *
                  torch.nn.functional.normalize(es, p=2, dim=-1, eps=1e-12)).sum(-1)
    lr = (1 / (1e-7 + cosd)).log()
    (lr * gl.double()).sum().backward()
    _soft_check(lik.detach(), lr.detach(), "lik")
    _soft_check(xd.grad, xr.grad, "dL/dx")
    _soft_check(encd.grad, er.grad, "dL/denc")
    for (name, p), pr in zip(m.named_parameters(), ref_pe.parameters()):
        _soft_check(p.grad, pr.grad, f"dL/d{name}")


@pytest.mark.parametrize("B,N,scale", [(3, 500, 1.0), (2, 77, 10.0), (1, 1, 1.0)])
def test_nn_measurement_backward_vs_autograd(B, N, scale, monkeypatch):
    """measurement_model_NN under autograd (HIP: nfdpf_nn_measurement_backward + the encoder
    backward) == float64 autograd of model/models.py:221-235 with likelihood_est of :119-128
    (d/d encodings, particles and every parameter of both nets)."""
    import torch.nn as nn
    from model.models import measurement_model_NN
    from nfdpf import ops
    calls = []
    real = ops.nn_measurement_backward
    monkeypatch.setattr(ops, "nn_measurement_backward", lambda *a, **k: calls.append(1) or real(*a, **k))
    torch.manual_seed(B * 31 + N)
    pe = nn.Sequential(nn.Linear(2, 16), nn.ReLU(), nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 32))
    le = nn.Sequential(nn.Linear(64, 64), nn.ReLU(), nn.Linear(64, 64), nn.ReLU(), nn.Linear(64, 1), nn.Sigmoid())
    ref_pe, ref_le = copy.deepcopy(pe).double(), copy.deepcopy(le).double()
    m = measurement_model_NN(pe.to(DEV), le.to(DEV))
    g = torch.Generator().manual_seed(N + 1)
    enc = torch.randn(B, 32, generator=g)
    x = torch.randn(B, N, 2, generator=g) * scale
    gl = torch.randn(B, N, generator=g)
    encd, xd = enc.to(DEV).requires_grad_(True), x.to(DEV).requires_grad_(True)
    lik = m(encd, xd)
    (lik * gl.to(DEV)).sum().backward()
    assert len(calls) == 1, "the backward did not run through nfdpf_nn_measurement_backward"
    er, xr = enc.double().requires_grad_(True), x.double().requires_grad_(True)
    h = torch.cat([er[:, None, :].repeat(1, N, 1), ref_pe(xr)], dim=-1)
    lr = ref_le(h)[..., 0].log()
    (lr * gl.double()).sum().backward()
    _soft_check(lik.detach(), lr.detach(), "lik")
    _soft_check(xd.grad, xr.grad, "dL/dx")
    _soft_check(encd.grad, er.grad, "dL/denc")
    refs = list(ref_pe.parameters()) + list(ref_le.parameters())
    for (name, p), pr in zip(m.named_parameters(), refs):
        _soft_check(p.grad, pr.grad, f"dL/d{name}")


@pytest.mark.parametrize("B,N,std", [(3, 500, 0.3), (2, 70, 0.01)])
def test_crnvp_measurement_backward_vs_autograd(B, N, std, monkeypatch):
    """measurement_model_cnf under autograd (HIP: encoder forward/backward + stack backward)
    == float64 autograd of model/models.py:256-278 (d/d encodings, particles, every parameter)."""
    import torch.nn as nn
    from model.models import build_conditional_nf, measurement_model_cnf
    from nfdpf import ops
    calls = []
    real = ops.particle_encoder_backward
    monkeypatch.setattr(ops, "particle_encoder_backward", lambda *a, **k: calls.append(1) or real(*a, **k))
    torch.manual_seed(B * 7 + N)
    pe = nn.Sequential(nn.Linear(2, 16), nn.ReLU(), nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 32))
    cnf = build_conditional_nf(2, 32, 32, init_var=std, prior_std=2.5)
    ref_pe, ref_flows = copy.deepcopy(pe).double(), [copy.deepcopy(f).cpu() for f in cnf.flows]
    m = measurement_model_cnf(pe.to(DEV), cnf.to(DEV))
    g = torch.Generator().manual_seed(N)
    enc = torch.randn(B, 32, generator=g)
    x = torch.randn(B, N, 2, generator=g) * 5
    gl = torch.randn(B, N, generator=g)
    encd, xd = enc.to(DEV).requires_grad_(True), x.to(DEV).requires_grad_(True)
    lik = m(encd, xd)
    (lik * gl.to(DEV)).sum().backward()
    assert len(calls) == 1, "the backward did not run through the HIP encoder backward"
    am = (lik.detach() == 0).float().argmax(-1).cpu()
    refs = {}
    for dt in (torch.float32, torch.float64):
        rpe = copy.deepcopy(ref_pe).to(dt)
        rfl = [copy.deepcopy(f).to(dt) for f in ref_flows]
        er, xr = enc.to(dt).clone().requires_grad_(True), x.to(dt).clone().requires_grad_(True)
        es = rpe(xr).reshape(-1, 32)
        eo = er[:, None, :].repeat(1, N, 1).reshape(-1, 32)
        _, ld, lp = _ref_stack(rfl, eo, es, False, (0.0, 2.5), dt)
        u = (lp + ld).reshape(B, N)
        # the row max taken at OUR argmax (lik == 0 there exactly): at the reference init the
        # particles' u differ by less than fp32 resolves, and a different argmax routes the
        # -sum g elsewhere -- a valid gradient of a different (tied) max
        lr = u - u.gather(1, am[:, None])
        (lr * gl.to(dt)).sum().backward()
        refs[dt] = (u.detach(), lr.detach(), xr.grad, er.grad,
                    list(rpe.parameters()) + [p for f in rfl for p in f.parameters()])
    u64, lr64, gx64, ge64, p64 = refs[torch.float64]
    _, _, gx32, ge32, p32 = refs[torch.float32]
    # lik is a difference of two log-densities ~ -60: its fp32 error scales with |u|, not |lik|
    d = (lik.detach().double().cpu() - lr64).abs()
    assert float(d.max()) <= 1e-6 * float(u64.abs().max()) + 1e-6, f"lik: max |d| {float(d.max()):.3g}"
    # the gradients cancel strongly at the reference init (sum_n dL/du_n = 0 after the row max):
    # measured against 4x the float32 autograd's own error, max and mean (_check_tensor)
    # reference init (std 0.01): activations ~1e-3, where the fast tanh's absolute error is a
    # 1e-4 relative one (see _check_tensor); wide init: the default bounds
    rel = dict(rmax=5e-4, rmean=2e-4) if std < 0.1 else {}
    _check_tensor(xd.grad, gx32, gx64, "dL/dx", **rel)
    _check_tensor(encd.grad, ge32, ge64, "dL/denc", **rel)
    for (name, p), q32, q64 in zip(m.named_parameters(), p32, p64):
        _check_tensor(p.grad, q32.grad, q64.grad, f"dL/d{name}", **rel)
