"""The split suffix of a flow blob (nfdpf.pack.split_flow_tensors, csrc/split.hpp) read the
way the kernel reads it reproduces each coupling net of the module (CPU, numpy)."""
import numpy as np
import torch

from nf.flows import RealNVP_cond
from nfdpf.pack import filter_flow_tensors, flows_tensors, split_flow_tensors, splittable


def _net_split(w, u, cb):
    """csrc/split.hpp net_split on one particle: w = the net's 90 floats, cb = its 8 folded
    first-layer biases; float64 here (layout check, not rounding)."""
    w1 = w[0:8].reshape(4, 2)
    w2 = w[8:72].reshape(4, 8, 2)
    b2 = w[72:80].reshape(4, 2)
    w3 = w[80:88].reshape(4, 2)
    b3 = w[88]
    h = np.tanh(w1 * u + cb.reshape(4, 2)).reshape(8)
    g = np.tanh(np.einsum("mkp,k->mp", w2, h) + b2)
    return float((w3 * g).sum() + b3)


def test_split_suffix_reproduces_nets():
    torch.manual_seed(0)
    O = 36
    flows = [RealNVP_cond(dim=2, hidden_dim=8, obser_dim=O) for _ in range(2)]
    for f in flows:
        for p in f.parameters():
            p.data.normal_(0, 0.3)
    assert splittable(flows)
    suffix = torch.cat([t.reshape(-1) for t in split_flow_tensors(flows)]).detach().double().numpy()
    assert suffix.size == 2 * 4 * 90
    full = torch.cat([t.reshape(-1) for t in filter_flow_tensors(flows)])
    prefix = torch.cat([t.reshape(-1) for t in flows_tensors(flows)])
    assert full.numel() == prefix.numel() + suffix.size
    u = 0.7
    ctx = torch.randn(O, dtype=torch.float64)
    for fi, f in enumerate(flows):
        for ni, net in enumerate((f.t1, f.s1, f.t2, f.s2)):
            w = suffix[(fi * 4 + ni) * 90:(fi * 4 + ni + 1) * 90]
            (w1, b1), (w2, b2), (w3, b3) = [(m.weight.detach().double().numpy(), m.bias.detach().double().numpy())
                                            for m in net.network.modules() if isinstance(m, torch.nn.Linear)]
            c = ctx.numpy()
            cb = w1[:, 1:] @ c + b1
            x = np.concatenate([[u], c])
            ref = float((w3 @ np.tanh(w2 @ np.tanh(w1 @ x + b1) + b2) + b3)[0])
            assert abs(_net_split(w, u, cb) - ref) < 1e-9


def test_maf_stack_not_split():
    from nf.flows import MAF
    assert not splittable([MAF(dim=2, hidden_dim=8)])


def test_blob_grad_scatter_matches_autograd_of_pack():
    """The HIP backward returns d/d(blob); nfdpf.pack.blob_grad_to_params maps it back to the
    parameters by one scatter -- equal to differentiating the packing itself."""
    import torch
    from nf.flows import RealNVP_cond, RealNVP
    from nfdpf.pack import blob_grad_to_params, flows_tensors
    torch.manual_seed(0)
    for fl in ([RealNVP_cond(2, 8, obser_dim=36) for _ in range(2)], [RealNVP(32, 8) for _ in range(3)]):
        for f in fl:
            f.zero_initialization(0.3)
        params = [p for f in fl for p in f.parameters()]
        flat = torch.cat([t.reshape(-1) for t in flows_tensors(fl)])
        assert flat.numel() == sum(p.numel() for p in params)
        g = torch.randn_like(flat)
        ref = torch.autograd.grad(flat, params, g)
        ours = blob_grad_to_params(fl[0], "t", params, lambda get: flows_tensors(fl, get), g)
        assert all(torch.equal(a, b) for a, b in zip(ref, ours))


def test_hip_backward_declines_unsupported_stacks():
    """CouplingStack.hip_backward returns None (autograd then differentiates the PyTorch
    restatement) for what nfdpf_cond_stack_backward is not built for -- before any device call."""
    import torch
    from nf.flows import CouplingStack, RealNVP_cond
    wide = [RealNVP_cond(2, 16, obser_dim=4)]             # hidden 16
    many = [RealNVP_cond(2, 8, obser_dim=4) for _ in range(5)]  # 5 flows
    x, c = torch.zeros(3, 2), torch.zeros(3, 4)
    g = (torch.zeros(3, 2), torch.zeros(3))
    assert CouplingStack(wide[0], wide, 2, 4, 16, False).hip_backward(x, c, g) is None
    assert CouplingStack(many[0], many, 2, 4, 8, True).hip_backward(x, c, g) is None
    # a broadcast (per-batch) condition is not the per-row layout the kernel takes
    one = [RealNVP_cond(2, 8, obser_dim=4)]
    assert CouplingStack(one[0], one, 2, 4, 8, False).hip_backward(x, torch.zeros(1, 4), g) is None
