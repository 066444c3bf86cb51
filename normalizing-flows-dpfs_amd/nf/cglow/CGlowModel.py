"""Conditional GLOW (nf/cglow/CGlowModel.py of the reference): same modules and state_dict
keys (flow.layers.{k}...., new_mean, new_logs), same forward / reverse API.

``CondGlowModel.forward(x, y)`` -- the likelihood the DPF's CGLOW measurement evaluates (squeeze
-> K x [cond-actnorm, cond-1x1 conv with a per-sample 12x12 slogdet, cond-affine coupling] ->
Gaussian log-prob, CGlowModel.py:167-176) -- runs as one HIP kernel (csrc/cglow.hip,
nfdpf_cglow_flow) for the configuration the reference's flags give (K = 1, L = 1, x_size =
y_size = (3, 8, 8), learn_top off) and returns the reference's (z, nll).  Under autograd its
backward differentiates ``torch_forward``, a PyTorch restatement of the same math run on the
saved inputs (nfdpf.autograd; the forward value is the kernel's).  ``reverse=True`` (sampling;
the DPF never calls it) runs the layers' PyTorch reverse."""
import numpy as np
import torch
import torch.nn as nn

from nf.cglow import modules
from nfdpf import autograd as _ag
from nfdpf._lib import NfdpfError


class CondGlowStep(nn.Module):
    def __init__(self, x_size, y_size, x_hidden_channels, x_hidden_size, y_hidden_channels):
        super().__init__()
        self.actnorm = modules.CondActNorm(x_size=x_size, y_channels=y_size[0], x_hidden_channels=x_hidden_channels,
                                           x_hidden_size=x_hidden_size)
        self.invconv = modules.Cond1x1Conv(x_size=x_size, x_hidden_channels=x_hidden_channels,
                                           x_hidden_size=x_hidden_size, y_channels=y_size[0])
        self.affine = modules.CondAffineCoupling(x_size=x_size, y_size=[y_size[0] // 2, y_size[1], y_size[2]],
                                                 hidden_channels=y_hidden_channels)

    def forward(self, x, y, logdet=None, reverse=False):
        """actnorm -> 1x1 conv -> affine coupling, or the reverse chain (CGlowModel.py:24-54)."""
        stages = (self.actnorm, self.invconv, self.affine)
        for st in (reversed(stages) if reverse else stages):
            y, logdet = st(x, y, logdet, reverse=reverse)
        return y, logdet


class CondGlow(nn.Module):
    def __init__(self, x_size, y_size, x_hidden_channels, x_hidden_size, y_hidden_channels, K, L):
        super().__init__()
        self.layers = nn.ModuleList()
        self.output_shapes = []
        self.K, self.L = K, L
        C, H, W = y_size
        for level in range(L):
            C, H, W = C * 4, H // 2, W // 2
            self.layers.append(modules.SqueezeLayer(factor=2))
            self.output_shapes.append([-1, C, H, W])
            for _ in range(K):
                self.layers.append(CondGlowStep(x_size, [C, H, W], x_hidden_channels, x_hidden_size,
                                                y_hidden_channels))
                self.output_shapes.append([-1, C, H, W])
            if level < L - 1:
                self.layers.append(modules.Split2d(num_channels=C))
                self.output_shapes.append([-1, C // 2, H, W])
                C = C // 2

    def forward(self, x, y, logdet=0.0, reverse=False, eps_std=1.0):
        """encode (squeeze / steps / split in order) or decode (reversed), CGlowModel.py:98-120."""
        if not reverse:
            for layer in self.layers:
                if isinstance(layer, (modules.Split2d, modules.SqueezeLayer)):
                    y, logdet = layer(y, logdet, reverse=False)
                else:
                    y, logdet = layer(x, y, logdet, reverse=False)
            return y, logdet
        for layer in reversed(self.layers):
            if isinstance(layer, modules.Split2d):
                y, logdet = layer(y, logdet=logdet, reverse=True, eps_std=eps_std)
            elif isinstance(layer, modules.SqueezeLayer):
                y, logdet = layer(y, logdet=logdet, reverse=True)
            else:
                y, logdet = layer(x, y, logdet=logdet, reverse=True)
        return y, logdet


class _FlowRunner:
    """nfdpf.autograd runner: the HIP kernel forward, the PyTorch restatement for backward."""

    def __init__(self, model):
        self.model = model

    def hip(self, x, y):
        from nfdpf import ops
        from nfdpf.pack import blob, cglow_tensors
        m = self.model
        glow = blob(m, "glow", m, lambda: cglow_tensors(m), x.device)
        return ops.cglow_flow(glow, x, y)

    def torch(self, x, y):
        return self.model.torch_forward(x, y)

    def hip_backward(self, x, y, gouts):
        """d/d(x, y, parameters) on nfdpf_cglow_flow_backward (csrc/cglow_bwd.hip)."""
        from nfdpf import ops
        from nfdpf.pack import blob, blob_param_grads, cglow_tensors
        m = self.model
        glow = blob(m, "glow", m, lambda: cglow_tensors(m), x.device)
        g_z, g_nll = gouts
        gx, gy, g_glow = ops.cglow_flow_backward(glow, x, y, g_z, g_nll)
        res = blob_param_grads(m, "glow_grad", list(m.parameters()), lambda get: cglow_tensors(m, get), g_glow)
        return (gx, gy), res


class CondGlowModel(nn.Module):
    def __init__(self, args):
        super().__init__()
        self.flow = CondGlow(x_size=args.x_size, y_size=args.y_size, x_hidden_channels=args.x_hidden_channels,
                             x_hidden_size=args.x_hidden_size, y_hidden_channels=args.y_hidden_channels,
                             K=args.flow_depth, L=args.num_levels)
        self.learn_top = args.learn_top
        shp = self.flow.output_shapes[-1]
        self.register_parameter("new_mean", nn.Parameter(torch.zeros([1, shp[1], shp[2], shp[3]])))
        self.register_parameter("new_logs", nn.Parameter(torch.zeros([1, shp[1], shp[2], shp[3]])))
        self.n_bins = args.y_bins

    def prior(self):
        """(mean, logs) of the top Gaussian: learnt when learn_top, else zeros (:161-166)."""
        if self.learn_top:
            return self.new_mean, self.new_logs
        return torch.zeros_like(self.new_mean), torch.zeros_like(self.new_mean)

    def kernel_supported(self) -> bool:
        """The configuration csrc/cglow.hip is built for: the reference's defaults
        (arguments.py:61-70) K = 1, L = 1, 3x8x8 x and y, hidden 8 / 16 / 8, learn_top off."""
        f = self.flow
        return (f.K == 1 and f.L == 1 and not self.learn_top and float(self.n_bins) == 256.0
                and list(f.output_shapes[-1][1:]) == [12, 4, 4])

    def forward(self, x=0.0, y=None, eps_std=1.0, reverse=False):
        """reverse=False: (z, nll) of y given the condition x (CGlowModel.py:167-176), on the
        HIP kernel.  reverse=True: a sample (or the inverse of a given y) and its log-det
        (:178-184), PyTorch (off the DPF path)."""
        if reverse:
            with torch.no_grad():
                mean, logs = self.prior()
                if y is None:
                    y = modules.GaussianDiag.batchsample(x.size(0), mean, logs, eps_std)
                return self.flow(x, y, eps_std=eps_std, reverse=True)
        if not self.kernel_supported():
            raise NfdpfError("CondGlowModel.forward: the HIP kernel is built for K = 1, L = 1, 3x8x8 inputs, "
                             "learn_top off and 256 bins (the reference's defaults)")
        z, nll = _ag.apply(_FlowRunner(self), (x.float().contiguous(), y.float().contiguous()),
                           list(self.parameters()))
        return z, nll

    def torch_forward(self, x, y):
        """The PyTorch restatement of forward (CGlowModel.py:167-176) -- the backward of the
        kernel path differentiates this on the saved inputs."""
        dims = y.size(1) * y.size(2) * y.size(3)
        logdet = torch.zeros_like(y[:, 0, 0, 0]) + float(-np.log(self.n_bins) * dims)
        z, obj = self.flow(x, y, logdet=logdet, reverse=False)
        mean, logs = self.prior()
        obj = obj + modules.GaussianDiag.logp(mean, logs, z)
        return z, -obj / float(np.log(2.0) * dims)
