"""Conditional-GLOW building blocks (nf/cglow/modules.py of the reference): the parameter
structure and initialisation of each layer, so checkpoints keep their state_dict keys, and
each layer's forward / reverse in PyTorch.

The likelihood evaluation the DPF runs (CondGlowModel.forward, K = 1, L = 1) is ONE HIP kernel
(csrc/cglow.hip).  The PyTorch forwards below are not on that path: they are what autograd
differentiates when CGLOW is trained (nfdpf.autograd re-runs them on the saved inputs, the
forward value still being the kernel's) and the reverse (sampling) direction, which the DPF
never calls."""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


def split_feature(t, kind="split"):
    """Channel halves ("split") or even / odd channels ("cross") (nf/cglow/utils.py:5-13)."""
    C = t.size(1)
    if kind == "split":
        return t[:, :C // 2], t[:, C // 2:]
    return t[:, 0::2], t[:, 1::2]


class ActNorm(nn.Module):
    """bias, logs ~ N(0, 0.05^2) per channel; y = (x + bias) e^logs (modules.py:8-35)."""

    def __init__(self, num_channels):
        super().__init__()
        size = [1, num_channels, 1, 1]
        self.register_parameter("bias", nn.Parameter(torch.normal(torch.zeros(*size), torch.ones(*size) * 0.05)))
        self.register_parameter("logs", nn.Parameter(torch.normal(torch.zeros(*size), torch.ones(*size) * 0.05)))

    def forward(self, input, logdet=0, reverse=False):
        hw = input.size(2) * input.size(3)
        if not reverse:
            return (input + self.bias) * torch.exp(self.logs), logdet + torch.sum(self.logs) * hw
        return input * torch.exp(-self.logs) - self.bias, logdet - torch.sum(self.logs) * hw


class Conv2dZeros(nn.Conv2d):
    """3x3 'same' conv, weights N(0, 0.1^2) (modules.py:38-44)."""

    def __init__(self, in_channel, out_channel, kernel_size=(3, 3), stride=(1, 1)):
        super().__init__(in_channel, out_channel, kernel_size=kernel_size, stride=stride,
                         padding=(kernel_size[0] - 1) // 2)
        self.weight.data.normal_(mean=0.0, std=0.1)


class Conv2dResize(nn.Conv2d):
    """Strided conv mapping in_size -> out_size, zero weights (modules.py:47-61)."""

    def __init__(self, in_size, out_size):
        stride = [in_size[1] // out_size[1], in_size[2] // out_size[2]]
        k = [in_size[1] - (out_size[1] - 1) * stride[0], in_size[2] - (out_size[2] - 1) * stride[1]]
        super().__init__(in_channels=in_size[0], out_channels=out_size[0], kernel_size=k, stride=stride)
        self.weight.data.zero_()


class Conv2dNormy(nn.Conv2d):
    """Bias-free conv + ActNorm, weights N(0, 0.05^2) (modules.py:214-230)."""

    def __init__(self, in_channels, out_channels, kernel_size=(3, 3), stride=(1, 1)):
        super().__init__(in_channels, out_channels, kernel_size, stride,
                         [(kernel_size[0] - 1) // 2, (kernel_size[1] - 1) // 2], bias=False)
        self.weight.data.normal_(mean=0.0, std=0.05)
        self.actnorm = ActNorm(out_channels)

    def forward(self, input):
        return self.actnorm(super().forward(input))[0]


class Conv2dZerosy(nn.Conv2d):
    """Zero-initialised conv with learnt output scale exp(3 logs) (modules.py:233-253)."""

    def __init__(self, in_channels, out_channels, kernel_size=(3, 3), stride=(1, 1)):
        super().__init__(in_channels, out_channels, kernel_size, stride,
                         [(kernel_size[0] - 1) // 2, (kernel_size[1] - 1) // 2])
        self.logscale_factor = 3.0
        self.register_parameter("logs", nn.Parameter(torch.zeros(out_channels, 1, 1)))
        self.register_parameter("newbias", nn.Parameter(torch.zeros(out_channels, 1, 1)))
        self.weight.data.zero_()
        self.bias.data.zero_()

    def forward(self, input):
        return (super().forward(input) + self.newbias) * torch.exp(self.logs * self.logscale_factor)


class LinearZeros(nn.Linear):
    def __init__(self, in_channels, out_channels):
        super().__init__(in_channels, out_channels)
        self.weight.data.zero_()
        self.bias.data.zero_()


class LinearNorm(nn.Linear):
    def __init__(self, in_channels, out_channels):
        super().__init__(in_channels, out_channels)
        self.weight.data.normal_(mean=0.0, std=0.1)
        self.bias.data.normal_(mean=0.0, std=0.1)


def _cond_net(x_size, hidden_channels, hidden_size, out_features, last):
    C, H, W = x_size
    con = nn.Sequential(
        Conv2dResize([C, H, W], [hidden_channels, H // 2, W // 2]), nn.ReLU(),
        Conv2dResize([hidden_channels, H // 2, W // 2], [hidden_channels, H // 4, W // 4]), nn.ReLU(),
        Conv2dResize([hidden_channels, H // 4, W // 4], [hidden_channels, H // 8, W // 8]), nn.ReLU())
    lin = nn.Sequential(LinearZeros(hidden_channels * H * W // 64, hidden_size), nn.ReLU(),
                        LinearZeros(hidden_size, hidden_size), nn.ReLU(), last(hidden_size, out_features),
                        nn.Tanh())
    return con, lin


class CondActNorm(nn.Module):
    """Per-sample actnorm whose (logs, bias) come from the conditioning x (modules.py:76-132)."""

    def __init__(self, x_size, y_channels, x_hidden_channels, x_hidden_size):
        super().__init__()
        self.x_Con, self.x_Linear = _cond_net(x_size, x_hidden_channels, x_hidden_size, 2 * y_channels,
                                              LinearZeros)

    def forward(self, x, y, logdet=0, reverse=False):
        B = x.size(0)
        h = self.x_Linear(self.x_Con(x).view(B, -1)).view(B, -1, 1, 1)
        logs, bias = split_feature(h)
        hw = y.size(2) * y.size(3)
        dld = hw * torch.sum(logs, dim=(1, 2, 3))
        if not reverse:
            return (y + bias) * torch.exp(logs), logdet + dld
        return y * torch.exp(-logs) - bias, logdet - dld


class Cond1x1Conv(nn.Module):
    """Per-sample invertible 1x1 conv with a y_channels^2 weight from x (modules.py:136-211)."""

    def __init__(self, x_size, x_hidden_channels, x_hidden_size, y_channels):
        super().__init__()
        self.x_Con, self.x_Linear = _cond_net(x_size, x_hidden_channels, x_hidden_size, y_channels * y_channels,
                                              LinearNorm)

    def get_weight(self, x, y, reverse):
        B, C = x.size(0), y.size(1)
        w = self.x_Linear(self.x_Con(x).view(B, -1)).view(B, C, C)
        dld = torch.slogdet(w)[1] * (y.size(2) * y.size(3))
        if reverse:
            w = torch.inverse(w.double()).float()
        return w, dld

    def forward(self, x, y, logdet=None, reverse=False):
        w, dld = self.get_weight(x, y, reverse)
        z = torch.einsum("boc,bchw->bohw", w, y)  # the grouped 1x1 conv2d of :195-209
        if logdet is not None:
            logdet = logdet - dld if reverse else logdet + dld
        return z, logdet


class CondAffineCoupling(nn.Module):
    """Affine coupling conditioned on resized x (modules.py:258-303)."""

    def __init__(self, x_size, y_size, hidden_channels):
        super().__init__()
        self.resize_x = nn.Sequential(Conv2dZeros(x_size[0], 16), nn.ReLU(),
                                      Conv2dResize((16, x_size[1], x_size[2]), out_size=y_size), nn.ReLU(),
                                      Conv2dZeros(y_size[0], y_size[0]), nn.ReLU())
        self.f = nn.Sequential(Conv2dNormy(y_size[0] * 2, hidden_channels), nn.ReLU(),
                               Conv2dNormy(hidden_channels, hidden_channels, kernel_size=[1, 1]), nn.ReLU(),
                               Conv2dZerosy(hidden_channels, 2 * y_size[0]), nn.Tanh())

    def forward(self, x, y, logdet=0.0, reverse=False):
        z1, z2 = split_feature(y, "split")
        h = self.f(torch.cat((self.resize_x(x), z1), dim=1))
        shift, scale = split_feature(h, "cross")
        scale = torch.sigmoid(scale + 2.0)
        dld = torch.sum(torch.log(scale), dim=(1, 2, 3))
        if not reverse:
            return torch.cat((z1, (z2 + shift) * scale), dim=1), dld + logdet
        return torch.cat((z1, z2 / scale - shift), dim=1), -dld + logdet


class SqueezeLayer(nn.Module):
    def __init__(self, factor):
        super().__init__()
        self.factor = factor

    def forward(self, input, logdet=None, reverse=False):
        f = self.factor
        if f == 1:
            return input, logdet
        B, C, H, W = input.shape
        if not reverse:  # (C, H, W) -> (C f^2, H/f, W/f), channel = c f^2 + a f + b (modules.py:319-328)
            x = input.view(B, C, H // f, f, W // f, f).permute(0, 1, 3, 5, 2, 4)
            return x.reshape(B, C * f * f, H // f, W // f), logdet
        x = input.view(B, C // (f * f), f, f, H, W).permute(0, 1, 4, 2, 5, 3)
        return x.reshape(B, C // (f * f), H * f, W * f), logdet


class GaussianDiag:
    Log2PI = float(np.log(2 * np.pi))

    @staticmethod
    def likelihood(mean, logs, x):
        return -0.5 * (logs * 2.0 + ((x - mean) ** 2.0) / torch.exp(logs * 2.0) + GaussianDiag.Log2PI)

    @staticmethod
    def logp(mean, logs, x):
        return torch.sum(GaussianDiag.likelihood(mean, logs, x), dim=(1, 2, 3))

    @staticmethod
    def sample(mean, logs, eps_std=None):
        eps = torch.normal(mean=torch.zeros_like(mean), std=torch.ones_like(logs) * (eps_std or 1))
        return mean + torch.exp(logs) * eps

    @staticmethod
    def batchsample(batchsize, mean, logs, eps_std=None):
        return torch.cat([GaussianDiag.sample(mean, logs, eps_std) for _ in range(batchsize)], dim=0)


class Split2d(nn.Module):
    def __init__(self, num_channels):
        super().__init__()
        self.conv = nn.Sequential(Conv2dZeros(num_channels // 2, num_channels), nn.Tanh())

    def split2d_prior(self, z):
        return split_feature(self.conv(z), "cross")

    def forward(self, input, logdet=0.0, reverse=False, eps_std=None):
        if not reverse:
            z1, z2 = split_feature(input, "split")
            mean, logs = self.split2d_prior(z1)
            return z1, GaussianDiag.logp(mean, logs, z2) + logdet
        mean, logs = self.split2d_prior(input)
        return torch.cat((input, GaussianDiag.sample(mean, logs, eps_std)), dim=1), logdet
