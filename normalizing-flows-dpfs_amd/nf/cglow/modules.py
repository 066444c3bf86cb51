"""Conditional-GLOW building blocks (nf/cglow/modules.py of the reference): the parameter
structure and initialisation of each layer, so checkpoints keep their state_dict keys.
The forward computation of the whole model is a HIP kernel (nf/cglow/CGlowModel.py)."""
import numpy as np
import torch
import torch.nn as nn


class ActNorm(nn.Module):
    """bias, logs ~ N(0, 0.05^2) per channel (modules.py:8-35)."""

    def __init__(self, num_channels):
        super().__init__()
        size = [1, num_channels, 1, 1]
        self.register_parameter("bias", nn.Parameter(torch.normal(torch.zeros(*size), torch.ones(*size) * 0.05)))
        self.register_parameter("logs", nn.Parameter(torch.normal(torch.zeros(*size), torch.ones(*size) * 0.05)))


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


class Cond1x1Conv(nn.Module):
    """Per-sample invertible 1x1 conv with a y_channels^2 weight from x (modules.py:136-211)."""

    def __init__(self, x_size, x_hidden_channels, x_hidden_size, y_channels):
        super().__init__()
        self.x_Con, self.x_Linear = _cond_net(x_size, x_hidden_channels, x_hidden_size, y_channels * y_channels,
                                              LinearNorm)


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


class SqueezeLayer(nn.Module):
    def __init__(self, factor):
        super().__init__()
        self.factor = factor


class Split2d(nn.Module):
    def __init__(self, num_channels):
        super().__init__()
        self.conv = nn.Sequential(Conv2dZeros(num_channels // 2, num_channels), nn.Tanh())


class GaussianDiag:
    Log2PI = float(np.log(2 * np.pi))
