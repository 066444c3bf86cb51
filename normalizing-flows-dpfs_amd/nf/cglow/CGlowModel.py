"""Conditional GLOW (nf/cglow/CGlowModel.py of the reference): same modules and state_dict
keys (flow.layers.{k}...., new_mean, new_logs).  The likelihood evaluation (squeeze ->
K x [cond-actnorm, cond-1x1conv with a per-particle 12x12 slogdet, cond-affine coupling]
-> Gaussian log-prob) runs on the HIP device (nfdpf; BASELINE config 5)."""
import torch
import torch.nn as nn

from nf.cglow import modules
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

    def forward(self, x=0.0, y=None, eps_std=1.0, reverse=False):
        raise NfdpfError("the conditional-GLOW measurement kernel (BASELINE config 5) is not in this build yet")
