"""Small frame encoder / decoder for the DPF.forward / DPF.testing fixtures.

The reference's CNN encoder and decoder (model/models.py:10-117) hold ~1.6 M parameters --
too large for a committed fixture -- and are per-image work outside the hot path (SURVEY.md
§2).  The forward-path fixtures (tests/golden/gen_golden.py gen_forward) swap both for these
modules, in the reference's DPF and in ours alike, so DPF.forward / .testing run end to end on
128x128 frames with a few hundred parameters."""
import torch
from torch import nn


class TinyEncoder(nn.Module):
    """(B, 3, 128, 128) -> (B, H): 32x32 average pooling, then a Linear."""

    def __init__(self, H):
        super().__init__()
        self.pool = nn.AvgPool2d(32)
        self.lin = nn.Linear(48, H)

    def forward(self, x):
        return self.lin(self.pool(x).flatten(1))


class TinyDecoder(nn.Module):
    """(B, H) -> (B, 3, 128, 128): a Linear to a 3x4x4 sigmoid image, upsampled 32x."""

    def __init__(self, H):
        super().__init__()
        self.lin = nn.Linear(H, 48)

    def forward(self, z):
        return torch.sigmoid(self.lin(z)).view(-1, 3, 4, 4).repeat_interleave(32, 2).repeat_interleave(32, 3)
