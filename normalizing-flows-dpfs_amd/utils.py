"""utils.py of the reference: densities, weight normalisation, initialisation, checkpoints.

``normalize_log_probs`` runs the HIP kernel on device tensors (utils.py:39-44); the
initialisation draws from the CPU generator exactly as the reference does (utils.py:46-62)
-- the fused filter uses the device-RNG kernel instead unless run in parity mode.
"""
import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


def et_distance(encoding_input, e_t):
    """Cosine distance after L2 normalisation (utils.py:8-15)."""
    a = F.normalize(encoding_input, p=2, dim=-1, eps=1e-12)
    b = F.normalize(e_t, p=2, dim=-1, eps=1e-12)
    return 1.0 - torch.sum(a * b, dim=-1)


class compute_normal_density(nn.Module):
    """Isotropic Gaussian log-density of (pos, vel) noise (utils.py:17-37)."""

    def __init__(self, pos_noise=1.0, vel_noise=1.0):
        super().__init__()
        self.pos_noise = pos_noise
        self.vel_noise = vel_noise

    def forward(self, noise, std_pos=None, std_vel=None):
        sp = torch.tensor(self.pos_noise if std_pos is None else std_pos)
        sv = torch.tensor(self.vel_noise if std_vel is None else std_vel)
        log_c = -0.5 * torch.log(torch.tensor(2 * np.pi))
        d = noise.shape[-1]
        pos, vel = noise[:, :, :2], noise[:, :, 2:]
        return (d * log_c - 2 * torch.log(sp) - torch.sum(pos ** 2 / (2 * sp ** 2), dim=-1)
                + -(d - 2) * torch.log(sv) - torch.sum(vel ** 2 / (2 * sv ** 2), dim=-1))


def normalize_log_probs(probs):
    """exp(p - rowmax) / rowsum (utils.py:39-44); HIP kernel on device tensors."""
    if probs.is_cuda and not (torch.is_grad_enabled() and probs.requires_grad):
        from nfdpf import ops
        return ops.normalize_log_probs(probs)[0]
    e = (probs - probs.max(dim=1, keepdim=True)[0]).exp()
    return e / torch.sum(e, dim=1, keepdim=True)


def particle_initialization(start_state, width, num_particles, state_dim=2, init_with_true_state=False):
    """Uniform on [-width/2, width/2)^2 (or start + N(0,1)); log-weights log(1/N) (utils.py:46-62)."""
    B = start_state.shape[0]
    dev = start_state.device
    if init_with_true_state:
        x = start_state[:, None, :].repeat(1, num_particles, 1) + \
            torch.randn(B, num_particles, state_dim).to(dev)
    else:
        hi, lo = width / 2.0, -width / 2.0
        x = torch.tensor(hi - lo).to(dev) * torch.rand(B, num_particles, 2).to(dev) + torch.tensor(lo).to(dev)
        torch.randn(B, num_particles, 2)  # the reference draws (and discards) initial velocities
    return x, torch.log(torch.ones([B, num_particles]).to(dev) / num_particles)


def freeze_model(model):
    for p in model.parameters():
        p.requires_grad = False


def unfreeze_model(model):
    for p in model.parameters():
        p.requires_grad = True


def checkpoint_state(model, epoch):
    """{model, model_optim, model_optim_scheduler, epoch} (utils.py:72-79)."""
    return {"model": model.state_dict(), "model_optim": model.optim.state_dict(),
            "model_optim_scheduler": model.optim_scheduler.state_dict(), "epoch": epoch}


def load_model(model, ckpt_e2e):
    model.load_state_dict(ckpt_e2e["model"])
    model.optim.load_state_dict(ckpt_e2e["model_optim"])
    model.optim_scheduler.load_state_dict(ckpt_e2e["model_optim_scheduler"])
