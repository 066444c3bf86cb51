"""losses.py of the reference: RMSE (the benchmark's accuracy metric), AE and
pseudo-likelihood losses (training)."""
import numpy as np
import torch
from torch import nn


def autoencoder_loss(image, train, encoder, decoder):
    """MSE of the frame auto-encoder (losses.py:5-16)."""
    b, s, c, h, w = image.shape
    x = image.reshape(b * s, c, h, w)
    return nn.MSELoss()(decoder(encoder(x)), x)


def supervised_loss(particle_list, particle_weight_list, true_state, mask, train, labeledRatio=1.0):
    """Weighted-mean prediction and RMSE against the true position (losses.py:18-31)."""
    prediction = torch.sum(particle_list * particle_weight_list[:, :, :, None], dim=2)
    err2 = (prediction - true_state[:, :, :2]) ** 2
    if not train:
        return torch.sqrt(torch.mean(err2)), prediction
    if labeledRatio > 0:
        return torch.sqrt(torch.mean(mask[:, :, None] * err2) / labeledRatio), prediction
    return 0


def _block_density(weights, lik, index, prior_terms, block_len):
    """Shared block recursion of compute_block_density(_nf) (losses.py:37-68, 75-105)."""
    B, T, N = weights.shape
    Q, nb, eta = 0, 0, 0
    for k in range(T):
        if (k + 1) % block_len:
            continue
        idx = None
        for j in range(k, k - block_len, -1):
            if j == k:
                idx = index[:, j, :]
                l, pr = lik[:, j, :], prior_terms(j, None)
            else:
                l = lik[:, j, :].reshape(B * N)[idx]
                pr = prior_terms(j, idx)
                idx = index[:, j, :].reshape(B * N)[idx]
            eta = eta + pr + l
        Q = Q + torch.sum(weights[:, k, :] * eta, dim=-1)
        nb += 1
    return Q / nb


def _block_density_nf_torch(particle_weight_list, likelihood_list, index_list, prior_list, block_len):
    B, T, N = particle_weight_list.shape

    def prior_terms(j, idx):
        p = prior_list[:, j, :]
        return p if idx is None else p.reshape(B * N)[idx]
    return _block_density(particle_weight_list, likelihood_list, index_list, prior_terms, block_len)


class _PseudoLikNf(torch.autograd.Function):
    """compute_block_density_nf on the HIP kernels (csrc/pseudo_lik.hip): the ancestry walks
    and the row sums forward, the chain scatter backward; a non-monotone ancestor map (never
    produced by the filter) is differentiated through the PyTorch restatement instead."""

    @staticmethod
    def forward(ctx, w, lik, prior, index, block_len):
        from nfdpf import ops
        ctx.save_for_backward(w, lik, prior, index)
        ctx.block_len = block_len
        return ops.pseudo_lik_forward(w, lik, prior, index, block_len).to(w.dtype)

    @staticmethod
    def backward(ctx, gQ):
        from nfdpf import ops
        w, lik, prior, index = ctx.saved_tensors
        if ops.pseudo_lik_monotone(index):
            gw, gl, gp = ops.pseudo_lik_backward(w, lik, prior, index, ctx.block_len, gQ.float())
        else:
            with torch.enable_grad():
                leaves = [t.detach().requires_grad_(True) for t in (w, lik, prior)]
                Q = _block_density_nf_torch(leaves[0], leaves[1], index, leaves[2], ctx.block_len)
                gw, gl, gp = torch.autograd.grad(Q, leaves, gQ)
        need = ctx.needs_input_grad
        return (gw if need[0] else None, gl if need[1] else None, gp if need[2] else None, None, None)


def compute_block_density_nf(particle_weight_list, noise_list, likelihood_list, index_list, jac_list, prior_list,
                             block_len=10):
    """losses.py:37-68 (the reference's positional accumulation of eta across blocks kept).  On
    the HIP device: the pseudo_lik kernels; elsewhere the PyTorch restatement."""
    w = particle_weight_list
    if w.is_cuda and w.shape[1] // block_len > 0 and w.shape[2] <= 12288:
        return _PseudoLikNf.apply(w, likelihood_list, prior_list, index_list, block_len)
    return _block_density_nf_torch(w, likelihood_list, index_list, prior_list, block_len)


def pseudolikelihood_loss_nf(particle_weight_list, noise_list, likelihood_list, index_list, jac_list, prior_list,
                             block_len=10):
    return -1. * torch.mean(compute_block_density_nf(particle_weight_list, noise_list, likelihood_list, index_list,
                                                     jac_list, prior_list, block_len))


def compute_block_density(particle_weight_list, noise_list, likelihood_list, index_list, block_len=10,
                          std_pos=1.0, std_vel=1.0):
    B, T, N = particle_weight_list.shape
    log_c = -0.5 * torch.log(torch.tensor(2 * np.pi))

    def gauss(v, s):
        return 2 * log_c - 2 * torch.log(torch.tensor(s)) - torch.sum(v ** 2 / (2 * torch.tensor(s) ** 2), dim=-1)

    def prior_terms(j, idx):
        pos = noise_list[:, j, :, :2]
        vel = noise_list[:, j, :, 2:]
        if idx is not None:
            pos = pos.reshape(B * N, -1)[idx, :]
            vel = vel.reshape(B * N, -1)[idx, :]
        return gauss(pos, std_pos) + gauss(vel, std_vel)
    return _block_density(particle_weight_list, likelihood_list, index_list, prior_terms, block_len)


def pseudolikelihood_loss(particle_weight_list, noise_list, likelihood_list, index_list, block_len=10, std_pos=1.0,
                          std_vel=1.0):
    return -1. * torch.mean(compute_block_density(particle_weight_list, noise_list, likelihood_list, index_list,
                                                  block_len, std_pos, std_vel))
