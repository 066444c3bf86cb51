"""Pack nn.Module parameters into the flat fp32 blobs the kernels read (include/nfdpf.h).

Blobs are cached per module and rebuilt only when a parameter changes (tensor version
counter or storage), so an optimizer step is picked up and an unchanged model pays nothing.
"""
from __future__ import annotations

import torch
import torch.nn as nn


def _linears(seq: nn.Module):
    return [m for m in seq.modules() if isinstance(m, nn.Linear)]


def fcnn_tensors(fcnn: nn.Module):
    """FCNN(in, out, H): W1 b1 W2 b2 W3 b3 (nf/flows.py:101-114)."""
    out = []
    for lin in _linears(fcnn.network):
        out += [lin.weight, lin.bias]
    return out


def coupling_net_tensors(net: nn.Module, half: int):
    """One coupling net FCNN(half + O, half, H) (nf/flows.py:101-114, 183-190) in the kernel
    layout: core [W1[:, :half], W2, b2, W3, b3] then context [W1[:, half:], b1], so the
    per-particle path reads the core at compile-time offsets and the context columns are
    folded into a bias once per row (csrc/flows.hpp)."""
    l1, l2, l3 = _linears(net.network)
    w1 = l1.weight
    return [w1[:, :half], l2.weight, l2.bias, l3.weight, l3.bias, w1[:, half:], l1.bias]


def realnvp_tensors(flow: nn.Module):
    """RealNVP / RealNVP_cond flow: nets t1, s1, t2, s2 (nf/flows.py:123-129, 183-190)."""
    out = []
    for net in (flow.t1, flow.s1, flow.t2, flow.s2):
        out += coupling_net_tensors(net, flow.dim // 2)
    return out


def maf_tensors(flow: nn.Module):
    """MAF flow: initial_param[2] then FCNN(i, 2, H) for i = 1..dim-1 (nf/flows.py:247-254)."""
    out = [flow.initial_param]
    for layer in flow.layers:
        out += fcnn_tensors(layer)
    return out


def mlp_tensors(seq: nn.Module):
    """nn.Sequential of Linear layers (+activations): W, b per Linear."""
    out = []
    for lin in _linears(seq):
        out += [lin.weight, lin.bias]
    return out


def flows_tensors(flows):
    out = []
    for f in flows:
        if hasattr(f, "initial_param"):
            out += maf_tensors(f)
        else:
            out += realnvp_tensors(f)
    return out


class BlobCache:
    """Flat fp32 copy of a parameter list on one device, refreshed on change."""

    def __init__(self):
        self._key = None
        self._blob = None

    def get(self, tensors, device) -> torch.Tensor:
        key = (str(device),) + tuple((t.data_ptr(), t._version, t.numel()) for t in tensors)
        if key != self._key:
            with torch.no_grad():
                flat = [t.detach().reshape(-1).to(device=device, dtype=torch.float32) for t in tensors]
                self._blob = torch.cat(flat).contiguous() if flat else torch.zeros(1, device=device)
            self._key = key
        return self._blob


def blob(owner: nn.Module, name: str, tensors, device) -> torch.Tensor:
    """Cached blob stored on ``owner`` under ``name`` (not a registered buffer)."""
    caches = owner.__dict__.setdefault("_nfdpf_blobs", {})
    cache = caches.get(name)
    if cache is None:
        cache = caches[name] = BlobCache()
    return cache.get(tensors, device)
