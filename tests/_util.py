"""Shared helpers for the test-suite (fixture loading, tape RNG, tolerances)."""
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name)))


def group(fx, prefix):
    p = prefix + "/"
    return {k[len(p):]: v for k, v in fx.items() if k.startswith(p)}


def weights(fx, prefix="w"):
    return {k: torch.from_numpy(v) for k, v in group(fx, prefix).items()}


def t(a):
    return torch.from_numpy(np.asarray(a))


def close(a, b, rtol, atol):
    """|a-b| <= rtol*|b| + atol elementwise; returns (ok, worst excess)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    err = np.abs(a - b) - (rtol * np.abs(b) + atol)
    return bool(np.all(err <= 0)), float(err.max()) if err.size else 0.0


def assert_close(a, b, rtol, atol, what=""):
    ok, worst = close(a, b, rtol, atol)
    assert ok, f"{what}: tolerance |d| <= {rtol}*|ref| + {atol} exceeded by {worst:.3e}"


class TapeRNG:
    """Replays the CPU-generator draws recorded in an e2e golden fixture."""

    def __init__(self, fx):
        self.tape_noise = torch.from_numpy(fx["noise"])      # (B,T,N,2)
        self.tape_off = torch.from_numpy(fx["offsets"])      # (B,T)
        self.t_noise = 0
        self.t_off = 0
        self.gen = None

    def offsets(self, B, N):
        # an offsets draw belongs to the step whose noise is drawn next
        return self.tape_off[:, self.t_noise].clone()

    def noise(self, B, N, std):
        v = self.tape_noise[:, self.t_noise].clone()
        self.t_noise += 1
        return v


def e2e_cfg(fx):
    flag = lambda k: fx[f"flag/{k}"].item()
    m = flag("measurement")
    return dict(N=int(fx["N"]), NF_dyn=bool(flag("NF_dyn")), NF_cond=bool(flag("NF_cond")), measurement=m,
                resampler=flag("resampler_type"), alpha=0.5, eps=0.1, scaling=0.75, threshold=1e-3,
                max_iter=100, pos_noise=20.0, vel_noise=20.0, width=128, n_flows=2, cglow_K=1,
                dyn_flow=str(flag("NF_dyn_flow")) if "flag/NF_dyn_flow" in fx else "RealNVP", H=int(fx["H"]))
