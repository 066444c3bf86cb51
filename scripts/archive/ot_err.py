"""OT x' error of the HIP Sinkhorn against the fp64 oracle (golden + stress cases); prints
max |d| and max |d| / (1e-4 |ref| + 2e-3).  NFDPF_LIB selects the library."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normalizing-flows-dpfs_amd"), ROOT, os.path.join(ROOT, "tests")]
from _util import group, load, t  # noqa: E402
from nfdpf import ops  # noqa: E402
from oracle import dpf_oracle as O  # noqa: E402

DEV = torch.device("cuda:0")
cases = []
fx = load("ot.npz")
for i in range(int(fx["n_cases"])):
    c = group(fx, f"c{i}")
    cases.append((f"golden{i}", t(c["x"]), t(c["p"])))
for B, N, kind in [(2, 1000, "peaked"), (3, 777, "outliers"), (2, 1500, "uniform"), (4, 64, "peaked"),
                   (1, 300, "clusters")]:
    g = torch.Generator().manual_seed(N + B)
    x = torch.randn(B, N, 2, generator=g) * 30
    if kind == "outliers":
        x[:, :5] *= 40
    if kind == "clusters":
        x[:, : N // 2] += 400
    s = {"peaked": 12.0, "outliers": 3.0, "uniform": 0.0, "clusters": 2.0}[kind]
    p = torch.softmax(torch.randn(B, N, generator=g) * s, -1) + 1e-12
    cases.append((f"{kind}{B}x{N}", x, p))
for name, x, p in cases:
    xo, _, _, it = ops.ot_resample(x.to(DEV), p.to(DEV))
    _, fb = ops.ot_stats(DEV)
    xr, _, _, info = O.ot_resample(x.double(), p.double(), return_info=True)
    d = (xo.cpu().double() - xr).abs()
    tol = 1e-4 * xr.abs() + 2e-3
    print(f"{name:>18}: iters {int(it.item())} vs {info['iters']}  max|d| {float(d.max()):.3e}  "
          f"mean|d| {float(d.mean()):.3e}  worst/tol {float((d / tol).max()):.3f}  exact-fallbacks {fb}")
