"""Time the CGLOW measurement's backward at the C5 per-GPU size (64 rows x N particles):
the HIP kernel (nfdpf_cglow_measurement_backward) against the PyTorch recompute backward it
replaces (nfdpf.autograd with HIP_BACKWARD off).  Prints one JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-dpfs_amd"))


def main():
    from arguments import parse_args
    from model.models import build_particle_encoder_cglow, measurement_model_cglow
    from nf.cglow.CGlowModel import CondGlowModel
    from nfdpf import autograd as ag
    B, N = int(os.environ.get("CGB_B", 64)), int(os.environ.get("CGB_N", 10000))
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = measurement_model_cglow(build_particle_encoder_cglow(192, 2), CondGlowModel(parse_args([]))).to(dev)
    g = torch.Generator().manual_seed(1)
    enc = torch.randn(B, 192, generator=g).to(dev).requires_grad_(True)
    x = (torch.randn(B, N, 2, generator=g) * 20).to(dev).requires_grad_(True)
    gl = torch.randn(B, N, generator=g).to(dev)
    out = {"B": B, "N": N}
    modes = (True,) if os.environ.get("CGB_HIP_ONLY") else (True, False)
    for mode in modes:
        ag.HIP_BACKWARD = mode
        times = []
        for it in range(4):
            m.zero_grad(set_to_none=True)
            enc.grad = x.grad = None
            lik = m(enc, x)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            (lik * gl).sum().backward()
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        out["hip_backward_ms" if mode else "recompute_backward_ms"] = 1e3 * min(times[1:])
        print(json.dumps(out), flush=True)
    ag.HIP_BACKWARD = True
    if "recompute_backward_ms" in out:
        out["speedup"] = out["recompute_backward_ms"] / out["hip_backward_ms"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
