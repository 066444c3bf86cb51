"""Training-path timings on one GPU -> one JSON line per measurement.

1. nfdpf_cond_stack_backward alone vs the PyTorch-recompute backward of the same stack
   (NormalizingFlowModel_cond.inverse, D=2): the proposal flow (O=36) and nf_dyn (O=4) at
   M = B*N rows, HIP events around each.
2. One training pass of the reference loop (DPF.filtering_pos under autograd + loss.backward)
   with the HIP flow backward vs the recompute backward.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-dpfs_amd"))

DEV = torch.device("cuda:0")


def _time(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def stack_bench(M, O, reps):
    from nf.flows import RealNVP_cond
    from nf.models import NormalizingFlowModel_cond
    from nfdpf import autograd as ag
    torch.manual_seed(0)
    flows = [RealNVP_cond(2, 8, obser_dim=O) for _ in range(2)]
    for f in flows:
        f.zero_initialization(0.3)
    prior = torch.distributions.MultivariateNormal(torch.zeros(2, device=DEV), torch.eye(2, device=DEV))
    model = NormalizingFlowModel_cond(prior, flows, device=DEV)
    x = torch.randn(M, 2, device=DEV, requires_grad=True)
    c = torch.randn(M, O, device=DEV, requires_grad=True)
    w = torch.randn(M, 2, device=DEV)
    out = {}
    for mode in (True, False):
        ag.HIP_BACKWARD = mode

        def step():
            z, ld = model.inverse(x, c)
            ((z * w).sum() + ld.sum()).backward()
        out["hip" if mode else "recompute"] = _time(step, reps)
    ag.HIP_BACKWARD = True
    with torch.no_grad():
        fwd = _time(lambda: model.inverse(x, c), reps)
    # per row: forward of the stack (2 flows x 2 halves x (t,s) nets) + ~2x for the backward
    return {"what": "cond_stack inverse fwd+bwd", "rows": M, "obser_dim": O, "ms_fwd_only": fwd,
            "ms_fwd_bwd_hip": out["hip"], "ms_fwd_bwd_recompute": out["recompute"],
            "speedup": out["recompute"] / out["hip"]}


def train_pass(B, N, T, reps):
    from bench import make_args, synthetic_disk
    from DPFs import DPF
    from nfdpf import autograd as ag
    flags = dict(NF_dyn=True, NF_cond=True, measurement="cos", resampler_type="soft")
    torch.manual_seed(5)
    a = make_args(flags, B, N, T, {})
    dpf = DPF(a).to(DEV)
    dpf.encoder = nn.Identity()
    start, state, vel_in, enc = (x.to(DEV) for x in synthetic_disk(B, T, 3, a.hiddensize))
    res = {}
    for mode in (True, False):
        ag.HIP_BACKWARD = mode

        def step():
            dpf.zero_grad(set_to_none=True)
            out = dpf.filtering_pos(enc, start, vel_in)
            pred = (out[0] * out[1][..., None]).sum(2)
            loss = ((pred - state[:, :, :2]) ** 2).mean()
            loss.backward()
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            step()
        torch.cuda.synchronize()
        res["hip" if mode else "recompute"] = (time.perf_counter() - t0) / reps * 1e3
    ag.HIP_BACKWARD = True
    return {"what": "training pass (filtering_pos under autograd + backward), c2 flags", "B": B, "N": N, "T": T,
            "ms_hip_bwd": res["hip"], "ms_recompute_bwd": res["recompute"],
            "particle_steps_per_s_hip": B * N * T / (res["hip"] * 1e-3),
            "speedup": res["recompute"] / res["hip"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=64000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--train", type=str, default="64,1000,10")
    args = ap.parse_args()
    for O in (36, 4):
        print(json.dumps(stack_bench(args.rows, O, args.reps)), flush=True)
    B, N, T = (int(v) for v in args.train.split(","))
    print(json.dumps(train_pass(B, N, T, max(2, args.reps // 10))), flush=True)


if __name__ == "__main__":
    main()
