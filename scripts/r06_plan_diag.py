"""Diagnostic: the plan pass given the gated pass's gates (counts, flags, gates side by side)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normalizing-flows-dpfs_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np
import torch
import _fullsize as F
from nfdpf.engine import FilterConfig, FilterEngine

DEV = "cuda:0"
B, N, T = 8, 1000, 16
wl = F.workload("c2_full", B=B, N=N, T=T)
models = wl["models"].to(DEV)
inp = (wl["enc"].to(DEV), wl["start"].to(DEV), wl["vel"].to(DEV))
mk = lambda **kw: FilterEngine(FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft",
                                            seed=5, kernel="tiled", **kw), models)
eg = mk(speculate_gate=False)
g = eg.run(*inp)
gates = eg.last_gates.cpu().numpy()
print("gated: gates", gates.tolist(), "launches", eg.pass_launches)
ep = mk()
p = ep.run(*inp, plan=gates, finish=False)
pend = ep.take_pending()
torch.cuda.synchronize()
v = pend[6]
fl = v[2] if v[0] is None else v[0]
print("plan pass: flags", [int(x) for x in fl[:3]], "actual gates", pend[10].cpu().tolist())
for f in ("particles", "probs", "index", "lik", "noise", "jac", "prior"):
    a, b = getattr(p, f), getattr(g, f)
    if torch.equal(a, b):
        print(f, "equal")
    else:
        bad = (a != b).reshape(B, T, -1).any(-1)
        t0 = int(bad.any(0).nonzero()[0])
        print(f, f"differ: first slot {t0}, rows {bad[:, t0].nonzero().flatten().tolist()}, max abs diff at it "
                 f"{float((a - b).reshape(B, T, -1)[:, t0].abs().max()) if a.is_floating_point() else 'idx'}")
import nfdpf.ops as ops
parts_p = pend[0]
