"""Diagnostic: the bench's trained-like C3 line (bench.trained_like on the synthetic disk data) --
per-step prediction error, particle spread, and one of its Sinkhorn calls against the oracle
(FP64) on the same inputs (2 rows)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normalizing-flows-dpfs_amd"), ROOT]
import torch
import bench
from DPFs import DPF
from nfdpf import ops
from nfdpf.engine import FilterEngine

dev = torch.device("cuda:0")
flags, B, N, T, _, _ = bench.CONFIGS["c3"]
B, T = 8, 20
torch.manual_seed(2)
a = bench.make_args(flags, B, N, T, {})
dpf = DPF(a).to(dev).eval()
start, state, vel_in, enc = bench.synthetic_disk(B, T, 2, a.hiddensize)
start, state, vel_in = start.to(dev), state.to(dev), vel_in.to(dev)
dpf_i, enc_i = bench.trained_like(dpf, state)
eng = FilterEngine(dpf.filter_config(), dpf_i)
res = eng.run(enc_i, start, vel_in)
torch.cuda.synchronize()
err = ((res.pred - state[:, :, :2]) ** 2).sum(-1).sqrt()  # [B, T]
print("OT calls", eng.last_ot_calls)
print("pred error per step (mean over rows):", [round(float(v), 1) for v in err.mean(0)])
spread = res.particles.std(2).mean(-1)  # [B, T]
print("particle std per step (mean over rows):", [round(float(v), 1) for v in spread.mean(0)])
print("max |x|:", float(res.particles.abs().max()), "lik range", float(res.lik.min()), float(res.lik.max()))
# one Sinkhorn call on step 5's input vs the oracle, 2 rows
t = 5
x = res.particles[:2, t - 1].contiguous()
p = res.probs[:2, t - 1].contiguous()
xo, wo, idx, it = ops.ot_resample(x, p)
torch.cuda.synchronize()
from oracle import dpf_oracle as O
O.OT_POTENTIALS = 2
with torch.no_grad():
    xr, wr, ir, info = O.ot_resample(x.double().cpu(), p.double().cpu(), return_info=True)
print("iters ours", int(it), "oracle", info["iters"])
d = (xo.cpu().double() - xr).abs()
print("x' max err", float(d.max()), "row scale", float(xr.abs().max()), "x' max |.|", float(xo.abs().max()))
print("p row max", [float(v) for v in p.max(1).values], "ESS", [float(v) for v in 1 / (p.double() ** 2).sum(1)])
