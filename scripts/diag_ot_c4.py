"""Diagnostic: the C4-shaped full-size case's OT calls, ours vs the oracle's fp64 Sinkhorn on
identical inputs (the oracle's own step inputs), to separate OT error from flow amplification."""
import sys
import numpy as np
import torch
sys.path[:0] = ["tests", "normalizing-flows-dpfs_amd", "."]
torch.set_num_threads(16)
import _fullsize as F
from oracle import dpf_oracle as O
from nfdpf import _lib, ops
_lib.load()
O.OT_POTENTIALS = 2
w = F.build("c4_n4000")
ref = w["ref"]
x_in = [w["init"][0]] + [ref[0][:, t] for t in range(w["T"] - 1)]
p_in = [O.normalize_log_probs(w["init"][1])] + [ref[1][:, t] for t in range(w["T"] - 1)]
for t in range(w["T"]):
    x, p = x_in[t].float().contiguous(), p_in[t].float().contiguous()
    xo, _, _, it = ops.ot_resample(x.cuda(), p.cuda())
    xr, _, _, info = O.ot_resample(x.double(), p.double(), return_info=True)
    e = (xo.cpu().double() - xr).abs()
    print(f"step {t}: |x| max {float(x.abs().max()):.1f}  iters ours {int(it.item())} ref {info['iters']}  "
          f"OT max abs err {float(e.max()):.3e}  rel {float((e / xr.abs().clamp_min(1)).max()):.3e}", flush=True)
