"""Experiment: per-step phase timestamps of the one-launch pass (lib built with
-DNFDPF_EXP_PTRACE, loaded through NFDPF_LIB; scripts/archive/exp_build.sh PTRACE -DNFDPF_EXP_PTRACE).
C2 bench workload, the last of 3 passes; durations in us, median over the 256 workgroups and
steps 4..45.
Chain waves 0-3: 0 step start, 1 A published, 2 nf_dyn context folded (fA), 3 nf_dyn inverse
done, 4 proposal folded (fB), 5 proposal handed over (qf); wave 0 also 7 A swept, 8 B swept.
Prior waves 4-7: 0 step start, 1 proposal received, 2 prior done.  Encoder wave 8: 0 step
start, 4 proposal received, 5 encoder done, 2 C(t-1) swept, 3 slot t-1 normalised, 6 log-weight,
7 C(t) published (the gated pass's order)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-dpfs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from nfdpf import _lib  # noqa: E402

force = "--force" in sys.argv
flags, B, N, T, _, _ = bench.CONFIGS["c2"]
torch.manual_seed(2)
a = bench.make_args(flags, B, N, T, {"force_resample": force})
from DPFs import DPF  # noqa: E402
from nfdpf.engine import FilterEngine, ShardInfo  # noqa: E402
dev = torch.device("cuda", 0)
dpf = DPF(a).to(dev).eval()
start, state, vel, enc = (t.to(dev) for t in bench.synthetic_disk(B, T, 2, a.hiddensize))
eng = FilterEngine(dpf.filter_config(), dpf)
for _ in range(3):
    eng.run(enc, start, vel, shard=ShardInfo.from_env(B))
torch.cuda.synchronize()
print("pass ran as one launch:", eng.last_pass)
buf = np.zeros((256, 16, 64, 20), dtype=np.uint64)
assert _lib.lib().nfdpf_exp_ptrace_read(buf.ctypes.data_as(ctypes.c_void_p)) == 0
tr = buf.astype(np.int64)
S = slice(4, 46)


def med(x):
    return float(np.median(x / 100.0))


for wv, name, order in ((0, "chain w0", range(6)), (3, "chain w3", range(6)), (4, "prior w4", range(3)),
                        (7, "prior w7", range(3)), (8, "enc w8", (0, 4, 5, 2, 3, 6, 7)), (15, "enc w15", (0, 4, 5, 3, 6, 7))):
    order = list(order)
    nph = len(order)
    x = tr[:, wv][:, :, order]
    d = np.diff(x, axis=-1)[:, S]
    step = x[:, 5:47, 0] - x[:, 4:46, 0]
    print(f"{name}: step {med(step):.2f} us |", " ".join(f"{order[k]}->{order[k + 1]} {med(d[..., k]):.2f}" for k in range(nph - 1)))
ch = tr[:, 0:4, S]  # (wg, wave, step, k)
print("chain step start rel. wave 0 (us):", [round(med(ch[:, k, :, 0] - ch[:, 0, :, 0]), 2) for k in range(4)])
pub = ch[..., 1].reshape(-1, 4 * 4, ch.shape[2])  # (row, tile*wave, step)
last = pub.max(1)
w0 = tr[:, 0, S].reshape(-1, 4, ch.shape[2], tr.shape[-1])  # (row, tile, step, k)
print(f"A: publish spread in a row {med(pub.max(1) - pub.min(1)):.2f}; swept {med(w0[..., 7] - last[:, None, :]):.2f} after the last "
      f"publish; ctx + fold {med(w0[..., 2] - w0[..., 7]):.2f}")
pt = ch[..., 1].reshape(-1, 4, 4, ch.shape[2])  # (row, tile, wave, step)
rowmin = pt.min(axis=(1, 2))[:, None, None, :]
print("A publish rel. the row's first, median per tile:", [round(med(pt[:, k] - rowmin[:, 0]), 2) for k in range(4)])
st0 = ch[..., 0].reshape(-1, 4, 4, ch.shape[2])
print("chain step start rel. the row's first, median per tile:", [round(med(st0[:, k] - st0.min(axis=(1, 2))[:, None, :]), 2) for k in range(4)])
fb = tr[:, 0, S, 4].reshape(-1, 4, ch.shape[2])
print("fB set rel. the row's first, median per tile:", [round(med(fb[:, k] - fb.min(1)), 2) for k in range(4)])
bp = tr[:, 0:4, S, 3].reshape(-1, 16, ch.shape[2]).max(1)
print(f"B: swept {med(w0[..., 8] - bp[:, None, :]):.2f} after the last nf_dyn inverse; fold + fB {med(w0[..., 4] - w0[..., 8]):.2f}")
if force:
    z = tr[:, 0, S]
    pts = [0, 12] + [k for k in range(13, 20) if np.median(z[..., k]) > 0] + [1]
    print("forced: chain w0 resample marks", pts, "|", " ".join(f"{pts[k]}->{pts[k + 1]} {med(z[..., pts[k + 1]] - z[..., pts[k]]):.2f}" for k in range(len(pts) - 1)))
en = tr[:, 8, S]
print(f"prior done after qf: {med(tr[:, 4, S, 2] - tr[:, 0, S, 5]):.2f}; enc C(t) published after qf: {med(en[..., 7] - tr[:, 0, S, 5]):.2f}")
ef = [med(tr[:, w, S, 6] - tr[:, 0, S, 5]) for w in range(8, 16)]
print("encoder waves 8-15: log-weight (ef) after qf(t):", [round(v, 2) for v in ef])
