"""Experiment: where a step of the GATED one-launch pass (kModeGate; --spec: the speculative pass,
--force: the forced pass) waits -- per-step phase
timestamps (lib built with -DNFDPF_EXP_PTRACE: scripts/archive/exp_build.sh PTRACE -DNFDPF_EXP_PTRACE,
loaded through NFDPF_LIB).  C2 bench workload ([--informative]: frame encodings = the particle
encoder at the true positions, the gate fires), the last of 3 passes; medians over the 256
workgroups and steps 4..45, us.  Times are relative to the chain's hand-over of step t-1 (qf)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-dpfs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from nfdpf import _lib  # noqa: E402

flags, B, N, T, _, _ = bench.CONFIGS["c2"]
torch.manual_seed(2)
a = bench.make_args(flags, B, N, T, {"force_resample": "--force" in sys.argv})
from DPFs import DPF  # noqa: E402
from nfdpf.engine import FilterEngine, ShardInfo  # noqa: E402
dev = torch.device("cuda", 0)
dpf = DPF(a).to(dev).eval()
start, state, vel, enc = (t.to(dev) for t in bench.synthetic_disk(B, T, 2, a.hiddensize))
if "--informative" in sys.argv:
    with torch.no_grad():
        enc = dpf.particle_encoder(state[:, :, :2].float()).contiguous()
cfg = dpf.filter_config()
if "--spec" in sys.argv:
    cfg.speculate_gate = True
eng = FilterEngine(cfg, dpf)
for _ in range(3):
    eng.run(enc, start, vel, shard=ShardInfo.from_env(B))
torch.cuda.synchronize()
print("pass:", eng.last_pass, "gated:", eng.last_gate_pass, "fired:", None if eng.last_gates is None else
      int(eng.last_gates.sum()))
buf = np.zeros((256, 16, 64, 20), dtype=np.uint64)
assert _lib.lib().nfdpf_exp_ptrace_read(buf.ctypes.data_as(ctypes.c_void_p)) == 0
tr = buf.astype(np.int64)
S = np.arange(4, 46)


def med(x):
    return round(float(np.median(x / 100.0)), 2)


q_prev = tr[:, 0, S - 1, 5]  # chain wave 0: step t-1 handed over (qf)
ev = {
    "prior(t-1) done": tr[:, 4, S - 1, 2],
    "enc w8: encode(t-1) done": tr[:, 8, S - 1, 5],
    "enc w8: C(t-1) published": tr[:, 8, S - 1, 7],
    "enc w15: C(t-1) published": tr[:, 15, S - 1, 7],
    "enc w8: C(t-1) swept": tr[:, 8, S, 10],
    "enc w8: decision(t)": tr[:, 8, S, 2],
    "chain w0: A(t) swept": tr[:, 0, S, 7],
    "chain w0: B(t) swept": tr[:, 0, S, 8],
    "chain w0: proposal(t) starts (fB)": tr[:, 0, S, 4],
    "chain w0: decision(t) in hand": tr[:, 0, S, 9],
    "chain w0: qf(t)": tr[:, 0, S, 5],
}
for k, v in ev.items():
    print(f"{k:40s} {med(v - q_prev):7.2f}")
print("step (qf to qf)", med(tr[:, 0, S, 5] - q_prev))
# the batch-wide spread: the last row's C(t-1) publish vs the median row's
pubC = tr[:, 8, S - 1, 7].reshape(-1, 4, len(S)).max(1)  # per row: its last tile's wave-8 publish
print("C(t-1) publish spread over rows (max - median):", med(pubC.max(0) - np.median(pubC, 0)))
# raw timestamps for offline analysis (100 MHz ticks relative to the first, int32): every wave, steps 0..51
if "--save" in sys.argv:
    out = sys.argv[sys.argv.index("--save") + 1]
    sub = tr[:, :, :52, :]
    base = sub[sub > 0].min()
    rel = np.where(sub > 0, sub - base, -1).astype(np.int32)
    np.savez_compressed(out, tr=rel)
    print("saved", out, rel.shape)
