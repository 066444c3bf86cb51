"""Experiment: per-wave phase timestamps of the quad proposal launch (lib built with
-DNFDPF_EXP_QTRACE, loaded through NFDPF_LIB), last step of a C2 pass.  Phases (us, median /
max over workgroups): encoder: layer 2 (8), layer 3 (9), fp64 sums done (11);
 flow waves 0-7: prologue end (1), proposal published (2), nf_dyn
forward end (3); encoder waves 8-15: proposal received (2), encoder end (3); all: final
barrier (4), end (5)."""
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
a = bench.make_args(flags, B, N, T, {})
from DPFs import DPF  # noqa: E402
from nfdpf.engine import FilterEngine, ShardInfo  # noqa: E402
dev = torch.device("cuda", 0)
dpf = DPF(a).to(dev).eval()
start, state, vel, enc = (t.to(dev) for t in bench.synthetic_disk(B, T, 2, a.hiddensize))
eng = FilterEngine(dpf.filter_config(), dpf)
for _ in range(3):
    eng.run(enc, start, vel, shard=ShardInfo.from_env(B))
torch.cuda.synchronize()
buf = np.zeros((1024, 16, 16), dtype=np.uint64)
assert _lib.lib().nfdpf_exp_qtrace_read(buf.ctypes.data_as(ctypes.c_void_p)) == 0
nwg = B * ((N + 255) // 256)
tr = buf[:nwg].astype(np.int64)
t0 = tr[:, :, 0].min(axis=1, keepdims=True)  # per workgroup: its first wave's start
x = (tr - t0[:, :, None]) / 100.0
for name, ws in (("flow", slice(0, 8)), ("enc", slice(8, 16))):
    for p in ((1, 2, 3, 4, 5) if name == 'flow' else (1, 2, 8, 9, 11, 3, 4, 5)):
        v = x[:, ws, p]
        print(f"{name:4s} P{p}: med {np.median(v):6.2f} max {v.max():6.2f} us")
