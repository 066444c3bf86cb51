"""Experiment: the merged front launch's phase 0->1 split into the gate wave and the
speculative-motion waves (lib built with -DNFDPF_EXP_TRACE, loaded through NFDPF_LIB)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-dpfs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from nfdpf import _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
flags, _, N, T, _, _ = bench.CONFIGS["c2"]
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
buf = np.zeros((4, 2048, 8), dtype=np.uint64)
assert _lib.lib().nfdpf_exp_trace_read(buf.ctypes.data_as(ctypes.c_void_p)) == 0
nwg = B * ((N + 255) // 256)
tr = buf[0, :nwg, :].astype(np.int64)
for name, slot in (("gate wave", 4), ("motion wave 1", 5), ("motion wave 7", 6), ("barrier", 1), ("fold", 2), ("end", 3)):
    d = (tr[:, slot] - tr[:, 0]) / 100.0
    print(f"fdyn 0->{name:14s} med {np.median(d):6.2f} us  max {d.max():6.2f} us")
