"""Experiment: per-workgroup phase timestamps of the tiled step (lib built with
-DNFDPF_EXP_TRACE, loaded through NFDPF_LIB).  Prints, per kernel, the start skew and the
phase durations in microseconds (median / max over workgroups) for the last step of a pass."""
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
SPLIT = int(sys.argv[2]) if len(sys.argv) > 2 else 1
CFG = os.environ.get("TRACE_CONFIG", "c2")
flags, _, N, T, _, _ = bench.CONFIGS[CFG]
torch.manual_seed(2)
a = bench.make_args(flags, B, N, T, {})
from DPFs import DPF  # noqa: E402
from nfdpf.engine import FilterEngine, ShardInfo  # noqa: E402
dev = torch.device("cuda", 0)
dpf = DPF(a).to(dev).eval()
start, state, vel, enc = (t.to(dev) for t in bench.synthetic_disk(B, T, 2, a.hiddensize))
cfg = dpf.filter_config()
cfg.split_nets = bool(SPLIT)
eng = FilterEngine(cfg, dpf)
for _ in range(3):
    eng.run(enc, start, vel, shard=ShardInfo.from_env(B))
torch.cuda.synchronize()
buf = np.zeros((4, 2048, 8), dtype=np.uint64)
assert _lib.lib().nfdpf_exp_trace_read(buf.ctypes.data_as(ctypes.c_void_p)) == 0
nwg = B * ((N + 255) // 256)
tr = buf[:, :nwg, :8].astype(np.int64)
t0 = tr[:, :, 0][tr[:, :, 0] > 0].min()
for k, name in enumerate(["motion", "dyn", "prop", "norm"]):
    x = (tr[k] - t0) / 100.0  # 100 MHz -> us
    st = x[:, 0]
    print(f"{name:7s} start min {st.min():7.2f} med {np.median(st):7.2f} max {st.max():7.2f} | end max "
          f"{x[:, 3].max():7.2f}", end="")
    order = [0, 1, 4, 2, 3] if (tr[k][:, 4] > 0).all() else [0, 1, 2, 3]
    for a, p in zip(order[:-1], order[1:]):
        if (tr[k][:, p] > 0).all() and (tr[k][:, a] > 0).all():
            dd = x[:, p] - x[:, a]
            print(f" | {a}->{p} med {np.median(dd):6.2f} max {dd.max():6.2f}", end="")
    print()
