"""Per-call Sinkhorn diagnostics over one bench pass of a config (default c4): iterations and
exact-fallback counts of every nfdpf_ot_resample call, and the OT wall time."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normalizing-flows-dpfs_amd"), ROOT]
import bench  # noqa: E402
from nfdpf import ops  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
flags, B, N, T, _, _ = bench.CONFIGS[cfg]
dev = torch.device("cuda:0")
torch.manual_seed(2)
a = bench.make_args(flags, B, N, T, {})
from DPFs import DPF  # noqa: E402
from nfdpf.engine import FilterEngine, ShardInfo  # noqa: E402

dpf = DPF(a).to(dev).eval()
start, state, vel_in, enc = (t.to(dev) for t in bench.synthetic_disk(B, T, 2, a.hiddensize))
eng = FilterEngine(dpf.filter_config(), dpf)
orig = ops.ot_resample
log = []


def wrapped(*args, **kw):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = orig(*args, **kw)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    log.append((dt,) + ops.ot_stats(dev))
    return out


ops.ot_resample = wrapped
eng.run(enc, start, vel_in, shard=ShardInfo.from_env(B))
log.clear()
res = eng.run(enc, start, vel_in, shard=ShardInfo.from_env(B))
tot = sum(x[0] for x in log)
print(f"{cfg}: {len(log)} OT calls, {tot * 1e3:.1f} ms, iterations {[x[1] for x in log]}")
print(f"exact fallbacks per call {[x[2] for x in log]} (of {B * N} lanes x softmins)")
