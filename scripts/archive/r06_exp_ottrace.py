"""Experiment: per-phase wall time of the Sinkhorn iteration launches (ot_iter_kernel) at a given
shape, from an -DNFDPF_EXP_OTTRACE build (never shipped):

    SRC=resample_ot scripts/archive/exp_build_fast.sh OTT -DNFDPF_EXP_OTTRACE
    NFDPF_LIB=exp/lib_OTT.so OT_B=64 OT_N=1000 python scripts/archive/r06_exp_ottrace.py

Phases (lane 0 of wave 0 of every workgroup; s_memrealtime, 10 ns ticks): 0 launch start ->
1 after the stop check -> 2 end of the wave's pair loop -> 3 after the LDS combine and the
log-sum-exps -> 4 potentials written -> 5 after the state tables (emit_state_tables).
Prints the median over workgroups of each phase per iteration, and the spread of the start
and end stamps across workgroups (the launch's ramp and drain)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "normalizing-flows-dpfs_amd"))
import torch  # noqa: E402

from nfdpf import _lib, ops  # noqa: E402

B, N = int(os.environ.get("OT_B", 64)), int(os.environ.get("OT_N", 1000))
g = torch.Generator().manual_seed(0)
x = (torch.randn(B, N, 2, generator=g) * 3.0).cuda()
w = torch.rand(B, N, generator=g) + 0.05
w = (w / w.sum(1, keepdim=True)).cuda()
gate = torch.ones(1, dtype=torch.int32, device="cuda")
for _ in range(3):
    out = ops.ot_resample(x, w, 0.1, 0.75, 1e-3, 100, 0, gate=gate)
torch.cuda.synchronize()
K = int(out[3].item()) - 2
buf = np.zeros((1024, 64, 8), dtype=np.uint64)
lib = _lib.lib()
fn = lib.nfdpf_exp_ottrace
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
wgs = B * ((N + 255) // 256)
tr = buf[:wgs].astype(np.int64)
print(f"B {B} N {N}: {K} iterations, {wgs} workgroups; us per phase (median over workgroups)")
names = ["stop-check", "pair loop", "combine+lse", "pot write", "tables"]
tot = []
for k in range(min(K, 64)):
    t = tr[:, k, :6]
    ph = np.diff(t, axis=1) * 0.01  # 100 MHz ticks -> us
    med = np.median(ph, axis=0)
    ramp = (t[:, 0].max() - t[:, 0].min()) * 0.01
    span = (t[:, 5].max() - t[:, 0].min()) * 0.01
    tot.append(span)
    print(f"  k={k:2d} " + " ".join(f"{n} {m:5.2f}" for n, m in zip(names, med)) +
          f" | start spread {ramp:5.2f} | first start -> last end {span:5.2f}")
print(f"median first-start -> last-end {np.median(tot):.2f} us")
print("ot_stats (iterations, exact fallbacks -- per-mille of wave-slices on the two-exp path in an "
      "-DNFDPF_OT_RISKSTAT build):", ops.ot_stats())
# per-workgroup spread at one iteration: total time vs placement (HW_ID / XCC_ID of wave 0)
k = min(K, 64) // 2
t = tr[:, k, :]
tot_wg = (t[:, 5] - t[:, 0]) * 0.01
loop_wg = (t[:, 2] - t[:, 1]) * 0.01
hw = t[:, 6].astype(np.int64)
xcc = t[:, 7].astype(np.int64) & 0xF
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
S = (N + 255) // 256
print(f"iteration {k}: per-WG total us p10/p50/p90/max {np.percentile(tot_wg, [10, 50, 90, 100]).round(2)}; "
      f"loop p10/p50/p90/max {np.percentile(loop_wg, [10, 50, 90, 100]).round(2)}")
for x in range(8):
    sel = xcc == x
    if sel.any():
        print(f"  XCC {x}: {sel.sum()} WGs, total p50 {np.median(tot_wg[sel]):.2f} max {tot_wg[sel].max():.2f}")
key = xcc * 1000 + se * 100 + cu
u, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
share = cnt[inv]
for c in sorted(set(share)):
    sel = share == c
    print(f"  WGs sharing a CU with {c - 1} other(s): {sel.sum()}, total p50 {np.median(tot_wg[sel]):.2f}")
rows = np.arange(len(tot_wg)) // S
slices = np.arange(len(tot_wg)) % S
print("  total p50 by slice index:", [round(float(np.median(tot_wg[slices == q])), 1) for q in range(S)])
print("  end stamp spread (us) first/last WG end:", (t[:, 5].min() - t[:, 0].min()) * 0.01, (t[:, 5].max() - t[:, 0].min()) * 0.01)
