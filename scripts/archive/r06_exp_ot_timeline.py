"""Experiment (round 6): wall time of one Sinkhorn call at the C3 shape (64 rows x 1000, gate on) against
its kernels (run under rocprofv3 --kernel-trace for the per-kernel timeline)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "normalizing-flows-dpfs_amd"))
import torch  # noqa: E402

from nfdpf import ops  # noqa: E402

B, N = int(os.environ.get("OT_B", 64)), int(os.environ.get("OT_N", 1000))
g = torch.Generator().manual_seed(0)
x = (torch.randn(B, N, 2, generator=g) * 3.0).cuda()
w = torch.rand(B, N, generator=g) + 0.05
w = (w / w.sum(1, keepdim=True)).cuda()
gate = torch.ones(1, dtype=torch.int32, device="cuda")
for poll in (1, 0):
    for _ in range(3):
        ops.ot_resample(x, w, 0.1, 0.75, 1e-3, 100, 0, gate=gate, poll=bool(poll))
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    a.record()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = ops.ot_resample(x, w, 0.1, 0.75, 1e-3, 100, 0, gate=gate, poll=bool(poll))
    b.record()
    torch.cuda.synchronize()
    it = out[3]
    print(f"B {B} N {N} poll {poll}: {1000 * a.elapsed_time(b) / reps:.1f} us per call (events), "
          f"{1e6 * (time.perf_counter() - t0) / reps:.1f} us host, iters {int(it.item()) if it is not None else None}",
          flush=True)
