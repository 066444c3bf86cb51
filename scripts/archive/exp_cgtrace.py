"""Experiment: per-phase timestamps of the CGLOW kernel (lib built with -DNFDPF_EXP_CGTRACE,
loaded through NFDPF_LIB), the third tile of every workgroup, C5 shape (64 rows x 10000).
Phases (between the CGTRACE points): encoder, cond conv1, conv2, conv3, linear 1 + 2, last
layer + tanh, phase_y, resize, phase_f + store."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-dpfs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from nfdpf import _lib, ops  # noqa: E402
from nfdpf.pack import cglow_tensors, encoder_tensors  # noqa: E402

flags, B, N, T, _, _ = bench.CONFIGS["c5"]
a = bench.make_args(flags, B, N, T, {})
from DPFs import DPF  # noqa: E402
dev = torch.device("cuda", 0)
torch.manual_seed(0)
dpf = DPF(a).to(dev).eval()
mm = dpf.measurement_model
pe = torch.cat([t.detach().reshape(-1) for t in encoder_tensors(mm.particle_encoder)]).to(dev)
glow = torch.cat([t.detach().reshape(-1) for t in cglow_tensors(mm.CGLOW)]).to(dev)
enc = torch.randn(B, 192, device=dev)
x = torch.randn(B, N, 2, device=dev) * 30
for _ in range(3):
    ops.cglow_measurement(pe, glow, enc, x)
torch.cuda.synchronize()
buf = np.zeros((1024, 16), dtype=np.uint64)
assert _lib.lib().nfdpf_exp_cgtrace_read(buf.ctypes.data_as(ctypes.c_void_p)) == 0
tr = buf.astype(np.int64)
ok = (tr[:, 0] > 0) & (tr[:, 9] > 0)
tr = tr[ok]
names = ["encoder", "cond conv1", "cond conv2", "cond conv3", "linear 1+2", "last layer", "phase_y",
         "resize", "phase_f"]
d = np.diff(tr[:, :10], axis=1) / 100.0
tot = (tr[:, 9] - tr[:, 0]) / 100.0
print(f"workgroups {len(tr)}, tile total med {np.median(tot):.2f} us")
for k, n in enumerate(names):
    print(f"{n:14s} med {np.median(d[:, k]):6.2f} us  ({100 * np.median(d[:, k]) / np.median(tot):4.1f} %)")
