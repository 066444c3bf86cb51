"""Experiment: per-phase timestamps of the CGLOW backward kernel (lib built with
-DNFDPF_EXP_CBTRACE via scripts/exp_build.sh, loaded through NFDPF_LIB), the third tile of
every workgroup, C5 shape (64 rows x 10000 particles)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-dpfs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from arguments import parse_args  # noqa: E402
from model.models import build_particle_encoder_cglow  # noqa: E402
from nf.cglow.CGlowModel import CondGlowModel  # noqa: E402
from nfdpf import _lib, ops  # noqa: E402
from nfdpf.pack import cglow_tensors, encoder_tensors  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
glow = CondGlowModel(parse_args([])).to(dev)
pe = build_particle_encoder_cglow(192, 2).to(dev)
peb = torch.cat([t.detach().reshape(-1) for t in encoder_tensors(pe)])
glb = torch.cat([t.detach().reshape(-1) for t in cglow_tensors(glow)])
B, N = 64, 10000
enc = torch.randn(B, 192, device=dev)
x = torch.randn(B, N, 2, device=dev) * 20
g = torch.randn(B, N, device=dev)
for _ in range(2):
    ops.cglow_measurement_backward(peb, glb, enc, x, g)
torch.cuda.synchronize()
buf = np.zeros((256, 24), dtype=np.uint64)
assert _lib.lib().nfdpf_exp_cbtrace_read(buf.ctypes.data_as(ctypes.c_void_p)) == 0
tr = buf.astype(np.int64)[:, :13]
ok = (tr[:, 0] > 0) & (tr[:, 12] > 0)
tr = tr[ok]
names = ["encoder", "cond nets fwd", "actnorm/1x1/GJ", "resize fwd", "f fwd", "f4 bwd", "f2+f0 bwd",
         "r4 bwd", "resize rounds", "1x1/actnorm bwd", "cond nets bwd", "encoder bwd"]
d = np.diff(tr, axis=1) / 100.0
tot = (tr[:, 12] - tr[:, 0]) / 100.0
print(f"workgroups {len(tr)}, tile total med {np.median(tot):.2f} us")
for k, n in enumerate(names):
    print(f"  {n:18s} med {np.median(d[:, k]):8.2f} us  max {np.max(d[:, k]):8.2f}")
full = buf.astype(np.int64)[ok]
if (full[:, 13] > 0).all():  # round 0 of the resize stage: r1 staged, r2w, d r1 staged
    sub = [full[:, 8], full[:, 13], full[:, 14], full[:, 15]]
    for a, b, n in zip(sub[:-1], sub[1:], ["round0 r1 + stage", "round0 r2w", "round0 d r1 + stage"]):
        print(f"  {n:18s} med {np.median((b - a) / 100.0):8.2f} us")
if (full[:, 16] > 0).all():  # inside the actnorm / 1x1 / GJ phase
    sub = [full[:, 2], full[:, 16], full[:, 17], full[:, 3]]
    for a, b, n in zip(sub[:-1], sub[1:], ["actnorm + 1x1", "Gauss-Jordan", "resize1 + conv2"]):
        print(f"  {n:18s} med {np.median((b - a) / 100.0):8.2f} us")
