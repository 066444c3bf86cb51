"""Experiment: the C5 CGLOW likelihood outlier.  Builds the c5_n10000
workload (tests/_fullsize.py: the oracle's teacher-forced run, CPU), evaluates OUR CGLOW kernel on
the reference's own particles of every step (the kernel-alone comparison of
test_fullsize_teacher_forced) and saves the raw (unshifted) kernel likelihoods with the
particles, encodings and the oracle float32 likelihoods, for a layer-by-layer analysis on the CPU
(scripts/r05_cglow_layers.py).  GPU box: python scripts/archive/r05_cglow_dump.py gpurun_out/r05_cglow.npz"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-dpfs_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _fullsize as F  # noqa: E402
from nfdpf import _lib, ops  # noqa: E402
from nfdpf.pack import cglow_tensors, encoder_tensors  # noqa: E402

torch.set_num_threads(16)
_lib.load()
DEV = torch.device("cuda:0")
w = F.build("c5_n10000")
m = w["models"]
pe = torch.cat([a.detach().reshape(-1) for a in encoder_tensors(m.particle_encoder)]).float().to(DEV)
glow = torch.cat([a.detach().reshape(-1) for a in cglow_tensors(m.cglow_measurement)]).float().to(DEV)
x = w["ref"][0]
raw = []
for t in range(x.shape[1]):
    raw.append(ops.cglow_measurement(pe, glow, w["enc"][:, t].float().contiguous().to(DEV),
                                     x[:, t].float().contiguous().to(DEV)).cpu().numpy())
np.savez_compressed(sys.argv[1], raw=np.stack(raw, 1), x=x.numpy(), enc=w["enc"].numpy(), lik32=w["ref"][3].numpy())
print("saved", sys.argv[1], np.stack(raw, 1).shape)
