"""Experiment: dump OUR CGLOW kernel's per-particle 1x1-conv W, its
log|det W| (the in-kernel LU's) and the actnorm outputs for the outlier particle
(NFDPF_CG_TARGET of the exp build: SRC=cglow scripts/archive/exp_build_fast.sh CGD -DNFDPF_EXP_CGDUMP
-DNFDPF_CG_TARGET=68339), on the c5_n10000 workload's step-2 reference particles (exp/cg_in.npz,
cut from scripts/archive/r05_cglow_dump.py's output).  GPU box:
NFDPF_LIB=exp/lib_CGD.so python scripts/archive/r05_cglow_w.py gpurun_out/r05_cgw.npz"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-dpfs_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _fullsize as F  # noqa: E402
from nfdpf import _lib, ops  # noqa: E402
from nfdpf.pack import cglow_tensors, encoder_tensors  # noqa: E402

lib = _lib.load()
DEV = torch.device("cuda:0")
m = F.workload("c5_n10000")["models"]
pe = torch.cat([a.detach().reshape(-1) for a in encoder_tensors(m.particle_encoder)]).float().to(DEV)
glow = torch.cat([a.detach().reshape(-1) for a in cglow_tensors(m.cglow_measurement)]).float().to(DEV)
d = np.load(os.path.join(ROOT, "exp", "cg_in.npz"))
lik = ops.cglow_measurement(pe, glow, torch.from_numpy(d["enc"]).to(DEV), torch.from_numpy(d["x"]).to(DEV))
torch.cuda.synchronize()
buf = np.zeros(256, np.float32)
fn = lib.nfdpf_exp_cgdump_read
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
np.savez(sys.argv[1], dump=buf, lik=lik.cpu().numpy())
print("W[0,:4]", buf[:4], "ldw", buf[200], "ld", buf[201], "part", buf[202])
