import sys, os, torch
sys.path[:0] = ["/root/repo", "/root/repo/tests", "/root/repo/normalizing-flows-dpfs_amd"]
from test_gpu_pass import _models, _inputs, _run
m = _models("e2e_c2.npz")
enc, start, vel = _inputs(6, 8, seed=6 * 1000 + 1000)
eng, a = _run(m, 1000, enc, start, vel, spec=True)
print("last_pass", eng.last_pass)
ref = (a.probs[..., None].double() * a.particles.double()).sum(2)
d = (a.pred.double() - ref).abs()
print("max diff per t", d.amax(dim=(0, 2)).tolist())
print("pred[0,:3]", a.pred[0, :3].tolist(), "ref", ref[0, :3].tolist())
