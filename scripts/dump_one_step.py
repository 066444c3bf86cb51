"""Debug helper (GPU box): teacher-forced one-step outputs of both kernels plus the oracle's
float32 fixture values and float64 re-evaluation, saved for offline error analysis."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "normalizing-flows-dpfs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import test_gpu_parity as G  # noqa: E402
from _util import load, t  # noqa: E402


class MP:
    def setattr(self, obj, name, val):
        setattr(obj, name, val)


out = {}
soft = G.O.soft_resample
for name in sys.argv[1:] or ["c2", "c2w", "c3n"]:
    fx = load(f"e2e_{name}.npz")
    for kernel in G.KERNELS:
        eng, c = G._engine(fx, kernel)
        res = eng.run(t(fx["enc"]).to(G.DEV), t(fx["start"]).to(G.DEV), t(fx["vel"]).to(G.DEV),
                      host=G._TapeDraws(fx), init=(t(fx["init_x"]), t(fx["logw0"])),
                      teacher={"x": t(fx["x"]), "p": t(fx["p"])})
        for k, v in dict(x=res.particles, p=res.probs, lik=res.lik, jac=res.jac, prior=res.prior).items():
            if v is not None:
                out[f"{name}_{kernel}_{k}"] = v.cpu().numpy()
    G.O.soft_resample = soft
    r64 = G._oracle64_one_step(fx, MP())
    G.O.soft_resample = soft
    for k, v in r64.items():
        out[f"{name}_ref64_{k}"] = v
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/one_step_dump.npz", **out)
print("saved", len(out))
