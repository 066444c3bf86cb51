"""Diagnostic (GPU box): where the C5-shaped teacher-forced likelihood error comes from.

Runs tests/_fullsize.py case c5_n10000 teacher-forced, then separates
  * the CGLOW kernel's own error: the kernel on the float64 oracle's particles (cast to f32) vs
    the float64 likelihood, next to the oracle's float32 CGLOW on the same f32 particles;
  * the inherited error: our proposal particles differ from the float64 ones by rounding, and the
    likelihood's slope in x amplifies it.
Prints the worst elements of the end-to-end comparison with both parts."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normalizing-flows-dpfs_amd"), ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import _fullsize as F  # noqa: E402
from oracle import dpf_oracle as O  # noqa: E402


def main():
    from nfdpf import _lib, ops
    import test_gpu_parity_full as T
    _lib.load()
    torch.set_num_threads(16)
    dev = torch.device("cuda:0")
    w = F.build("c5_n10000")
    eng = T._engine(w)
    res = T._run(w, teacher=True)
    torch.cuda.synchronize()
    r64 = T._oracle64_teacher(w)
    ref = w["ref"]
    lik_o = res.lik.cpu().numpy().astype(np.float64)
    lik_r = ref[3].numpy().astype(np.float64)
    e_o, e_r = np.abs(lik_o - r64["lik"]), np.abs(lik_r - r64["lik"])
    x_o = res.particles.cpu().numpy().astype(np.float64)
    x_r = ref[0].numpy().astype(np.float64)
    ex_o = np.abs(x_o - r64["x"]).max(-1)
    ex_r = np.abs(x_r - r64["x"]).max(-1)
    print(f"end to end: lik max err ours {e_o.max():.3e} ref32 {e_r.max():.3e}; mean ours {e_o.mean():.3e} "
          f"ref32 {e_r.mean():.3e}; particle max err ours {ex_o.max():.3e} ref32 {ex_r.max():.3e}")
    for flat in np.argsort(e_o.ravel())[-10:][::-1]:
        b, t, n = np.unravel_index(flat, e_o.shape)
        print(f"  ({b},{t},{n}) lik64 {r64['lik'][b, t, n]:.5f} err ours {e_o[b, t, n]:.3e} ref {e_r[b, t, n]:.3e} "
              f"| x64 {r64['x'][b, t, n]} x err ours {ex_o[b, t, n]:.2e} ref {ex_r[b, t, n]:.2e}")
    # the kernel alone on identical particles (the float64 oracle's, rounded to f32)
    _, _, pe, glow = eng._blobs(dev)
    ek, er = [], []
    for t in range(w["T"]):
        x32 = torch.from_numpy(r64["x"][:, t]).float()
        raw = ops.cglow_measurement(pe, glow, w["enc"][:, t].to(dev), x32.to(dev))
        lk = (raw - raw.max(-1, keepdim=True)[0]).cpu().numpy().astype(np.float64)
        with O.precision(torch.float32), torch.no_grad():
            p32 = O.cast_params(w["params"], torch.float32)
            lr32 = O.meas_cglow(O.sub(p32, "particle_encoder"), O.sub(p32, "cglow_measurement"), 1,
                                w["enc"][:, t].float(), x32).numpy().astype(np.float64)
        with O.precision(torch.float64), torch.no_grad():
            p64 = O.cast_params(w["params"], torch.float64)
            l64 = O.meas_cglow(O.sub(p64, "particle_encoder"), O.sub(p64, "cglow_measurement"), 1,
                               w["enc"][:, t].double(), x32.double()).numpy()
        ek.append(np.abs(lk - l64))
        er.append(np.abs(lr32 - l64))
    ek, er = np.stack(ek), np.stack(er)
    print(f"kernel alone on the same f32 particles: max err ours {ek.max():.3e} oracle f32 {er.max():.3e}; "
          f"mean ours {ek.mean():.3e} oracle f32 {er.mean():.3e}")
    # slope: d lik / dx estimated by a finite difference of the float64 oracle at the worst element
    flat = np.argmax(e_o.ravel())
    b, t, n = np.unravel_index(flat, e_o.shape)
    with O.precision(torch.float64), torch.no_grad():
        p64 = O.cast_params(w["params"], torch.float64)
        xx = torch.from_numpy(r64["x"][b:b + 1, t]).clone()
        base = O.meas_cglow(O.sub(p64, "particle_encoder"), O.sub(p64, "cglow_measurement"), 1,
                            w["enc"][b:b + 1, t].double(), xx)[0, n].item()
        for k in range(2):
            x2 = xx.clone()
            x2[0, n, k] += 1e-4
            v = O.meas_cglow(O.sub(p64, "particle_encoder"), O.sub(p64, "cglow_measurement"), 1,
                             w["enc"][b:b + 1, t].double(), x2)[0, n].item()
            print(f"  worst element d lik / d x{k} ~ {(v - base) / 1e-4:.3f}")


if __name__ == "__main__":
    main()
