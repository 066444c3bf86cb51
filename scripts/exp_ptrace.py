"""Experiment: per-step phase timestamps of the one-launch pass (lib built with
-DNFDPF_EXP_PTRACE, loaded through NFDPF_LIB; scripts/exp_build.sh PTRACE -DNFDPF_EXP_PTRACE).
C2 bench workload, the last of 3 passes; phases as durations (us), median over the 256
workgroups and steps 4..45.
Flow waves 0 (t-net + exchange poller) and 1 (s-net): 0 step start, 1 A published, 2 nf_dyn
context folded (fA), 3 nf_dyn inverse done, 4 proposal folded (fB), 5 proposal inverse done,
6 nf_dyn forward + densities done.  Encoder wave 8: 0 step start, 1 C(t-1) swept, 2 encoding
fold (fE), 3 slot t-1 normalised, 4 proposal received, 5 encoder done, 6 log-weight, 7 C(t)
published."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-dpfs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from nfdpf import _lib  # noqa: E402

force = "--force" in sys.argv
flags, B, N, T, _, _ = bench.CONFIGS["c2"]
torch.manual_seed(2)
a = bench.make_args(flags, B, N, T, {"force_resample": force})
from DPFs import DPF  # noqa: E402
from nfdpf.engine import FilterEngine, ShardInfo  # noqa: E402
dev = torch.device("cuda", 0)
dpf = DPF(a).to(dev).eval()
start, state, vel, enc = (t.to(dev) for t in bench.synthetic_disk(B, T, 2, a.hiddensize))
eng = FilterEngine(dpf.filter_config(), dpf)
for _ in range(3):
    eng.run(enc, start, vel, shard=ShardInfo.from_env(B))
torch.cuda.synchronize()
print("pass ran as one launch:", eng.last_pass)
buf = np.zeros((256, 16, 64, 20), dtype=np.uint64)
assert _lib.lib().nfdpf_exp_ptrace_read(buf.ctypes.data_as(ctypes.c_void_p)) == 0
tr = buf.astype(np.int64)[:, [0, 1, 8, 2, 4, 6]]  # waves 0, 1, 8, then role-0 waves 2, 4, 6
steps = slice(4, 46)
for wi, name, nph in ((0, "flow w0", 7), (1, "flow w1", 7), (2, "enc w8", 8)):
    x = tr[:, wi, :, :nph]
    d = (np.diff(x, axis=-1) / 100.0)[:, steps]
    per_step = (x[:, 5:47, 0] - x[:, 4:46, 0]) / 100.0
    print(f"{name}: step {np.median(per_step):.2f} us |", " ".join(
        f"{k}->{k + 1} {np.median(d[..., k]):.2f}" for k in range(nph - 1)))
x = tr[:, 0, steps]
print(f"flow w0: A poll wait {np.median((x[..., 7] - x[..., 1]) / 100):.2f} us, A ctx + fold {np.median((x[..., 2] - x[..., 7]) / 100):.2f} us")
# skew between the row's tiles: A published (flow w0 phase 1) by the row's 4 workgroups
pub = tr[:, 0, steps, 1].reshape(-1, 4, tr[:, 0, steps, 1].shape[-1])  # (row, tile, step)
print(f"A publish skew within a row: med {np.median((pub.max(1) - pub.min(1)) / 100):.2f} us")
done = tr[:, 0, steps, 7].reshape(-1, 4, pub.shape[-1])
print(f"A poll done after the row's last publish: med {np.median((done - pub.max(1)[:, None, :]) / 100):.2f} us")
st = tr[:, 0, steps, 8].reshape(done.shape)
iss = tr[:, 0, steps, 9].reshape(done.shape)
print(f"A store acked after own publish: med {np.median((x[..., 8] - x[..., 1]) / 100):.2f} us; "
      f"poll iterations med {np.median(x[..., 10]):.0f}")
print(f"successful A load: issued {np.median((iss - pub.max(1)[:, None, :]) / 100):.2f} us after the row's last "
      f"publish, {np.median((iss - st.max(1)[:, None, :]) / 100):.2f} us after its last store ack; "
      f"round trip {np.median((done - iss) / 100):.2f} us")
allpub = tr[:, [0, 3, 4, 5]][:, :, steps, 1]  # (wg, wave, step)
allpub = allpub.reshape(-1, 4, 4, allpub.shape[-1]).reshape(-1, 16, allpub.shape[-1])  # (row, tile*wave, step)
lastall = allpub.max(1)
print(f"A: last publish of all 16 role-0 waves after wave 0's last: med {np.median((lastall - pub.max(1)) / 100):.2f} us; "
      f"poll done after it {np.median((done - lastall[:, None, :]) / 100):.2f} us; "
      f"successful load issued after it {np.median((iss - lastall[:, None, :]) / 100):.2f} us")
w0s = tr[:, [0, 3, 4, 5]][:, :, steps, 0]
print("step start per role-0 wave rel. wave 0 (med us):", [round(float(np.median((w0s[:, k] - w0s[:, 0]) / 100)), 2) for k in range(4)])
print("A publish per role-0 wave rel. wave 0 (med us):", [round(float(np.median((tr[:, [0, 3, 4, 5]][:, k, steps, 1] - tr[:, 0, steps, 1]) / 100)), 2) for k in range(4)])
fl = tr[:, 0, steps]
en = tr[:, 2, steps]
print(f"B: poll done after wave 0's B publish-ready (phase 3) {np.median((fl[..., 11] - fl[..., 3]) / 100):.2f} us; "
      f"fE set {np.median((en[..., 2] - fl[..., 3]) / 100):.2f} us after phase 3; fB set {np.median((fl[..., 4] - fl[..., 11]) / 100):.2f} us after the B poll")
print(f"fraction of steps where fE is set after the B poll: {np.mean(en[..., 2] > fl[..., 11]):.2f}")
full = buf.astype(np.int64)
for wv in (0, 1, 4, 5):
    z = full[:, wv, steps]
    print(f"wave {wv} first nf_dyn coupling: net {np.median((z[..., 13] - z[..., 12]) / 100):.2f} swap {np.median((z[..., 14] - z[..., 13]) / 100):.2f} "
          f"net {np.median((z[..., 15] - z[..., 14]) / 100):.2f} swap {np.median((z[..., 16] - z[..., 15]) / 100):.2f} | "
          f"start rel. wave 0 {np.median((z[..., 12] - full[:, 0, steps, 12]) / 100):.2f}")
# cross-wave: encoder's C(t) publish vs the flow step end
f_end = tr[:, 0, :, 6]
e_pub = tr[:, 2, :, 7]
print(f"enc C(t) published after flow step end: med {np.median((e_pub - f_end)[:, steps]) / 100:.2f} us")
print(f"enc proposal received after flow qf set: med {np.median((tr[:, 2, :, 4] - tr[:, 0, :, 5])[:, steps]) / 100:.2f} us")
