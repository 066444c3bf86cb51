"""Golden vector for the Sinkhorn stop rule at a C4 rank's share: ONE OT call on 32 rows x N = 4000
(BASELINE configs[3]: B = 256 over 8 GPUs), whose batch-coupled stop (resamplers.py:126-129:
the loop ends when ANY row has converged) depends on the batch -- tests/test_gpu_parity_full.py
checks the HIP resampler's iteration count and x' against this.

    python tests/golden/gen_ot_share.py        # writes tests/golden/ot_c4_share.npz (~10 min, ~20 GB RAM)

The input is regenerated from its seed by ``ot_share_input`` (numpy's PCG64: the same bits on
every machine), so only the oracle's outputs are stored: the iteration count (``total_iter + 2``
as the reference returns it) and x' (float32 of the FP64 result).  The oracle
(oracle/dpf_oracle.py, pinned to the reference's own OT fixture G4) runs with its two live
potentials (the other two never reach the output, resamplers.py:139-147).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "tests", "golden", "ot_c4_share.npz")
SEED = 20261018
B, N = 32, 4000


def ot_share_input(seed: int = SEED, B: int = B, N: int = N):
    """32 particle clouds of a C4-like spread (rows 10^0.5 .. 10^2.5 px wide, a third of them
    bimodal) with likelihood weights of varied degeneracy: float32 x [B, N, 2], w [B, N]."""
    g = np.random.default_rng(seed)
    x = np.empty((B, N, 2), np.float64)
    lw = np.empty((B, N), np.float64)
    for b in range(B):
        c = g.uniform(-64, 64, size=2)
        sd = 10 ** g.uniform(0.5, 2.5)
        xb = c + sd * g.normal(size=(N, 2))
        if b % 3 == 0:  # bimodal: a second cloud
            k = N // 3
            xb[:k] += sd * g.uniform(2, 4, size=2)
        tgt = c + sd * g.normal(size=2) * 0.5
        r = sd * g.uniform(0.15, 1.0)
        x[b] = xb
        lw[b] = -((xb - tgt) ** 2).sum(-1) / (2 * r * r)
    lw -= lw.max(1, keepdims=True)
    w = np.exp(lw)
    w /= w.sum(1, keepdims=True)
    return x.astype(np.float32), w.astype(np.float32)


def main():
    sys.path.insert(0, ROOT)
    import torch
    from oracle import dpf_oracle as O
    torch.set_num_threads(len(os.sched_getaffinity(0)))
    O.OT_POTENTIALS = 2
    x, w = ot_share_input()
    t0 = time.time()
    xt, wt = torch.from_numpy(x), torch.from_numpy(w)
    with torch.no_grad():
        _, _, _, info = O.ot_resample(xt, wt, return_info=True)
        xr64 = torch.matmul(info["T"].double(), xt.double())  # x' with the transport applied in fp64
    print(f"iterations {info['iters']}, {time.time() - t0:.0f} s")
    np.savez_compressed(OUT, seed=np.int64(SEED), iters=np.int64(info["iters"]), xr=xr64.numpy().astype(np.float32))


if __name__ == "__main__":
    main()
