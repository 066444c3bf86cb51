"""CPU-baseline faithfulness record: the bench's `cpu_baseline` times the
oracle (oracle/dpf_oracle.py, a timing-faithful PyTorch-CPU restatement of DPF.filtering_pos)
because the reference itself cannot travel to the GPU box.  This script times BOTH here, in
the build container, on the same bounded samples bench.py's cpu_baseline uses (C1-C3), and
records the restatement / reference time ratio (target: within +-20 %).

    python scripts/cpu_baseline_fidelity.py [--threads 8] [--out profiles/r04/cpu_baseline_fidelity.json]

Build container only (reads /root/reference; never run on the GPU box).  Each leg runs in its
own subprocess: the reference and this repo both have a top-level ``DPFs`` module.
"""
import argparse
import json
import os
import subprocess
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def sample(cfg_name):
    """bench.cpu_baseline's sample for a config: (flags, B, N, T, Bs, Ts)."""
    sys.path.insert(0, ROOT)
    from bench import CONFIGS
    flags, B, N, T, _, _ = CONFIGS[cfg_name]
    Bs, Ts = B, T
    if flags["resampler_type"] == "ot":
        Bs, Ts = max(1, B // 16), min(T, 10)
    return flags, B, N, T, Bs, Ts


def inputs_file(cfg_name):
    """The leg's inputs, written by the parent (the reference leg must not import bench.py: it
    puts this repo's package -- whose regular packages shadow the reference's namespace
    packages -- on sys.path)."""
    import torch
    flags, B, N, T, Bs, Ts = sample(cfg_name)
    from bench import synthetic_disk
    start, state, vel, enc = synthetic_disk(B, T, 2, 32)
    path = f"/tmp/nfdpf_fidelity_{cfg_name}.pt"
    torch.save({"flags": flags, "B": B, "N": N, "T": T, "Bs": Bs, "Ts": Ts, "enc": enc[:Bs, :Ts],
                "start": start[:Bs], "vel": vel[:Bs, :Ts]}, path)
    return path


def leg(which, cfg_name, threads, reps):
    import torch
    torch.set_num_threads(threads)
    inp = torch.load(f"/tmp/nfdpf_fidelity_{cfg_name}.pt", weights_only=True)
    flags, B, N, T, Bs, Ts = (inp[k] for k in ("flags", "B", "N", "T", "Bs", "Ts"))
    enc, start, vel = inp["enc"], inp["start"], inp["vel"]
    if which == "reference":
        sys.dont_write_bytecode = True
        sys.path.insert(0, REF)
        for name in ("cv2", "torch.utils.tensorboard"):  # imported, unused on this path (gen_golden.py)
            sys.modules.setdefault(name, types.ModuleType(name))
        sys.modules["torch.utils.tensorboard"].SummaryWriter = object
        import arguments
        from DPFs import DPF
        saved = sys.argv
        sys.argv = ["fidelity"]
        a = arguments.parse_args()
        sys.argv = saved
        a.num_particles, a.batchsize, a.sequence_length = N, Bs, Ts
        for k, v in flags.items():
            setattr(a, k, v)
        torch.manual_seed(2)
        dpf = DPF(a).eval()
        dpf.encoder = torch.nn.Identity()  # precomputed encodings, as bench.py and BASELINE.md
        run = lambda: dpf.filtering_pos(enc, start, vel)  # noqa: E731
    else:
        sys.path.insert(0, ROOT)
        from bench import make_args
        from DPFs import DPF
        from oracle import dpf_oracle as O
        torch.manual_seed(2)
        dpf = DPF(make_args(flags, B, N, T, {}))
        params = {k: v.detach().float().cpu() for k, v in dpf.state_dict().items()}
        cfg = dict(N=N, NF_dyn=flags["NF_dyn"], NF_cond=flags["NF_cond"], measurement=flags["measurement"],
                   resampler=flags["resampler_type"], alpha=0.5, eps=0.1, scaling=0.75, threshold=1e-3, max_iter=100,
                   pos_noise=20.0, vel_noise=20.0, width=128, n_flows=2, cglow_K=1,
                   dyn_flow=flags.get("NF_dyn_flow", "RealNVP"))
        run = lambda: O.filtering(cfg, params, enc, start, vel, rng=O.HostRNG())  # noqa: E731
    times = []
    with torch.no_grad():
        torch.manual_seed(3)
        run()  # warm-up
        for _ in range(reps):
            torch.manual_seed(3)
            t0 = time.perf_counter()
            run()
            times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2]
    return {"which": which, "config": cfg_name, "sample": f"B={Bs} N={N} T={Ts}", "median_s": med, "times_s": times,
            "particle_steps_per_s": Bs * N * Ts / med, "threads": threads}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--configs", default="c1,c2,c3")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r04", "cpu_baseline_fidelity.json"))
    ap.add_argument("--leg", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--config", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.leg:
        print(json.dumps(leg(args.leg, args.config, args.threads, args.reps)))
        return
    rows = []
    for c in args.configs.split(","):
        r = {}
        inputs_file(c)
        for which in ("reference", "oracle"):
            out = subprocess.run([sys.executable, __file__, "--leg", which, "--config", c, "--threads",
                                  str(args.threads), "--reps", str(args.reps)], capture_output=True, text=True,
                                 check=True).stdout
            r[which] = json.loads(out.strip().splitlines()[-1])
        ratio = r["oracle"]["median_s"] / r["reference"]["median_s"]
        rows.append({"config": c, "sample": r["oracle"]["sample"], "reference_s": r["reference"]["median_s"],
                     "oracle_s": r["oracle"]["median_s"], "oracle_over_reference_time": ratio,
                     "within_20pct": abs(ratio - 1.0) <= 0.2, "reference": r["reference"], "oracle": r["oracle"]})
        print(json.dumps(rows[-1]))
    import platform
    rec = {"what": "cpu_baseline faithfulness: oracle (restatement) vs reference DPF.filtering_pos wall time, "
                   "same sample, same thread count, build container (SURVEY.md §8(d))",
           "host": platform.processor() or platform.machine(), "threads": args.threads, "rows": rows}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
