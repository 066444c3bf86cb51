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
    """bench.cpu_baseline's sample for a config: (flags, B, N, T, Bs, Ts).  "<cfg>inf": the same
    sample on INFORMATIVE frame encodings (the particle encoder at the true positions, as
    bench.py --enc-from-state), where the ESS gate fires and -- with OT -- the FP64 Sinkhorn runs."""
    sys.path.insert(0, ROOT)
    from bench import CONFIGS
    if cfg_name == "c3fire":  # tests/_fullsize.py's c3_full workload at B = 4: the OT gate fires
        flags, B, N, T, _, _ = CONFIGS["c3"]
        return flags, B, N, T, 4, 10
    flags, B, N, T, _, _ = CONFIGS[cfg_name.replace("inf", "")]
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
    if cfg_name.endswith("inf"):  # the particle encoder (DPF(args) at seed 2, both legs) at the truth
        from bench import make_args
        sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-dpfs_amd"))
        from DPFs import DPF
        torch.manual_seed(2)
        dpf = DPF(make_args(flags, B, N, T, {}))
        with torch.no_grad():
            enc = dpf.particle_encoder(state[:, :, :2].float()).contiguous()
    sd = None
    if cfg_name == "c3fire":
        # the workload's perturbed weights (CRNVP measurement std 0.1, flows 0.05: informative enough
        # that the ESS gate fires and the FP64 Sinkhorn runs), mapped onto the DPF's state_dict names
        sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "normalizing-flows-dpfs_amd")]
        import _fullsize as F
        wl = F.workload("c3_full", B=Bs, N=N, T=Ts)
        enc, start, vel = wl["enc"], wl["start"], wl["vel"]
        sd = {}
        for k, v in wl["models"].state_dict().items():
            sd[k] = v.detach().float().cpu()
            sd["measurement_model." + k] = sd[k]
    path = f"/tmp/nfdpf_fidelity_{cfg_name}.pt"
    torch.save({"flags": flags, "B": B, "N": N, "T": T, "Bs": Bs, "Ts": Ts, "enc": enc[:Bs, :Ts],
                "start": start[:Bs], "vel": vel[:Bs, :Ts], "sd": sd}, path)
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
        if inp["sd"] is not None:
            known = dpf.state_dict()
            dpf.load_state_dict({k: v for k, v in inp["sd"].items() if k in known}, strict=False)
        dpf.encoder = torch.nn.Identity()  # precomputed encodings, as bench.py and BASELINE.md
        calls = []
        fwd = dpf.resampler.forward
        dpf.resampler.forward = lambda *x: (calls.append(1), fwd(*x))[1]  # counts the gate's firings
        run = lambda: dpf.filtering_pos(enc, start, vel)  # noqa: E731
    else:
        sys.path.insert(0, ROOT)
        from bench import make_args
        from DPFs import DPF
        from oracle import dpf_oracle as O
        torch.manual_seed(2)
        dpf = DPF(make_args(flags, B, N, T, {}))
        if inp["sd"] is not None:
            known = dpf.state_dict()
            dpf.load_state_dict({k: v for k, v in inp["sd"].items() if k in known}, strict=False)
        params = {k: v.detach().float().cpu() for k, v in dpf.state_dict().items()}
        cfg = dict(N=N, NF_dyn=flags["NF_dyn"], NF_cond=flags["NF_cond"], measurement=flags["measurement"],
                   resampler=flags["resampler_type"], alpha=0.5, eps=0.1, scaling=0.75, threshold=1e-3, max_iter=100,
                   pos_noise=20.0, vel_noise=20.0, width=128, n_flows=2, cglow_K=1,
                   dyn_flow=flags.get("NF_dyn_flow", "RealNVP"))
        calls = []
        for name in ("soft_resample", "ot_resample"):
            f0 = getattr(O, name)
            setattr(O, name, (lambda f: lambda *x, **k: (calls.append(1), f(*x, **k))[1])(f0))
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
            "particle_steps_per_s": Bs * N * Ts / med, "threads": threads,
            "resampler_calls_per_pass": len(calls) / (reps + 1), "resampler": flags["resampler_type"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--configs", default="c1,c2,c3,c2inf,c3fire")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05", "cpu_baseline_fidelity.json"))
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
                     "within_20pct": abs(ratio - 1.0) <= 0.2,
                     "resampler_calls_per_pass": {"reference": r["reference"]["resampler_calls_per_pass"],
                                                  "oracle": r["oracle"]["resampler_calls_per_pass"],
                                                  "kind": r["oracle"]["resampler"]},
                     "reference": r["reference"], "oracle": r["oracle"]})
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
