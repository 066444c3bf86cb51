"""Batch sharding through nfdpf.engine.FilterEngine on the GPU: two ranks (gloo, both on
cuda:0 -- RCCL refuses two ranks on one device; the exchange code is the same) each filter
half of the batch's rows and must return exactly the unsharded pass's rows (SURVEY.md §4.4,
§8(e); DPFs.py:163-166 batch-global ESS gate, resamplers.py:126-129 batch-coupled Sinkhorn
stop).  GPU box only.

Cases (tests/_fullsize.py workloads, device RNG keyed on the GLOBAL row):
  * soft_gated -- C2 flags (NF dyn + NF proposal, cos, soft), aligned frame encodings: the ESS
    gate fires on some steps, so the auto mode's speculative pass misses and reruns with the
    per-step exchange of the tiled partials;
  * ot_gated -- C3 flags (CRNVP, OT): the speculative OT pass misses, the per-step pass reads
    every gate and runs the two-phase sharded Sinkhorn (ops.ot_resample_sharded);
  * ot_forced -- C4 flags (MAF dyn flow, NF proposal, cos, OT every step).
Histories and indices must be bit-identical; the obs-likelihood is an fp64 sum reduced in a
different order (per rank, then across ranks), then rounded to float32: 1e-6 relative.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

# name: (_fullsize case, B, N, T)
CASES = {
    "soft_gated": ("c2_full", 8, 1000, 12),
    "ot_gated": ("c3_full", 8, 1000, 6),
    "ot_forced": ("c4_n4000", 4, 2000, 3),
}
FIELDS = ("particles", "probs", "noise", "lik", "index", "jac", "prior", "pred")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(case, rows, shard=None):
    import _fullsize as F
    from nfdpf.engine import FilterConfig, FilterEngine
    name, B, N, T = CASES[case]
    wl = F.workload(name, B=B, N=N, T=T)
    c = F.cfg_dict(wl["flags"], N)
    # (pass_gate off: the unsharded run's rerun after a fired gate is then the step launches, as the
    # sharded ranks' -- the gated one-launch pass needs the whole batch on one GPU)
    cfg = FilterConfig(N=N, NF_dyn=c["NF_dyn"], NF_cond=c["NF_cond"], measurement=c["measurement"],
                       resampler=c["resampler"], dyn_flow=c["dyn_flow"], force_resample=wl["force"], seed=123,
                       kernel="tiled", pass_gate=False)
    eng = FilterEngine(cfg, wl["models"].to(DEV))
    sl = slice(*rows)
    res = eng.run(wl["enc"][sl].to(DEV), wl["start"][sl].to(DEV), wl["vel"][sl].to(DEV), shard=shard)
    torch.cuda.synchronize()
    out = {f: getattr(res, f).cpu() for f in FIELDS if getattr(res, f) is not None}
    out["obs_likelihood"] = res.obs_likelihood.cpu()
    out["ot_calls"] = eng.last_ot_calls
    return out


def _worker(rank, world, port, case, path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "normalizing-flows-dpfs_amd"), root, os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nfdpf import _lib
        from nfdpf.engine import ShardInfo
        _lib.load()
        B = CASES[case][1] // world
        out = _run(case, (rank * B, (rank + 1) * B), ShardInfo.from_env(B))
        torch.save(out, f"{path}.{rank}")
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("case", list(CASES))
def test_sharded_engine_matches_unsharded(case, tmp_path):
    import torch.multiprocessing as mp
    from nfdpf import _lib
    _lib.load()
    B = CASES[case][1]
    full = _run(case, (0, B))
    world = 2
    path = str(tmp_path / "shard")
    mp.start_processes(_worker, args=(world, _free_port(), case, path), nprocs=world, start_method="spawn")
    parts = [torch.load(f"{path}.{r}", weights_only=True) for r in range(world)]
    h = B // world
    for f in FIELDS:
        if f not in full:
            continue
        for r, part in enumerate(parts):
            assert torch.equal(part[f], full[f][r * h:(r + 1) * h]), (case, f, r)
    for part in parts:
        a, b = float(part["obs_likelihood"]), float(full["obs_likelihood"])
        assert abs(a - b) <= 1e-6 * abs(b), (a, b)  # float32 of the fp64 sums
        assert part["ot_calls"] == full["ot_calls"]
    ident = torch.arange(CASES[case][2]) + CASES[case][2] * torch.arange(B)[:, None]
    fired = int((full["index"] != ident[:, None, :]).any(-1).any(0).sum())
    print(f"\n{case}: B={B} over {world} ranks, resampling fired in {fired} steps, OT calls {full['ot_calls']}")
    assert fired > 0 or full["ot_calls"] > 0


# ---- the one-launch pass, sharded (nfdpf_filter_pass_tiled + finish_pending's all-gather and
# batch gate): "quiet" = the bench's model at its init weights on N(0,1) encodings (no gate
# fires: the sharded passes ARE the result), "firing" = the c2_full workload (aligned encodings:
# the gathered verification catches the fired gate and every rank reruns with the per-step
# exchange)
# (firing_gated: the same, with the gated pass allowed -- the rerun after the missed speculation is
# then the gated pass on every rank, the batch gate exchanged inside the launches, round 6)
PASS_CASES = {"quiet": (8, 1000, 12), "firing": (8, 1000, 12), "firing_gated": (8, 1000, 12),
              "quiet_c3": (8, 1000, 12)}


def _pass_inputs(kind, rows):
    """-> (models on DEV, enc, start, vel) of the case's rows."""
    B, N, T = PASS_CASES[kind]
    sl = slice(*rows)
    if kind in ("quiet", "quiet_c3"):  # (quiet_c3: the C3 shape, tiled_pass_cm_kernel, OT resampler)
        import bench
        from DPFs import DPF
        flags = bench.CONFIGS["c2" if kind == "quiet" else "c3"][0]
        torch.manual_seed(2)
        models = DPF(bench.make_args(flags, B, N, T, {})).to(DEV).eval()
        g = torch.Generator().manual_seed(31)
        enc, start, vel = torch.randn(B, T, 32, generator=g), torch.randn(B, 4, generator=g) * 10, \
            torch.randn(B, T, 2, generator=g) * 3
    else:  # firing, firing_gated
        import _fullsize as F
        wl = F.workload("c2_full", B=B, N=N, T=T)
        models, enc, start, vel = wl["models"].to(DEV), wl["enc"], wl["start"], wl["vel"]
    return models, enc[sl].to(DEV), start[sl].to(DEV), vel[sl].to(DEV)


def _pass_run(kind, rows, shard=None, rank=0, world=1):
    """The auto-mode engine on the case's rows: a speculative one-launch pass (run(finish=False);
    sharded, the ranks' passes run one after the other -- they share the one GPU, and each grid
    must be resident by itself), then finish_pending (sharded: one all-gather of all steps'
    partials and the batch gate) and, if a gate fired, the per-step rerun."""
    import torch.distributed as dist
    from nfdpf.engine import FilterConfig, FilterEngine
    B, N, T = PASS_CASES[kind]
    models, enc, start, vel = _pass_inputs(kind, rows)
    if kind == "quiet_c3":
        cfg = FilterConfig(N=N, NF_dyn=False, NF_cond=False, measurement="CRNVP", resampler="ot", seed=321,
                           kernel="tiled")
    else:
        cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=321,
                           kernel="tiled",  # (firing: the unsharded rerun by the step launches, as the ranks')
                           pass_gate=None if kind == "firing_gated" else False)
    eng = FilterEngine(cfg, models)
    for r in range(world):
        if r == rank:
            res = eng.run(enc, start, vel, shard=shard, finish=False, speculate=True)
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
    launched = eng.last_pass
    verified = eng.finish_pending()
    eng._pending = None
    if not verified:
        res = eng.run(enc, start, vel, shard=shard, speculate=False)
    torch.cuda.synchronize()
    out = {f: getattr(res, f).cpu() for f in FIELDS if getattr(res, f) is not None}
    out["obs_likelihood"] = res.obs_likelihood.cpu()
    out["launched"], out["verified"], out["gated"] = launched, verified, eng.last_gate_pass
    return out


def _worker_pass(rank, world, port, kind, path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "normalizing-flows-dpfs_amd"), root, os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NFDPF_PASS_SHARED_OK="1")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nfdpf import _lib
        from nfdpf.engine import ShardInfo
        _lib.load()
        B = PASS_CASES[kind][0] // world
        out = _pass_run(kind, (rank * B, (rank + 1) * B), ShardInfo.from_env(B), rank, world)
        torch.save(out, f"{path}.{rank}")
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("kind", list(PASS_CASES))
def test_sharded_pass_matches_unsharded(kind, tmp_path):
    """The one-launch pass on two ranks (rows [0, 4) and [4, 8), device RNG keyed on the global
    row) == the unsharded pass, bit for bit: every history; the obs-likelihood to 1e-6 (an fp64
    sum reduced per rank, then across ranks).  quiet: the sharded passes verify and are the
    result; firing: the gathered verification catches the fired gate on both ranks alike and the
    per-step rerun is returned.  (The test-only NFDPF_PASS_SHARED_OK lets ranks that share the one
    GPU run the pass, serialised by barriers.)"""
    import torch.multiprocessing as mp
    from nfdpf import _lib
    _lib.load()
    B = PASS_CASES[kind][0]
    full = _pass_run(kind, (0, B))
    assert full["launched"], "the unsharded one-launch pass did not run"
    assert full["verified"] == (kind not in ("firing", "firing_gated"))
    assert full["gated"] == (kind == "firing_gated")
    world = 2
    path = str(tmp_path / "pass")
    mp.start_processes(_worker_pass, args=(world, _free_port(), kind, path), nprocs=world, start_method="spawn")
    parts = [torch.load(f"{path}.{r}", weights_only=True) for r in range(world)]
    h = B // world
    for r, part in enumerate(parts):
        assert part["launched"], f"rank {r}: the sharded one-launch pass did not run"
        assert part["verified"] == full["verified"], (r, part["verified"])
        assert part["gated"] == full["gated"], (r, part["gated"])  # firing_gated: the sharded GATED pass
        for f in FIELDS:
            if f in full:
                assert torch.equal(part[f], full[f][r * h:(r + 1) * h]), (kind, f, r)
        a, b = float(part["obs_likelihood"]), float(full["obs_likelihood"])
        assert abs(a - b) <= 1e-6 * abs(b), (a, b)


# ---- gate plans, sharded: the exact run (per-step exchange) records the batch's gates, the next
# pass follows them as one launch per rank (no exchange inside it) and one all-gather verifies it
def _plan_run(rows, shard=None, rank=0, world=1):
    import torch.distributed as dist
    from nfdpf.engine import FilterConfig, FilterEngine
    B, N, T = PASS_CASES["firing"]
    models, enc, start, vel = _pass_inputs("firing", rows)
    cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=321,
                       kernel="tiled", pass_plan=True)  # (unsharded: the gated pass's decisions, then plans)
    eng = FilterEngine(cfg, models)
    eng.run(enc, start, vel, shard=shard, speculate=False)  # exact; its gates become the plan
    plan = None if eng._plan is None else eng._plan.copy()
    for r in range(world):  # (the ranks share the one GPU: each pass's grid resident by itself)
        if r == rank:
            res = eng.run(enc, start, vel, shard=shard, finish=False)
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
    planned = eng.last_plan_pass
    verified = eng.finish_pending()
    eng._pending = None
    torch.cuda.synchronize()
    out = {f: getattr(res, f).cpu() for f in FIELDS if getattr(res, f) is not None}
    out["obs_likelihood"] = res.obs_likelihood.cpu() if verified else torch.tensor(float("nan"))
    out["planned"], out["verified"], out["plan"] = planned, verified, torch.from_numpy(plan)
    return out


def _worker_plan(rank, world, port, path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "normalizing-flows-dpfs_amd"), root, os.path.join(root, "tests")]
    # (NFDPF_XGATE=0: the exact sharded run is the step launches' per-step exchange, not the gated
    # pass through the cross-rank exchange -- test_sharded_gated_pass_matches_unsharded covers that)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NFDPF_PASS_SHARED_OK="1", NFDPF_XGATE="0")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nfdpf import _lib
        from nfdpf.engine import ShardInfo
        _lib.load()
        B = PASS_CASES["firing"][0] // world
        out = _plan_run((rank * B, (rank + 1) * B), ShardInfo.from_env(B), rank, world)
        torch.save(out, f"{path}.{rank}")
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_plan_pass_matches_unsharded(tmp_path):
    """The firing case on two ranks: the exact sharded run (step launches, one all-gather per
    step) records the same batch gates as the unsharded gated pass decides; the next pass on each
    rank follows them as ONE launch with no exchange inside (d.pass_plan) and the one all-gather
    after it verifies them -- bit for bit the unsharded plan pass (every history; obs to 1e-6)."""
    import torch.multiprocessing as mp
    from nfdpf import _lib
    _lib.load()
    B = PASS_CASES["firing"][0]
    full = _plan_run((0, B))
    assert full["planned"] and full["verified"] and int(full["plan"].sum()) > 0
    world = 2
    path = str(tmp_path / "plan")
    mp.start_processes(_worker_plan, args=(world, _free_port(), path), nprocs=world, start_method="spawn")
    parts = [torch.load(f"{path}.{r}", weights_only=True) for r in range(world)]
    h = B // world
    for r, part in enumerate(parts):
        assert torch.equal(part["plan"], full["plan"]), (r, part["plan"], full["plan"])
        assert part["planned"] and part["verified"], (r, part["planned"], part["verified"])
        for f in FIELDS:
            if f in full:
                assert torch.equal(part[f], full[f][r * h:(r + 1) * h]), (f, r)
        a, b = float(part["obs_likelihood"]), float(full["obs_likelihood"])
        assert abs(a - b) <= 1e-6 * abs(b), (a, b)


# ---- the gated pass, sharded: the batch-global gate through the cross-rank exchange (IPC-mapped
# buffers, ops.GateExchange) inside every rank's launch
def _xgate_run(rows, shard=None, world=1):
    from nfdpf.engine import FilterConfig, FilterEngine
    B, N, T = PASS_CASES["firing"]
    models, enc, start, vel = _pass_inputs("firing", rows)
    cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=321, kernel="tiled")
    eng = FilterEngine(cfg, models)
    outs = []
    for _ in range(2):  # (twice: the exchange's epoch carries from pass to pass)
        res = eng.run(enc, start, vel, shard=shard, speculate=False)
        torch.cuda.synchronize()
        out = {f: getattr(res, f).cpu() for f in FIELDS if getattr(res, f) is not None}
        out["obs_likelihood"] = res.obs_likelihood.cpu()
        out["gated"], out["launches"] = eng.last_gate_pass, eng.pass_launches
        out["gates"] = eng.last_gates.cpu() if eng.last_gates is not None else None
        outs.append(out)
    return outs


def _worker_xgate(rank, world, port, path):
    import sys
    import warnings
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "normalizing-flows-dpfs_amd"), root, os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NFDPF_PASS_SHARED_OK="1")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nfdpf import _lib
        from nfdpf.engine import ShardInfo
        _lib.load()
        B = PASS_CASES["firing"][0] // world
        with warnings.catch_warnings(record=True) as wl:
            warnings.simplefilter("always")
            outs = _xgate_run((rank * B, (rank + 1) * B), ShardInfo.from_env(B), world)
        outs[0]["warnings"] = [str(w.message) for w in wl]
        torch.save(outs, f"{path}.{rank}")
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_gated_pass_matches_unsharded(tmp_path):
    """The firing case on two ranks, their gated one-launch passes running CONCURRENTLY on the one
    GPU (each grid of 4 rows x 4 tiles; NFDPF_PASS_SHARED_OK): every step's batch-global gate is
    decided inside both launches from the 8 rows' terms swept through the IPC-mapped exchange
    buffers (d.gate_peers) -- no fallback, no per-step all-gather.  Both passes of each rank equal
    the unsharded gated pass bit for bit (every history and every decision; obs to 1e-6)."""
    import torch.multiprocessing as mp
    from nfdpf import _lib
    _lib.load()
    B = PASS_CASES["firing"][0]
    full = _xgate_run((0, B))
    assert full[0]["gated"] and full[0]["launches"] == 1 and int(full[0]["gates"].sum()) > 0
    world = 2
    path = str(tmp_path / "xgate")
    mp.start_processes(_worker_xgate, args=(world, _free_port(), path), nprocs=world, start_method="spawn")
    parts = [torch.load(f"{path}.{r}", weights_only=True) for r in range(world)]
    h = B // world
    for r, outs in enumerate(parts):
        assert not outs[0]["warnings"], (r, outs[0]["warnings"])
        for k, (o, f) in enumerate(zip(outs, full)):
            assert o["gated"] and o["launches"] == k + 1, (r, k, o["gated"], o["launches"])
            assert torch.equal(o["gates"], f["gates"]), (r, k, o["gates"], f["gates"])
            for fld in FIELDS:
                if fld in f:
                    assert torch.equal(o[fld], f[fld][r * h:(r + 1) * h]), (fld, r, k)
            a, b = float(o["obs_likelihood"]), float(f["obs_likelihood"])
            assert abs(a - b) <= 1e-6 * abs(b), (a, b)
