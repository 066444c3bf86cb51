"""Timing of the sharded gated pass on ONE GPU: 2 processes x 32 rows of the c2_full workload
(B = 64, N = 1000, T = 50; the gate fires on a mix of steps), their gated passes concurrent and
the batch gate exchanged through the IPC-mapped buffers every step -- against the unsharded gated
pass of the 64 rows, and the sharded plan pass (NFDPF_XGATE=0, cfg.pass_plan).  Prints one JSON
line per mode: ms per pass (max over ranks, barrier + synchronize around K passes).

    python scripts/r06_xgate_time.py [K]
"""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normalizing-flows-dpfs_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

B, N, T = 64, 1000, 50


def run(rank, world, K, mode, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NFDPF_PASS_SHARED_OK="1")
    if mode == "plan":
        os.environ["NFDPF_XGATE"] = "0"
    torch.cuda.set_device(0)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    import _fullsize as F
    from nfdpf import _lib
    from nfdpf.engine import FilterConfig, FilterEngine, ShardInfo
    _lib.load()
    wl = F.workload("c2_full", B=B, N=N, T=T)
    h = B // world
    sl = slice(rank * h, (rank + 1) * h)
    models = wl["models"].to("cuda:0")
    enc, start, vel = (wl[k][sl].to("cuda:0") for k in ("enc", "start", "vel"))
    shard = ShardInfo.from_env(h) if world > 1 else None
    cfg = FilterConfig(N=N, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", seed=5, kernel="tiled",
                       pass_plan=True if mode == "plan" else None)
    eng = FilterEngine(cfg, models)
    for _ in range(3):
        eng.run(enc, start, vel, shard=shard)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(K):
        eng.run(enc, start, vel, shard=shard)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ms = (time.perf_counter() - t0) / K * 1e3
    # the pass kernel itself (events in its own dispatch), K more passes, each after a barrier:
    # sharded, a kernel also waits for the other rank's to start -- the minimum is the closest
    # to no launch skew
    kms = []
    for _ in range(K):
        if world > 1:
            dist.barrier()
        eng.step_events = []
        eng.run(enc, start, vel, shard=shard)
        kms.append(eng.step_events[0].ms())
        eng.step_events = None
    kms.sort()
    out = dict(mode=mode, world=world, rank=rank, ms_per_pass=ms, kernel_ms_min=kms[0], kernel_ms_median=kms[len(kms) // 2],
               gated=eng.last_gate_pass, plan=eng.last_plan_pass,
               launches=eng.pass_launches, fired=None if eng.last_gates is None else int(eng.last_gates.sum()),
               plan_misses=eng.plan_misses, disabled=eng.pass_disabled)
    if world > 1:
        dist.destroy_process_group()
    q.put(out)


def main():
    import torch.multiprocessing as mp
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    ctx = mp.get_context("spawn")
    for mode, world in (("gated", 1), ("gated", 2), ("plan", 2)):
        q = ctx.Queue()
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        ps = [ctx.Process(target=run, args=(r, world, K, mode, port, q)) for r in range(world)]
        for p in ps:
            p.start()
        outs = [q.get(timeout=600) for _ in ps]
        for p in ps:
            p.join()
        ms = max(o["ms_per_pass"] for o in outs)
        print(json.dumps(dict(mode=mode, world=world, rows_per_rank=B // world, ms_per_pass=round(ms, 4),
                              kernel_ms_min=max(o["kernel_ms_min"] for o in outs),
                              kernel_ms_median=max(o["kernel_ms_median"] for o in outs),
                              particle_steps_per_s=B * N * T / (ms * 1e-3), ranks=outs)), flush=True)


if __name__ == "__main__":
    main()
