"""world_size-2 rehearsal (gloo, CPU) of the batch-sharded exchange logic of nfdpf.engine:
shard geometry, the per-step all-gather of per-row ESS terms feeding an identical gate on
every rank, host-draw slicing in parity mode, the MIN of the Sinkhorn stop iteration and the
end-of-sequence obs-likelihood reduce.
The RCCL/GPU path uses the same code with device tensors."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "normalizing-flows-dpfs_amd"), root]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nfdpf.engine import FilterEngine, HostDraws, ShardInfo
        B, N = 3, 50
        sh = ShardInfo.from_env(B)
        g = torch.Generator().manual_seed(7)
        inv_all = torch.rand(world * B, generator=g) * N
        mine = inv_all[sh.row_base:sh.row_base + B].contiguous()
        gathered = FilterEngine._gather(mine, sh)
        gate = FilterEngine._host_gate(gathered, N, False)
        # parity-mode draws: every rank draws the GLOBAL tensor and keeps its rows
        h = HostDraws(torch.Generator().manual_seed(11))
        nz = h.noise(sh.B_global, N, 20.0)[sh.row_base:sh.row_base + B]
        lw = torch.full((B, 4), float(rank + 1))
        tot = lw.double().sum(0)
        dist.all_reduce(tot)
        # speculative-gate verification: every step's [B, tiles, 4] partials gathered at once
        steps = torch.arange(5 * B * 3 * 4, dtype=torch.float64).reshape(5, B, 3, 4) + 1000 * rank
        allsteps = FilterEngine._gather_steps(steps, sh)
        # OT stop (engine._ot_global_stop): the MIN over ranks of the local iteration count
        it = torch.tensor([31 + 7 * rank], dtype=torch.int32)
        dist.all_reduce(it, op=dist.ReduceOp.MIN)
        q.put((rank, sh.world, sh.B_global, sh.row_base, gathered.numpy(), gate, nz.numpy(), tot.numpy(),
               int(it.item()), allsteps.numpy()))
    finally:
        dist.destroy_process_group()


def test_sharded_exchange_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "normalizing-flows-dpfs_amd"), root]
    from nfdpf.engine import FilterEngine, HostDraws
    B, N = 3, 50
    inv_all = torch.rand(world * B, generator=torch.Generator().manual_seed(7)) * N
    ref_gate = FilterEngine._host_gate(inv_all, N, False)
    ref_noise = HostDraws(torch.Generator().manual_seed(11)).noise(world * B, N, 20.0)
    steps = [torch.arange(5 * B * 3 * 4, dtype=torch.float64).reshape(5, B, 3, 4) + 1000 * r for r in range(world)]
    ref_steps = torch.cat(steps, 1).numpy()  # [T, B_global, tiles, 4], rows in rank order
    for rank, w, bg, base, gathered, gate, nz, tot, it, allsteps in res:
        np.testing.assert_array_equal(allsteps, ref_steps)
        assert it == 31
        assert (w, bg, base) == (world, world * B, rank * B)
        np.testing.assert_array_equal(gathered, inv_all.numpy())
        assert gate == ref_gate
        np.testing.assert_array_equal(nz, ref_noise[rank * B:(rank + 1) * B].numpy())
        np.testing.assert_array_equal(tot, np.full(4, 3.0 * (1 + 2)))


def test_single_process_shard_is_identity():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "normalizing-flows-dpfs_amd"), root]
    from nfdpf.engine import ShardInfo
    sh = ShardInfo.from_env(5)
    assert (sh.world, sh.B_global, sh.row_base) == (1, 5, 0)


def _grad_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "normalizing-flows-dpfs_amd"), root]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nfdpf.gradsync import GradBucket, global_mean
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.Tanh(), torch.nn.Linear(4, 2))
        x = torch.randn(5, 3, generator=torch.Generator().manual_seed(100 + rank))
        m(x).pow(2).mean().backward()
        m[2].bias.grad = None if rank == 1 else m[2].bias.grad  # a gradient missing on one rank
        GradBucket(m).sync()
        inv = torch.arange(3, dtype=torch.float32) + 10 * rank
        ess = global_mean(inv.sum(), inv.numel())
        q.put((rank, [p.grad.clone().numpy() for p in m.parameters()], float(ess)))
    finally:
        dist.destroy_process_group()


def test_grad_bucket_world2():
    """nfdpf.gradsync: one all-reduce averages the ranks' gradients (== the gradient of the
    mean loss over both shards); global_mean is the batch-global ESS mean."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.Tanh(), torch.nn.Linear(4, 2))
    grads = []
    for r in range(world):
        m.zero_grad()
        m(torch.randn(5, 3, generator=torch.Generator().manual_seed(100 + r))).pow(2).mean().backward()
        g = [p.grad.clone() for p in m.parameters()]
        if r == 1:
            g[3] = torch.zeros_like(g[3])
        grads.append(g)
    ref = [(a + b) / 2 for a, b in zip(*grads)]
    for rank, gs, ess in res:
        for a, b in zip(gs, ref):
            np.testing.assert_allclose(a, b.numpy(), rtol=1e-6, atol=1e-7)
        assert abs(ess - (0 + 1 + 2 + 10 + 11 + 12) / 6) < 1e-6


def _rmse_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "normalizing-flows-dpfs_amd"), root]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nfdpf.gradsync import GradBucket, sharded_supervised_loss
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.Tanh(), torch.nn.Linear(4, 2))
        unused = torch.nn.Linear(2, 2)  # touched by no rank: its .grad must stay None
        holder = torch.nn.ModuleDict({"m": m, "unused": unused})
        B, T, N = 3, 4, 5
        g = torch.Generator().manual_seed(100 + rank)
        x = torch.randn(B, T, N, 3, generator=g)
        w = torch.softmax(torch.randn(B, T, N, generator=g), -1)
        state = torch.randn(B, T, 4, generator=g)
        mask = (torch.rand(B, T, generator=g) > 0.3).float()
        loss, _ = sharded_supervised_loss(m(x), w, state, mask, True, 0.7)
        loss.backward()
        GradBucket(holder).sync()
        ev, _ = sharded_supervised_loss(m(x).detach(), w, state, mask, False)
        q.put((rank, float(loss), [p.grad.clone().numpy() for p in m.parameters()],
               [p.grad is None for p in unused.parameters()], float(ev)))
    finally:
        dist.destroy_process_group()


def test_sharded_rmse_gradient_world2():
    """The batch-sharded supervised RMSE (nfdpf.gradsync.sharded_supervised_loss + GradBucket)
    has the value AND the gradient of the single-device full-batch RMSE (losses.py:18-31) --
    not the average of per-shard RMSE gradients; a parameter no rank used keeps .grad None."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rmse_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "normalizing-flows-dpfs_amd"), root]
    from losses import supervised_loss
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.Tanh(), torch.nn.Linear(4, 2))
    B, T, N = 3, 4, 5
    xs, ws, ss, ms = [], [], [], []
    for r in range(world):
        g = torch.Generator().manual_seed(100 + r)
        xs.append(torch.randn(B, T, N, 3, generator=g))
        ws.append(torch.softmax(torch.randn(B, T, N, generator=g), -1))
        ss.append(torch.randn(B, T, 4, generator=g))
        ms.append((torch.rand(B, T, generator=g) > 0.3).float())
    x, w, s, mk = (torch.cat(v) for v in (xs, ws, ss, ms))
    loss, _ = supervised_loss(m(x), w, s, mk, True, 0.7)
    loss.backward()
    ev, _ = supervised_loss(m(x).detach(), w, s, mk, False)
    for rank, l, gs, unused_none, e in res:
        assert abs(l - loss.item()) < 1e-5 * loss.item()
        assert abs(e - float(ev)) < 1e-5 * float(ev)
        for a, p in zip(gs, m.parameters()):
            np.testing.assert_allclose(a, p.grad.numpy(), rtol=1e-5, atol=1e-7)
        assert all(unused_none)


def _ot_stop_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "normalizing-flows-dpfs_amd"), root]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import resamplers.resamplers as R
        calls = []

        def fake_local(x, w, eps, scaling, threshold, max_iter, ws, hist, gate=None, poll=None):
            # local stop rule: rank r's rows converge after 20 + 9 r iterations
            calls.append("local")
            return torch.tensor([20 + 9 * rank], dtype=torch.int32)

        def fake_finish(x, eps, scaling, threshold, max_iter, row_base, ws, hist, stop_at, gate=None):
            calls.append(int(stop_at.item()))
            return x + int(stop_at.item()), torch.full(x.shape[:2], 0.2), torch.zeros(x.shape[:2], dtype=torch.int64)

        R._ops.ot_sinkhorn_local, R._ops.ot_sinkhorn_finish = fake_local, fake_finish
        x = torch.zeros(2, 5, 2)
        w = torch.full((2, 5), 0.2)
        xo, _, _ = R.resampler_ot(x, w)
        q.put((rank, calls, float(xo[0, 0, 0])))
    finally:
        dist.destroy_process_group()


def test_ot_stop_exchange_in_autograd_loop_world2():
    """resampler_ot under batch sharding (the e2e_train loop, resamplers.py:126-129): each rank
    runs its local stop rule, the ranks take the MIN iteration, and every rank finishes at that
    state (ops.ot_resample_sharded: one local loop, no rerun)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ot_stop_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, calls, x0 in res:
        assert calls == ["local", 20], calls
        assert x0 == 20.0


def _worker_verify(rank, world, port, q):
    """FilterEngine._sharded_verify's plumbing (the summary layout, the rank-major row order of the
    gathered terms, the fault and step-sum reductions) on CPU tensors, with the two kernels
    restated in torch (their arithmetic is pinned on the GPU: test_row_terms_gates_match_gate_batch)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "normalizing-flows-dpfs_amd"), root]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nfdpf import ops
        from nfdpf.engine import FilterEngine, ShardInfo
        T, B, N = 5, 3, 50

        def row_terms(parts, N, t0=0, out=None):  # terms [T*B] (t-major) then the fault word
            terms = parts[..., 1].sum(-1).float().reshape(-1)
            fault = torch.tensor([rank + 2], dtype=torch.int32).view(torch.float32)
            return torch.cat([terms, fault])

        def gate_terms(terms, N, force=False, out=None):
            return (terms.mean(1) < 0.5 * N).to(torch.int32)
        ops.ess_row_terms, ops.ess_gate_terms = row_terms, gate_terms
        sh = ShardInfo.from_env(B)
        g = torch.Generator().manual_seed(3)
        parts_all = torch.rand(T, world * B, 2, 4, generator=g, dtype=torch.float64) * 40
        tot_all = torch.rand(world, T, generator=g, dtype=torch.float64)
        parts = parts_all[:, rank * B:(rank + 1) * B].contiguous()
        small, tot = FilterEngine._sharded_verify(parts, tot_all[rank].clone(), sh, N)
        q.put((rank, small.numpy(), tot.numpy(), parts_all.numpy(), tot_all.numpy()))
    finally:
        dist.destroy_process_group()


def test_sharded_verify_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_verify, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    T, N = 5, 50
    for rank, small, tot, parts_all, tot_all in out:
        terms = parts_all[..., 1].sum(-1).astype(np.float32)  # [T, world * B], global row order
        gates = (terms.mean(1) < 0.5 * N).astype(np.int64)
        assert np.array_equal(small[:T], gates), (rank, small[:T], gates)
        assert small[T] == sum(r + 2 for r in range(world))  # the fault words, summed over the ranks
        np.testing.assert_allclose(tot, tot_all.sum(0), rtol=0, atol=1e-12)
