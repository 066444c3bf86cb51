"""The fused step (tiled_step_fused_kernel: the merged front launch and the quad proposal launch
as ONE launch per step, the row's x_dyn partials exchanged between its four workgroups through
tagged granules) against the two-launch pipeline it replaces, on the C2 bench workload
(B=64, N=1000, device RNG).  GPU box only.

* gate never fires (the bench's synthetic encodings): the two paths run the same arithmetic
  in the same order -- every output bit-identical;
* --force-resample and a workload whose gate fires (encodings = the particle encoder at the
  true positions): the fused workgroup has 16 waves, so the resampling branch's row sums run
  over a different thread partition (fp64, another order): indices equal, floats within 1e-5;
* graph replay (the pass epoch advances per replay) gives the same bits twice;
* no hand-off gave up (the device fault counter stays 0).

The oracle parity of this path is covered by the rest of the GPU suite, which runs it for every
C2-shaped case (tests/test_gpu_parity*.py, tests/test_gpu_dpf_api.py).
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
FIELDS = ("particles", "probs", "lik", "index", "noise", "jac", "prior", "pred")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from nfdpf import _lib
    _lib.load()
    assert torch.cuda.is_available()


def _setup(T=12, force=False, from_state=False, B=64, N=1000):
    import bench
    from DPFs import DPF
    from nfdpf.engine import FilterEngine
    flags = dict(bench.CONFIGS["c2"][0])
    torch.manual_seed(2)
    a = bench.make_args(flags, B, N, T, {"force_resample": force})
    dpf = DPF(a).to(DEV).eval()
    start, state, vel, enc = (x.to(DEV) for x in bench.synthetic_disk(B, T, 2, a.hiddensize))
    if from_state:
        with torch.no_grad():
            enc = dpf.particle_encoder(state[:, :, :2].float()).contiguous()
    return FilterEngine(dpf.filter_config(), dpf), (enc, start, vel)


def _run(eng, inputs, fused, monkeypatch):
    from nfdpf import _lib
    monkeypatch.setenv("NFDPF_PASS", "0")  # the step launches (the one-launch pass would take over)
    monkeypatch.setenv("NFDPF_FUSED_STEP", "1" if fused else "0")
    res = eng.run(*inputs)
    torch.cuda.synchronize()
    assert eng.last_fused == fused
    assert _lib.lib().nfdpf_split_fault(1, _lib.stream_ptr(DEV)) == 0
    return {k: getattr(res, k).clone() for k in FIELDS}, float(res.obs_likelihood)


def test_fused_step_bit_identical_gated(monkeypatch):
    eng, inp = _setup()
    a, oa = _run(eng, inp, True, monkeypatch)
    b, ob = _run(eng, inp, False, monkeypatch)
    for k in FIELDS:
        assert torch.equal(a[k], b[k]), k
    assert oa == ob


@pytest.mark.parametrize("mode", ["force", "from_state"])
def test_fused_step_resampling(mode, monkeypatch):
    eng, inp = _setup(force=mode == "force", from_state=mode == "from_state")
    a, oa = _run(eng, inp, True, monkeypatch)
    b, ob = _run(eng, inp, False, monkeypatch)
    ident = torch.arange(1000, device=DEV) + 1000 * torch.arange(64, device=DEV)[:, None]
    fired = int((b["index"] != ident[:, None, :]).flatten(2).any(-1).any(0).sum())
    print(f"\n{mode}: steps that resampled {fired} of 12")
    assert fired >= (11 if mode == "force" else 1)  # step 0: uniform weights resample to the identity
    assert torch.equal(a["index"], b["index"])
    assert torch.equal(a["noise"], b["noise"])
    for k in ("particles", "probs", "lik", "jac", "prior", "pred"):
        torch.testing.assert_close(a[k], b[k], rtol=1e-5, atol=1e-5, msg=k)
    assert abs(oa - ob) <= 1e-5 * abs(ob) + 1e-5


def test_fused_step_graph_replay(monkeypatch):
    monkeypatch.setenv("NFDPF_PASS", "0")
    monkeypatch.setenv("NFDPF_FUSED_STEP", "1")
    eng, inp = _setup(T=8)
    eng.run(*inp)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        res = eng.run(*inp)
    outs = []
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        outs.append({k: getattr(res, k).clone() for k in FIELDS})
    ref, _ = _run(eng, inp, False, monkeypatch)
    for k in FIELDS:
        assert torch.equal(outs[0][k], outs[1][k]), k
        assert torch.equal(outs[0][k], ref[k]), k
    from nfdpf import _lib
    assert _lib.lib().nfdpf_split_fault(1, _lib.stream_ptr(DEV)) == 0
