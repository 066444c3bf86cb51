"""Speculative ESS gate on the OT configurations (engine.FilterEngine.run, auto mode): the pass
runs with every gate taken as off -- no host read of the gate per step, no Sinkhorn launch --
and the T gates are verified from the kept per-step partials afterwards; a fired gate reruns
the pass with the per-step gates (the reference's own control flow, DPFs.py:163-166).  GPU box.

* C3 workload (CRNVP, OT, B=64, N=1000), gate never fires at the init weights: the speculative
  pass equals the per-step pass bit for bit and launched no OT call;
* a C4-shaped workload (MAF dynamic flow, OT, N=500) whose gate fires: the auto pass returns
  the per-step pass's result (it reran), and the next auto pass skips the speculation.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
FIELDS = ("particles", "probs", "lik", "index", "noise", "pred")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from nfdpf import _lib
    _lib.load()
    assert torch.cuda.is_available()


def _setup(cfg, B, N, T):
    import bench
    from DPFs import DPF
    from nfdpf.engine import FilterEngine
    flags = dict(bench.CONFIGS[cfg][0])
    torch.manual_seed(2)
    a = bench.make_args(flags, B, N, T, {})
    dpf = DPF(a).to(DEV).eval()
    start, state, vel, enc = (x.to(DEV) for x in bench.synthetic_disk(B, T, 2, a.hiddensize))
    return FilterEngine(dpf.filter_config(), dpf), (enc, start, vel)


def _take(res):
    torch.cuda.synchronize()
    return {k: getattr(res, k).clone() for k in FIELDS}, float(res.obs_likelihood)


def test_ot_speculative_pass_equals_per_step():
    eng, inp = _setup("c3", 64, 1000, 10)
    a, oa = _take(eng.run(*inp, speculate=False))
    assert eng.last_ot_calls == 0  # the gate never fires here
    b, ob = _take(eng.run(*inp))   # auto: speculates
    assert eng.last_ot_calls == 0
    for k in FIELDS:
        assert torch.equal(a[k], b[k]), k
    assert oa == ob


def test_ot_speculation_miss_reruns():
    eng, inp = _setup("c4", 4, 500, 16)
    a, oa = _take(eng.run(*inp, speculate=False))
    calls = eng.last_ot_calls
    print(f"\nOT calls in the per-step pass: {calls} of 16 steps")
    assert calls >= 1
    eng._ot_fired = False          # as on a fresh engine: the auto pass speculates, misses, reruns
    b, ob = _take(eng.run(*inp))
    assert eng.last_ot_calls == calls
    for k in FIELDS:
        assert torch.equal(a[k], b[k]), k
    assert oa == ob
    assert eng._ot_fired           # so the next auto pass reads the gates step by step
