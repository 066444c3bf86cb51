"""Host logic of the gate plans (nfdpf.engine.FilterEngine._plan_*; the kernels are in
tests/test_gpu_pass.py): which passes follow a plan, the plan's device buffer rewritten in place
only when it changes, and the argument checks.  CPU only (the buffer lives where the pass runs)."""
import numpy as np
import pytest
import torch

from nfdpf import _lib as L
from nfdpf.engine import FilterConfig, FilterEngine


def _eng(**kw):
    cfg = FilterConfig(N=100, NF_dyn=True, NF_cond=True, measurement="cos", resampler="soft", **kw)
    return FilterEngine(cfg, models=None)


def test_plan_capability():
    e = _eng()
    assert e._plan_capable(True) and not e._plan_capable(False)
    assert e._plan_wanted(True, gate_ok=False)        # sharded, or rows beyond the resident grid
    assert not e._plan_wanted(True, gate_ok=True)     # one GPU, all rows resident: the gated pass
    assert _eng(pass_plan=True)._plan_wanted(True, gate_ok=True)
    assert not _eng(pass_plan=False)._plan_capable(True)
    assert not _eng(pass_gate=False)._plan_capable(True)
    assert not _eng(force_resample=True)._plan_capable(True)
    ot = FilterEngine(FilterConfig(N=100, NF_dyn=True, NF_cond=True, resampler="ot"), models=None)
    assert not ot._plan_capable(True)


def test_plan_env_switches(monkeypatch):
    monkeypatch.setenv("NFDPF_PASS_PLAN", "0")
    assert not _eng()._plan_capable(True)
    monkeypatch.setenv("NFDPF_PASS_PLAN", "1")
    assert _eng()._plan_wanted(True, gate_ok=True)


def test_plan_select_auto_and_buffer():
    e = _eng()
    T = 6
    assert e._plan_select(True, False, T, True, None, True, "cpu") == (None, None)  # no plan yet
    e._plan = np.zeros(T, np.int32)
    assert e._plan_select(True, False, T, True, None, True, "cpu") == (None, None)  # fires nothing
    e._plan = np.array([0, 1, 0, 1, 1, 0], np.int32)
    p, buf = e._plan_select(True, False, T, True, None, True, "cpu")
    assert np.array_equal(p, e._plan) and buf.tolist() == e._plan.tolist()
    p2, buf2 = e._plan_select(True, False, T, True, None, True, "cpu")
    assert buf2.data_ptr() == buf.data_ptr()  # one buffer: a captured pass reads the current plan
    e._plan = np.array([1, 1, 0, 0, 1, 0], np.int32)
    _, buf3 = e._plan_select(True, False, T, True, None, True, "cpu")
    assert buf3.data_ptr() == buf.data_ptr() and buf3.tolist() == [1, 1, 0, 0, 1, 0]  # rewritten in place
    assert e._plan_select(True, True, T, True, None, True, "cpu") == (None, None)  # gated pass applies
    assert e._plan_select(True, False, T, False, None, True, "cpu") == (None, None)  # not auto
    assert e._plan_select(True, False, T + 1, True, None, True, "cpu") == (None, None)  # other T


def test_explicit_plan_checks():
    e = _eng()
    p, buf = e._plan_select(True, True, 4, False, [0, 1, 1, 0], True, "cpu")  # explicit: any mode
    assert p.dtype == np.int32 and buf.tolist() == [0, 1, 1, 0]
    with pytest.raises(L.NfdpfError):
        e._plan_select(True, True, 5, False, [0, 1, 1, 0], True, "cpu")
    with pytest.raises(L.NfdpfError):
        _eng(pass_plan=False)._plan_select(True, True, 4, False, [0, 1, 1, 0], True, "cpu")
    with pytest.raises(L.NfdpfError):
        e._plan_select(False, True, 4, False, [0, 1, 1, 0], True, "cpu")  # no one-launch pass
