"""Checkpoint compatibility of the drop-in (checkpoint row): DPF(args).state_dict()
has exactly the reference's keys and shapes for every measurement model
(tests/golden/state_dict_keys.json, written by running the reference: gen_golden.py gen_keys)."""
import json
import os

import pytest
import torch

from _util import GOLDEN

REF = json.load(open(os.path.join(GOLDEN, "state_dict_keys.json")))


@pytest.mark.parametrize("meas", sorted(REF))
def test_state_dict_keys_match_reference(meas):
    from arguments import parse_args
    from DPFs import DPF
    a = parse_args([])
    a.measurement = meas
    a.hiddensize = 192 if meas == "CGLOW" else 32
    a.NF_dyn, a.NF_cond = True, meas != "CGLOW"
    torch.manual_seed(0)
    ours = {k: list(v.shape) for k, v in DPF(a).state_dict().items()}
    ref = REF[meas]
    assert sorted(ours) == sorted(ref), (sorted(set(ours) ^ set(ref)))[:10]
    assert ours == ref
