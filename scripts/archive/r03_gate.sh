#!/bin/bash
# Round 3: the gate wave's partials in registers (no scratch) and global reads of the partials --
# gate / parity tests on the default library, then the C2 A/B exp/lib_BASE vs exp/lib_NEW.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_parity_full.py tests/test_gpu_dist.py tests/test_gpu_ot_speculate.py -k "c2 or gate or spec or shard or rows" \
  > gpurun_out/r03_gate_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_gate_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="BASE NEW" bash scripts/archive/r03_ab.sh
