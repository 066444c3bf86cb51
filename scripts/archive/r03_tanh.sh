#!/bin/bash
# Round 3: branch-free tanh in CGLOW (exp/lib_BF.so) -- CGLOW parity on that build (golden +
# full size), then C5 A/B against the default (exp/lib_DEF.so).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_BF.so timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 500 \
  --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_parity_full.py -k "cglow or CGLOW or c5" \
  > gpurun_out/r03_tanh_tests.log 2>&1
rc=$?; grep -E "max \||golden|PASS|FAIL|passed|failed" gpurun_out/r03_tanh_tests.log | tail -14; [ $rc -eq 0 ] || exit $rc
CG_VARIANTS="DEF BF" bash scripts/archive/r03_cg.sh 2>&1 | grep "^c5"
