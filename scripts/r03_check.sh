#!/bin/bash
# round 3: the new sharded-OT / dist tests, then the full-size parity suite with the 1e-5 tables
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "ot_sharded or ot_poll or ot_resampler_golden" tests/test_gpu_dist.py tests/test_gpu_fused_step.py \
  > gpurun_out/r03_dist_tests.log 2>&1 || { echo "dist tests failed"; tail -40 gpurun_out/r03_dist_tests.log; exit 1; }
tail -5 gpurun_out/r03_dist_tests.log
rm -f gpurun_out/r03_parity_fractions.txt
NFDPF_PARITY_TABLE=gpurun_out/r03_parity_fractions.txt timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 \
  --timeout-method thread tests/test_gpu_parity_full.py > gpurun_out/r03_full_tests.log 2>&1 \
  || { echo "full-size tests failed"; tail -60 gpurun_out/r03_full_tests.log; exit 1; }
tail -15 gpurun_out/r03_full_tests.log
