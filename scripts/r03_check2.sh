#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_fused_step.py tests/test_gpu_parity.py -k "fused or rows_kernel or speculative or ot_sharded" \
  > gpurun_out/r03_dist_tests2.log 2>&1 || { echo "dist tests failed"; tail -40 gpurun_out/r03_dist_tests2.log; exit 1; }
tail -3 gpurun_out/r03_dist_tests2.log
for a in 1 2; do
  for sp in 1 0; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --speculate $sp > gpurun_out/r03_ab_spec${sp}_$a.json 2> gpurun_out/r03_ab_spec${sp}_$a.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r03_ab_spec${sp}_$a.json'));print('spec $sp', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['resample'].get('front_launch_ms'), d['rmse_informative_encodings'])"
  done
done
NFDPF_PARITY_TABLE=gpurun_out/r03_parity_fractions2.txt timeout -k 10 400 python -u -m pytest -v -s --timeout 300 \
  --timeout-method thread tests/test_gpu_parity_full.py -k "cglow_measurement_fullsize" > gpurun_out/r03_cglow_full.log 2>&1
rc=$?; tail -3 gpurun_out/r03_cglow_full.log; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python -u scripts/diag_c5.py > gpurun_out/r03_diag_c5.log 2>&1; rc=$?; tail -25 gpurun_out/r03_diag_c5.log
case $rc in 0|1) ;; *) exit $rc;; esac
NFDPF_PARITY_TABLE=gpurun_out/r03_parity_fractions2.txt timeout -k 10 700 python -u -m pytest -v -s --timeout 600 \
  --timeout-method thread tests/test_gpu_parity_full.py -k "ot_direct or free_running" > gpurun_out/r03_full_tests2.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r03_full_tests2.log | tail; exit $rc
