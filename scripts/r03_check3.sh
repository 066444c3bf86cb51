#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rm -f gpurun_out/r03_parity_fractions3.txt
NFDPF_PARITY_TABLE=gpurun_out/r03_parity_fractions3.txt timeout -k 10 600 python -u -m pytest -v -s --timeout 500 \
  --timeout-method thread tests/test_gpu_parity_full.py -k "c5_n10000 and teacher or cglow_measurement_fullsize" \
  > gpurun_out/r03_full_tests3.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r03_full_tests3.log | tail -5; case $rc in 0|1) ;; *) exit $rc;; esac
for cfg in c5 c4 c3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $cfg > gpurun_out/r03_bench_$cfg.json 2> gpurun_out/r03_bench_$cfg.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r03_bench_$cfg.json'));print('$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_avg_ms'], d['resample'].get('front_launch_ms'), d['rmse'], d['rmse_informative_encodings'])"
done
