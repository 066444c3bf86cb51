#!/bin/bash
# Round 3: deferred normalisation in speculative OT passes -- the OT speculation / parity tests,
# then C3 and C4 bench lines (compare profiles/ records of the previous build).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ot_speculate.py \
  tests/test_gpu_dist.py tests/test_gpu_parity.py -k "ot or OT or c3 or c4 or spec or crnvp" \
  > gpurun_out/r03_otdefer_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_otdefer_tests.log; [ $rc -eq 0 ] || exit $rc
val() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('value %.4g ms %.4f dom %s %.5f' % (d['value'], d['ms_per_step'], d['roofline'].get('kernel'), d['roofline']['kernel_avg_ms']))" $1; }
for cfg in c3 c4; do
  timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/otdefer_$cfg.log 2>&1 || exit 1
  echo "$cfg $(val gpurun_out/otdefer_$cfg.log)"
done
