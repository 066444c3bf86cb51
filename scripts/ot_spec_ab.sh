#!/bin/bash
# OT speculative gate: tests, then the C3 / C4 bench with and without it
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -rP --tb=short --timeout 300 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_ot_speculate.py > gpurun_out/otspec_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/otspec_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for spec in "" "--speculate 0"; do
    for c in c3 c4; do
      [ "$c" = c4 ] && [ -n "$spec" ] && continue
      timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline $spec > gpurun_out/osab.log 2>&1 || exit 1
      echo "$c [$spec]" $(python3 -c "
import json
d=json.loads(open('gpurun_out/osab.log').read().strip().splitlines()[-1])
print('value %.4g ms/pass %.3f kernel %s %.4f resampled %s | %s' % (d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_avg_ms'], d['resampled_steps'], d['config']['workload'][-60:]))")
    done
  done
done
