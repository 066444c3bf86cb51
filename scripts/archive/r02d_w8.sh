#!/bin/bash
# Round 2d: 8-wave Sinkhorn iteration launch -- OT tests, then A/B of NFDPF_OT_ITER_WAVES on C3 forced / C4.
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest -x -v -rP --tb=short --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_parity_full.py tests/test_gpu_ot_speculate.py tests/test_gpu_backward.py \
  -k "ot or c3 or c4" > gpurun_out/w8_tests.log 2>&1
rc=$?; [ -n "$SKIP_TESTS" ] || { echo "pytest rc=$rc"; tail -3 gpurun_out/w8_tests.log; [ $rc -eq 0 ] || exit $rc; }
for round in 1 2; do
  for cfg in c3:force c4; do
    c=${cfg%%:*}; extra=""; case "$cfg" in *:force) extra="--force-resample";; esac
    for w in 4 auto 8; do
      [ $c = c3 ] && [ $w = 8 ] && continue
      L=""; [ $w != auto ] && L="NFDPF_OT_ITER_WAVES=$w"
      env $L timeout -k 10 200 python bench.py --config $c $extra --steps 3 --warmup 1 --no-cpu-baseline \
        > gpurun_out/w8_${w}_${c}_$round.log 2>&1 || exit 1
      echo $cfg W=$w $(python3 -c "
import json
d=json.loads(open('gpurun_out/w8_${w}_${c}_$round.log').read().strip().splitlines()[-1])
r=d['resample']
print('value %.4g ms/pass %.2f iter_ms %.4f' % (d['value'], d['ms_per_step'], r['avg_ms']))")
    done
  done
done
