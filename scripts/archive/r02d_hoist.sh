#!/bin/bash
# ot_iter loads hoisted above the stop rule (HEAD) vs exp/lib_BASE.so: OT tests, then C3 forced / C4 A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out
NFDPF_LIB=$PWD/exp/lib_SLICE.so timeout -k 10 600 python -u -m pytest -x -v -rP --tb=short --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_parity_full.py tests/test_gpu_ot_speculate.py tests/test_gpu_backward.py \
  -k "ot or c3 or c4" > gpurun_out/hoist_tests.log 2>&1
rc=$?; echo "pytest SLICE rc=$rc"; tail -3 gpurun_out/hoist_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v -rP --tb=short --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_parity_full.py tests/test_gpu_ot_speculate.py tests/test_gpu_backward.py \
  -k "ot or c3 or c4" > gpurun_out/hoist_tests_head.log 2>&1
rc=$?; echo "pytest HEAD rc=$rc"; tail -3 gpurun_out/hoist_tests_head.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for round in 1 2; do
  for cfg in c3:force c4; do
    c=${cfg%%:*}; extra=""; case "$cfg" in *:force) extra="--force-resample";; esac
    for v in BASE HEAD SLICE; do
      L=""; [ $v = BASE ] && L="NFDPF_LIB=$PWD/exp/lib_BASE.so NFDPF_LIB_PARTIAL=1"
      [ $v = SLICE ] && L="NFDPF_LIB=$PWD/exp/lib_SLICE.so"
      env $L timeout -k 10 200 python bench.py --config $c $extra --steps 5 --warmup 1 --no-cpu-baseline \
        > gpurun_out/hoist_${v}_${c}_$round.log 2>&1 || exit 1
      echo $cfg $v $(python3 -c "
import json
d=json.loads(open('gpurun_out/hoist_${v}_${c}_$round.log').read().strip().splitlines()[-1])
r=d['resample']
print('value %.4g ms/pass %.2f iter_ms %.4f' % (d['value'], d['ms_per_step'], r['avg_ms']))")
    done
  done
done
