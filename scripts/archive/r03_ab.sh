#!/bin/bash
# A/B of experiment libraries (exp/lib_<V>.so) on one box: default C2 bench, alternating rounds,
# then (optional) the trace build's phase printout and the given parity tests on the default lib.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS ${KEXPR:+-k "$KEXPR"} \
    > gpurun_out/r03_ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/r03_ab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -f exp/lib_TRACE.so ]; then
  NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_TRACE.so timeout -k 10 200 python -u scripts/archive/exp_trace_fdyn.py > gpurun_out/r03_trace_fdyn.log 2>&1
  rc=$?; tail -8 gpurun_out/r03_trace_fdyn.log; [ $rc -eq 0 ] || exit $rc
fi
for round in 1 2; do
  for v in ${VARIANTS:-BASE NEW}; do
    NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_$v.so timeout -k 10 150 python bench.py ${BENCH_ARGS:---steps 20 --warmup 3 --no-cpu-baseline} > gpurun_out/ab_${v}_$round.log 2>&1 || exit 1
    echo $v $(python3 -c "
import json
d=json.loads(open('gpurun_out/ab_${v}_$round.log').read().strip().splitlines()[-1])
print('value %.4g prop_ms %.5f front_ms %.5f' % (d['value'], d['roofline']['kernel_avg_ms'], d['resample'].get('front_launch_ms') or -1))")
  done
done
