#!/bin/bash
# Tests of the fused step, then A/B: the C2 bench with the fused step vs the two launches.
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v -rP --tb=short --timeout 300 --timeout-method thread \
    -p no:cacheprovider $TESTS ${KEXPR:+-k "$KEXPR"} > gpurun_out/fused_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/fused_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for round in 1 2; do
  for f in 1 0; do
    NFDPF_FUSED_STEP=$f timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} \
      > gpurun_out/fab_${f}_$round.log 2>&1 || exit 1
    echo "fused=$f" $(python3 -c "
import json
d=json.loads(open('gpurun_out/fab_${f}_$round.log').read().strip().splitlines()[-1])
r=d['roofline']
print('value %.4g ms/pass %.4f kernel %s %.5f ms frac %.3f front %s' % (d['value'], d['ms_per_step'], r['kernel'], r['kernel_avg_ms'], r['frac'], d['resample'].get('front_launch_ms')))")
  done
done
