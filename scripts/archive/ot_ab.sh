#!/bin/bash
# OT tests on the default library, then A/B of experiment builds (VARIANTS) on C4 and C3 forced.
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v -rP --tb=short --timeout 300 --timeout-method thread \
    -p no:cacheprovider $TESTS ${KEXPR:+-k "$KEXPR"} > gpurun_out/ot_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ot_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for round in 1 2; do
  for cfg in ${CFGS:-c4 c3:force}; do
    c=${cfg%%:*}; extra=""; case "$cfg" in *:force) extra="--force-resample";; esac
    for v in ${VARIANTS:-OTL1 OTLDS}; do
      NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_$v.so timeout -k 10 200 python bench.py --config $c $extra \
        --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/otab_${v}_${c}_$round.log 2>&1 || exit 1
      echo $cfg $v $(python3 -c "
import json
d=json.loads(open('gpurun_out/otab_${v}_${c}_$round.log').read().strip().splitlines()[-1])
r=d['resample']
print('value %.4g ms/pass %.2f iter_ms %.4f frac %.3f fixed_ms %.4f' % (d['value'], d['ms_per_step'], r['avg_ms'], r['frac'], r.get('fixed_ms_per_call', -1)))")
    done
  done
done
