#!/bin/bash
# C3 (CRNVP) tests on the default library, then A/B of experiment builds on the C3 bench
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 700 python -u -m pytest -x -v -rP --tb=short --timeout 400 --timeout-method thread \
    -p no:cacheprovider $TESTS ${KEXPR:+-k "$KEXPR"} > gpurun_out/c3_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/c3_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for round in 1 2; do
  for v in ${VARIANTS:-CRVALU CRMFMA}; do
    NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_$v.so timeout -k 10 200 python bench.py --config c3 --steps 10 --warmup 3 \
      --no-cpu-baseline > gpurun_out/c3ab.log 2>&1 || exit 1
    echo "$v" $(python3 -c "
import json
d=json.loads(open('gpurun_out/c3ab.log').read().strip().splitlines()[-1])
r=d['roofline']
print('value %.4g ms/pass %.3f kernel %s %.4f ms frac %.3f' % (d['value'], d['ms_per_step'], r['kernel'], r['kernel_avg_ms'], r['frac']))")
  done
done
