#!/bin/bash
# 8-wave iteration at 4 waves per SIMD (exp/lib_W8O4.so: -DNFDPF_OT_ITER_WPS=4 -DNFDPF_OT_LDS1) vs the default.
export TMPDIR=/tmp
mkdir -p gpurun_out
NFDPF_LIB=$PWD/exp/lib_W8O4.so timeout -k 10 300 python -u -m pytest -x -v --tb=short --timeout 200 \
  --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "ot_iter_waves or ot_resampler" \
  > gpurun_out/w8o4_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/w8o4_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for cfg in c4 c3:force; do
    c=${cfg%%:*}; extra=""; case "$cfg" in *:force) extra="--force-resample";; esac
    for v in HEAD W8O4; do
      L=""; [ $v = W8O4 ] && L="NFDPF_LIB=$PWD/exp/lib_W8O4.so NFDPF_OT_ITER_WAVES=8"
      env $L timeout -k 10 200 python bench.py --config $c $extra --steps 3 --warmup 1 --no-cpu-baseline \
        > gpurun_out/w8o4_${v}_${c}_$round.log 2>&1 || exit 1
      echo $cfg $v $(python3 -c "
import json
d=json.loads(open('gpurun_out/w8o4_${v}_${c}_$round.log').read().strip().splitlines()[-1])
r=d['resample']
print('value %.4g ms/pass %.2f iter_ms %.4f' % (d['value'], d['ms_per_step'], r['avg_ms']))")
    done
  done
done
