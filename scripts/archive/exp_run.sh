#!/bin/bash
# Timing of experiment builds (exp/lib_<V>.so, scripts/archive/exp_build.sh) on one box: the default
# bench per variant, alternating rounds; prints value, live proposal-launch and front-launch ms.
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:---steps 20 --warmup 3 --no-cpu-baseline}
for round in 1 2; do
  for v in ${VARIANTS:-BASE}; do
    NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_$v.so timeout -k 10 120 python bench.py $ARGS > gpurun_out/exp_${v}_$round.log 2>&1 || exit 1
    echo $v $(python3 -c "
import json,sys
d=json.loads(open('gpurun_out/exp_${v}_$round.log').read().strip().splitlines()[-1])
print('value %.4g prop_ms %.5f front_ms %.5f' % (d['value'], d['roofline']['kernel_avg_ms'], d['resample'].get('front_launch_ms') or -1))")
  done
done
