#!/bin/bash
# A/B of bench flag sets on one box (FLAGSETS, separated by '|'), alternating rounds.
export TMPDIR=/tmp
mkdir -p gpurun_out
IFS='|' read -ra SETS <<< "${FLAGSETS:---speculate 0|--speculate 1}"
for round in 1 2; do
  k=0
  for f in "${SETS[@]}"; do
    k=$((k+1))
    timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $f > gpurun_out/ab_${k}_$round.log 2>&1 || exit 1
    echo "[$f]" $(python3 -c "
import json
d=json.loads(open('gpurun_out/ab_${k}_$round.log').read().strip().splitlines()[-1])
print('value %.4g ms/pass %.4f prop_ms %.5f front_ms %.5f' % (d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['resample'].get('front_launch_ms') or -1))")
  done
done
