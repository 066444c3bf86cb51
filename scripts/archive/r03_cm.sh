#!/bin/bash
# Round 3: the two-chain CRNVP proposal launch -- bit-identity tests, C3 A/B against the one-chain
# launch (NFDPF_CM_TWO_CHAIN=0 vs 1), then the C2 A/B of exp/lib_NEW vs exp/lib_RCP (ctx_from_sums).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "two_chain or crnvp or CRNVP or c3" > gpurun_out/r03_cm_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_cm_tests.log; [ $rc -eq 0 ] || exit $rc
val() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('value %.4g ms %.4f dom %s %.5f' % (d['value'], d['ms_per_step'], d['roofline'].get('kernel'), d['roofline']['kernel_avg_ms']))" $1; }
for round in 1 2; do
  for single in 1 0; do
    NFDPF_CM_TWO_CHAIN=$((1-single)) timeout -k 10 150 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/cm_${single}_$round.log 2>&1 || exit 1
    echo "c3 single=$single $(val gpurun_out/cm_${single}_$round.log)"
  done
done
for round in 1 2; do
  for v in NEW RCP; do
    NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_$v.so timeout -k 10 150 python bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline > gpurun_out/ab_${v}_$round.log 2>&1 || exit 1
    echo "c2 $v $(val gpurun_out/ab_${v}_$round.log)"
  done
done
