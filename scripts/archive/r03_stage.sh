#!/bin/bash
# Round 3: CRNVP weights staged in LDS (tiled_prop_kernel<..., true>) -- bit-identity and the C3
# parity tests, then the C3 A/B against the scalar-cache stream (NFDPF_CRNVP_STAGE=0 vs 1).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "staged or crnvp or CRNVP or c3" > gpurun_out/r03_stage_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_stage_tests.log; [ $rc -eq 0 ] || exit $rc
val() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('value %.4g ms %.4f dom %s %.5f' % (d['value'], d['ms_per_step'], d['roofline'].get('kernel'), d['roofline']['kernel_avg_ms']))" $1; }
for round in 1 2; do
  for scalar in 1 0; do
    NFDPF_CRNVP_STAGE=$((1-scalar)) timeout -k 10 150 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline \
      ${STAGE_ARGS} > gpurun_out/stage_${scalar}_$round.log 2>&1 || exit 1
    echo "c3 scalar=$scalar $(val gpurun_out/stage_${scalar}_$round.log)"
  done
done
