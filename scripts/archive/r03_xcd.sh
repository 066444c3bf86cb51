#!/bin/bash
# Round 3: XCD-aware (row, tile) remap of the tiled step (exp/lib_XCD.so, -DNFDPF_XCD_REMAP) --
# tiled parity tests on that build, then C2 / C3 / C5 A/B against exp/lib_BASE.so.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_XCD.so timeout -k 10 600 python -u -m pytest -x -q --timeout 500 \
  --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused_step.py -k "tiled or fused or rows or c2" \
  > gpurun_out/r03_xcd_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_xcd_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="BASE XCD" bash scripts/archive/r03_ab.sh
for v in BASE XCD; do
  NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_$v.so timeout -k 10 150 python bench.py --config c3 --steps 20 --warmup 3 \
    --no-cpu-baseline > gpurun_out/xcd_c3_$v.log 2>&1 || exit 1
  echo "c3 $v $(python3 -c "
import json
d=json.loads(open('gpurun_out/xcd_c3_$v.log').read().strip().splitlines()[-1]); print('%.4g' % d['value'])")"
done
