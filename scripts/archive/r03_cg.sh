#!/bin/bash
# Round 3: CGLOW pivot search (branch-free DPP max, rcp multiplier) -- parity tests on the
# default library, then C5 A/B: exp/lib_CGBASE (round-2 LU), lib_CGLU (default), lib_CGLU3.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_parity_full.py -k "cglow or CGLOW or c5" > gpurun_out/r03_cg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_cg_tests.log; [ $rc -eq 0 ] || exit $rc
val() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('value %.4g ms %.4f dom %s %.5f' % (d['value'], d['ms_per_step'], d['roofline'].get('kernel'), d['roofline']['kernel_avg_ms']))" $1; }
for round in 1 2; do
  for v in ${CG_VARIANTS:-CGBASE CGLU CGLU3}; do
    NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_$v.so timeout -k 10 200 python bench.py --config c5 --steps 3 \
      --warmup 1 --no-cpu-baseline > gpurun_out/cg_${v}_$round.log 2>&1 || exit 1
    echo "c5 $v $(val gpurun_out/cg_${v}_$round.log)"
  done
done
