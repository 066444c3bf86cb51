#!/bin/bash
# A/B of experiment libraries on the C2 bench (quiet line + informative line), one box:
#   [BENCH_EXTRA="--config c3"] scripts/archive/r05_ab.sh OUTTAG base S3 S3B ...   (base = the in-tree library)
OUT=$1; shift
mkdir -p gpurun_out
for tag in "$@"; do
  if [ "$tag" = base ]; then unset NFDPF_LIB; else export NFDPF_LIB=exp/lib_${tag}.so; fi
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-forced ${BENCH_EXTRA} > gpurun_out/${OUT}_${tag}.json 2> gpurun_out/${OUT}_${tag}.err || exit 1
  python -c "
import json; d = json.load(open('gpurun_out/${OUT}_${tag}.json')); i = d.get('informative') or {}
print('${tag}', 'quiet %.4g' % d['value'], 'pass %.4f ms' % d['roofline']['kernel_avg_ms'], '| informative %.4g' % i.get('value', 0), 'fired', i.get('resampled_steps'), 'pass', i.get('pass_kernel_avg_ms_live'))"
done
