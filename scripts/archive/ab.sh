#!/bin/bash
# A/B timing of two library builds on one box: A = the in-tree libnfdpf.so, B = $LIB_B
# (an exp/ build); alternating runs of the default bench, value and live prop-launch time.
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:---steps 20 --warmup 3 --no-cpu-baseline}
for v in A B A B A B; do
  if [ $v = A ]; then L=""; else L="NFDPF_LIB=$LIB_B"; fi
  env $L timeout -k 10 120 python bench.py $ARGS > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo $v $(grep -o "\"value\": [0-9.e+]*" gpurun_out/ab_$v.log) $(grep -o "\"kernel_avg_ms\": [0-9.e+-]*" gpurun_out/ab_$v.log)
done
