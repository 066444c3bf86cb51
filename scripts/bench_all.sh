#!/bin/bash
# GPU box: the bench line of every configuration (CPU baseline included) ->
# gpurun_out/bench_<config>.json; stops at the first failing run.
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CONFIGS:-c2 c3 c4 c5}; do
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --config $c ${BENCH_ARGS} > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  rc=$?
  echo "$c rc=$rc"; tail -c 1500 gpurun_out/bench_$c.json
  [ $rc -eq 0 ] || exit $rc
done
