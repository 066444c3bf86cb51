#!/bin/bash
# Round-2 measurement call: the tests fixed this round, then the bench lines (ESS-gated and
# --force-resample) of C2 and C3, then rocprofv3 kernel-trace summaries of the forced runs.
# Stops at the first GPU fault / abort / timeout.
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider $TESTS \
    > gpurun_out/r02_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/r02_tests.log; tail -5 gpurun_out/r02_tests.log
  fatal $rc && exit $rc
fi
for spec in ${RUNS:-c2 c2:force c3 c3:force}; do
  cfg=${spec%%:*}; extra=""; tag=$cfg
  case "$spec" in *:force) extra="--force-resample"; tag=${cfg}_force;; esac
  timeout -k 10 ${BENCH_TIMEOUT:-300} python -u bench.py --config $cfg $extra ${BENCH_ARGS} \
    > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
  rc=$?; echo "$tag rc=$rc"; tail -c 600 gpurun_out/bench_$tag.json; echo
  [ $rc -eq 0 ] || exit $rc
done
for spec in ${PROFS}; do
  cfg=${spec%%:*}; extra=""; tag=$cfg
  case "$spec" in *:force) extra="--force-resample"; tag=${cfg}_force;; esac
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
    python3 bench.py --config $cfg $extra --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1
  rc=$?; echo "prof $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
