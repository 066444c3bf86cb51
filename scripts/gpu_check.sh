#!/bin/bash
# GPU-box check: parity tests, then a short bench.  Stops at the first GPU fault /
# abort / timeout (exit 124, 134, 137, 139); plain test failures (rc 1) do not stop it.
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { case "$1" in 0|1|2|5) return 0;; *) return 1;; esac; }
timeout -k 10 ${TEST_TIMEOUT:-420} python -m pytest tests -m gpu -q ${PYTEST_ARGS:--x} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; tail -15 gpurun_out/gpu_tests.log
ok $rc || exit $rc
if [ -n "$SKIP_BENCH" ]; then exit 0; fi
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.log; tail -4 gpurun_out/bench.log
exit $rc
