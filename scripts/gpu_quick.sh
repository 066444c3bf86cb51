#!/bin/bash
# GPU box: selected tests (TESTS, pytest args) then the experiment timings (VARIANTS); stops at
# the first GPU fault / abort / timeout.
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest -x -v -rP --tb=short --timeout 300 --timeout-method thread \
    -p no:cacheprovider $TESTS ${KEXPR:+-k "$KEXPR"} > gpurun_out/quick_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/quick_tests.log; tail -4 gpurun_out/quick_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$VARIANTS" ]; then bash scripts/exp_run.sh || exit $?; fi
