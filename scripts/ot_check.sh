#!/bin/bash
# GPU-box check of the Sinkhorn kernels: accuracy vs the fp64 oracle, per-call diagnostics of
# a C4 pass, the GPU test-suite, then a rocprofv3 kernel trace of a short C4 bench.
# Stops at the first GPU fault / abort / timeout (plain test failures, rc 1, do not stop it).
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { case "$1" in 0|1) return 0;; *) return 1;; esac; }
timeout -k 10 200 python scripts/ot_err.py > gpurun_out/ot_err.log 2>&1; rc=$?; cat gpurun_out/ot_err.log; ok $rc || exit $rc
timeout -k 10 200 python scripts/ot_c4_stats.py ${CFG:-c4} > gpurun_out/ot_stats.log 2>&1; rc=$?; cat gpurun_out/ot_stats.log; ok $rc || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; ok $rc || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${CFG:-c4} -o run -- \
  python3 bench.py --config ${CFG:-c4} --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${CFG:-c4}.log 2>&1
rc=$?; tail -1 gpurun_out/prof_${CFG:-c4}.log; exit $rc
