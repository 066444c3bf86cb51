#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_TRACE.so timeout -k 10 200 python -u scripts/exp_trace_fdyn.py > gpurun_out/r03_trace_fdyn.log 2>&1
rc=$?; cat gpurun_out/r03_trace_fdyn.log | tail -9; [ $rc -eq 0 ] || exit $rc
NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_TRACE.so timeout -k 10 200 python -u scripts/exp_trace.py > gpurun_out/r03_trace.log 2>&1
rc=$?; cat gpurun_out/r03_trace.log | tail -6; [ $rc -eq 0 ] || exit $rc
NFDPF_PARITY_TABLE=gpurun_out/r03_parity_fractions4.txt timeout -k 10 600 python -u -m pytest -v -s --timeout 500 \
  --timeout-method thread tests/test_gpu_parity_full.py -k "c5_n10000 and teacher" > gpurun_out/r03_full_tests4.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/r03_full_tests4.log | tail -5; exit $rc
