#!/bin/bash
# OT prescaled-coordinate experiment: OT parity tests on exp/lib_EPIPS.so, then the A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out
NFDPF_LIB=$PWD/exp/lib_EPIPS.so timeout -k 10 600 python -u -m pytest -x -v -rP --tb=short --timeout 300 \
  --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_parity_full.py \
  tests/test_gpu_ot_speculate.py tests/test_gpu_backward.py -k "ot or c3 or c4" > gpurun_out/ot_ps_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ot_ps_tests.log
case $rc in 0|1|5) ;; *) exit $rc;; esac
VARIANTS="BASE EPI EPIPS NORISK" bash scripts/archive/ot_ab.sh
