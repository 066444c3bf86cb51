#!/bin/bash
# fused-step probe: phase trace, I-cache PMC of both paths, A/B timing
export TMPDIR=/tmp
mkdir -p gpurun_out
NFDPF_FUSED_STEP=1 NFDPF_LIB_PARTIAL=1 NFDPF_LIB=$PWD/exp/lib_TRACE.so timeout -k 10 200 python scripts/exp_trace.py > gpurun_out/trace_fused.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/trace_fused.txt | head -4
for f in 1 0; do
  NFDPF_FUSED_STEP=$f TAG=f$f bash scripts/pmc_icache.sh || exit 1
done
BENCH_ARGS= bash scripts/fused_ab.sh
