#!/bin/bash
# Round 2d: full GPU suite on the default library, then C3 gated / C3 forced / C2 A/B vs exp/lib_BASE.so (r02c).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --tb=short --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r02d_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r02d_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for cfg in c3 c3:force c2; do
    c=${cfg%%:*}; extra=""; case "$cfg" in *:force) extra="--force-resample";; esac
    for v in BASE HEAD; do
      L=""; [ $v = BASE ] && L="NFDPF_LIB=$PWD/exp/lib_BASE.so NFDPF_LIB_PARTIAL=1"
      env $L timeout -k 10 200 python bench.py --config $c $extra --steps 10 --warmup 2 --no-cpu-baseline \
        > gpurun_out/ab2d_${v}_${c}${extra:+f}_$round.log 2>&1 || exit 1
      echo $cfg $v $(grep -o "\"value\": [0-9.e+]*" gpurun_out/ab2d_${v}_${c}${extra:+f}_$round.log) \
        $(grep -o "\"kernel_avg_ms\": [0-9.e+-]*" gpurun_out/ab2d_${v}_${c}${extra:+f}_$round.log)
    done
  done
done
