#!/bin/bash
# Round-2 end-of-round measurement, part $PART:
#   1: full GPU test suite + smoke
#   2: bench lines (CPU baselines) C2 gated / forced, C3 gated / forced, C4, C5
#   3: rocprofv3 kernel-trace summaries + PMC passes (SQ, MFMA, FETCH, WRITE) per config
# Stops at the first GPU fault / abort / timeout.
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
case "$PART" in
1)
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --tb=short --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/final_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/final_tests.log; tail -3 gpurun_out/final_tests.log
  fatal $rc && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
  rc=$?; tail -2 gpurun_out/final_smoke.log; exit $rc
  ;;
2)
  for spec in ${RUNS:-c2 c2:force c3 c3:force c4 c5}; do
    cfg=${spec%%:*}; extra=""; tag=$cfg
    case "$spec" in *:force) extra="--force-resample"; tag=${cfg}_force;; esac
    timeout -k 10 420 python -u bench.py --config $cfg $extra ${BENCH_ARGS} > gpurun_out/final_bench_$tag.json \
      2> gpurun_out/final_bench_$tag.err
    rc=$?; echo "$tag rc=$rc"; tail -c 300 gpurun_out/final_bench_$tag.json; echo
    [ $rc -eq 0 ] || exit $rc
  done
  ;;
3)
  for spec in ${PROFS:-c2 c2:force c3:force c4 c5}; do
    cfg=${spec%%:*}; extra=""; tag=$cfg
    case "$spec" in *:force) extra="--force-resample"; tag=${cfg}_force;; esac
    A="--config $cfg $extra --steps 2 --warmup 1 --no-cpu-baseline"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof_$tag -o run -- \
      python3 bench.py $A > gpurun_out/fprof_$tag.log 2>&1
    rc=$?; echo "prof $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
    # keep only the summaries (the raw traces exceed gpurun's 64 MiB copy-back)
    find gpurun_out/fprof_$tag -name "*kernel_stats.csv" -exec cp {} gpurun_out/kstats_$tag.csv \;
    rm -rf gpurun_out/fprof_$tag
    for pass in "sq:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SMEM" \
                "mfma:SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                "fetch:FETCH_SIZE" "write:WRITE_SIZE"; do
      name=${pass%%:*}; ctr=${pass#*:}
      timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/fpmc_${tag}_$name -o run -- \
        python3 bench.py $A --graph 0 > gpurun_out/fpmc_${tag}_$name.log 2>&1
      rc=$?; echo "pmc $tag $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
    python3 scripts/pmc_summary.py gpurun_out/fpmc_${tag}_* > gpurun_out/pmc_$tag.csv && rm -rf gpurun_out/fpmc_${tag}_*/
  done
  ;;
esac
