#!/bin/bash
# Round-3 measurement, part $PART (one GPU call each; stops at the first fault / abort / timeout):
#   1: full GPU test suite (+ the 1e-5 fraction record) + smoke
#   2: bench lines (with CPU baselines) for $RUNS (default: C2 gated / forced, C3 gated / forced, C4, C5)
#   3: per config of $PROFS: rocprofv3 --kernel-trace --stats of the SAME bench command as part 2
#      (gpurun_out/rocprof_<tag>.csv) and the PMC passes SQ / MFMA / FETCH / WRITE, each alone
#      (gpurun_out/pmc_<tag>.csv); bench.py reads both back from profiles/ once committed there
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
case "$PART" in
1)
  rm -f gpurun_out/r03_parity_fractions.txt
  NFDPF_PARITY_TABLE=gpurun_out/r03_parity_fractions.txt timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rP \
    --tb=short --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/final_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/final_tests.log; tail -3 gpurun_out/final_tests.log
  fatal $rc && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
  rc=$?; tail -2 gpurun_out/final_smoke.log; exit $rc
  ;;
2)
  for spec in ${RUNS:-c2 c2:force c3 c3:force c4 c5}; do
    cfg=${spec%%:*}; extra=""; tag=$cfg
    case "$spec" in *:force) extra="--force-resample"; tag=${cfg}_force;; esac
    timeout -k 10 420 python -u bench.py --config $cfg $extra ${BENCH_ARGS} > gpurun_out/bench_$tag.json \
      2> gpurun_out/bench_$tag.err
    rc=$?; echo "$tag rc=$rc"; tail -c 400 gpurun_out/bench_$tag.json; echo
    [ $rc -eq 0 ] || exit $rc
  done
  ;;
3)
  for spec in ${PROFS:-c2 c2:force c3 c3:force c4 c5}; do
    cfg=${spec%%:*}; extra=""; tag=$cfg
    case "$spec" in *:force) extra="--force-resample"; tag=${cfg}_force;; esac
    A="--config $cfg $extra --no-cpu-baseline ${PROF_ARGS}"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof_$tag -o run -- \
      python3 bench.py $A > gpurun_out/fprof_$tag.log 2>&1
    rc=$?; echo "prof $tag rc=$rc"; tail -c 300 gpurun_out/fprof_$tag.log; echo; [ $rc -eq 0 ] || exit $rc
    # keep only the summaries (the raw traces exceed gpurun's 64 MiB copy-back)
    find gpurun_out/fprof_$tag -name "*kernel_stats.csv" -exec cp {} gpurun_out/rocprof_$tag.csv \;
    rm -rf gpurun_out/fprof_$tag
    [ -n "$NO_PMC" ] && continue
    for pass in "sq:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SMEM" \
                "mfma:SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                "fetch:FETCH_SIZE" "write:WRITE_SIZE"; do
      name=${pass%%:*}; ctr=${pass#*:}
      timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/fpmc_${tag}_$name -o run -- \
        python3 bench.py $A --steps 1 --warmup 1 --graph 0 > gpurun_out/fpmc_${tag}_$name.log 2>&1
      rc=$?; echo "pmc $tag $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
    python3 scripts/pmc_summary.py gpurun_out/fpmc_${tag}_* > gpurun_out/pmc_$tag.csv && rm -rf gpurun_out/fpmc_${tag}_*/
  done
  ;;
esac
