#!/bin/bash
# Round-4 GPU steps (one gpurun call per PART; stops at the first fault / abort / timeout):
#   pass   : the one-launch pass tests, then a C2 bench line without the CPU baseline
#   suite  : the full GPU suite (+ the 1e-5 fraction record) + smoke, log named by $TAG
#   bench  : bench lines for $RUNS (default c2 c2:force), args $BENCH_ARGS
#   prof   : rocprofv3 --kernel-trace --stats of the bench command for $PROFS (+ PMC passes unless NO_PMC)
#   tests  : pytest on $TESTS (-k $K)
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
case "$PART" in
pass)
  timeout -k 10 600 python -u -m pytest tests/test_gpu_pass.py -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider ${K:+-k "$K"} > gpurun_out/pass_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pass_tests.log; tail -15 gpurun_out/pass_tests.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_c2_pass.json 2> gpurun_out/bench_c2_pass.err
  rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench_c2_pass.json; tail -5 gpurun_out/bench_c2_pass.err; exit $rc
  ;;
tests)
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    ${K:+-k "$K"} > gpurun_out/tests_${TAG:-x}.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_${TAG:-x}.log; tail -25 gpurun_out/tests_${TAG:-x}.log; exit $rc
  ;;
suite)
  rm -f gpurun_out/parity_fractions_${TAG}.txt
  NFDPF_PARITY_TABLE=gpurun_out/parity_fractions_${TAG}.txt timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rP \
    --tb=short --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/suite_${TAG}.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/suite_${TAG}.log; tail -5 gpurun_out/suite_${TAG}.log
  fatal $rc && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_${TAG}.log 2>&1
  rc2=$?; tail -2 gpurun_out/smoke_${TAG}.log; [ $rc -eq 0 ] && exit $rc2; exit $rc
  ;;
bench)
  for spec in ${RUNS:-c2 c2:force}; do
    cfg=${spec%%:*}; extra=""; tag=$cfg
    case "$spec" in *:force) extra="--force-resample"; tag=${cfg}_force;; esac
    timeout -k 10 420 python -u bench.py --config $cfg $extra ${BENCH_ARGS} > gpurun_out/bench_${TAG}_$tag.json \
      2> gpurun_out/bench_${TAG}_$tag.err
    rc=$?; echo "$tag rc=$rc"; tail -c 600 gpurun_out/bench_${TAG}_$tag.json; echo
    [ $rc -eq 0 ] || exit $rc
  done
  ;;
prof)
  for spec in ${PROFS:-c2}; do
    cfg=${spec%%:*}; extra=""; tag=$cfg
    case "$spec" in *:force) extra="--force-resample"; tag=${cfg}_force;; esac
    A="--config $cfg $extra --no-cpu-baseline --no-forced ${PROF_ARGS}"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof_$tag -o run -- \
      python3 bench.py $A > gpurun_out/fprof_$tag.log 2>&1
    rc=$?; echo "prof $tag rc=$rc"; tail -c 300 gpurun_out/fprof_$tag.log; echo; [ $rc -eq 0 ] || exit $rc
    find gpurun_out/fprof_$tag -name "*kernel_stats.csv" -exec cp {} gpurun_out/rocprof_$tag.csv \;
    # OT: the iteration launches that ran an iteration, apart from the early-exit tail
    tr=$(find gpurun_out/fprof_$tag -name "*kernel_trace.csv" | head -n 1)
    [ -n "$tr" ] && python3 scripts/rocprof_ot_split.py "$tr" gpurun_out/rocprof_$tag.csv
    rm -rf gpurun_out/fprof_$tag
    [ -n "$NO_PMC" ] && continue
    for pass in "sq:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SMEM" \
                "mfma:SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                "fetch:FETCH_SIZE" "write:WRITE_SIZE" \
                "inst:SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"; do
      name=${pass%%:*}; ctr=${pass#*:}
      timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/fpmc_${tag}_$name -o run -- \
        python3 bench.py $A --steps 1 --warmup 1 --graph 0 > gpurun_out/fpmc_${tag}_$name.log 2>&1
      rc=$?; echo "pmc $tag $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
    python3 scripts/pmc_summary.py gpurun_out/fpmc_${tag}_* > gpurun_out/pmc_$tag.csv && rm -rf gpurun_out/fpmc_${tag}_*/
  done
  ;;
esac
