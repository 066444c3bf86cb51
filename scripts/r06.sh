#!/bin/bash
# Round-6 GPU steps, chained in one gpurun call (stops at the first failure / fault / timeout):
#   STEPS="tests:<pytest args> bench:<spec>[,<spec>] prof:<spec> pmc:<spec> suite smoke"
# spec = config[:force][:env=VAL...]  (e.g. c3, c2:force, c3:NFDPF_CM_MFMA=0)
#   tests  -> gpurun_out/r06/t_<n>.log          pytest (-x -v, thread timeouts)
#   bench  -> gpurun_out/r06/bench_<tag>.json    one bench line (BENCH_ARGS, default no CPU baseline)
#   prof   -> gpurun_out/r06/rocprof_<tag>.csv   rocprofv3 --kernel-trace --stats of the bench command
#   pmc    -> gpurun_out/r06/pmc_<tag>.csv       SQ / MFMA / FETCH / WRITE passes, each its own run
#   suite  -> gpurun_out/r06/suite.log           the whole GPU suite (+ parity fraction record)
#   smoke  -> gpurun_out/r06/smoke.log
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
n=0
spec_parse() {  # -> cfg, extra, tag, envs
  local s=$1; cfg=${s%%:*}; extra=""; tag=$cfg; envs=""
  local rest=${s#$cfg}; rest=${rest#:}
  IFS=':' read -ra parts <<< "$rest"
  for p in "${parts[@]}"; do
    case "$p" in
      force) extra="$extra --force-resample"; tag="${tag}_force";;
      *=*) envs="$envs $p"; tag="${tag}_${p//=/}";;
      "") ;;
      *) extra="$extra --$p"; tag="${tag}_$p";;
    esac
  done
}
for step in $STEPS; do
  kind=${step%%:*}; arg=${step#*:}
  n=$((n + 1))
  case "$kind" in
  tests)  # (pytest args comma-separated; "+" in a -k expression reads " or ")
    IFS=',' read -ra TA <<< "$arg"
    for i in "${!TA[@]}"; do TA[$i]="${TA[$i]//+/ or }"; done
    timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -v --timeout ${TEST_ONE:-300} --timeout-method thread \
      -p no:cacheprovider "${TA[@]}" > $O/t_$n.log 2>&1
    rc=$?; echo "tests $arg rc=$rc"; tail -3 $O/t_$n.log; [ $rc -eq 0 ] || exit $rc ;;
  bench)
    for s in ${arg//,/ }; do
      spec_parse $s
      env $envs timeout -k 10 ${BENCH_TIMEOUT:-420} python -u bench.py --config $cfg $extra ${BENCH_ARGS:---no-cpu-baseline} \
        > $O/bench_$tag.json 2> $O/bench_$tag.err
      rc=$?; echo "bench $tag rc=$rc"; tail -c 300 $O/bench_$tag.json; echo; [ $rc -eq 0 ] || exit $rc
    done ;;
  prof)
    for s in ${arg//,/ }; do
      spec_parse $s
      A="--config $cfg $extra --no-cpu-baseline ${PROF_ARGS}"
      env $envs timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fprof_$tag -o run -- \
        python3 bench.py $A > $O/fprof_$tag.log 2>&1
      rc=$?; echo "prof $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
      find $O/fprof_$tag -name "*kernel_stats.csv" -exec cp {} $O/rocprof_$tag.csv \;
      rm -rf $O/fprof_$tag
    done ;;
  pmc)
    for s in ${arg//,/ }; do
      spec_parse $s
      A="--config $cfg $extra --no-cpu-baseline --no-forced --no-informative ${PROF_ARGS}"
      for pass in "sq:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SMEM" \
                  "mfma:SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                  "br:SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" \
                  "fetch:FETCH_SIZE" "write:WRITE_SIZE"; do
        name=${pass%%:*}; ctr=${pass#*:}
        env $envs timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $O/fpmc_${tag}_$name -o run -- \
          python3 bench.py $A --steps 1 --warmup 1 --graph 0 > $O/fpmc_${tag}_$name.log 2>&1
        rc=$?; echo "pmc $tag $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done
      python3 scripts/pmc_summary.py $O/fpmc_${tag}_* > $O/pmc_$tag.csv && rm -rf $O/fpmc_${tag}_*/
    done ;;
  suite)
    rm -f $O/parity_fractions.txt
    NFDPF_PARITY_TABLE=$O/parity_fractions.txt timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rP \
      --tb=short --timeout 900 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1
    rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
