#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc run each, nothing else traced) of a short bench run
# -> gpurun_out/pmc_<tag>_<pass>/ ; summarise with scripts/pmc_summary.py
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${BENCH_ARGS:---steps 1 --warmup 1 --no-cpu-baseline}
mkdir -p gpurun_out
run() {
  timeout -k 10 ${PMC_TIMEOUT:-240} rocprofv3 --pmc $2 --output-format csv -d gpurun_out/pmc_${TAG}_$1 -o run -- \
    python3 bench.py $ARGS > gpurun_out/pmc_${TAG}_$1.log 2>&1
  rc=$?; echo "pmc $1 rc=$rc" >> gpurun_out/pmc_${TAG}_$1.log; return $rc
}
run sq "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_BUSY_CYCLES" &&
run fetch "FETCH_SIZE" &&
run write "WRITE_SIZE"
