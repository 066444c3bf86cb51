#!/bin/bash
# One GPU call: rocprofv3 kernel-trace summary of the default bench command of a config, then the
# PMC passes (FETCH / WRITE / SQ, each alone) -> gpurun_out/; copy summaries into profiles/ with
#   python scripts/pmc_summary.py gpurun_out/pmc_<tag>_* > profiles/pmc_<config>.csv
export TMPDIR=/tmp
CFG=${CFG:-c2}
TAG=${TAG:-r01_${CFG}}
export BENCH_ARGS="--config $CFG --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline"
TAG=$TAG bash scripts/profile.sh && BENCH_ARGS="$BENCH_ARGS --graph 0" TAG=$TAG bash scripts/pmc.sh
